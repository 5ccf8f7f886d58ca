"""The drop-in facades' device work at C2, for rocprofv3 --kernel-trace --stats: the
insertion-order link the DependencyLinker facade runs (its _capacity context, service ranks) and
InMemoryStorage.get_dependencies(endTs, lookback).execute() over a store holding the batch, each
`--reps` times after a warm-up, with host wall clock per phase printed.

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python3 tools/facade_prof.py
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from zipkin_amd import _native as N  # noqa: E402
from zipkin_amd import synth  # noqa: E402
from zipkin_amd.linker import _capacity  # noqa: E402
from zipkin_amd.storage import InMemoryStorage  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--traces", type=int, default=1_000_000)
    ap.add_argument("--no-store", action="store_true")
    ap.add_argument("--no-ord", action="store_true")
    a = ap.parse_args()
    import torch
    w = synth.C2.scaled(a.traces)
    cols = synth.generate(w)
    S = w.total_services
    names = synth.service_names(w)
    dev = torch.device("cuda", 0)
    keep = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev)
        for k in ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags", "timestamp")}
    doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
    ptrs = {k: v.data_ptr() for k, v in keep.items()}
    ptrs["timestamp"] = None
    torch.cuda.synchronize()
    if not a.no_ord:
        ictx = N.Context(_capacity(S), device=0, insertion_order=True)
        rk = np.empty(S, np.int32)
        rk[np.argsort(np.array(names, dtype=object), kind="stable")] = np.arange(S, dtype=np.int32)
        ictx.set_ranks(N.ZDL_DICT_SERVICE, rk)
        ts = []
        for r in range(a.reps + 1):
            t0 = time.perf_counter()
            ictx.reset()
            ictx.put_spans_device(ptrs, cols.n_spans, doff.data_ptr(), cols.n_traces)
            ictx.link(N.ZDL_ORDER_INSERTION)
            ts.append(time.perf_counter() - t0)
        ictx.close()
        print(f"insertion order step ms: {' '.join(f'{t * 1e3:.3f}' for t in ts[1:])}", flush=True)
    if not a.no_store:
        end_ms = int(cols.timestamp.max()) // 1000 + 1
        lookback = end_ms - int(cols.timestamp.min()) // 1000 + 1
        ims = InMemoryStorage(max_span_count=max(cols.n_spans, 500000), device=0)
        for nm in names:
            ims._linker.svc.id(nm)
        ims._st().append(cols)
        ims.get_dependencies(end_ms, lookback).execute()
        st = ims._st()
        ts, ss = [], []
        for r in range(a.reps):
            t0 = time.perf_counter()
            ims.get_dependencies(end_ms, lookback).execute()
            ts.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            st.select(N.ZDL_SELECT_NEWEST)
            ss.append(time.perf_counter() - t0)
        ims.close()
        print(f"facade get_dependencies ms: {' '.join(f'{t * 1e3:.3f}' for t in ts)}", flush=True)
        print(f"select ms: {' '.join(f'{t * 1e3:.3f}' for t in ss)}", flush=True)


if __name__ == "__main__":
    main()
