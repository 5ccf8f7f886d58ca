"""Host-side cost of an insertion-order step at C2 (the DependencyLinker facade's context):
reset + put enqueue, link(ZDL_ORDER_INSERTION) after the put has finished, and the whole
serial step, each averaged over back-to-back repetitions.

    python tools/ord_host.py [--steps 50]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch

    from zipkin_amd import _native as N
    from zipkin_amd import synth
    from zipkin_amd.linker import _capacity

    w = synth.CONFIGS["c2"]
    cols = synth.generate(w)
    dev = torch.device("cuda", 0)
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags", "timestamp")
    dcols = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
        np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
    doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
    ptrs = {k: v.data_ptr() for k, v in dcols.items()}
    ptrs["timestamp"] = None
    torch.cuda.synchronize(dev)
    S = w.total_services
    rk = np.arange(S, dtype=np.int32)
    ctx = N.Context(_capacity(S), device=0, insertion_order=True)
    ctx.set_ranks(N.ZDL_DICT_SERVICE, rk)

    def put():
        ctx.reset()
        ctx.put_spans_device(ptrs, cols.n_spans, doff.data_ptr(), cols.n_traces)

    def timed(name, fn, pre=None, n=a.steps):
        ts = []
        for i in range(n + 3):
            if pre:
                pre()
                ctx.sync()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ctx.sync()
        print(f"{name:34s} {np.median(ts[3:]) * 1e6:8.1f} us median", flush=True)

    out = N.Links()
    timed("step (reset + put + link)", lambda: (put(), ctx.link(N.ZDL_ORDER_INSERTION)))
    timed("reset + put (enqueue only)", put, pre=lambda: None)
    timed("link() after a finished put", lambda: ctx.link(N.ZDL_ORDER_INSERTION), pre=put)
    timed("link(copy=False) after a put", lambda: ctx.link(N.ZDL_ORDER_INSERTION, copy=False), pre=put)
    timed("raw zdl_link after a put", lambda: ctx._L.zdl_link(ctx.h, N.ZDL_ORDER_INSERTION, N.C.byref(out)), pre=put)
    ctx.close()


if __name__ == "__main__":
    main()
