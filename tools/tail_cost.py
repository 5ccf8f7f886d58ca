"""k_tail cost model: put time for workloads whose traces all have n spans (n > 64: every
trace is k_tail's big-trace path). Prints one JSON line per n: traces, spans, ms per put,
us per trace per workgroup (x 256 CUs), ns per span.

    python tools/tail_cost.py [--sizes 65,128,...] [--services 10000]
"""
import argparse
import json
import os
import sys
import time
from dataclasses import replace

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="65,128,256,512,1024,2048,8192,32768,131072")
    ap.add_argument("--services", type=int, default=10000)
    ap.add_argument("--spans", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from zipkin_amd import _native as N
    from zipkin_amd import synth
    dev = torch.device("cuda", 0)
    for n in [int(x) for x in args.sizes.split(",")]:
        T = max(256, min(200_000, args.spans // n))
        w = replace(synth.C5, n_traces=T, n_services=args.services, size_dist=2, max_size=n)
        cols = synth.generate(w)
        names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
        d = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
            np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
        doff = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
        ptrs = {k: v.data_ptr() for k, v in d.items()}
        ptrs["timestamp"] = None
        ctx = N.Context(w.total_services, device=0)
        torch.cuda.synchronize(dev)
        best = 1e9
        for r in range(args.reps + 1):
            ctx.reset()
            ctx.sync()
            t0 = time.perf_counter()
            ctx.put_spans_device(ptrs, cols.n_spans, doff.data_ptr(), cols.n_traces)
            ctx.sync()
            dt = time.perf_counter() - t0
            if r:
                best = min(best, dt)
        links = ctx.link()
        print(json.dumps({"n": n, "traces": T, "spans": int(cols.n_spans), "ms": best * 1e3,
                          "us_per_trace_wg": best * 1e6 * 256 / T, "ns_per_span": best * 1e9 / cols.n_spans,
                          "links": len(links[0]) if isinstance(links, tuple) else len(links)}), flush=True)
        del ctx, d, doff


if __name__ == "__main__":
    main()
