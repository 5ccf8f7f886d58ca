"""Wall-clock breakdown of one bench step (reset / put / link) on the C2 batch.

    python tools/step_breakdown.py [--steps 50]

Each part is timed over `steps` back-to-back repetitions with a stream sync at the end,
without events, with the k_link events (ZDL_FLAG_TIMING) and with every kernel's
(ZDL_FLAG_TIMING_ALL), so launch gaps and host-side
costs show next to the kernel times of bench.py.
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
    ap.add_argument("--config", default="c2")
    ap.add_argument("--traces", type=int, default=0)
    a = ap.parse_args()
    import torch

    from zipkin_amd import _native as N
    from zipkin_amd import synth

    w = synth.CONFIGS[a.config]
    if a.traces:
        w = w.scaled(a.traces)
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

    def put(ctx):
        ctx.put_spans_device(ptrs, cols.n_spans, doff.data_ptr(), cols.n_traces)

    for timing in (0, 1, 2):
        ctx = N.Context(S, device=0, timing=timing == 1, timing_all=timing == 2)
        parts = {
            "reset": lambda: ctx.reset(),
            "put": lambda: put(ctx),
            "reset+put": lambda: (ctx.reset(), put(ctx)),
            "link": lambda: ctx.link(),
            "sync": lambda: ctx.sync(),
            "raw_link": lambda: ctx._L.zdl_link(ctx.h, N.ZDL_ORDER_SORTED, N.C.byref(N.Links())),
            "step": lambda: (ctx.reset(), put(ctx), ctx.link()),
        }
        for name, fn in parts.items():
            for _ in range(3):
                fn()
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fn()
            ctx.sync()
            dt = (time.perf_counter() - t0) / a.steps * 1e6
            print(f"timing={int(timing)} {name:10s} {dt:8.1f} us", flush=True)
        if timing == 2:
            kt = ctx.kernel_times()
            print("  kernel us: " + " ".join(f"{f}={getattr(kt, f) * 1e3:.1f}" for f in
                                             ("plan_ms", "tiles_ms", "full_ms", "reduce_ms", "big_ms", "compact_ms")))
        ctx.close()


if __name__ == "__main__":
    main()
