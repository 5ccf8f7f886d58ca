"""What zdl_reset's kernel costs the in-flight C2 step: the headline loop (two contexts in flight,
reset + put + link) against the same loop without the reset (counts accumulate: timing only).

    python tools/reset_probe.py [--steps 400]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    import torch
    from zipkin_amd import _native as N
    from zipkin_amd import synth
    w = synth.C2
    cols = synth.generate(w)
    dev = torch.device("cuda", 0)
    names = ("id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags")
    bs = []
    for _ in range(2):
        dc = {k: torch.from_numpy(np.ascontiguousarray(getattr(cols, k)).view(
            np.int64 if getattr(cols, k).dtype.itemsize == 8 else np.int32)).to(dev) for k in names}
        off = torch.from_numpy(cols.offsets.view(np.int64)).to(dev)
        p = {k: v.data_ptr() for k, v in dc.items()}
        p["timestamp"] = None
        bs.append((p, off, dc))
    torch.cuda.synchronize(dev)
    ctxs = [N.Context(w.total_services, device=0) for _ in range(2)]

    def run(k, reset):
        for i in range(k):
            c = ctxs[i % 2]
            if reset:
                c.reset()
            c.put_spans_device(bs[i % 2][0], cols.n_spans, bs[i % 2][1].data_ptr(), cols.n_traces)
            if i >= 1:
                ctxs[(i - 1) % 2].link(copy=False)
        ctxs[(k - 1) % 2].link(copy=False)
        for c in ctxs:
            c.sync()

    run(2000, True)  # warm
    for r in range(3):
        for reset in (True, False):
            t0 = time.perf_counter()
            run(a.steps, reset)
            print(f"reset={int(reset)} {(time.perf_counter() - t0) / a.steps * 1e3:.4f} ms/step", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
