"""Bisects a GPU/oracle link mismatch down to one trace and saves it (debugging aid).

    python tools/debug_bisect.py c5 20000 [max_size]

Runs the engine and the C++ restatement on the synthetic workload; on a mismatch, halves
the trace range until a single trace reproduces it, and writes its columns to
gpurun_out/bisect_<cfg>.npz.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref  # noqa: E402
from zipkin_amd import _native as N  # noqa: E402
from zipkin_amd import synth  # noqa: E402
from zipkin_amd.columnar import Columns  # noqa: E402

FIELDS = ("trace_lo", "id", "parent_id", "local_svc", "remote_svc", "local_ip4", "local_ip6", "port_flags",
          "timestamp")


def sub(cols, a, b):
    o = cols.offsets
    lo, hi = int(o[a]), int(o[b])
    return Columns(*(np.ascontiguousarray(getattr(cols, f)[lo:hi]) for f in FIELDS),
                   np.ascontiguousarray(o[a:b + 1] - o[a]))


def links_gpu(cols, S):
    ctx = N.Context(S)
    ctx.put_spans(cols)
    p, c, n, e = ctx.link()
    ctx.close()
    return sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def links_cpu(cols):
    st, p, c, n, e = ref.link(cols, threads=8)
    assert st == 0
    return sorted(zip(p.tolist(), c.tolist(), n.tolist(), e.tolist()))


def main():
    cfg, n = sys.argv[1], int(sys.argv[2])
    w = synth.CONFIGS[cfg].scaled(n)
    if len(sys.argv) > 3:
        w = synth.Workload(**{**w.__dict__, "max_size": int(sys.argv[3])})
    cols = synth.generate(w)
    S = w.total_services
    a, b = 0, cols.n_traces
    if links_gpu(cols, S) == links_cpu(cols):
        print("no mismatch")
        return
    while b - a > 1:
        m = (a + b) // 2
        if links_gpu(sub(cols, a, m), S) != links_cpu(sub(cols, a, m)):
            b = m
        elif links_gpu(sub(cols, m, b), S) != links_cpu(sub(cols, m, b)):
            a = m
        else:
            print(f"mismatch needs traces from both halves of [{a}, {b})")
            break
    one = sub(cols, a, b)
    print(f"traces [{a}, {b}): {one.n_spans} spans")
    print("gpu", links_gpu(one, S))
    print("cpu", links_cpu(one))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"bisect_{cfg}.npz"), offsets=one.offsets,
             **{f: getattr(one, f) for f in FIELDS})


if __name__ == "__main__":
    main()
