"""Runs one synthetic batch through the engine many times and counts runs whose links
differ from the C++ restatement (nondeterminism hunt; debugging aid).

    python tools/debug_repeat.py c5 20000 50 [max_size]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ref  # noqa: E402
from zipkin_amd import _native as N  # noqa: E402
from zipkin_amd import synth  # noqa: E402


def main():
    cfg, n, reps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    w = synth.CONFIGS[cfg].scaled(n)
    if len(sys.argv) > 4:
        w = synth.Workload(**{**w.__dict__, "max_size": int(sys.argv[4])})
    cols = synth.generate(w)
    st, op, oc, on, oe = ref.link(cols, threads=8)
    exp = sorted(zip(op.tolist(), oc.tolist(), on.tolist(), oe.tolist()))
    ctx = N.Context(w.total_services)
    bad = 0
    for r in range(reps):
        ctx.reset()
        ctx.put_spans(cols)
        p, c, k, e = ctx.link()
        got = sorted(zip(p.tolist(), c.tolist(), k.tolist(), e.tolist()))
        if got != exp:
            bad += 1
            ge, ee = set(got), set(exp)
            print(f"run {r}: gpu-only {sorted(ge - ee)[:4]} cpu-only {sorted(ee - ge)[:4]}", flush=True)
    ctx.close()
    print(f"{cfg}: {bad}/{reps} runs differ ({cols.n_spans} spans, {len(exp)} links)", flush=True)


if __name__ == "__main__":
    main()
