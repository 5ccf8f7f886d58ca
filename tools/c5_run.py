"""C5 (BASELINE configs[4]) steps on one GPU for profiling: bench.py's c5_leg with a chosen
giant-tier threshold, printing the step time and the phase times as one JSON line.

    python tools/c5_run.py [--giant-min N] [--steps K] [--no-parity]
    rocprofv3 --kernel-trace --stats -d gpurun_out/c5 -o run -- python3 tools/c5_run.py --no-parity
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--giant-min", default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--host-threads", type=int, default=2, choices=(1, 2))
    a = ap.parse_args()
    if a.giant_min is not None:
        os.environ["ZDL_GIANT_MIN"] = str(a.giant_min)
    import bench
    r = bench.c5_leg(0, steps=a.steps, parity=not a.no_parity, host_threads=a.host_threads)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
