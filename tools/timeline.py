"""Prints a rocprofv3 kernel(+memory-copy) trace as a timeline: start-end (ms from the first
event), kernel name, queue and stream - the events longer than --min-us, optionally only those
between the N-th and M-th launch of a marker kernel (to look at steps in flight).

    python tools/timeline.py DIR [--min-us 60] [--marker k_link] [--from 3] [--to 5]
"""
import argparse
import csv
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=60)
    ap.add_argument("--marker", default=None)
    ap.add_argument("--from", dest="a", type=int, default=0)
    ap.add_argument("--to", dest="b", type=int, default=10 ** 9)
    x = ap.parse_args()
    ev = []
    for f in ("run_kernel_trace.csv", "run_memory_copy_trace.csv"):
        p = os.path.join(x.dir, f)
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name") or ("copy " + r.get("Direction", ""))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0][:48],
                       r.get("Queue_Id", "-"), r.get("Stream_Id", "-")))
    ev.sort()
    t0 = ev[0][0]
    lo, hi = ev[0][0], ev[-1][1]
    if x.marker:
        m = [e for e in ev if x.marker in e[2]]
        lo = m[min(x.a, len(m) - 1)][0] - 1_000_000
        hi = m[min(x.b, len(m) - 1)][0]
    for s, e, n, q, st in ev:
        if lo <= s <= hi and (e - s) / 1e3 >= x.min_us:
            print(f"{(s - t0) / 1e6:10.3f} - {(e - t0) / 1e6:10.3f}  {(e - s) / 1e3:8.1f} us  {n:48s} q{q} s{st}")


if __name__ == "__main__":
    main()
