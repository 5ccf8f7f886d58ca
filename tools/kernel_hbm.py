"""Per-kernel achieved HBM GB/s against the MI355X peak, from one rocprofv3 kernel-trace stats
run (durations) and two PMC runs of the same command (FETCH_SIZE, WRITE_SIZE; one counter block
each). HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB): the gfx950 FETCH_SIZE
correction calibrated by tools/calib_fetch.hip for 4/8/16-B lanes (MI355X_MICROARCH.md, HBM).

    python tools/kernel_hbm.py STATS_CSV FETCH_DIR WRITE_DIR [--json OUT] [--label L]

STATS_CSV: rocprofv3 --stats kernel_stats.csv; FETCH_DIR / WRITE_DIR: -d directories of the PMC
runs (their *counter_collection.csv is found below them).
"""
import argparse
import collections
import csv
import json
import os

PEAK_GBS = 8000.0


def short(name: str) -> str:
    n = name.split("(")[0]
    for p in ("void ", "zdl::", "zp3::zjs::", "zp3::", "rocprim::detail::", "(anonymous namespace)::"):
        n = n.replace(p, "")
    return n[:70]


def counters(d: str, counter: str):
    per = collections.defaultdict(list)
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    if r["Counter_Name"] == counter:
                        per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--json", default=None)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    fetch, write = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
    rows = []
    for r in csv.DictReader(open(a.stats)):
        name = r["Name"]
        ns = float(r["AverageNs"])
        f, w = fetch.get(name), write.get(name)
        hbm = 2 * f + w if f is not None and w is not None else None
        gbs = hbm / ns if hbm is not None and ns > 0 else None  # bytes / ns = GB/s
        rows.append({"kernel": short(name), "calls": int(r["Calls"]), "avg_us": ns / 1e3,
                     "total_us": float(r["TotalDurationNs"]) / 1e3, "hbm_bytes_per_launch": hbm,
                     "hbm_gbs": gbs, "frac_of_8tbs": gbs / PEAK_GBS if gbs is not None else None})
    rows.sort(key=lambda x: -x["total_us"])
    print(f"{'kernel':70s} {'calls':>5s} {'avg us':>9s} {'MB/launch':>10s} {'GB/s':>7s} {'frac':>6s}")
    for x in rows:
        mb = f"{x['hbm_bytes_per_launch'] / 1e6:10.1f}" if x["hbm_bytes_per_launch"] is not None else f"{'-':>10s}"
        g = f"{x['hbm_gbs']:7.0f} {x['frac_of_8tbs']:6.3f}" if x["hbm_gbs"] is not None else f"{'-':>7s} {'-':>6s}"
        print(f"{x['kernel']:70s} {x['calls']:5d} {x['avg_us']:9.1f} {mb} {g}")
    if a.json:
        json.dump({"label": a.label, "peak_gbs": PEAK_GBS, "how": "durations: rocprofv3 --kernel-trace --stats; "
                   "HBM bytes: 2 x FETCH_SIZE + WRITE_SIZE from separate --pmc runs of the same command",
                   "kernels": rows}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
