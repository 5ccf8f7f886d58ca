"""Copies one GPU session's rocprofv3 output into profiles/ and condenses the PMC passes.

    python tools/prof_summary.py TAG [--kernel k_link] [--workload c2_...] [--n-spans N]

Reads gpurun_out/prof_TAG/run_kernel_stats.csv (kernel-trace --stats) and the
FETCH_SIZE / WRITE_SIZE passes gpurun_out/pmc_{fetch,write}_TAG/run_counter_collection.csv,
writes profiles/TAG_kernel_stats.csv, profiles/TAG_pmc.json and (for the dominant
kernel) profiles/pmc_<kernel>.json, which bench.py reads for roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes). The factor 2 is the
gfx950 correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE counts 128-B requests at 64 B).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n.replace("zdl::", "")


def pmc(path: str) -> dict:
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    # the mean over the dispatches of the largest grid of work: a bench run also links smaller
    # batches with the same kernel (the putTrace leg's 1M-span puts), which must not dilute the
    # headline put's figure (dispatches within half of the largest value)
    def big_mean(v):
        top = max(v)
        w = [x for x in v if x >= 0.5 * top]
        return sum(w) / len(w)
    return {k: {c: big_mean(v) for c, v in d.items()} for k, d in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_link")
    ap.add_argument("--workload", default="c2_10M_spans_1M_traces_50_services")
    ap.add_argument("--n-spans", type=int, default=10001749)
    a = ap.parse_args()
    g = os.path.join(ROOT, "gpurun_out")
    p = os.path.join(ROOT, "profiles")
    os.makedirs(p, exist_ok=True)
    stats = os.path.join(g, f"prof_{a.tag}", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(p, f"{a.tag}_kernel_stats.csv"))
    stats3 = os.path.join(g, f"prof_c3_{a.tag}", "run_kernel_stats.csv")
    if os.path.exists(stats3):
        shutil.copy(stats3, os.path.join(p, f"{a.tag}_c3_kernel_stats.csv"))
    calib = os.path.join(g, f"calib_{a.tag}", "run_counter_collection.csv")
    if os.path.exists(calib):  # tools/calib_fetch: 1 GiB streamed once per load width
        cal = {}
        for r in csv.DictReader(open(calib)):
            n = r["Kernel_Name"]
            if "k_stream" in n:
                w = {"unsigned int": "4B", "unsigned long": "8B"}.get(n.split("<")[1].split(">")[0], "16B")
                cal[w + "_per_lane"] = {"bytes_read": 1 << 30, "fetch_size_bytes": float(r["Counter_Value"]) * 1024,
                                        "factor": (1 << 30) / (float(r["Counter_Value"]) * 1024)}
        json.dump(cal, open(os.path.join(p, f"{a.tag}_fetch_calibration.json"), "w"), indent=1)
    for f in ("gpu_tests", "smoke", "bench", "bench_c3"):
        src = os.path.join(g, f"{f}_{a.tag}.log")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(p, f"{a.tag}_{f}.log"))
    counters = {}
    for sub in os.listdir(g):
        if sub.startswith("pmc_") and sub.endswith(a.tag) and os.path.isdir(os.path.join(g, sub)):
            for k, d in pmc(os.path.join(g, sub, "run_counter_collection.csv")).items():
                counters.setdefault(k, {}).update(d)
    json.dump(counters, open(os.path.join(p, f"{a.tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    kern = [k for k in counters if k.startswith(a.kernel + "<") or k == a.kernel]
    if kern:
        d = counters[kern[0]]
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            fetch = d["FETCH_SIZE"] * 1024
            write = d["WRITE_SIZE"] * 1024
            out = {"kernel": kern[0], "workload": a.workload, "n_spans": a.n_spans, "tag": a.tag,
                   "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
                   "hbm_bytes_per_launch": 2 * fetch + write,
                   "note": "2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md §HBM; "
                           "the factor 2 holds for k_link's 4 and 8 B/lane loads too: profiles/*_fetch_calibration.json)"}
            json.dump(out, open(os.path.join(p, f"pmc_{a.kernel}.json"), "w"), indent=1)
            print(json.dumps(out))
    print(f"wrote profiles/{a.tag}_*")


if __name__ == "__main__":
    main()
