"""Prints per-kernel PMC averages from gpurun_out/<glob>/run_counter_collection.csv."""
import collections
import csv
import glob
import sys

pat, kern = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_link<")
for f in sorted(glob.glob(f"gpurun_out/{pat}/run_counter_collection.csv")):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[1], " ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(d.items())))
