"""Prints a rocprofv3 kernel_stats.csv as name / calls / average us (the names hold commas)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:10.1f} us")
