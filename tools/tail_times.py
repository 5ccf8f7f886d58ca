"""Per-dispatch durations of the named kernels from a rocprofv3 kernel_trace.csv, in launch
order (run tail_cost.py under rocprofv3 --kernel-trace).

    python tools/tail_times.py gpurun_out/tc_x/run_kernel_trace.csv [k_tail] [per_group]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "k_tail"
    group = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    for g in range(0, len(d), group):
        part = d[g:g + group]
        print(f"{g // group}: " + " ".join(f"{x:9.1f}" for x in part) + f"   min {min(part):9.1f} us")


if __name__ == "__main__":
    main()
