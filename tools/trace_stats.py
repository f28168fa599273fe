"""Per-kernel statistics keyed by (name, grid) from a rocprofv3 --kernel-trace
CSV (run_kernel_trace.csv), in the layout of --stats' kernel_stats.csv:

    python tools/trace_stats.py gpurun_out/prof_c2/stats/run_kernel_trace.csv > profiles/rNN/x_kernel_stats.csv
"""
import collections
import csv
import sys


def main(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in acc.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for (n, g), v in sorted(acc.items(), key=lambda x: -sum(x[1])):
        w.writerow([n, g, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
