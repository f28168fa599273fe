"""Print one train step's kernel timeline from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv [--step -3]
    python tools/timeline.py gpurun_out/prof/run_results.db [--step -3]

Steps are delimited by the frontier's first kernel.  For the chosen step
every dispatch is listed with its queue, start offset and duration (µs)
relative to the step's first kernel, so gaps between dependent launches and
the overlap of the side streams are visible.
"""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"\(.*", "", n.replace("void ", ""))
    return n[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--delim", default="bits_top_set_kernel",
                    help="kernel that starts a step (the step ends before its next launch)")
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocpd database (rocprofv3's default output on ROCm 7)
        import sqlite3
        c = sqlite3.connect(a.trace)
        keys = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Grid_Size_X",
                "Workgroup_Size_X"]
        rows = [dict(zip(keys, r)) for r in
                c.execute("select name, start, end, queue_id, grid_x, workgroup_x from kernels")]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.delim in r["Kernel_Name"]]
    lo = starts[a.step - 1]
    k = starts[a.step] - 1
    t0 = int(rows[lo]["Start_Timestamp"])
    busy = 0
    last_end = t0
    for r in rows[lo:k + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"q{r['Queue_Id']:>2} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {grid:6d}  "
              f"{short(r['Kernel_Name'])}")
    total = (max(int(r["End_Timestamp"]) for r in rows[lo:k + 1]) - t0) / 1e3
    print(f"step span {total:.1f} us, some kernel running {busy / 1e3:.1f} us")


if __name__ == "__main__":
    main()
