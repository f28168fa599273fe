"""Per-kernel statistics from a rocprofv3 rocpd database (the default output
format of rocprofv3 on ROCm 7), in the column layout of `--stats`'
kernel_stats.csv, keyed by kernel name AND grid size so that launches of one
template with different shapes stay apart.

    python tools/rocpd_stats.py gpurun_out/prof_c2/run_results.db > profiles/rNN/x_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(db, by_grid=True):
    c = sqlite3.connect(db)
    key = "name, grid_x" if by_grid else "name"
    rows = c.execute(f"select name, {'grid_x' if by_grid else '0'}, count(*), sum(duration), "
                     f"min(duration), max(duration) from kernels group by {key} "
                     f"order by sum(duration) desc").fetchall()
    total = sum(r[3] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, grid, n, tot, mn, mx in rows:
        w.writerow([name, grid, n, tot, tot / n, 100.0 * tot / total, mn, mx])


if __name__ == "__main__":
    main(sys.argv[1], by_grid="--by-name" not in sys.argv)
