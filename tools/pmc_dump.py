"""Mean of every collected counter per kernel (name, grid) from rocprofv3 --pmc CSVs.

    rocprofv3 --pmc <counters> --output-format csv -d gpurun_out/pmcX -o run -- python3 ...
    python tools/pmc_dump.py gpurun_out/pmcX/run_counter_collection.csv [--match gemm_f32_kernel]

Also prints the mean dispatch duration and, when GRBM_GUI_ACTIVE is present, the
clock it implies (GUI_ACTIVE / 8 XCDs / duration).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--xcds", type=int, default=8)
    a = ap.parse_args()
    for path in a.csv:
        cnt = collections.defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(path)):
            if a.match not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            cnt[k][r["Counter_Name"]] = cnt[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[k] = (r["Kernel_Name"].split("(")[0].replace("void ", "")[:90], int(r["Grid_Size"]),
                       (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
        groups = collections.defaultdict(list)
        for k, c in sorted(cnt.items()):
            name, grid, dur = meta[k]
            groups[(name, grid)].append((dur, c))
        print(f"# {path}")
        for (name, grid), rows in groups.items():
            n = len(rows)
            dur = sum(r[0] for r in rows) / n
            print(f"{name} grid={grid} launches={n} dur_us={dur * 1e6:.2f}")
            keys = sorted(rows[0][1])
            for key in keys:
                v = sum(r[1].get(key, 0.0) for r in rows) / n
                extra = ""
                if key == "GRBM_GUI_ACTIVE":
                    extra = f"  clock_GHz={v / a.xcds / dur / 1e9:.3f}"
                print(f"  {key:32s} {v:16.4e}{extra}")


if __name__ == "__main__":
    main()
