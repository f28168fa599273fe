"""MFMA-busy fraction per GEMM launch from one rocprofv3 --pmc pass.

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \\
        --output-format csv -d gpurun_out/pmc_mfma -o run -- python3 tools/gemm_bench.py ...
    python tools/pmc_mfma.py gpurun_out/pmc_mfma/run_counter_collection.csv [--match gemm_f32_kernel]

SQ_VALU_MFMA_BUSY_CYCLES sums, over all SIMDs, 64 cycles per v_mfma_f32_32x32x2_f32
(its issue time); GRBM_GUI_ACTIVE sums the active cycles of the 8 XCDs.  So
busy / (GUI_ACTIVE / 8 * 1024 SIMDs) is the fraction of the launch's SIMD-cycles
the matrix pipes were busy, and GUI_ACTIVE / 8 / duration is the clock held.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="gemm_f32_kernel")
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--last", type=int, default=0, help="keep each group's last N dispatches")
    a = ap.parse_args()
    cnt = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(a.csv)):
        if a.match not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        cnt[k][r["Counter_Name"]] = cnt[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"].split("(")[0].replace("void ", ""), int(r["Grid_Size"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    groups = collections.defaultdict(list)
    for k, c in sorted(cnt.items()):
        name, grid, dur = meta[k]
        cyc = c["GRBM_GUI_ACTIVE"] / a.xcds
        groups[(name, grid)].append((dur, c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * a.simds), cyc / dur / 1e9,
                                     c["SQ_VALU_MFMA_BUSY_CYCLES"] / 64))
    print(f"# {a.csv}: per kernel/grid, mean over launches")
    print(f"{'kernel':60s} {'grid':>8s} {'n':>3s} {'us':>8s} {'mfma_busy':>9s} {'GHz':>5s} {'mfma_insts':>11s}")
    for (name, grid), v in sorted(groups.items()):
        if a.last > 0:
            v = v[-a.last:]
        n = len(v)
        m = [sum(x[i] for x in v) / n for i in range(4)]
        print(f"{name:60s} {grid:8d} {n:3d} {m[0] * 1e6:8.1f} {m[1]:9.3f} {m[2]:5.2f} {m[3]:11.0f}")


if __name__ == "__main__":
    main()
