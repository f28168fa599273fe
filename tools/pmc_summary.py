"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc1/{fetch,write,sq}/run_counter_collection.csv

Kernels are keyed by (name, grid size) so launches of one template with
different shapes stay apart.  FETCH_SIZE/WRITE_SIZE are rocprofv3's KB units;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads
(MI355X_MICROARCH.md, HBM), so `fetch_bytes_x2` doubles it.
"""
import collections
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name.replace("void ", ""))
    return name[:70]


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for key, cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        rows.append((key, n, d))
    rows.sort(key=lambda x: -x[2].get("SQ_WAVE_CYCLES", x[2].get("FETCH_SIZE", 0)))
    for (name, grid), n, d in rows:
        extra = ""
        if "FETCH_SIZE" in d:
            extra += f" fetch_bytes_x2={2 * d['FETCH_SIZE'] * 1024:.3e}"
        if "WRITE_SIZE" in d:
            extra += f" write_bytes={d['WRITE_SIZE'] * 1024:.3e}"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "GRBM_GUI_ACTIVE" in d and d["GRBM_GUI_ACTIVE"] > 0:
            extra += f" mfma_busy/gui={d['SQ_VALU_MFMA_BUSY_CYCLES'] / d['GRBM_GUI_ACTIVE']:.3f}"
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"] > 0:
            w = d["SQ_WAVE_CYCLES"]
            extra += (f" wait={d.get('SQ_WAIT_ANY', 0) / w:.2f} issue_stall="
                      f"{d.get('SQ_WAIT_INST_ANY', 0) / w:.2f} active={d.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")
        print(f"{name:70s} grid={grid:8d} n={n:4d}{extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
