"""Per-site PMC summaries (HBM bytes and MFMA busy of fwd.q_gemm.l0,
fwd.aggw.l0, bwd.q_wgrad.l0) of one tools/profile_config.sh output directory,
written as profiles/<round>/pmc_<key>_<site>.json (bench.py reads them):

    python tools/pmc_sites_all.py gpurun_out/prof_c2 c2 profiles/r02
"""
import collections
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
TAGS = {"fwd.q_gemm.l0": "q_gemm", "fwd.aggw.l0": "aggw", "bwd.q_wgrad.l0": "q_wgrad"}


def occurrences(trace, kernel, grid):
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    holds = [i for i, r in enumerate(rows) if "stream_hold" in r["Kernel_Name"]]
    step = rows[holds[-1] + 1:]
    return [r for r in step if r["Kernel_Name"].replace("void ", "").split("(")[0] == kernel
            and int(r["Grid_Size_X"]) == grid]


def algo(bench, site):
    for key in ("roofline", "roofline_other"):  # (round 6: the bench line names both launches)
        r = bench.get(key) or {}
        if r.get("kernel", "").startswith(site):
            return r["algorithmic_bytes_per_launch"]
    if site == "fwd.q_gemm.l0":
        return bench["roofline"]["algorithmic_bytes_per_launch"]
    if site == "fwd.aggw.l0":
        return bench["gather_kernel"]["algorithmic_bytes"]
    U0, d = bench["frontier"]["U0_mean"], bench["config"]["d_in"]
    return 4.0 * (U0 * 512 + U0 * d + 512 * d + 512)


def main(prof, key, outdir):
    trace = os.path.join(prof, "stats", "run_kernel_trace.csv")
    sites = json.loads(subprocess.check_output([sys.executable, os.path.join(HERE, "site_kernels.py"), trace]))
    bench = json.load(open(os.path.join(prof, "bench.json")))
    for site, v in sites.items():
        occ = occurrences(trace, v["kernel"], v["grid"])
        stride = len(occ)
        # this site's position among its template + grid's launches in a step
        starts = sorted(int(r["Start_Timestamp"]) for r in occ)
        offset = 0 if site != "bwd.q_wgrad.l0" else stride - 1
        out = subprocess.check_output([
            sys.executable, os.path.join(HERE, "pmc_site.py"), "--config", key, "--site", site,
            "--kernel", v["kernel"].replace("ps::", ""),
            "--fetch", os.path.join(prof, "pmc_FETCH_SIZE", "run_counter_collection.csv"),
            "--write", os.path.join(prof, "pmc_WRITE_SIZE", "run_counter_collection.csv"),
            "--grid", str(v["grid"]), "--last", "5", "--stride", str(stride), "--offset", str(offset),
            "--algorithmic", str(algo(bench, site))])
        d = json.loads(out)
        cnt = collections.defaultdict(dict)
        dur = {}
        for r in csv.DictReader(open(os.path.join(prof, "pmc_SQ_VALU_MFMA_BUSY_CYCLES", "run_counter_collection.csv"))):
            if v["kernel"].replace("ps::", "") in r["Kernel_Name"] and int(r["Grid_Size"]) == v["grid"]:
                i = int(r["Dispatch_Id"])
                cnt[i][r["Counter_Name"]] = cnt[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                dur[i] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        keys = sorted(cnt)[-5 * stride:][offset::stride]
        if keys:
            busy = [cnt[i]["SQ_VALU_MFMA_BUSY_CYCLES"] / (cnt[i]["GRBM_GUI_ACTIVE"] / 8 * 1024) for i in keys]
            ghz = [cnt[i]["GRBM_GUI_ACTIVE"] / 8 / dur[i] / 1e9 for i in keys]
            d["mfma_busy"] = round(sum(busy) / len(busy), 3)
            d["mfma_busy_ghz"] = round(sum(ghz) / len(ghz), 2)
            d["mfma_busy_method"] = ("rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES (own "
                                     "pass): busy / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs), the last 5 launches of the site "
                                     "(eager timing pass), GEMM choices pinned to the stats run's")
        d["stats_run_us"] = v["us"]
        path = os.path.join(outdir, f"pmc_{key}_{TAGS[site]}.json")
        json.dump(d, open(path, "w"), indent=1)
        print(path, d["launches"], round(d["hbm_bytes_per_launch"] / 1e6, 1), "MB",
              round(d.get("traffic_over_algorithmic", 0), 2), d.get("mfma_busy"), v["us"])


if __name__ == "__main__":
    main(*sys.argv[1:4])
