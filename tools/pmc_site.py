"""HBM bytes per launch of one bench kernel site from rocprofv3 --pmc passes.

    python tools/pmc_site.py --config c2 --site fwd.q_gemm.l0 \\
        --kernel "gemm_f32_kernel<true, true, 2, 2, 1, 2, 32>" \\
        --fetch gpurun_out/pmc_fetch/run_counter_collection.csv \\
        --write gpurun_out/pmc_write/run_counter_collection.csv > profiles/rNN/pmc_c2_q_gemm.json

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one
pass's TCC slots); FETCH_SIZE is doubled (gfx950 counts half of wide
coalesced reads, MI355X_MICROARCH.md HBM section); sizes are KB = 1024 B.
Launches of the kernel are averaged (every launch of this template in the
bench is this site).
"""
import argparse
import csv
import json


def mean_counter(path, kernel, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            key = r.get("Dispatch_Id") or r.get("Correlation_Id") or len(vals)
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return (sum(vals.values()) / len(vals), len(vals)) if vals else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--site", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    a = ap.parse_args()
    f, nf = mean_counter(a.fetch, a.kernel, "FETCH_SIZE")
    w, nw = mean_counter(a.write, a.kernel, "WRITE_SIZE")
    out = {"config": a.config, "site": a.site, "kernel": a.kernel, "launches": min(nf, nw),
           "fetch_size_kb": f, "write_size_kb": w,
           "hbm_bytes_per_launch": (2 * f + w) * 1024 if f is not None and w is not None else None,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "FETCH_SIZE doubled (gfx950 counts half of wide coalesced reads); KB = 1024 B"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
