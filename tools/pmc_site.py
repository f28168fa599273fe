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


def mean_counter(path, kernel, counter, grid=None, last=0, stride=1, offset=0):
    """Mean per dispatch of `counter` over the dispatches of `kernel` (and grid
    size); last > 0 keeps the last `last` dispatches only (bench.py's eager
    timing pass runs each site once per step at the end of the run, after the
    tuner's probe launches of the same templates)."""
    vals = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter and \
                (grid is None or int(r["Grid_Size"]) == grid):
            key = int(r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    keys = sorted(vals)[-last * stride:] if last > 0 else sorted(vals)
    # a template + grid launched `stride` times per step: this site is the
    # `offset`-th of them in dispatch order
    keys = keys[offset::stride]
    return (sum(vals[k] for k in keys) / len(keys), len(keys)) if keys else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--site", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--offset", type=int, default=0)
    ap.add_argument("--algorithmic", type=float, default=None,
                    help="algorithmic bytes per launch (bench.py), for the traffic ratio")
    a = ap.parse_args()
    f, nf = mean_counter(a.fetch, a.kernel, "FETCH_SIZE", a.grid, a.last, a.stride, a.offset)
    w, nw = mean_counter(a.write, a.kernel, "WRITE_SIZE", a.grid, a.last, a.stride, a.offset)
    out = {"config": a.config, "site": a.site, "kernel": a.kernel, "grid": a.grid, "launches": min(nf, nw),
           "fetch_size_kb": f, "write_size_kb": w,
           "hbm_bytes_per_launch": (2 * f + w) * 1024 if f is not None and w is not None else None,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "FETCH_SIZE doubled (gfx950 counts half of wide coalesced reads); KB = 1024 B"}
    if a.algorithmic and out["hbm_bytes_per_launch"]:
        out["algorithmic_bytes_per_launch"] = a.algorithmic
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / a.algorithmic
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
