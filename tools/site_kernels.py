"""(kernel, grid, duration) of the main bench sites in the last eager step of a
rocprofv3 kernel trace of bench.py (the per-kernel timing pass runs each step
eagerly behind a stream hold, after the timed graph replays):

    python tools/site_kernels.py gpurun_out/prof_c2/stats/run_kernel_trace.csv

fwd.q_gemm.l0 = the step's first gemm_f32_kernel<true, true, ...> (gathered
rows x Q^T), fwd.aggw.l0 = its first agg_w*_kernel, bwd.q_wgrad.l0 = the last
gemm_f32_kernel<false, false, ...> before the publish kernel (dQ0 closes the
backward on the main stream, pinsage engine_backward); with the long-K weight
gradients (wgrad.hip) it is the first wgrad_kw_kernel on the main queue after
that queue's last dq kernel (the side stream runs wgrad_kw_kernel launches of
the same grid for the other weights)."""
import csv
import json
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    holds = [i for i, r in enumerate(rows) if "stream_hold" in r["Kernel_Name"]]
    step = rows[holds[-1] + 1:]
    end = next((i for i, r in enumerate(step) if "step_publish" in r["Kernel_Name"]), len(step))
    step = step[:end]

    def rec(r):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        return {"kernel": name, "grid": int(r["Grid_Size_X"]),
                "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3}
    out = {}
    for r in step:
        n = r["Kernel_Name"]
        if "fwd.q_gemm.l0" not in out and "gemm_f32_kernel<true, true" in n:
            out["fwd.q_gemm.l0"] = rec(r)
        if "fwd.aggw.l0" not in out and "agg_w" in n:  # agg_w_kernel or agg_w32_kernel
            out["fwd.aggw.l0"] = rec(r)
        if "gemm_f32_kernel<false, false" in n:
            out["bwd.q_wgrad.l0"] = rec(r)
    dq = [i for i, r in enumerate(step) if "dq_combine_kernel" in r["Kernel_Name"] or "dq_chunk_kernel" in r["Kernel_Name"]]
    if dq:
        q = step[dq[-1]]["Queue_Id"] if "Queue_Id" in step[dq[-1]] else None
        for r in step[dq[-1] + 1:]:
            if "wgrad_kw_kernel" in r["Kernel_Name"] and (q is None or r.get("Queue_Id") == q):
                out["bwd.q_wgrad.l0"] = rec(r)
                break
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
