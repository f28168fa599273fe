"""Cosine kNN throughput (eval.py save_knn over PinSage embeddings, k = 1000):
all n rows of an [n, d] embedding table queried against the whole table.

    python tools/bench_knn.py [--n 100000] [--d 128] [--k 1000] [--reps 3]

Prints one JSON line: queries/s for the HIP path (pinsage_knn_cosine: fp32
MFMA dot products + per-row radix select), the roofline of its two phases
(GEMM 2*n*n*d FLOP vs fp32 MFMA peak; select bytes = 4 passes over each
query's row of n dot products + the final write) and the reference's CPU
restatement (baselines.py knn_from_emb, torch CPU) timed on a sample of
queries on the host cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gcn-song-embeddings_amd"))
sys.path.insert(0, REPO)

PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-queries", type=int, default=256)
    a = ap.parse_args()
    import baselines
    rng = np.random.default_rng(0)
    emb_h = torch.from_numpy(rng.standard_normal((a.n, a.d), dtype=np.float32))
    emb = emb_h.cuda()
    q = torch.arange(a.n, device="cuda")
    baselines.knn_from_emb(emb, q[:1024], a.k)  # warm-up (module load, allocator)
    torch.cuda.synchronize()
    times = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        w, nb = baselines.knn_from_emb(emb, q, a.k)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1e-3)
    t = min(times)
    flops = 2.0 * a.n * a.n * a.d
    sel_bytes = a.n * a.n * 4 * 4.0 + a.n * (a.k + 1) * 12
    res = {"metric": "cosine kNN queries/s (save_knn, k=1000)", "value": a.n / t, "unit": "queries/s",
           "n": a.n, "d": a.d, "k": a.k, "seconds": t,
           "bound_if_gemm_only_s": flops / (PEAK_FP32_TFLOPS * 1e12),
           "bound_if_select_hbm_only_s": sel_bytes / (PEAK_HBM_GBS * 1e9),
           "dtype": "f32", "data": "synthetic N(0,1) embeddings"}
    # reference restatement on the host (torch CPU, same ops as baselines.py:69-103)
    from oracle import oracle as orc
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    qs = np.arange(a.cpu_queries, dtype=np.int64)
    t0 = time.time()
    orc.knn_from_emb(emb_h, qs, a.k)
    tc = time.time() - t0
    res["cpu_baseline"] = {"value": a.cpu_queries / tc, "unit": "queries/s", "cores": threads,
                           "kind": "port", "sample": f"{a.cpu_queries} queries against all {a.n} rows"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
