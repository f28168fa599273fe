"""Precompute (precompute_neighborhoods_topt, pinsage_model.py:109-132) wall
time and device time of the fused sampler at a bench config.

    python tools/precompute_probe.py [--config c2] [--rng philox|mt19937] [--reps 3]

Prints the cold (first) and warm wall times of the whole precompute, and the
HIP-event time of the sampler kernels (pinsage_ppr_topk over all sources)
alone, on the launch stream."""
import argparse
import contextlib
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "gcn-song-embeddings_amd"))
sys.path.insert(0, R)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rng", default="philox")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import bench
    import pinsage_model as pm
    cfg = bench.CONFIGS[a.config]
    pg, g, feats, pos = bench.build_problem(cfg)
    n = cfg["n_tracks"]
    pm.set_rng_mode(a.rng)
    for r in range(a.reps):
        torch.manual_seed(0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(sys.stderr):
            w, nb = pm.precompute_neighborhoods_topt(g, n, pm.DEF_HOPS, pm.DEF_ALPHA, pm.DEF_T_PRECOMP, None)
        torch.cuda.synchronize()
        print(f"precompute {a.config} {a.rng} rep {r}: wall {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    ids = torch.arange(n, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.reps):
        torch.manual_seed(0)
        e0.record()
        pm._ppr_topk_device(g, ids, pm.DEF_HOPS, pm.DEF_ALPHA, pm.DEF_T_PRECOMP,
                            philox=None if a.rng == "mt19937" else (1234, 0))
        e1.record()
        torch.cuda.synchronize()
        print(f"ppr_topk {n} sources x {pm.DEF_HOPS} hops, top-{pm.DEF_T_PRECOMP}: "
              f"{e0.elapsed_time(e1):.2f} ms (events, includes the host MT expansion in mt19937 mode)",
              flush=True)


if __name__ == "__main__":
    main()
