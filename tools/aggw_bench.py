"""Microbenchmark of the aggregation + projection kernel (pinsage_conv_agg_project,
pinsage_model.py:195-210) on uniformly random slot lists (no reuse of popular
rows beyond chance: a lower bound on the in-step rate, where popular tracks'
q rows repeat).  Prints one JSON line per shape: µs per launch (HIP events,
median of repeats), algorithmic bytes (distinct q rows + slot lists + self rows
+ W planes + agg / y / norm writes) and logical bytes (every slot's row).

    python tools/aggw_bench.py [--shapes c2l0,c2l1,c4l0,c4sl0] [--reps 50]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gcn-song-embeddings_amd"))

SHAPES = {  # n_rows (F), d, hid, T, U (distinct q rows), h rows
    "c2l0": (5704, 512, 512, 10, 10550, 100000),
    "c2l1": (1450, 128, 512, 10, 4600, 5704),
    "c4l0": (8570, 128, 512, 10, 23190, 8000000),
    "c4sl0": (58640, 128, 512, 10, 151820, 8000000),
    "c3l0": (53000, 512, 512, 25, 200000, 1000000),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="c2l0,c2l1,c4l0,c4sl0")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--agg-only", action="store_true",
                    help="time the aggregation alone (pinsage_weighted_agg; PINSAGE_AGG_SLICED=0/1)")
    args = ap.parse_args()
    import _native as nat
    lib = nat.lib()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name in args.shapes.split(","):
        F, d, hid, T, U, nh = SHAPES[name]
        g = torch.Generator(device="cuda").manual_seed(1)
        h = torch.randn(nh, d, device="cuda", generator=g)
        q = torch.randn(U, hid, device="cuda", generator=g)
        loc = torch.randint(0, U, (F, T), device="cuda", generator=g, dtype=torch.int32)
        w = torch.rand(F, T, device="cuda", generator=g)
        self_src = torch.randint(0, nh, (F,), device="cuda", generator=g, dtype=torch.int32)
        W = torch.randn(128, d + hid, device="cuda", generator=g) * 0.05
        bias = torch.zeros(128, device="cuda")
        y = torch.empty(F, 128, device="cuda")
        nrm = torch.empty(F, device="cuda")
        agg = torch.empty(F, hid, device="cuda")
        planes = torch.empty(3 * 128 * (d + hid), dtype=torch.int16, device="cuda")

        def run_agg():
            nat.check(lib.pinsage_weighted_agg(vp(q), hid, vp(loc), vp(w), F, T, vp(agg), st), "weighted_agg")

        def run():
            if args.agg_only:
                return run_agg()
            nat.check(lib.pinsage_conv_agg_project(vp(h), d, d, vp(self_src), vp(q), hid, U, vp(loc), vp(w), F, T,
                                                   vp(W), vp(bias), 128, vp(planes), vp(y), vp(nrm), vp(agg), st),
                      "conv_agg_project")
        for _ in range(5):
            run()
        times = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b) * 1e3)
        times.sort()
        us = times[len(times) // 2]
        distinct = min(U, F * T)
        alg = distinct * hid * 4 + F * T * 8 + F * d * 4 + 128 * (d + hid) * 4 + F * (hid + 129) * 4
        logical = F * T * hid * 4 + F * T * 8 + F * d * 4 + F * (hid + 129) * 4
        if args.agg_only:
            alg = distinct * hid * 4 + F * T * 8 + F * hid * 4
            logical = F * T * hid * 4 + F * T * 8 + F * hid * 4
            print(json.dumps({"shape": name, "agg_only": True, "sliced": os.environ.get("PINSAGE_AGG_SLICED", "1"),
                              "us": round(us, 2), "alg_frac_hbm": round(alg / us / 1e3 / 8000, 3),
                              "logical_TBs": round(logical / us / 1e6, 2)}), flush=True)
            continue
        print(json.dumps({"shape": name, "F": F, "d": d, "T": T, "U": U, "us": round(us, 2),
                          "alg_GBs": round(alg / us / 1e3, 1), "alg_frac_hbm": round(alg / us / 1e3 / 8000, 3),
                          "logical_TBs": round(logical / us / 1e6, 2),
                          "tflops": round(2 * F * (d + hid) * 128 / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
