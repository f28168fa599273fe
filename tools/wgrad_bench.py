"""Microbenchmark of the long-K weight-gradient kernel (pinsage_wgrad, csrc/wgrad.hip)
against the split-K GEMM + slab reduction it replaced (pinsage_gemm_ex kEpiPartial),
on the engine's weight-gradient shapes, with HIP events on the launch stream.

    python tools/wgrad_bench.py [--reps 20]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gcn-song-embeddings_amd"))
import _native as nat  # noqa: E402

SHAPES = [  # name, M, N, K rows, gathered table rows (0: B ungathered)
    ("C2 dQ0", 512, 512, 10541, 100000),
    ("C2 dW0", 128, 1024, 5716, 100000),
    ("C4 dQ0", 512, 128, 15000, 8000000),
    ("C2 dQ0 ungathered", 512, 512, 10541, 0),
]


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    L = nat.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, M, N, K, R in SHAPES:
        n1 = N if name != "C2 dW0" else 512
        A = torch.randn(K, M, device="cuda")
        B = torch.randn(R if R else K, n1, device="cuda") if R < 2_000_000 else \
            torch.randn(R, n1, device="cuda")
        B2 = torch.randn(K, N - n1, device="cuda") if n1 < N else None
        idx = torch.randint(0, R, (K,), device="cuda", dtype=torch.int32).sort().values if R else None
        K_dev = torch.tensor([K], dtype=torch.int32, device="cuda")
        dst = torch.empty(M, N, device="cuda")
        db = torch.empty(M, device="cuda")
        sc = torch.zeros(int(L.pinsage_wgrad_scratch_bytes(M, N)), dtype=torch.uint8, device="cuda")
        res = {}
        for S in (0, 2, 4, 8, 16):
            def kw():
                nat.check(L.pinsage_wgrad(M, N, vp(K_dev), K, vp(A), M, vp(B), n1, vp(idx), n1 if B2 is not None else -1,
                                          vp(B2), (N - n1) if B2 is not None else 0, vp(dst), N, vp(db), S, vp(sc),
                                          None, None, None, None, None, None, None, 0.9, 0.999, 1e-8, st), "wgrad")
            res[f"kw S={S or 'auto'}"] = timed(kw, a.reps)
        os.environ["PINSAGE_KW_FORM"] = "1"  # 4 waves, 64-KiB ring
        for S in (0, 4, 8, 16):
            res[f"f1 S={S or 'auto'}"] = timed(lambda: nat.check(L.pinsage_wgrad(
                M, N, vp(K_dev), K, vp(A), M, vp(B), n1, vp(idx), n1 if B2 is not None else -1, vp(B2),
                (N - n1) if B2 is not None else 0, vp(dst), N, vp(db), S, vp(sc), None, None, None, None, None,
                None, None, 0.9, 0.999, 1e-8, st), "wgrad"), a.reps)
        os.environ.pop("PINSAGE_KW_FORM")
        os.environ["PINSAGE_KW_WAVES"] = "1"  # the register-ring k loop
        for S in (0, 4, 8):
            res[f"reg S={S or 'auto'}"] = timed(lambda: nat.check(L.pinsage_wgrad(
                M, N, vp(K_dev), K, vp(A), M, vp(B), n1, vp(idx), n1 if B2 is not None else -1, vp(B2),
                (N - n1) if B2 is not None else 0, vp(dst), N, vp(db), S, vp(sc), None, None, None, None, None,
                None, None, 0.9, 0.999, 1e-8, st), "wgrad"), a.reps)
        os.environ.pop("PINSAGE_KW_WAVES")
        if n1 == N:  # timing-only k loops (pinsage_wgrad_probe: results wrong by construction)
            for probe in (1, 2, 3, 4):
                res[f"probe{probe} S=auto"] = timed(lambda: nat.check(L.pinsage_wgrad_probe(
                    M, N, vp(K_dev), K, vp(A), vp(B), vp(idx), vp(dst), vp(db), 0, vp(sc), probe, st),
                    "wgrad_probe"), a.reps)
        if n1 == N:  # both operands pre-split (pinsage_wgrad_planes)
            A3 = torch.empty((3, A.shape[0], M), dtype=torch.int16, device="cuda")
            B3 = torch.empty((3, B.shape[0], N), dtype=torch.int16, device="cuda")
            nat.check(L.pinsage_split_planes(vp(A), A.shape[0], M, M, vp(A3), st), "split")
            nat.check(L.pinsage_split_planes(vp(B), B.shape[0], N, N, vp(B3), st), "split")
            for S in (0, 4, 8):
                res[f"planes S={S or 'auto'}"] = timed(lambda: nat.check(L.pinsage_wgrad_planes(
                    M, N, vp(K_dev), K, vp(A3), A3[0].numel(), M, vp(B3), B3[0].numel(), N, vp(idx), vp(dst), N,
                    vp(db), S, vp(sc), st), "wgrad_planes"), a.reps)
            del A3, B3
        flops = 2.0 * M * N * K
        print(name, {k: f"{v:.1f} us {flops / v / 1e6:.0f} TF/s" for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
