"""Microbenchmark of the fp32 MFMA GEMM through the C-ABI (pinsage_gemm_ex).

    python tools/gemm_bench.py [--reps 50] [--shapes M,N,K,ak,bk[,gather] ...]

Times each shape under every tile configuration (and the size-based pick)
with HIP events on the launch stream; prints µs per launch and TF/s.  The
default shapes are the C2 train step's projections (bench.py config c2).
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gcn-song-embeddings_amd"))
import _native as nat  # noqa: E402

DEFAULT = [
    "10541,512,512,1,1,1",    # fwd Q l0: gathered h rows x Q^T
    "5716,128,1024,1,1,1",    # fwd W l0 (first K segment gathered)
    "2600,512,128,1,1,1",     # fwd Q l1
    "1500,128,640,1,1,1",     # fwd W l1
    "5716,1024,128,1,0,0",    # bwd dcat l0 = dY W
    "10541,512,512,1,0,0",    # bwd dh l0 = dpq Q (scatter-add in the engine)
    "8192,512,512,1,1,0",     # reference square-ish shape: 512 tiles of 64x128
]


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def run(shape, cfg, sk, reps, lib, stream, pool=0, sets=1, bias_act=False, sort_idx=False, presplit=False,
        graph=False):
    # M,N,K,ak,bk[,gather[,splits]]: gather = rows of A (K-major A) or k-rows
    # of B (N-major B, the weight-gradient form); splits > 1 = split-K slabs
    M, N, K, ak, bk, *g = [int(x) for x in shape.split(",")]
    gather = bool(g and g[0])
    splits = g[1] if len(g) > 1 else 1
    dev = "cuda"
    rows = max(M, pool) if (ak and gather) else M
    A = torch.randn((rows if ak else K), (K if ak else M), device=dev)
    B = torch.randn((N if bk else K), (K if bk else N), device=dev)
    C = torch.empty(splits, M, N, device=dev)
    # pool > M: gathered rows from a larger table, `sets` different row sets
    # cycled over the repetitions (cold: sets x M rows exceed the Infinity Cache)
    idx_sets = [torch.randperm(rows, device=dev)[:M].to(torch.int32) for _ in range(sets)] \
        if gather and ak else [None]
    if sort_idx and idx_sets[0] is not None:  # the frontier's sorted distinct rows
        idx_sets = [ix.sort().values for ix in idx_sets]
    bias = torch.randn(N, device=dev) if bias_act else None
    a_idx = idx_sets[0]
    b_idx = torch.randperm(K, device=dev).to(torch.int32) if gather and not ak and not bk else None
    args = (M, N, K, ak, bk, vp(A), A.shape[1], vp(a_idx), vp(B), B.shape[1], vp(b_idx), vp(C), N,
            vp(bias), int(bias_act), 3 if splits > 1 else 0, splits, cfg, sk, ctypes.c_void_p(stream.cuda_stream))
    call = lib.pinsage_gemm_ex
    if presplit == "ilv":  # the A table and W as interleaved plane tables (pinsage_split_ilv), A's split once
        assert ak and bk and splits == 1 and sk == 0
        cs0 = ctypes.c_void_p(stream.cuda_stream)
        at = torch.empty(A.shape[0], 3 * K, dtype=torch.int16, device=dev)
        wt = torch.empty(N, 3 * K, dtype=torch.int16, device=dev)
        nat.check(lib.pinsage_split_ilv(vp(A), A.shape[1], A.shape[0], K, vp(at), 3 * K, cs0), "split A")
        nat.check(lib.pinsage_split_ilv(vp(B), B.shape[1], N, K, vp(wt), 3 * K, cs0), "split W")
        args = (vp(at), 3 * K, vp(a_idx), M, None, M, K, vp(B), vp(wt), 3 * K, vp(bias), N, int(bias_act), vp(C), N,
                cs0)
        call = lib.pinsage_linear_ilv
        ai = 2
    elif presplit:  # B (K-major, [N][K]) read as pre-split bf16 planes: pinsage_linear_split_b
        assert ak and bk and splits == 1 and sk == 0, "pre-split B: K-major operands, no split-K/stream-K"
        planes = torch.empty(3, N, K, dtype=torch.int16, device=dev)
        nat.check(lib.pinsage_split_planes(vp(B), N, K, K, vp(planes), ctypes.c_void_p(stream.cuda_stream)),
                  "split_planes")
        args = (vp(A), A.shape[1], vp(a_idx), M, K, vp(B), vp(planes), K, vp(bias), N, int(bias_act), vp(C),
                N, cfg, ctypes.c_void_p(stream.cuda_stream))
        call = lib.pinsage_linear_split_b
    rc = call(*args)
    if rc != 0:
        raise RuntimeError(lib.pinsage_last_error().decode())
    ref = ((A[a_idx.long()] if a_idx is not None else A) if ak else A.t()).double()
    ref = ref @ ((B.t() if bk else (B[b_idx.long()] if b_idx is not None else B))).double()
    if bias_act:
        ref = torch.nn.functional.leaky_relu(ref + bias.double())
    err = ((C.sum(0).double() - ref).norm() / ref.norm()).item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        call(*args)
    if presplit != "ilv":
        ai = 2 if presplit else 7  # position of a_idx
    all_args = [tuple(vp(ix) if i == ai else a for i, a in enumerate(args)) for ix in idx_sets] \
        if idx_sets[0] is not None else [args]
    if graph:  # the reps captured once and replayed: device time without the host's launch rate
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                cs = ctypes.c_void_p(side.cuda_stream)
                for r in range(reps):
                    a = all_args[r % len(all_args)]
                    call(*(a[:-1] + (cs,)))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
    else:
        e0.record(stream)
        for r in range(reps):
            call(*all_args[r % len(all_args)])
        e1.record(stream)
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    return us, 2.0 * M * N * K / us / 1e6, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shapes", nargs="*", default=DEFAULT)
    ap.add_argument("--cfgs", default="-1,0,1,2")
    ap.add_argument("--sk", default="0,1", help="stream-K settings (-1 auto, 0 off, 1 on)")
    ap.add_argument("--pool", type=int, default=0, help="rows of the gathered table (0 = M)")
    ap.add_argument("--sets", type=int, default=1, help="row sets cycled over repetitions")
    ap.add_argument("--bias-act", action="store_true", help="bias + LeakyReLU epilogue (the Q projection)")
    ap.add_argument("--sorted", action="store_true", help="gathered rows in ascending order")
    ap.add_argument("--graph", action="store_true", help="time a hipGraph of the reps (no host launch rate)")
    ap.add_argument("--prec", default="1",
                    help="product arithmetic(s): 0 fp32 MFMA, 1 split bf16, 2 split bf16 with pre-split B planes, "
                         "3 interleaved plane tables of A (split once) and W (pinsage_linear_ilv)")
    a = ap.parse_args()
    lib = nat.lib()
    stream = torch.cuda.current_stream()
    for s in a.shapes:
      for prec in [int(x) for x in a.prec.split(",")]:
        lib.pinsage_gemm_set_prec(min(prec, 1))
        for cfg in [int(c) for c in a.cfgs.split(",")]:
            for sk in [int(c) for c in a.sk.split(",")]:
                if sk == 1 and cfg == 0:
                    continue
                us, tf, err = run(s, cfg, sk, a.reps, lib, stream, a.pool, a.sets, a.bias_act, a.sorted,
                                  presplit="ilv" if prec == 3 else prec == 2, graph=a.graph)
                print(f"{s:24s} prec={prec} cfg={cfg:2d} sk={sk:2d} {us:9.2f} us {tf:7.1f} TF/s  relerr={err:.2e}",
                      flush=True)


if __name__ == "__main__":
    main()
