"""The fp32 MFMA GEMM behind every projection (pinsage_model.py:196,201,208,
211,223-224 forward; their autograd products backward) through the C-ABI
entry pinsage_gemm_ex: every operand layout x tile configuration x schedule
(data-parallel tiles / stream-K), ragged shapes, gathered rows, epilogues,
against an fp64 product of the same fp32 operands.  Tolerance: the north
star's 1e-4 relative (Frobenius), and stream-K results must be bitwise
repeatable (its combine order is fixed, whichever workgroup arrives last).
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _gemm(M, N, K, ak, bk, A, a_idx, B, C, bias=None, act=0, epi=0, splits=1, cfg=-1, sk=0, b_idx=None):
    import _native as nat
    lib = nat.lib()
    rc = lib.pinsage_gemm_ex(M, N, K, ak, bk, _vp(A), A.shape[1], _vp(a_idx), _vp(B), B.shape[1],
                             _vp(b_idx), _vp(C), C.shape[-1], _vp(bias), act, epi, splits, cfg, sk,
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    nat.check(rc, "gemm_ex")


def _ref(M, N, K, ak, bk, A, a_idx, B, bias, act):
    A64, B64 = A.double(), B.double()
    if ak:
        a = A64[a_idx.long()] if a_idx is not None else A64[:M]
    else:
        a = A64[:K, :M].t()
    b = B64[:N, :K].t() if bk else B64[:K, :N]
    r = a @ b
    if bias is not None:
        r = r + bias.double()
    if act:
        r = torch.nn.functional.leaky_relu(r, 0.01)
    return r


def _rel(x, r):
    return ((x.double() - r).norm() / r.norm().clamp_min(1e-30)).item()


SHAPES = [  # M, N, K: ragged M / K tails, N = 128 and multi-tile N, long K
    (1, 128, 4),
    (37, 128, 132),
    (200, 256, 516),
    (1000, 384, 128),
    (64 * 9 + 5, 128, 2048),
    (3000, 512, 512),
]


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("sk", [0, 1])
def test_gemm_layouts_configs_schedules(ak, bk, cfg, sk):
    """Every block-tile config (0: 128x128x16, 1: 64x128x32, 2: 32x128x32,
    3: 64x128x16 three per CU, 4: four per CU -- K-major operands only, other
    layouts are refused) under both schedules."""
    if sk and cfg == 0:
        pytest.skip("stream-K runs the 64- and 32-row tiles")
    if cfg == 4 and not (ak and bk):
        A = torch.randn(64, 64, device="cuda")
        C = torch.empty(64, 64, device="cuda")
        with pytest.raises(RuntimeError, match="cfg 4"):
            _gemm(64, 64, 64, ak, bk, A, None, A, C, cfg=4, sk=sk)
        return
    g = torch.Generator(device="cuda").manual_seed(1234 + 10 * cfg + sk)
    for M, N, K in SHAPES:
        if not ak and M % 4:
            M += 4 - M % 4  # M-major A needs M % 4 == 0 (launch_gemm)
        A = torch.randn((M, K) if ak else (K, M), device="cuda", generator=g)
        B = torch.randn((N, K) if bk else (K, N), device="cuda", generator=g)
        a_idx = None
        if ak and M > 1:
            a_idx = torch.randint(0, M, (M,), device="cuda", generator=g, dtype=torch.int32)
        bias = torch.randn(N, device="cuda", generator=g)
        C = torch.full((M, N), float("nan"), device="cuda")
        _gemm(M, N, K, ak, bk, A, a_idx, B, C, bias=bias, act=1, cfg=cfg, sk=sk)
        torch.cuda.synchronize()
        r = _ref(M, N, K, ak, bk, A, a_idx, B, bias, 1)
        assert torch.isfinite(C).all(), (M, N, K)
        assert _rel(C, r) < REL_TOL, (M, N, K, _rel(C, r))


@pytest.mark.parametrize("cfg", [1, 2])
def test_stream_k_accumulate_and_repeatable(cfg):
    # few tiles, long K: many workgroups per tile, combine by the last arriver
    g = torch.Generator(device="cuda").manual_seed(7)
    M, N, K = 100, 256, 8192
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g)
    C0 = torch.randn(M, N, device="cuda", generator=g)
    outs = []
    for _ in range(3):
        C = C0.clone()
        _gemm(M, N, K, 1, 1, A, None, B, C, epi=1, cfg=cfg, sk=1)
        outs.append(C)
    torch.cuda.synchronize()
    r = C0.double() + A.double() @ B.double().t()
    assert _rel(outs[0], r) < REL_TOL
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_stream_k_matches_data_parallel_schedule():
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = 10541, 512, 512
    A = torch.randn(M, K, device="cuda", generator=g)
    idx = torch.randint(0, M, (M,), device="cuda", generator=g, dtype=torch.int32)
    B = torch.randn(N, K, device="cuda", generator=g)
    C_dp = torch.empty(M, N, device="cuda")
    C_sk = torch.empty(M, N, device="cuda")
    _gemm(M, N, K, 1, 1, A, idx, B, C_dp, cfg=1, sk=0)
    _gemm(M, N, K, 1, 1, A, idx, B, C_sk, cfg=1, sk=1)
    torch.cuda.synchronize()
    r = A.double()[idx.long()] @ B.double().t()
    assert _rel(C_dp, r) < REL_TOL and _rel(C_sk, r) < REL_TOL
    assert ((C_dp - C_sk).abs().max() / r.abs().max()).item() < 1e-5


def test_split_k_partials():
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, K, S = 128, 256, 3000, 6  # M-major A, N-major B: weight-gradient form
    A = torch.randn(K, M, device="cuda", generator=g)
    B = torch.randn(K, N, device="cuda", generator=g)
    C = torch.empty(S, M, N, device="cuda")
    _gemm(M, N, K, 0, 0, A, None, B, C, epi=3, splits=S)
    torch.cuda.synchronize()
    r = A.double().t() @ B.double()
    assert _rel(C.sum(0), r) < REL_TOL


@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
@pytest.mark.parametrize("S", [1, 2, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("shape", [(512, 512, 10552), (128, 640, 1500), (128, 128, 1536), (512, 128, 2600)])
def test_weight_gradient_split_k_every_config(cfg, S, shape):
    """The weight-gradient form the engine tunes over (pinsage_engine_set_gemm_choice):
    M-major A (dpq / dp), N-major B with gathered k-rows (h[q_src], h[self]), split-K
    slabs summed afterwards, for every config and split count (empty splits
    included: S > K / BK)."""
    M, N, K = shape
    g = torch.Generator(device="cuda").manual_seed(17 + cfg + 10 * S)
    A = torch.randn(K, M, device="cuda", generator=g)
    rows = 3 * K
    B = torch.randn(rows, N, device="cuda", generator=g)
    b_idx = torch.randint(0, rows, (K,), device="cuda", generator=g, dtype=torch.int32)
    C = torch.full((S, M, N), float("nan"), device="cuda")
    _gemm(M, N, K, 0, 0, A, None, B, C, epi=3, splits=S, cfg=cfg, b_idx=b_idx)
    torch.cuda.synchronize()
    r = A.double().t() @ B.double()[b_idx.long()]
    assert torch.isfinite(C).all()
    assert _rel(C.sum(0), r) < REL_TOL, _rel(C.sum(0), r)


@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4])
def test_split_bf16_products_are_fp32_accurate(ak, bk, cfg):
    """The split-bf16 product path (x = hi + mid + lo bf16, six 32x32x16 bf16
    MFMAs per 16-k step, fp32 accumulation) against float64, next to the
    exact-fp32 MFMA path on the same data, for every operand layout (K-major
    images read as float4 fragments, M-/N-major images as four k-rows): its
    error is the fp32 path's order (measured below it), with ragged M / K
    tails, gathered rows / k-rows, wide-range magnitudes and both schedules."""
    if cfg == 4 and not (ak and bk):
        pytest.skip("cfg 4 takes K-major operands only")
    import _native as nat
    lib = nat.lib()
    g = torch.Generator(device="cuda").manual_seed(99 + cfg + 7 * ak + 13 * bk)
    old = lib.pinsage_gemm_get_prec()
    try:
        for M, N, K in SHAPES:
            if not ak and M % 4:
                M += 4 - M % 4
            A = torch.randn((M, K), device="cuda", generator=g)
            A *= torch.exp2(torch.randint(-20, 20, (M, 1), device="cuda", generator=g).float())
            if not ak:
                A = A.t().contiguous()
            B = torch.randn((N, K) if bk else (K, N), device="cuda", generator=g)
            a_idx = torch.randint(0, M, (M,), device="cuda", generator=g, dtype=torch.int32) \
                if (ak and M > 1) else None
            b_idx = None
            if not bk:
                B = torch.cat([B, torch.randn(K, N, device="cuda", generator=g)])
                b_idx = torch.randint(0, 2 * K, (K,), device="cuda", generator=g, dtype=torch.int32)
            bias = torch.randn(N, device="cuda", generator=g)
            Bv = B if b_idx is None else B[b_idx.long()]
            r = _ref(M, N, K, ak, bk, A, a_idx, Bv, bias, 1)
            errs = {}
            for prec in (0, 1):
                assert lib.pinsage_gemm_set_prec(prec) == 0
                # stream-K takes no gathered k-rows (launch_gemm falls back to tiles)
                for sk in ((0, 1) if cfg else (0,)):
                    C = torch.full((M, N), float("nan"), device="cuda")
                    _gemm(M, N, K, ak, bk, A, a_idx, B, C, bias=bias, act=1, cfg=cfg, sk=sk, b_idx=b_idx)
                    torch.cuda.synchronize()
                    assert torch.isfinite(C).all()
                    errs[(prec, sk)] = _rel(C, r)
            assert max(errs[k] for k in errs if k[0] == 1) <= 2.0 * max(errs[k] for k in errs if k[0] == 0) + 1e-9, errs
            assert max(errs.values()) < 2e-6, errs
    finally:
        lib.pinsage_gemm_set_prec(old)


@pytest.mark.parametrize("prec", [0, 1])
def test_split_k_weight_gradient_both_arithmetics(prec):
    """The engine's weight-gradient form (M-major A, gathered N-major B, split-K
    slabs) under both product arithmetics."""
    import _native as nat
    lib = nat.lib()
    old = lib.pinsage_gemm_get_prec()
    g = torch.Generator(device="cuda").manual_seed(5 + prec)
    M, N, K, S = 512, 512, 10552, 32
    A = torch.randn(K, M, device="cuda", generator=g)
    B = torch.randn(3 * K, N, device="cuda", generator=g)
    b_idx = torch.randint(0, 3 * K, (K,), device="cuda", generator=g, dtype=torch.int32)
    try:
        assert lib.pinsage_gemm_set_prec(prec) == 0
        C = torch.full((S, M, N), float("nan"), device="cuda")
        _gemm(M, N, K, 0, 0, A, None, B, C, epi=3, splits=S, cfg=0, b_idx=b_idx)
        torch.cuda.synchronize()
    finally:
        lib.pinsage_gemm_set_prec(old)
    r = A.double().t() @ B.double()[b_idx.long()]
    assert _rel(C.sum(0), r) < 1e-6


def _split_planes_ref(W):
    """hi / mid / lo bf16 pieces by round-to-nearest-even (torch's fp32 -> bf16
    cast), each difference exact in fp32 (gemm.hip split_pair)."""
    H = W.to(torch.bfloat16)
    r = W - H.float()
    Mp = r.to(torch.bfloat16)
    L = (r - Mp.float()).to(torch.bfloat16)
    return torch.stack([H, Mp, L]).view(torch.int16)


@pytest.mark.parametrize("cfg", [0, 3, 1, -1])
def test_presplit_b_planes_bitwise(cfg):
    """The Q projection with its weight read as pre-split bf16 planes
    (pinsage_split_planes + pinsage_linear_split_b) is bitwise the
    in-register split-bf16 GEMM (same tiles, same products in the same order)
    for cfg 0 / 3, which run the plane form, and for the configs that fall back
    to the in-register split (1, and the size-picked one).  The planes
    themselves are the RN-even split of torch's bf16 cast."""
    import _native as nat
    lib = nat.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(31 + cfg)
    old = lib.pinsage_gemm_get_prec()
    try:
        assert lib.pinsage_gemm_set_prec(1) == 0
        for M, N, K in [(1, 128, 8), (37, 128, 136), (200, 256, 520), (3000, 512, 512),
                        (10541, 512, 512), (24369, 512, 128), (500, 200, 264), (77, 72, 40)]:
            A = torch.randn(M + 7, K, device="cuda", generator=g)
            A *= torch.exp2(torch.randint(-20, 20, (M + 7, 1), device="cuda", generator=g).float())
            W = torch.randn(N, K, device="cuda", generator=g) * 0.05
            bias = torch.randn(N, device="cuda", generator=g)
            a_idx = torch.randint(0, M + 7, (M,), device="cuda", generator=g, dtype=torch.int32)
            planes = torch.empty(3, N, K, dtype=torch.int16, device="cuda")
            nat.check(lib.pinsage_split_planes(_vp(W), N, K, K, _vp(planes), stream), "split_planes")
            torch.cuda.synchronize()
            assert torch.equal(planes, _split_planes_ref(W)), (M, N, K)
            C0 = torch.full((M, N), float("nan"), device="cuda")
            C1 = torch.full((M, N), float("nan"), device="cuda")
            _gemm(M, N, K, 1, 1, A, a_idx, W, C0, bias=bias, act=1, cfg=cfg, sk=0)
            nat.check(lib.pinsage_linear_split_b(_vp(A), K, _vp(a_idx), M, K, _vp(W), _vp(planes), K,
                                                 _vp(bias), N, 1, _vp(C1), N, cfg, stream),
                      "linear_split_b")
            torch.cuda.synchronize()
            assert torch.isfinite(C1).all(), (M, N, K)
            assert torch.equal(C0, C1), (M, N, K, (C0 - C1).abs().max().item())
            r = _ref(M, N, K, 1, 1, A, a_idx, W, bias, 1)
            assert _rel(C1, r) < 2e-6, (M, N, K, _rel(C1, r))
    finally:
        lib.pinsage_gemm_set_prec(old)


def test_presplit_b_argument_checks():
    import _native as nat
    lib = nat.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    W = torch.randn(128, 12, device="cuda")
    planes = torch.empty(3, 128, 12, dtype=torch.int16, device="cuda")
    assert lib.pinsage_split_planes(_vp(W), 128, 12, 12, _vp(planes), stream) != 0  # cols % 8
    A = torch.randn(16, 12, device="cuda")
    C = torch.empty(16, 128, device="cuda")
    assert lib.pinsage_linear_split_b(_vp(A), 12, None, 16, 12, _vp(W), _vp(planes), 12, None, 128, 0,
                                      _vp(C), 128, 3, stream) != 0  # K % 8


@pytest.mark.parametrize("M,N,K", [(1, 128, 16), (37, 128, 144), (200, 256, 528), (3000, 512, 512),
                                   (10541, 512, 512), (24369, 512, 128), (500, 200, 272), (77, 72, 48)])
def test_interleaved_tables_bitwise(M, N, K):
    """The Q projection from interleaved split-bf16 tables (pinsage_split_ilv
    of the whole row table, split once, and of W -- or W fp32 split in
    registers; pinsage_linear_ilv gathers the rows): bitwise the in-register split-bf16 GEMM of cfg 0 (the same
    128 x 128 tiles, products and k order), with M static and as a device-side
    count below M_max (the engine's form), within 2e-6 of float64; the table
    holds the RN-even split of torch's bf16 cast; bad arguments are refused."""
    import _native as nat
    lib = nat.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    old = lib.pinsage_gemm_get_prec()
    try:
        assert lib.pinsage_gemm_set_prec(1) == 0
        pool = M + 7
        A = torch.randn(pool, K + 4, device="cuda", generator=g)  # (row stride K + 4: the first K columns)
        A *= torch.exp2(torch.randint(-20, 20, (pool, 1), device="cuda", generator=g).float())
        W = torch.randn(N, K, device="cuda", generator=g) * 0.05
        bias = torch.randn(N, device="cuda", generator=g)
        a_idx = torch.randint(0, pool, (M,), device="cuda", generator=g, dtype=torch.int32)
        C0 = torch.full((M, N), float("nan"), device="cuda")
        _gemm(M, N, K, 1, 1, A, a_idx, W, C0, bias=bias, act=1, cfg=0, sk=0)
        lda = 3 * K + 8  # a padded table row
        at = torch.full((pool, lda), 0x7fff, dtype=torch.int16, device="cuda")
        wt = torch.empty(N, 3 * K, dtype=torch.int16, device="cuda")
        nat.check(lib.pinsage_split_ilv(_vp(A), K + 4, pool, K, _vp(at), lda, stream), "split A")
        nat.check(lib.pinsage_split_ilv(_vp(W), K, N, K, _vp(wt), 3 * K, stream), "split W")
        torch.cuda.synchronize()
        # table row = K/16 stages x (hi0 hi1 mid0 mid1 lo0 lo1) chunks of 8
        ref = _split_planes_ref(A[:, :K].contiguous()).view(3, pool, K // 16, 2, 8)
        got = at[:, :3 * K].view(pool, K // 16, 3, 2, 8).permute(2, 0, 1, 3, 4)
        assert torch.equal(got, ref)
        m_dev = torch.tensor([M], dtype=torch.int32, device="cuda")
        for dev_m, w_tab in [(False, True), (True, True), (True, False)]:  # W as a table or fp32
            C1 = torch.full((M, N), float("nan"), device="cuda")
            nat.check(lib.pinsage_linear_ilv(_vp(at), lda, _vp(a_idx), 0 if dev_m else M,
                                             _vp(m_dev) if dev_m else None, M + 300, K, _vp(W),
                                             _vp(wt) if w_tab else None, 3 * K, _vp(bias), N, 1, _vp(C1), N, stream),
                      "linear_ilv")
            torch.cuda.synchronize()
            assert torch.isfinite(C1).all(), (M, N, K, dev_m, w_tab)
            assert torch.equal(C0, C1), (M, N, K, dev_m, w_tab, (C0 - C1).abs().max().item())
        assert _rel(C1, _ref(M, N, K, 1, 1, A[:, :K], a_idx, W, bias, 1)) < 2e-6
        # K % 16, a row stride below 3K, negative sizes
        assert lib.pinsage_split_ilv(_vp(A), K + 4, 8, K - 8, _vp(at), lda, stream) != 0
        assert lib.pinsage_split_ilv(_vp(A), K + 4, 8, K, _vp(at), 3 * K - 8, stream) != 0
        assert lib.pinsage_linear_ilv(_vp(at), lda, None, M, None, M, K - 8, _vp(W), _vp(wt), 3 * K, None, N, 0,
                                      _vp(C1), N, stream) != 0
        assert lib.pinsage_linear_ilv(_vp(at), lda, None, -1, None, M, K, _vp(W), _vp(wt), 3 * K, None, N, 0,
                                      _vp(C1), N, stream) != 0
    finally:
        lib.pinsage_gemm_set_prec(old)


@pytest.mark.parametrize("M,N,K", [(1, 128, 32), (63, 128, 128), (1000, 256, 512), (10541, 512, 512),
                                   (3000, 512, 128), (700, 128, 1024)])
def test_warp_specialised_gemm_is_bitwise_cfg3(M, N, K):
    """cfg 5 (gemm_ws_kernel: producer waves split each element once into LDS
    bf16 planes, consumer waves run the products) computes the same products
    in the same k order as the split-bf16 tiles: bitwise cfg 3's output, for
    gathered rows with the Q projection's bias + LeakyReLU epilogue, within
    1e-4 of float64."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    pool = M + 37
    A = torch.randn(pool, K, device="cuda", generator=g)
    a_idx = torch.randperm(pool, device="cuda", generator=g)[:M].to(torch.int32)
    B = torch.randn(N, K, device="cuda", generator=g) * 0.05
    bias = torch.randn(N, device="cuda", generator=g)
    out = []
    for cfg in (5, 3):
        C = torch.full((M, N), float("nan"), device="cuda")
        _gemm(M, N, K, 1, 1, A, a_idx, B, C, bias=bias, act=1, cfg=cfg)
        torch.cuda.synchronize()
        out.append(C)
    assert torch.isfinite(out[0]).all()
    assert torch.equal(out[0], out[1])
    assert _rel(out[0], _ref(M, N, K, 1, 1, A, a_idx, B, bias, 1)) < REL_TOL


def test_warp_specialised_gemm_argument_checks():
    A = torch.randn(64, 96, device="cuda")
    C = torch.empty(64, 128, device="cuda")
    B = torch.randn(128, 96, device="cuda")
    for args in [dict(K=80), dict(ak=0), dict(N=64)]:  # K % 32, M-major A, N % 128
        K = args.get("K", 64)
        N = args.get("N", 128)
        with pytest.raises(RuntimeError, match="cfg 5"):
            _gemm(64, N, K, args.get("ak", 1), 1, A, None, B, C, cfg=5)


@pytest.mark.parametrize("site", ["q0", "q1", "dyw", "wgrad_q0", "wgrad_w1"])
def test_tuner_candidates_are_bitwise_equal(site):
    """the step's in-context tuner picks, per site, among tile
    configs 0-3 and 5 without stream-K (pinsage_training._tune_choices); the
    default step's bitwise reproducibility rests on every candidate summing
    each output element in the same k order.  At the C2 step's site shapes --
    gathered A with bias + LeakyReLU (the Q projections), N-major B (dY W), and
    the weight gradients' split-K slabs with gathered k-rows at the size
    model's split counts -- every candidate's output is bitwise equal."""
    g = torch.Generator(device="cuda").manual_seed(7)
    outs = []
    if site in ("q0", "q1"):
        M, N, K = (10541, 512, 512) if site == "q0" else (2600, 512, 128)
        rows = 3 * M
        A = torch.randn(rows, K, device="cuda", generator=g)
        a_idx = torch.randint(0, rows, (M,), device="cuda", generator=g, dtype=torch.int32)
        B = torch.randn(N, K, device="cuda", generator=g) * 0.05
        bias = torch.randn(N, device="cuda", generator=g)
        for cfg in (0, 1, 2, 3, 5):
            C = torch.full((M, N), float("nan"), device="cuda")
            _gemm(M, N, K, 1, 1, A, a_idx, B, C, bias=bias, act=1, cfg=cfg, sk=0)
            outs.append(C)
    elif site == "dyw":
        M, N, K = 5709, 640, 128
        A = torch.randn(M, K, device="cuda", generator=g)
        B = torch.randn(K, N, device="cuda", generator=g) * 0.05
        for cfg in (0, 1, 2, 3):
            C = torch.full((M, N), float("nan"), device="cuda")
            _gemm(M, N, K, 1, 0, A, None, B, C, cfg=cfg, sk=0)
            outs.append(C)
    else:
        # (the engine's size model, choose_wgrad: C2 layer-0 Q weight 32 splits, layer-1 W weight 11)
        (M, N, K), S = ((512, 512, 10544), 32) if site == "wgrad_q0" else ((128, 640, 1452), 11)
        A = torch.randn(K, M, device="cuda", generator=g)
        rows = 3 * K
        B = torch.randn(rows, N, device="cuda", generator=g)
        b_idx = torch.randint(0, rows, (K,), device="cuda", generator=g, dtype=torch.int32)
        for cfg in (0, 1, 2):
            C = torch.full((S, M, N), float("nan"), device="cuda")
            _gemm(M, N, K, 0, 0, A, None, B, C, epi=3, splits=S, cfg=cfg, b_idx=b_idx)
            outs.append(C)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
