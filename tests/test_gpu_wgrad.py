"""The long-K weight-gradient kernel (csrc/wgrad.hip, pinsage_wgrad): the
AddmmBackward of every nn.Linear weight of the model (pinsage_model.py:196-201,
208-210) -- dW = A^T [B || B2] over a device-side row count with gathered B
rows, db = column sums of A, splits combined inside the launch, torch.optim.Adam
fused -- against a float64 product of the same fp32 operands (the north star's
1e-4 relative; split-bf16 products are fp32-accurate, measured ~1e-7), and
bitwise repeatable whichever split arrives last.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class _Scratch:
    def __init__(self, M, N):
        import _native as nat
        n = nat.lib().pinsage_wgrad_scratch_bytes(M, N)
        self.buf = torch.zeros(int(n), dtype=torch.uint8, device="cuda")


def _wgrad(M, N, K_dev, K_max, A, B, b_idx, dst, dst_b=None, N1=-1, B2=None, splits=0, scratch=None, adam=None):
    import _native as nat
    lib = nat.lib()
    sc = scratch or _Scratch(M, N)
    ad = adam or {}
    rc = lib.pinsage_wgrad(M, N, _vp(K_dev), K_max, _vp(A), A.shape[1], _vp(B), B.shape[1], _vp(b_idx),
                           N1, _vp(B2), B2.shape[1] if B2 is not None else 0, _vp(dst), dst.shape[1], _vp(dst_b),
                           splits, _vp(sc.buf), _vp(ad.get("p")), _vp(ad.get("m")), _vp(ad.get("v")),
                           _vp(ad.get("pb")), _vp(ad.get("mb")), _vp(ad.get("vb")), _vp(ad.get("coef")),
                           ad.get("b1", 0.9), ad.get("b2", 0.999), ad.get("eps", 1e-8),
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    nat.check(rc, "wgrad")
    return sc


def _rel(x, r):
    return ((x.double() - r).norm() / r.norm().clamp_min(1e-30)).item()


CASES = [  # M, N, N1, K, rows of the gathered table
    (512, 512, -1, 3001, 5000),      # Q0 weight gradient (C2-like, ragged K)
    (512, 128, -1, 777, 2000),       # Q1
    (128, 1024, 512, 2345, 4000),    # W0: [h_self (gathered) || agg]
    (128, 640, 128, 613, 900),       # W1
    (128, 128, -1, 1500, 1500),      # head G1 / G2
    (512, 512, -1, 40, 100),         # fewer rows than splits
]


@pytest.mark.parametrize("M,N,N1,K,R", CASES)
def test_wgrad_matches_float64_and_repeats_bitwise(M, N, N1, K, R):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn((K + 16, M), device="cuda", generator=g)
    A *= torch.exp2(torch.randint(-10, 10, (K + 16, 1), device="cuda", generator=g).float())
    n1 = N if N1 < 0 else N1
    B = torch.randn((R, n1), device="cuda", generator=g)
    b_idx = torch.randint(0, R, (K + 16,), device="cuda", generator=g, dtype=torch.int32)
    B2 = torch.randn((K + 16, N - n1), device="cuda", generator=g) if N1 >= 0 else None
    K_dev = torch.tensor([K], dtype=torch.int32, device="cuda")
    Bf = B.double()[b_idx[:K].long()]
    if B2 is not None:
        Bf = torch.cat([Bf, B2.double()[:K]], 1)
    ref = A.double()[:K].t() @ Bf
    ref_b = A.double()[:K].sum(0)
    outs = []
    for splits in (0, 1, 3, 0):
        dst = torch.full((M, N), float("nan"), device="cuda")
        db = torch.full((M,), float("nan"), device="cuda")
        _wgrad(M, N, K_dev, K + 16, A, B, b_idx, dst, db, N1=N1, B2=B2, splits=splits)
        torch.cuda.synchronize()
        assert torch.isfinite(dst).all() and torch.isfinite(db).all()
        assert _rel(dst, ref) < 2e-6, (splits, _rel(dst, ref))
        assert _rel(db, ref_b) < 2e-6, (splits, _rel(db, ref_b))
        outs.append((dst, db))
    assert torch.equal(outs[0][0], outs[3][0]) and torch.equal(outs[0][1], outs[3][1])  # same splits: bitwise


def test_wgrad_zero_rows_and_scratch_reuse():
    """K = 0 on the device gives zero gradients; the tickets a launch leaves
    behind are zero again (the next launch on the same scratch is correct)."""
    M, N = 512, 512
    A = torch.randn((300, M), device="cuda")
    B = torch.randn((300, N), device="cuda")
    sc = None
    for k in (0, 300, 0, 299):
        K_dev = torch.tensor([k], dtype=torch.int32, device="cuda")
        dst = torch.full((M, N), float("nan"), device="cuda")
        db = torch.full((M,), float("nan"), device="cuda")
        sc = _wgrad(M, N, K_dev, 300, A, B, None, dst, db, scratch=sc)
        torch.cuda.synchronize()
        ref = A.double()[:k].t() @ B.double()[:k]
        if k == 0:
            assert float(dst.abs().max()) == 0.0 and float(db.abs().max()) == 0.0
        else:
            assert _rel(dst, ref) < 2e-6
    assert int(sc.buf[:4 * 64].view(torch.int32).abs().sum()) == 0


def test_wgrad_fused_adam_matches_torch():
    """The fused Adam step (Q0's, the step's last gradient) against
    torch.optim.Adam's formula on the same gradient (fp32, as the engine's
    reduce_slabs_2d applies it), and a refused step (bc2 = 0) leaves the
    parameters and moments untouched."""
    M, N, K = 512, 512, 2000
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn((K, M), device="cuda", generator=g)
    B = torch.randn((K, N), device="cuda", generator=g)
    K_dev = torch.tensor([K], dtype=torch.int32, device="cuda")
    p = torch.randn((M, N), device="cuda", generator=g)
    m = torch.randn((M, N), device="cuda", generator=g) * 1e-3
    v = torch.rand((M, N), device="cuda", generator=g) * 1e-3
    pb, mb, vb = torch.randn(M, device="cuda"), torch.zeros(M, device="cuda"), torch.zeros(M, device="cuda")
    b1, b2, eps, lr, t = 0.9, 0.999, 1e-8, 1e-3, 3
    coef = torch.tensor([lr / (1 - b1 ** t), (1 - b2 ** t) ** 0.5], dtype=torch.float32, device="cuda")
    dst = torch.empty((M, N), device="cuda")
    db = torch.empty(M, device="cuda")
    P, Mo, V = p.clone(), m.clone(), v.clone()
    Pb, Mb, Vb = pb.clone(), mb.clone(), vb.clone()
    _wgrad(M, N, K_dev, K, A, B, None, dst, db,
           adam=dict(p=P, m=Mo, v=V, pb=Pb, mb=Mb, vb=Vb, coef=coef, b1=b1, b2=b2, eps=eps))
    torch.cuda.synchronize()

    def adam(pp, gg, mm, vv):
        mm = mm + (1 - b1) * (gg - mm)
        vv = vv * b2 + (1 - b2) * gg * gg
        return pp - coef[0] * (mm / (vv.sqrt() / coef[1] + eps)), mm, vv

    rp, rm, rv = adam(p, dst, m, v)
    assert torch.allclose(P, rp, rtol=1e-6, atol=1e-7) and torch.allclose(Mo, rm, rtol=1e-6, atol=1e-9)
    assert torch.allclose(V, rv, rtol=1e-6, atol=1e-12)
    rpb, _, _ = adam(pb, db, mb, vb)
    assert torch.allclose(Pb, rpb, rtol=1e-6, atol=1e-7)
    # refused step
    coef[1] = 0.0
    P2, M2, V2 = P.clone(), Mo.clone(), V.clone()
    _wgrad(M, N, K_dev, K, A, B, None, dst, db,
           adam=dict(p=P2, m=M2, v=V2, pb=Pb.clone(), mb=Mb.clone(), vb=Vb.clone(), coef=coef))
    torch.cuda.synchronize()
    assert torch.equal(P2, P) and torch.equal(M2, Mo) and torch.equal(V2, V)


def _planes(X):
    """hi / mid / lo bf16 planes of a row-major fp32 matrix (pinsage_split_planes)."""
    import _native as nat
    R, C = X.shape
    out = torch.empty((3, R, C), dtype=torch.int16, device="cuda")
    nat.check(nat.lib().pinsage_split_planes(_vp(X), R, C, X.stride(0), _vp(out),
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "split_planes")
    return out


@pytest.mark.parametrize("M,N,K,R", [(512, 512, 3001, 5000), (512, 128, 5000, 20000), (512, 256, 40, 100),
                                     (128, 128, 2345, 0)])
def test_wgrad_planes_equal_fp32_form_bitwise(M, N, K, R, monkeypatch):
    """pinsage_wgrad_planes (both operands pre-split, no conversions in the k
    loop: the engine's layer-0 Q weight gradient) gives the fp32 form's 4-wave
    launch bit for bit -- the planes hold exactly the in-register split, the
    products and the per-wave stage order are the same -- over gathered and
    ungathered B rows, ragged K and a K tail inside a 2048-row pass; the bias
    (summed from the planes' value) within 2^-22 of it, and both against
    float64."""
    import _native as nat
    lib = nat.lib()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn((K + 16, M), device="cuda", generator=g)
    A *= torch.exp2(torch.randint(-10, 10, (K + 16, 1), device="cuda", generator=g).float())
    B = torch.randn((R if R else K + 16, N), device="cuda", generator=g)
    b_idx = torch.randint(0, R, (K + 16,), device="cuda", generator=g, dtype=torch.int32) if R else None
    K_dev = torch.tensor([K], dtype=torch.int32, device="cuda")
    A3, B3 = _planes(A), _planes(B)
    Bf = B.double()[b_idx[:K].long()] if R else B.double()[:K]
    ref = A.double()[:K].t() @ Bf
    ref_b = A.double()[:K].sum(0)
    for splits in (0, 1, 3):
        monkeypatch.setenv("PINSAGE_KW_WAVES", "4")
        dst = torch.full((M, N), float("nan"), device="cuda")
        db = torch.full((M,), float("nan"), device="cuda")
        _wgrad(M, N, K_dev, K + 16, A, B, b_idx, dst, db, splits=splits)
        monkeypatch.delenv("PINSAGE_KW_WAVES")
        dp = torch.full((M, N), float("nan"), device="cuda")
        dbp = torch.full((M,), float("nan"), device="cuda")
        sc = _Scratch(M, N)
        nat.check(lib.pinsage_wgrad_planes(M, N, _vp(K_dev), K + 16, _vp(A3), A3[0].numel(), M, _vp(B3),
                                           B3[0].numel(), N, _vp(b_idx), _vp(dp), N, _vp(dbp), splits, _vp(sc.buf),
                                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                  "wgrad_planes")
        torch.cuda.synchronize()
        assert torch.equal(dp, dst), (splits, (dp - dst).abs().max().item())
        assert ((dbp - db).abs() <= 2.0 ** -22 * A[:K].abs().sum(0)).all(), splits
        assert _rel(dp, ref) < 2e-6 and _rel(dbp, ref_b) < 2e-6
