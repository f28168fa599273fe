"""The convolution's aggregation + projection kernel (pinsage_model.py:195-210:
importance-weighted mean of the neighbours' q rows, [h_self || agg] W^T + b,
LeakyReLU, row L2 norm) through the C-ABI entry pinsage_conv_agg_project,
against a float64 restatement of the same fp32 inputs.

agg is the fp32 fma chain in slot order (t = 0, 1, ...): held to 1e-6
row-relative (it differs from the f64 sum only by fp32 rounding); y and the
norms to the north star's 1e-4 (row-norm relative; the projection runs on
split-bf16 products, fp32-level error).  Shapes: the C2 layer-0 / layer-1 and
C4 shapes, fanouts below, at and above the kernel's 10-slot register group
(3, 10, 25, 50, 64), ragged row counts (1, 33, tiles that do not divide the
rows), rows whose slots repeat one q row, and padded self rows (ldh > d).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _run(h, d, self_src, q, loc, w, W, bias, planes=True):
    import _native as nat
    n_rows, T = loc.shape
    hid = q.shape[1]
    out = W.shape[0]
    y = torch.full((n_rows, out), float("nan"), device="cuda")
    nrm = torch.full((n_rows,), float("nan"), device="cuda")
    agg = torch.full((n_rows, hid), float("nan"), device="cuda")
    planes = torch.empty(3 * out * (d + hid), dtype=torch.int16, device="cuda") if planes else None
    rc = nat.lib().pinsage_conv_agg_project(
        _vp(h), h.shape[1], d, _vp(self_src), _vp(q), hid, q.shape[0], _vp(loc), _vp(w), n_rows, T, _vp(W),
        _vp(bias), out, _vp(planes), _vp(y), _vp(nrm), _vp(agg),
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    nat.check(rc, "conv_agg_project")
    torch.cuda.synchronize()
    return y, nrm, agg


def _ref(h, d, self_src, q, loc, w, W, bias):
    h64, q64 = h.double()[:, :d], q.double()
    agg = (w.double()[:, :, None] * q64[loc.long()]).sum(1)
    a = torch.cat([h64[self_src.long()], agg], 1)
    z = torch.nn.functional.leaky_relu(a @ W.double().t() + bias.double(), 0.01)
    n = z.norm(dim=1)
    return z / n[:, None], n, agg


def _rowrel(x, r):
    return ((x.double() - r).norm(dim=1) / r.norm(dim=1).clamp_min(1e-30)).max().item()


CASES = [  # n_rows, d, ldh, hid, T, U (q rows), n_h (h rows)
    (5704, 512, 512, 512, 10, 10550, 100000),   # C2 layer 0
    (1450, 128, 128, 512, 10, 4600, 5704),      # C2 layer 1 / C4 (d 128)
    (1, 512, 512, 512, 10, 7, 50),
    (33, 128, 132, 512, 3, 40, 90),             # padded h rows, fanout 3 (C1)
    (777, 256, 256, 512, 25, 3000, 4000),       # C3 fanout, d 256
    (300, 256, 256, 512, 50, 2000, 1000),       # C5 fanout
    (250, 64, 64, 128, 64, 500, 600),           # max fanout, small dims (uneven k-steps)
    (70, 32, 32, 96, 7, 90, 80),                # K = 128: fewer units than waves
]


@pytest.fixture(params=["s32", "s32reg", "lds16"])
def form(request, monkeypatch):
    """the kernel form behind pinsage_conv_agg_project: the 32-row tile
    (agg_w32s_kernel: each A fragment split once per two column groups, W read
    from its fragment-order bf16 planes; the default from 16 rows per CU), the
    same tile splitting W in registers (no planes), or the 16-row tile"""
    monkeypatch.setenv("PINSAGE_AGGW32_MIN_ROWS", "0" if request.param.startswith("s32") else "1000000000")
    return request.param


@pytest.mark.parametrize("n_rows,d,ldh,hid,T,U,n_h", CASES)
def test_agg_project_matches_f64(n_rows, d, ldh, hid, T, U, n_h, form):
    g = torch.Generator().manual_seed(n_rows * 7 + T)
    h = torch.randn(n_h, ldh, generator=g).cuda()
    q = torch.nn.functional.leaky_relu(torch.randn(U, hid, generator=g), 0.01).cuda()
    loc = torch.randint(0, U, (n_rows, T), generator=g, dtype=torch.int32)
    if n_rows > 4:
        loc[3, :] = loc[3, 0]  # one row whose slots all name one q row
    w = torch.rand(n_rows, T, generator=g, dtype=torch.float64) + 0.01
    w = (w / w.sum(1, keepdim=True)).float()
    self_src = torch.randint(0, n_h, (n_rows,), generator=g, dtype=torch.int32)
    bound = (6.0 / (d + hid + 128)) ** 0.5  # xavier_uniform, bias 0.3 (pinsage_model.py:184-187)
    W = (torch.rand(128, d + hid, generator=g) * 2 - 1) * bound
    bias = torch.full((128,), 0.3)
    loc, w, self_src, W, bias = loc.cuda(), w.cuda(), self_src.cuda(), W.cuda(), bias.cuda()
    y, nrm, agg = _run(h, d, self_src, q, loc, w, W, bias, planes=form != "s32reg")
    ry, rn, ragg = _ref(h, d, self_src, q, loc, w, W, bias)
    assert torch.isfinite(y).all() and torch.isfinite(agg).all()
    assert _rowrel(agg, ragg) <= 1e-6
    assert _rowrel(y, ry) <= 1e-4
    assert ((nrm.double() - rn).abs() / rn).max().item() <= 1e-4


def test_agg_project_agg_is_the_slot_order_fma_chain(form):
    """agg equals the unfused aggregation kernel (pinsage_weighted_agg, the same
    fma chain in slot order) bitwise."""
    import _native as nat
    g = torch.Generator().manual_seed(3)
    n_rows, d, hid, T, U = 517, 128, 512, 10, 900
    h = torch.randn(700, d, generator=g).cuda()
    q = torch.randn(U, hid, generator=g).cuda()
    loc = torch.randint(0, U, (n_rows, T), generator=g, dtype=torch.int32).cuda()
    w = torch.rand(n_rows, T, generator=g).cuda()
    self_src = torch.randint(0, 700, (n_rows,), generator=g, dtype=torch.int32).cuda()
    W = torch.randn(128, d + hid, generator=g).cuda() * 0.05
    bias = torch.zeros(128).cuda()
    _, _, agg = _run(h, d, self_src, q, loc, w, W, bias, planes=form != "s32reg")
    ref = torch.empty(n_rows, hid, device="cuda")
    rc = nat.lib().pinsage_weighted_agg(_vp(q), hid, _vp(loc), _vp(w), n_rows, T, _vp(ref),
                                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    nat.check(rc, "weighted_agg")
    torch.cuda.synchronize()
    assert torch.equal(agg, ref)


@pytest.mark.parametrize("n_rows,d,hid,T,U", [(5704, 512, 512, 10, 10550), (8570, 128, 512, 10, 23190),
                                              (777, 256, 512, 25, 3000), (300, 256, 512, 50, 2000),
                                              (45, 128, 512, 3, 40), (100, 128, 384, 7, 90)])
def test_planes_tile_is_bitwise_the_register_split_tile(n_rows, d, hid, T, U, monkeypatch):
    """agg_w32s_kernel with W read from its fragment-order planes (written once
    by split_wplanes_kernel) equals the same tile splitting W in registers
    (W_planes null): the planes hold split3's pieces, the products and their
    order are the same -- y, norms and agg bitwise equal."""
    g = torch.Generator().manual_seed(n_rows + d)
    h = torch.randn(900, d, generator=g).cuda()
    q = torch.nn.functional.leaky_relu(torch.randn(U, hid, generator=g), 0.01).cuda()
    loc = torch.randint(0, U, (n_rows, T), generator=g, dtype=torch.int32).cuda()
    w = torch.rand(n_rows, T, generator=g).cuda()
    self_src = torch.randint(0, 900, (n_rows,), generator=g, dtype=torch.int32).cuda()
    W = torch.randn(128, d + hid, generator=g).cuda() * 0.05
    bias = torch.rand(128, generator=g).cuda()
    monkeypatch.setenv("PINSAGE_AGGW32_MIN_ROWS", "0")
    out = [_run(h, d, self_src, q, loc, w, W, bias, planes=pl) for pl in (True, False)]
    for a, b in zip(*out):
        assert torch.isfinite(a).all()
        assert torch.equal(a, b)


def test_agg_project_rejects_unsupported_shapes():
    import _native as nat
    dummy = torch.zeros(16, device="cuda")
    for d, hid, out, T in [(100, 512, 128, 10), (128, 512, 64, 10), (128, 512, 128, 65), (128, 512, 128, 0)]:
        rc = nat.lib().pinsage_conv_agg_project(_vp(dummy), d, d, _vp(dummy), _vp(dummy), hid, 1, _vp(dummy),
                                                _vp(dummy), 1, T, _vp(dummy), _vp(dummy), out, _vp(dummy),
                                                _vp(dummy), _vp(dummy), _vp(dummy), None)
        assert rc == -2


@pytest.mark.parametrize("hid,T,n_rows,U", [(512, 10, 5704, 10550), (256, 50, 333, 2000), (128, 3, 1, 5),
                                            (512, 64, 77, 300)])
def test_xcd_sliced_aggregation_is_bitwise_the_row_kernel(hid, T, n_rows, U, monkeypatch):
    """pinsage_weighted_agg on the XCD-sliced kernel (column slice b % 8 per
    block) equals the one-wave-per-row kernel bitwise: same fma chain per
    element, slot order t = 0, 1, ..."""
    import _native as nat
    g = torch.Generator().manual_seed(hid + T)
    q = torch.randn(U, hid, generator=g).cuda()
    loc = torch.randint(0, U, (n_rows, T), generator=g, dtype=torch.int32).cuda()
    w = torch.rand(n_rows, T, generator=g).cuda()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = []
    for sliced in ("1", "0"):
        monkeypatch.setenv("PINSAGE_AGG_SLICED", sliced)
        a = torch.full((n_rows, hid), float("nan"), device="cuda")
        nat.check(nat.lib().pinsage_weighted_agg(_vp(q), hid, _vp(loc), _vp(w), n_rows, T, _vp(a), st), "agg")
        torch.cuda.synchronize()
        out.append(a)
    assert torch.isfinite(out[0]).all()
    assert torch.equal(out[0], out[1])
    ref = (w.double()[:, :, None] * q.double()[loc.long()]).sum(1)
    assert ((out[0].double() - ref).norm() / ref.norm()).item() < 1e-6
