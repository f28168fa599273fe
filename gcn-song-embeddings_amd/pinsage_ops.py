"""torch.ops.pinsage: the hot path's kernels as PyTorch-ROCm operators.

``libpinsage_torch.so`` (csrc/torch_ops.cpp, built in-tree by csrc/Makefile)
registers the schemas of SURVEY.md §8(b2) -- walk, ppr_topk, frontier,
gather_rows / scatter_add_rows, linear, concat_linear_lrelu_l2norm (+
norm_lrelu_backward), gemm, weighted_agg (+ weighted_agg_backward),
segment_wmean -- on the HIP device, each calling libpinsage_hip.so's C-ABI on
the current stream.  walk / ppr_topk take rng_mode "mt19937" (the reference's
own draws from torch's global generator, advanced as the reference advances
it) or "philox" (seed, offset, src_base: counter-based, generator untouched).  This
module loads it and registers the autograd formulas of the differentiable ops
(torch.library.register_autograd), so ``conv_layer`` below -- the standalone
ConvLayer forward (pinsage_model.py:189-212) -- trains through torch autograd
with every product, aggregation and transposed aggregation on the HIP kernels.
There is no CPU implementation: the ops raise on non-device tensors.
"""
from __future__ import annotations

import os

import torch

_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_DIR, "libpinsage_torch.so")
_loaded = False


def load():
    """Load the operator library once (raises if it was not built)."""
    global _loaded
    if _loaded:
        return
    if not os.path.isfile(_LIB):
        raise RuntimeError(f"{_LIB} missing: build it with `make -C gcn-song-embeddings_amd/csrc`")
    import _native  # the C-ABI library first (the operator library links it by $ORIGIN)
    _native.lib()
    torch.ops.load_library(_LIB)
    _register_autograd()
    _loaded = True


def _pad4(t, fill=0):
    r = (-t.shape[0]) % 4
    return t if r == 0 else torch.cat([t, t.new_full((r,) + tuple(t.shape[1:]), fill)])


def _linear_setup(ctx, inputs, output):
    x, rows, W, b, lrelu = inputs
    ctx.save_for_backward(x, rows, W, output)
    ctx.lrelu = lrelu
    ctx.has_b = b is not None


def _linear_backward(ctx, dy):
    """y = act(x[rows] W^T + b): dz = dy * act'(y); dW = dz^T x[rows], db = sum dz,
    dx[rows] += dz W (the GEMMs on pinsage::gemm)."""
    x, rows, W, y = ctx.saved_tensors
    N, K = W.shape
    dz = (dy * torch.where(y > 0, 1.0, 0.01)) if ctx.lrelu else dy
    dz = dz.contiguous()
    n = dz.shape[0]
    ops = torch.ops.pinsage
    dW = db = dx = None
    if ctx.needs_input_grad[2]:
        idx = rows if rows is not None else torch.arange(n, dtype=torch.int32, device=dz.device)
        dz4, idx4 = _pad4(dz), _pad4(idx)
        dW = ops.gemm(dz4, False, None, x, False, idx4, N, K, dz4.shape[0])
    if ctx.has_b and ctx.needs_input_grad[3]:
        db = dz.sum(0)
    if ctx.needs_input_grad[0]:
        d_rows = ops.gemm(dz, True, None, W, False, None, n, K, N)
        dx = torch.zeros_like(x)
        if rows is None:
            dx[:n, :K] += d_rows
        else:
            dx[:, :K].index_add_(0, rows.to(torch.int64), d_rows)
    return dx, None, dW, db, None


def _agg_setup(ctx, inputs, output):
    q, loc, w = inputs
    ctx.save_for_backward(loc, w)
    ctx.n_q = q.shape[0]


def _agg_backward(ctx, dagg):
    loc, w = ctx.saved_tensors
    return torch.ops.pinsage.weighted_agg_backward(dagg.contiguous(), loc, w, ctx.n_q), None, None


def _gather_setup(ctx, inputs, output):
    h, idx, width = inputs
    ctx.save_for_backward(idx)
    ctx.shape = tuple(h.shape)


def _gather_backward(ctx, dout):
    """get_embeddings' gradient: index_add of the rows' cotangents (repeated ids summed)."""
    idx, = ctx.saved_tensors
    n, w = ctx.shape
    return torch.ops.pinsage.scatter_add_rows(dout.contiguous(), idx, n, w), None, None


def _scatter_setup(ctx, inputs, output):
    grad, idx, n_rows, width = inputs
    ctx.save_for_backward(idx)
    ctx.d = grad.shape[1]


def _scatter_backward(ctx, dout):
    idx, = ctx.saved_tensors
    return torch.ops.pinsage.gather_rows(dout.contiguous(), idx, ctx.d), None, None, None


def _cat_setup(ctx, inputs, output):
    h, rows, agg, W, b = inputs
    y, norms = output
    ctx.save_for_backward(h, rows, agg, W, y, norms)
    ctx.mark_non_differentiable(norms)


def _cat_backward(ctx, dy, _dnorms):
    """y = normalize(lrelu([h[rows, :d] || agg] W^T + b)) (pinsage_model.py:208-210):
    dp = norm_lrelu_backward(dy); dW = dp^T [h[rows] || agg], db = sum dp,
    dh[rows, :d] += dp W[:, :d], dagg = dp W[:, d:] (products on pinsage::gemm)."""
    h, rows, agg, W, y, norms = ctx.saved_tensors
    ops = torch.ops.pinsage
    out, K = W.shape
    hid = agg.shape[1]
    d = K - hid
    n = y.shape[0]
    dp = ops.norm_lrelu_backward(dy.contiguous(), y, norms)
    dh = dagg = dW = db = None
    if ctx.needs_input_grad[3]:
        dp4 = _pad4(dp)
        idx = rows.to(torch.int32) if rows is not None else torch.arange(n, dtype=torch.int32, device=dp.device)
        idx4 = _pad4(idx)
        dW = torch.cat([ops.gemm(dp4, False, None, h, False, idx4, out, d, dp4.shape[0]),
                        ops.gemm(dp4, False, None, _pad4(agg.contiguous()), False, None, out, hid, dp4.shape[0])], 1)
    if ctx.needs_input_grad[4]:
        db = dp.sum(0)
    if ctx.needs_input_grad[0]:
        d_rows = ops.gemm(dp, True, None, W[:, :d], False, None, n, d, out)
        if rows is None:
            dh = torch.zeros_like(h)
            dh[:n, :d] += d_rows
        else:
            dh = ops.scatter_add_rows(d_rows, rows, h.shape[0], h.shape[1])
    if ctx.needs_input_grad[2]:
        dagg = ops.gemm(dp, True, None, W[:, d:], False, None, n, hid, out)
    return dh, None, dagg, dW, db


def _register_autograd():
    torch.library.register_autograd("pinsage::linear", _linear_backward, setup_context=_linear_setup)
    torch.library.register_autograd("pinsage::weighted_agg", _agg_backward, setup_context=_agg_setup)
    torch.library.register_autograd("pinsage::gather_rows", _gather_backward, setup_context=_gather_setup)
    torch.library.register_autograd("pinsage::scatter_add_rows", _scatter_backward, setup_context=_scatter_setup)
    torch.library.register_autograd("pinsage::concat_linear_lrelu_l2norm", _cat_backward,
                                    setup_context=_cat_setup)


def conv_layer(h, nodeset, nb_nodes, nb_weights, Qw, Qb, Ww, Wb):
    """ConvLayer.forward (pinsage_model.py:189-212) on torch.ops.pinsage:

        q   = lrelu(h[u] Q^T + b_Q)        u = the distinct neighbours
        agg = sum_t w[f,t] q[loc[f,t]]     w normalised by its f64 row sum
        y   = normalize(lrelu([h[f] || agg] W^T + b_W))

    Differentiable in the parameters and in h (rows :in_dim)."""
    load()
    import _native
    ops = torch.ops.pinsage
    dev = _native.device()
    # parameters may live on the host (a standalone layer): .to is differentiable
    Qw, Qb, Ww, Wb = (p.to(dev, torch.float32) for p in (Qw, Qb, Ww, Wb))
    hid, d = Qw.shape
    hd = h if (h.device == dev and h.dtype == torch.float32 and h.stride(1) == 1) else \
        h.to(dev, torch.float32).contiguous()
    ns = torch.as_tensor(nodeset).reshape(-1).to(dev, torch.int64)
    nb = torch.as_tensor(nb_nodes).to(dev, torch.int64)
    n, T = nb.shape
    if ns.shape[0] != n:
        raise ValueError("nodeset and nb_nodes rows differ")
    if n and (int(torch.cat([ns, nb.reshape(-1)]).min()) < 0 or
              int(torch.cat([ns, nb.reshape(-1)]).max()) >= hd.shape[0]):
        raise IndexError("node ids out of range of h")
    w64 = torch.as_tensor(nb_weights).to(dev, torch.float64)
    wn = (w64 / w64.sum(1, keepdim=True)).to(torch.float32).contiguous()
    uniq, inv = torch.unique(nb.reshape(-1), return_inverse=True)
    loc = inv.view(n, T).to(torch.int32).contiguous()
    q = ops.linear(hd, uniq.to(torch.int32).contiguous(), Qw, Qb, True)
    agg = ops.weighted_agg(q, loc, wn)
    # [h[nodeset, :d] || agg] W^T + b, lrelu, row L2 norm: the concat read in place
    y, _ = ops.concat_linear_lrelu_l2norm(hd, ns, agg, Ww, Wb)
    return y.to(h.device)
