"""torch.ops.pinsage: the hot path's kernels as PyTorch-ROCm operators.

``libpinsage_torch.so`` (csrc/torch_ops.cpp, built in-tree by csrc/Makefile)
registers the schemas of SURVEY.md §8(b2) -- ppr_topk, frontier, linear,
gemm, weighted_agg (+ weighted_agg_backward), segment_wmean -- on the HIP
device, each calling libpinsage_hip.so's C-ABI on the current stream.  This
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


def _register_autograd():
    torch.library.register_autograd("pinsage::linear", _linear_backward, setup_context=_linear_setup)
    torch.library.register_autograd("pinsage::weighted_agg", _agg_backward, setup_context=_agg_setup)


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
    cat = torch.cat([hd[ns, :d], agg], 1).contiguous()
    z = ops.linear(cat, None, Ww, Wb, True)
    y = z / z.norm(dim=1, keepdim=True)
    return y.to(h.device)
