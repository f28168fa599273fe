"""CPU oracle for the PinSage train-step path -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module; the product (``gcn-song-embeddings_amd/``) never does.
It restates the reference algorithm on the CPU:

* integer/RNG work in C (``oracle_core.c``): torch's MT19937 stream, the walk
  (``pinsage_model.py:32-53``), libstdc++ top-k (``pinsage_model.py:107``),
  Philox twin of the product's fast RNG mode;
* dense visit counts (``pinsage_model.py:88-101``), frontier construction
  (``pinsage_model.py:156-168``), batch sampling (``pinsage_training.py:53-97``)
  in numpy;
* the model (``pinsage_model.py:171-265``), loss (``pinsage_training.py:31-41``)
  and one train step (``pinsage_training.py:181-214``) in torch-CPU fp32 with
  f64 aggregation and the reference's clone/detach ``put_embeddings`` semantics
  (``pinsage_model.py:24-30``) -- this is also the timed "refcpu" baseline.

Parity pin: checked against tests/golden/*.npz, which were produced by running
the real reference in the dev container (tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """Load (building if needed) oracle/build/liboracle.so."""
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "build", "liboracle.so")
        src = os.path.join(HERE, "oracle_core.c")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", HERE, "build/liboracle.so"])
        L = ctypes.CDLL(path)
        vp, i64, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float
        L.orc_mt_size.restype = ctypes.c_int
        L.orc_mt_draw.restype = ctypes.c_uint32
        L.orc_mt_draw.argtypes = [vp]
        L.orc_mt_seed.argtypes = [vp, ctypes.c_uint64]
        L.orc_mt_from_torch.argtypes = [vp, vp]
        L.orc_mt_to_torch.argtypes = [vp, vp]
        L.orc_mt_draws.argtypes = [vp, vp, i64]
        L.orc_randperm.argtypes = [vp, i64, vp]
        L.orc_walk_mt.restype = i64
        L.orc_walk_mt.argtypes = [vp, vp, vp, vp, i64, i64, f32, vp]
        L.orc_walk_philox.restype = i64
        L.orc_walk_philox.argtypes = [ctypes.c_uint64, ctypes.c_uint32, vp, vp, vp, i64, i64, i64,
                                      f32, vp]
        L.orc_philox.argtypes = [ctypes.c_uint64, vp, vp]
        L.orc_topk.argtypes = [vp, i64, i64, i64, vp, vp]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------- RNG
class MT:
    """torch's CPU MT19937 generator, restated (state shared with torch via bytes)."""

    def __init__(self, seed=None):
        self.buf = np.zeros(lib().orc_mt_size(), np.uint8)
        if seed is not None:
            lib().orc_mt_seed(_p(self.buf), seed)

    @classmethod
    def from_torch(cls):
        g = cls()
        st = torch.get_rng_state().numpy().copy()
        lib().orc_mt_from_torch(_p(g.buf), _p(st))
        return g

    def to_torch(self):
        st = torch.get_rng_state().numpy().copy()
        lib().orc_mt_to_torch(_p(self.buf), _p(st))
        torch.set_rng_state(torch.from_numpy(st))

    def draws(self, n):
        out = np.empty(n, np.uint32)
        lib().orc_mt_draws(_p(self.buf), _p(out), n)
        return out

    def randperm(self, n):
        out = np.empty(n, np.int64)
        lib().orc_randperm(_p(self.buf), n, _p(out))
        return out


def philox(key, ctr):
    c = np.asarray(ctr, np.uint32)
    out = np.empty(4, np.uint32)
    lib().orc_philox(ctypes.c_uint64(key), _p(c), _p(out))
    return out


# ----------------------------------------------------------------------------- sampler
def walk_mt(indptr, indices, sources, n_hops, alpha, mt):
    indptr = np.ascontiguousarray(indptr, np.int64)
    indices = np.ascontiguousarray(indices, np.int32)
    sources = np.ascontiguousarray(sources, np.int64)
    trace = np.zeros((sources.shape[0], n_hops), np.int64)
    rc = lib().orc_walk_mt(_p(mt.buf), _p(indptr), _p(indices), _p(sources), sources.shape[0],
                           n_hops, np.float32(alpha), _p(trace))
    if rc != 0:
        raise RuntimeError(f"zero-degree node met while walking from source {-rc - 1}")
    return trace


def walk_philox(indptr, indices, sources, n_hops, alpha, seed, offset=0, src_base=0):
    indptr = np.ascontiguousarray(indptr, np.int64)
    indices = np.ascontiguousarray(indices, np.int32)
    sources = np.ascontiguousarray(sources, np.int64)
    trace = np.zeros((sources.shape[0], n_hops), np.int64)
    rc = lib().orc_walk_philox(ctypes.c_uint64(seed), ctypes.c_uint32(offset), _p(indptr),
                               _p(indices), _p(sources), sources.shape[0], src_base, n_hops,
                               np.float32(alpha), _p(trace))
    if rc != 0:
        raise RuntimeError("zero-degree node met")
    return trace


def visit_prob(trace, sources, n_all):
    """Dense normalised visit counts with the self column zeroed (pinsage_model.py:96-99)."""
    n_s, n_hops = trace.shape
    vc = np.zeros((n_s, n_all), np.float64)
    np.add.at(vc, (np.repeat(np.arange(n_s), n_hops), trace.reshape(-1)), 1.0)
    vp = vc / vc.sum(1, keepdims=True)
    vp[np.arange(n_s), np.asarray(sources)] = 0.0
    return vp


def topk(mat, k):
    """Tensor.topk(k, 1) on CPU f64 with libstdc++ tie order (restated in C)."""
    mat = np.ascontiguousarray(mat, np.float64)
    rows, n = mat.shape
    vals = np.zeros((rows, k), np.float64)
    idx = np.zeros((rows, k), np.int64)
    lib().orc_topk(_p(mat), rows, n, k, _p(vals), _p(idx))
    return vals, idx


def sample_neighborhood_topt(indptr, indices, n_all, sources, n_hops, alpha, T, mt):
    trace = walk_mt(indptr, indices, sources, n_hops, alpha, mt)
    return topk(visit_prob(trace, sources, n_all), T)


def ppr_knn(indptr, indices, n_all, nodeset, k, mt, n_hops=1000, alpha=0.85):
    """PersPageRank.knn (baselines.py:114-151): the same walk / visit_prob as
    sample_neighborhood (1000 hops, restart 0.85), then topk(k, 1)."""
    return sample_neighborhood_topt(indptr, indices, n_all, nodeset, n_hops, alpha, k, mt)


def cosine_sim_ab(a, b, eps=1e-16):
    """baselines.py:69-77 (torch CPU fp32, the reference's ops)."""
    dot = torch.mm(a, b.transpose(1, 0))
    lengths = torch.mm(torch.norm(a, dim=1).unsqueeze(1), torch.norm(b, dim=1).unsqueeze(0)) + eps
    return dot / lengths


def knn_from_emb(emb, q, k):
    """baselines.py:91-103: batches of 128 queries, topk(k+1) largest, first column dropped."""
    emb = torch.as_tensor(emb)
    q = torch.as_tensor(q)
    ws, ns = [], []
    for i in range(0, len(q), 128):
        sim = cosine_sim_ab(emb[q[i:i + 128], :], emb)
        w, n = sim.topk(k + 1, dim=1, largest=True)
        ws.append(w[:, 1:])
        ns.append(n[:, 1:])
    return torch.cat(ws, 0).numpy(), torch.cat(ns, 0).numpy()


def precompute_topt(indptr, indices, n_all, n_items, n_hops, alpha, T, mt, batch=256):
    """precompute_neighborhoods_topt (pinsage_model.py:109-132) without the file cache."""
    W = np.zeros((n_items, T), np.float64)
    N = np.zeros((n_items, T), np.int64)
    for i in range(0, n_items, batch):
        src = np.arange(i, min(i + batch, n_items), dtype=np.int64)
        w, nb = sample_neighborhood_topt(indptr, indices, n_all, src, n_hops, alpha, T, mt)
        W[src], N[src] = w, nb
    return W, N


def frontier(nodeset, n_layers, T, w_table, nb_table):
    """relevant_nodes_per_layer_precomp (pinsage_model.py:156-168): index 0 = bottom."""
    S = []
    cur = np.asarray(nodeset, np.int64)
    for _ in range(n_layers):
        w, nb = w_table[cur, :T], nb_table[cur, :T]
        S.insert(0, (cur, w, nb))
        cur = np.unique(np.concatenate([nb.reshape(-1), cur]))
    return S


# ----------------------------------------------------------------------------- batches
def sample_batch_easy(mt, positives, n_items, batch_size):
    """sample_batch with easy negatives (pinsage_training.py:53-77,89-97)."""
    P = positives.shape[0]
    pos = positives[mt.randperm(P)[:batch_size]]
    members = np.unique(pos.reshape(-1))
    mask = np.ones(n_items, bool)
    mask[members] = False
    possible = np.arange(n_items, dtype=np.int64)[mask]
    neg = possible[mt.randperm(possible.shape[0])[:pos.shape[0]]]
    batch = np.concatenate([pos, neg[:, None]], 1)
    return batch, np.unique(batch.reshape(-1))


# ----------------------------------------------------------------------------- model
SLOPE = 0.01  # nn.functional.leaky_relu default


def param_names(n_layers):
    names = []
    for i in range(n_layers):
        names += [f"conv_layers.{i}.Q.weight", f"conv_layers.{i}.Q.bias",
                  f"conv_layers.{i}.W.weight", f"conv_layers.{i}.W.bias"]
    return names + ["G1.weight", "G1.bias", "G2.weight"]


class _PutLast(torch.autograd.Function):
    """``out[idx] = rows`` with the serial order's last write winning for a
    repeated index.  torch-CPU's index_put_ gives no order for duplicates (it
    becomes a parallel scatter: on a 16-thread host the winner changed from
    run to run), the serial semantics are the last write; the backward is
    index_put's: every row, winner or not, gets out's cotangent at its index."""

    @staticmethod
    def forward(ctx, h, idx, rows):
        out = h.clone()
        n = idx.shape[0]
        _, first_rev = np.unique(idx.numpy()[::-1], return_index=True)
        keep = torch.from_numpy(np.ascontiguousarray(n - 1 - first_rev))
        out[idx[keep]] = rows[keep]
        ctx.save_for_backward(idx)
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return None, None, g[idx]


def _put(h, rows_idx, rows):
    """put_embeddings semantics (pinsage_model.py:24-30): detached copy,
    zero-padded row overwrite, last write wins for repeated ids."""
    pad = h.shape[1] - rows.shape[1]
    padded = torch.cat([rows, torch.zeros(rows.shape[0], pad, dtype=rows.dtype)], 1)
    return _PutLast.apply(h.detach(), rows_idx, padded)


# Test infrastructure only: when a list, every projection of model_forward
# appends (weight key, bias key or None, its input, its output) so a parity
# test can weigh a gradient's error by the magnitude of the terms it sums
# (parity_util.cond_grads).
_TAPS = None


def _linear(p, wk, bk, x):
    y = F.linear(x, p[wk], p[bk] if bk else None)
    if _TAPS is not None:
        _TAPS.append((wk, bk, x.detach(), y))
    return y


def conv_layer(p, i, h, nodes, nb, w, in_dim):
    """One ConvLayer (pinsage_model.py:189-212): f64 weighted mean, fp32 projections."""
    Fn, T = nb.shape
    self_h = h[nodes, :in_dim]
    nbr = h[nb.reshape(-1), :in_dim].reshape(Fn, T, in_dim)
    q = F.leaky_relu(_linear(p, f"conv_layers.{i}.Q.weight", f"conv_layers.{i}.Q.bias", nbr))
    agg = (w[:, :, None] * q).sum(1) / w.sum(1, keepdim=True)
    z = F.leaky_relu(_linear(p, f"conv_layers.{i}.W.weight", f"conv_layers.{i}.W.bias",
                             torch.cat([self_h, agg], 1).float()))
    return z / z.norm(dim=1, keepdim=True)


def relevant_nodes_fly(indptr, indices, n_all, nodeset, n_layers, n_hops, alpha, T, mt):
    """relevant_nodes_per_layer (pinsage_model.py:142-154): every layer's
    nodeset walked with the MT19937 stream (top layer first, draws in nodeset
    order), index 0 = bottom."""
    S = []
    cur = np.asarray(nodeset, np.int64)
    for _ in range(n_layers):
        w, nb = sample_neighborhood_topt(indptr, indices, n_all, cur, n_hops, alpha, T, mt)
        S.insert(0, (cur, w, nb))
        cur = np.unique(np.concatenate([nb.reshape(-1), cur]))
    return S


def model_forward(p, feats, nodeset, n_layers, T, w_table, nb_table, out_dim, layers=None):
    """PinSageModel.forward (pinsage_model.py:246-265) on torch-CPU tensors;
    `layers` (relevant_nodes_fly) replaces the table's frontier (:247-249)."""
    if layers is None:
        layers = frontier(np.asarray(nodeset), n_layers, T, w_table, nb_table)
    in_dims = [feats.shape[1]] + [out_dim] * (n_layers - 1)
    h = feats
    y = None
    for i, (ns, w, nb) in enumerate(layers):
        ns_t, w_t, nb_t = (torch.from_numpy(np.ascontiguousarray(a)) for a in (ns, w, nb))
        y = conv_layer(p, i, h, ns_t, nb_t, w_t, in_dims[i])
        h = _put(h, ns_t, y)
    z = _linear(p, "G2.weight", None, F.leaky_relu(_linear(p, "G1.weight", "G1.bias", y)))
    idx = torch.from_numpy(np.asarray(nodeset, np.int64))
    h = _put(h, idx, z)
    return h[idx, :out_dim]


def max_margin_loss(hq, hp, hn, margin):
    """pinsage_training.py:31-41 (hinge on normalised dot products, batch mean)."""
    hq, hp, hn = (F.normalize(x, dim=1) for x in (hq, hp, hn))
    d = (hq * hn).sum(1) - (hq * hp).sum(1) + margin
    return torch.clamp(d, min=0.0).mean()


def triplet_monitors(feats, hq, batch):
    """train_batch monitors (pinsage_training.py:200-212)."""
    fq, fp, fn = (F.normalize(feats[batch[:, c]], dim=1) for c in range(3))
    dpos = 1 - F.cosine_similarity(fq, fp)
    dneg = 1 - F.cosine_similarity(fq, fn)
    nfl = torch.clamp(dpos - dneg + 1e-4, min=0.0).mean()
    var = ((hq - hq.mean(0)) ** 2).sum() / (hq.shape[0] - 1)
    return nfl, var


class RefTrainer:
    """One reference train step, restated: 3 forwards, hinge loss, Adam (CPU)."""

    def __init__(self, state, feats, w_table, nb_table, n_layers=2, T=3, out_dim=128, lr=1e-4,
                 margin=1e-5):
        self.p = {k: torch.tensor(np.asarray(v), dtype=torch.float32).requires_grad_()
                  for k, v in state.items()}
        self.order = param_names(n_layers)
        self.opt = torch.optim.Adam([self.p[k] for k in self.order], lr=lr)
        self.feats = feats
        self.w, self.nb = w_table, nb_table
        self.L, self.T, self.out, self.margin = n_layers, T, out_dim, margin

    def step(self, batch):
        b = np.asarray(batch)
        hs = [model_forward(self.p, self.feats, b[:, c], self.L, self.T, self.w, self.nb, self.out)
              for c in range(3)]
        loss = max_margin_loss(*hs, self.margin)
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.order}
        self.opt.step()
        with torch.no_grad():
            nfl, var = triplet_monitors(self.feats, hs[0], torch.from_numpy(b))
        return float(loss), float(nfl), float(var), grads

    def step_fly(self, batch, graph, n_hops, alpha, mt):
        """The reference train step with on-the-fly sampling: each of the three
        model calls walks its own nodeset (q, pos, neg in order) with the MT
        stream `mt`; graph = (indptr, indices, n_all).  Returns (loss,
        grads, per-call layers)."""
        b = np.asarray(batch)
        indptr, indices, n_all = graph
        hs, lays = [], []
        for c in range(3):
            lay = relevant_nodes_fly(indptr, indices, n_all, b[:, c], self.L, n_hops, alpha, self.T, mt)
            lays.append(lay)
            hs.append(model_forward(self.p, self.feats, b[:, c], self.L, self.T, None, None, self.out,
                                    layers=lay))
        loss = max_margin_loss(*hs, self.margin)
        self.opt.zero_grad()
        loss.backward()
        grads = {k: self.p[k].grad.detach().clone() for k in self.order}
        self.opt.step()
        return float(loss.detach()), grads, lays

    def step_dp(self, batch, world):
        """Data-parallel restatement of one step: ``world`` ranks each run the
        reference train step's forwards and backward on their contiguous slice
        of the global batch (so put_embeddings' repeated-id semantics hold per
        rank), the gradients are averaged (the all-reduce), then one Adam step.
        Returns the per-rank losses."""
        b = np.asarray(batch)
        B = b.shape[0] // world
        self.opt.zero_grad()
        losses = []
        for r in range(world):
            sl = b[r * B:(r + 1) * B]
            hs = [model_forward(self.p, self.feats, sl[:, c], self.L, self.T, self.w, self.nb,
                                self.out) for c in range(3)]
            loss = max_margin_loss(*hs, self.margin)
            (loss / world).backward()
            losses.append(float(loss.detach()))
        self.opt.step()
        return losses


# ----------------------------------------------------------------------------- lib/gnns
def gnns_mean_aggregate(nodes, emb, unique, samp, adj_indptr, adj_indices, adj_data, gcn):
    """``GNN_model.aggregate`` with agg_func 'MEAN', gat False
    (lib/gnns/GNNs_unsupervised.py:537-588) as the reference computes it: a
    dense [F, U] float32 mask of ones at the sampled neighbours (the node itself
    dropped unless gcn, :543-544), times sqrt(edge count) (:553-554, float32),
    L1-normalised per row with eps 1e-12 (F.normalize, :572), then mask @ emb
    (:577) where emb is the unique-node rows unless it already has U rows
    (:546-549).  ``samp`` is a list of iterables (the sampled sets).
    Returns (agg [F, d], mask [F, U], emb_rows) so a test can form gradients."""
    U = len(unique)
    col_of = {int(u): j for j, u in enumerate(unique)}
    mask = np.zeros((len(nodes), U), np.float32)
    for i, s in enumerate(samp):
        s = {int(x) for x in s}
        if not gcn:
            s = s - {int(nodes[i])}
        for v in s:
            mask[i, col_of[v]] = 1.0
    # edge_counts = adj_matrix[nodes][:, unique_nodes_list].toarray() (:553)
    ec = np.zeros((len(nodes), U), np.float32)
    for i, r in enumerate(nodes):
        for p in range(int(adj_indptr[r]), int(adj_indptr[r + 1])):
            c = int(adj_indices[p])
            if c in col_of:
                ec[i, col_of[c]] = np.float32(adj_data[p])
    mask = mask * np.sqrt(ec, dtype=np.float32)
    den = np.maximum(np.abs(mask).sum(1, keepdims=True, dtype=np.float32), np.float32(1e-12))
    mask = (mask / den).astype(np.float32)
    rows = np.arange(U) if len(emb) == U else np.asarray(unique, np.int64)
    agg = (mask.astype(np.float64) @ np.asarray(emb, np.float64)[rows]).astype(np.float32)
    return agg, mask, rows


def gnns_mean_aggregate_grad(mask, rows, G, n_emb):
    """d(sum(agg * G)) / d emb for gnns_mean_aggregate: mask^T G scattered to
    the embedding rows it read."""
    g = np.zeros((n_emb, G.shape[1]), np.float64)
    np.add.at(g, rows, mask.T.astype(np.float64) @ np.asarray(G, np.float64))
    return g.astype(np.float32)
