"""The lib/gnns MEAN aggregator on the GPU.

``GNN_model.aggregate`` (lib/gnns/GNNs_unsupervised.py:537-588, agg_func
'MEAN', gat False) builds a dense [F, U] mask -- ones at each sampled
neighbour (the node itself removed unless ``gcn``), times sqrt(edge count)
from the adjacency matrix, L1-normalised per row (``F.normalize(p=1)``) -- and
returns ``mask.mm(embed_matrix)``.  The mask holds a handful of non-zeros per
row, so here it stays a CSR and the product is the segmented weighted mean
``pinsage_segment_wmean`` (csrc/gnns.hip): one gather-and-accumulate pass over
the neighbour rows, no [F, U] buffer.  Gradients flow to ``pre_hidden_embs``
through the transposed CSR (same kernel, fixed summation order, no atomics).

Host-side neighbour sampling (``_get_unique_neighs_list``,
GNNs_unsupervised.py:522-535) stays Python, with the reference's own
``random.sample`` / set semantics, so the unique-node order and the sampled
sets are the reference's.  Compute runs in HIP only (no CPU fallback).
"""
from __future__ import annotations

import random

import numpy as np
import torch

import _native as nat


def get_unique_neighs_list(adj_lists, nodes, num_sample=10, gcn=False, gat=False):
    """``GNN_model._get_unique_neighs_list`` (GNNs_unsupervised.py:522-535):
    returns ``(unique_nodes_list, samp_neighs, unique_nodes)`` with the same
    ``random.sample`` draws and set orders as the reference."""
    to_neighs = [adj_lists[int(node)] for node in nodes]
    if gcn or gat:
        samp_neighs = to_neighs
    else:
        samp_neighs = [set(random.sample(tuple(to_neigh), num_sample)) if len(to_neigh) >= num_sample
                       else to_neigh for to_neigh in to_neighs]
    samp_neighs = [samp_neigh | {nodes[i]} for i, samp_neigh in enumerate(samp_neighs)]
    unique_nodes_list = list(set.union(*samp_neighs))
    unique_nodes = dict(zip(unique_nodes_list, range(len(unique_nodes_list))))
    return unique_nodes_list, samp_neighs, unique_nodes


def mask_csr(nodes, pre_neighs, adj_matrix, gcn=False, gat=False):
    """The aggregation mask of GNNs_unsupervised.py:540-574 as a CSR over the
    unique-node columns: (seg_ptr int64 [F+1], cols int64, w float32).  The
    weights are the mask entries before normalisation: 1 * sqrt(edge count),
    in float32 as the reference (edge counts go through torch.FloatTensor)."""
    unique_nodes_list, samp_neighs, unique_nodes = pre_neighs
    assert len(nodes) == len(samp_neighs)
    assert all(nodes[i] in samp_neighs[i] for i in range(len(samp_neighs)))
    if not gat and not gcn:
        samp_neighs = [samp_neighs[i] - {nodes[i]} for i in range(len(samp_neighs))]
    counts = [len(s) for s in samp_neighs]
    seg_ptr = np.zeros(len(samp_neighs) + 1, np.int64)
    np.cumsum(counts, out=seg_ptr[1:])
    rows = np.repeat(np.asarray([int(n) for n in nodes], np.int64), counts)
    members = [n for s in samp_neighs for n in s]
    cols = np.fromiter((unique_nodes[n] for n in members), np.int64, count=len(members))
    # edge_counts = adj_matrix[nodes][:, unique_nodes_list] at the mask's non-zeros
    adj = adj_matrix.tocsr()
    ec = np.asarray(adj[rows, np.asarray(members, np.int64)]).reshape(-1) if len(members) else \
        np.zeros(0)
    w = np.sqrt(ec.astype(np.float32))
    return seg_ptr, cols, w


class _SegmentWMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, seg_ptr, cols, w, n_seg, fwd_T):
        out = torch.empty((n_seg, h.shape[1]), dtype=torch.float32, device=h.device)
        nat.check(nat.lib().pinsage_segment_wmean(
            nat.ptr(h), h.stride(0), h.shape[0], h.shape[1], nat.ptr(seg_ptr), nat.ptr(cols), nat.ptr(w),
            n_seg, 1, nat.ptr(out), out.stride(0), nat.stream_ptr()), "segment_wmean")
        ctx.n_h = h.shape[0]
        ctx.fwd_T = fwd_T
        return out

    @staticmethod
    def backward(ctx, dout):
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        dout = dout.contiguous()
        rows_u, segT, colsT, wT = ctx.fwd_T
        du = torch.empty((rows_u.numel(), dout.shape[1]), dtype=torch.float32, device=dout.device)
        nat.check(nat.lib().pinsage_segment_wmean(
            nat.ptr(dout), dout.stride(0), dout.shape[0], dout.shape[1], nat.ptr(segT), nat.ptr(colsT),
            nat.ptr(wT), rows_u.numel(), 0, nat.ptr(du), du.stride(0), nat.stream_ptr()), "segment_wmean_bwd")
        dh = torch.zeros((ctx.n_h, dout.shape[1]), dtype=torch.float32, device=dout.device)
        dh.index_copy_(0, rows_u, du)
        return dh, None, None, None, None, None


def _transpose(seg_ptr, hrows, w, n_h):
    """CSR of the mask's transpose over the touched h rows, with the row
    normalisation folded into the weights (the backward's dH = mask^T dOut)."""
    F = len(seg_ptr) - 1
    counts = np.diff(seg_ptr)
    seg_of = np.repeat(np.arange(F, dtype=np.int64), counts)
    den = np.zeros(F, np.float32)
    np.add.at(den, seg_of, np.abs(w))
    wn = (w / np.maximum(den, np.float32(1e-12))[seg_of]).astype(np.float32)
    order = np.argsort(hrows, kind="stable")
    hs = hrows[order]
    rows_u, start = np.unique(hs, return_index=True)
    segT = np.append(start, len(hs)).astype(np.int64)
    return rows_u, segT, seg_of[order].astype(np.int32), wn[order]


def mean_aggregate(nodes, pre_hidden_embs, pre_neighs, adj_matrix, gcn=False, gat=False):
    """``GNN_model.aggregate`` with agg_func 'MEAN' (GNNs_unsupervised.py:537-588):
    returns ``mask.mm(embed_matrix)`` as float32 [len(nodes), d] on the GPU,
    differentiable w.r.t. ``pre_hidden_embs``.  ``embed_matrix`` is
    ``pre_hidden_embs`` itself when it has exactly len(unique_nodes) rows (the
    reference's shortcut at :546-549), otherwise its unique-node rows."""
    if gat:
        raise NotImplementedError("the GAT attention mask (GNNs_unsupervised.py:555-565) is not built; "
                                  "only the MEAN aggregator is on this path")
    dev = nat.device()
    unique_nodes_list, _, unique_nodes = pre_neighs
    seg_ptr, cols, w = mask_csr(nodes, pre_neighs, adj_matrix, gcn=gcn)
    h = pre_hidden_embs
    if not torch.is_tensor(h):
        h = torch.as_tensor(np.asarray(h))
    if h.dtype != torch.float32 or h.device != dev or not h.is_contiguous():
        h = h.to(device=dev, dtype=torch.float32).contiguous()
    if len(h) == len(unique_nodes):
        hrows = cols
    else:
        hrows = np.asarray(unique_nodes_list, np.int64)[cols]
    if len(hrows) and (hrows.min() < 0 or hrows.max() >= len(h)):
        raise IndexError("aggregate: neighbour row out of range of pre_hidden_embs")
    fwd_T = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev)
                  for a in _transpose(seg_ptr, hrows, w, len(h)))
    return _SegmentWMean.apply(h, torch.from_numpy(seg_ptr).to(dev),
                               torch.from_numpy(hrows.astype(np.int32)).to(dev),
                               torch.from_numpy(w.astype(np.float32)).to(dev), len(nodes), fwd_T)


class MeanAggregator:
    """The aggregation half of ``GNN_model`` (GNNs_unsupervised.py:467-588) for
    agg_func 'MEAN': holds the adjacency matrix / lists and the gcn flag, and
    exposes the reference's ``_get_unique_neighs_list`` and ``aggregate``."""

    def __init__(self, adj_matrix, adj_lists, gcn=False, num_sample=10):
        self.adj_matrix = adj_matrix
        self.adj_lists = adj_lists
        self.gcn = gcn
        self.gat = False
        self.agg_func = "MEAN"
        self.num_sample = num_sample

    def _get_unique_neighs_list(self, nodes, num_sample=None):
        return get_unique_neighs_list(self.adj_lists, nodes, self.num_sample if num_sample is None
                                      else num_sample, gcn=self.gcn, gat=self.gat)

    def aggregate(self, nodes, pre_hidden_embs, pre_neighs):
        return mean_aggregate(nodes, pre_hidden_embs, pre_neighs, self.adj_matrix, gcn=self.gcn)
