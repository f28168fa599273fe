"""lib/gnns MEAN aggregator (GNNs_unsupervised.py:537-588).

CPU: the oracle restatement and the product's host side (neighbour sampling
with the reference's random.sample / set semantics, the mask CSR) against the
fixtures made by running the reference (tests/golden/make_golden_gnns.py).
GPU: ``gnns.mean_aggregate`` (HIP pinsage_segment_wmean) forward and gradient
against the same fixtures, fp32 tolerance 1e-5 relative (the reference is an
fp32 dense mm; the kernel sums the same products in a different order).
"""
import random

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden
from oracle import oracle as orc

CASES = ("sage", "gcn", "sage_odd_d")


def _load():
    d = golden("gnns_mean")
    n = int(d["n"])
    adj = sp.csr_matrix((d["adj_data"], d["adj_indices"], d["adj_indptr"]), shape=(n, n))
    return d, adj


def _case(d, c):
    g = {k.split("__", 1)[1]: v for k, v in d.items() if k.startswith(c + "__")}
    sp_ = g["samp_ptr"]
    g["samp_sets"] = [set(int(x) for x in g["samp"][sp_[i]:sp_[i + 1]]) for i in range(len(sp_) - 1)]
    return g


def _adj_lists(adj):
    # DataLoader.get_adj_list (GNNs_unsupervised.py:245-251): ascending column ids
    return {i: set(int(x) for x in adj.indices[adj.indptr[i]:adj.indptr[i + 1]])
            for i in range(adj.shape[0])}


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    d, adj = _load()
    g = _case(d, case)
    agg, mask, rows = orc.gnns_mean_aggregate(g["nodes"], g["emb"], g["unique"], g["samp_sets"],
                                              d["adj_indptr"], d["adj_indices"], d["adj_data"],
                                              bool(g["gcn"]))
    assert _rel(agg, g["agg"]) < 1e-6
    grad = orc.gnns_mean_aggregate_grad(mask, rows, g["G"], len(g["emb"]))
    assert _rel(grad, g["grad"]) < 1e-6
    # the isolated nodes' rows (no neighbours once the node itself is dropped) are zero
    if not g["gcn"]:
        iso = [i for i, v in enumerate(g["nodes"]) if adj.indptr[v] == adj.indptr[v + 1]]
        assert np.all(g["agg"][iso] == 0)
        assert iso or case != "sage"


@pytest.mark.parametrize("case", CASES)
def test_host_sampling_matches_reference(case):
    import gnns
    d, adj = _load()
    g = _case(d, case)
    random.seed(int(g["seed"]))
    uniq, samp, _ = gnns.get_unique_neighs_list(_adj_lists(adj), [int(x) for x in g["nodes"]],
                                                int(g["num_sample"]), gcn=bool(g["gcn"]))
    assert [int(x) for x in uniq] == g["unique"].tolist()
    assert [set(int(x) for x in s) for s in samp] == g["samp_sets"]


@pytest.mark.parametrize("case", CASES)
def test_mask_csr_matches_oracle_mask(case):
    import gnns
    d, adj = _load()
    g = _case(d, case)
    uniq = [int(x) for x in g["unique"]]
    pre = (uniq, g["samp_sets"], {u: j for j, u in enumerate(uniq)})
    nodes = [int(x) for x in g["nodes"]]
    seg, cols, w = gnns.mask_csr(nodes, pre, adj, gcn=bool(g["gcn"]))
    _, mask, _ = orc.gnns_mean_aggregate(nodes, g["emb"], uniq, g["samp_sets"], d["adj_indptr"],
                                         d["adj_indices"], d["adj_data"], bool(g["gcn"]))
    dense = np.zeros_like(mask)
    for i in range(len(nodes)):
        dense[i, cols[seg[i]:seg[i + 1]]] = w[seg[i]:seg[i + 1]]
    den = np.maximum(np.abs(dense).sum(1, keepdims=True), np.float32(1e-12))
    assert np.array_equal(dense / den, mask)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_mean_aggregate_matches_reference(case):
    import torch

    import gnns
    d, adj = _load()
    g = _case(d, case)
    uniq = [int(x) for x in g["unique"]]
    pre = (uniq, g["samp_sets"], {u: j for j, u in enumerate(uniq)})
    emb = torch.from_numpy(g["emb"]).cuda().requires_grad_(True)
    agg = gnns.MeanAggregator(adj, _adj_lists(adj), gcn=bool(g["gcn"])).aggregate(
        [int(x) for x in g["nodes"]], emb, pre)
    assert agg.is_cuda and agg.dtype == torch.float32
    assert _rel(agg.detach().cpu().numpy(), g["agg"]) < 1e-5
    (agg * torch.from_numpy(g["G"]).cuda()).sum().backward()
    assert _rel(emb.grad.cpu().numpy(), g["grad"]) < 1e-5


@pytest.mark.gpu
def test_gpu_segment_wmean_sizes_and_edges():
    """Larger random CSR (ragged rows incl. empty ones, a hub row of 5000
    entries, d not a multiple of 4) against a float64 restatement."""
    import torch

    import _native as nat
    rng = np.random.default_rng(0)
    n_h, F = 20000, 3000
    counts = rng.integers(0, 40, F)
    counts[:50] = 0
    counts[70] = 5000
    seg = np.zeros(F + 1, np.int64)
    np.cumsum(counts, out=seg[1:])
    cols = rng.integers(0, n_h, seg[-1]).astype(np.int32)
    w = rng.random(seg[-1]).astype(np.float32) + 0.1
    dev = [torch.from_numpy(a).cuda() for a in (seg, cols, w)]
    for d in (128, 30):
        h = rng.standard_normal((n_h, d)).astype(np.float32)
        ref = np.zeros((F, d))
        for i in range(F):
            s = slice(seg[i], seg[i + 1])
            den = max(float(np.abs(w[s]).sum(dtype=np.float32)), 1e-12)
            ref[i] = (w[s].astype(np.float64) / den) @ h[cols[s]].astype(np.float64)
        ht = torch.from_numpy(h).cuda()
        out = torch.full((F, d), float("nan"), device="cuda")
        nat.check(nat.lib().pinsage_segment_wmean(nat.ptr(ht), d, n_h, d, nat.ptr(dev[0]), nat.ptr(dev[1]),
                                                  nat.ptr(dev[2]), F, 1, nat.ptr(out), d, nat.stream_ptr()),
                  "segment_wmean")
        o = out.cpu().numpy()
        assert np.all(o[:50] == 0)
        assert np.abs(o - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max())
