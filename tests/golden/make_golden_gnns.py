"""Golden fixtures for the lib/gnns MEAN aggregator, from the REAL reference.

Runs only in the development container (it imports
/root/reference/lib/gnns/GNNs_unsupervised.py, which never travels to the GPU
box).  Calls the reference's ``GNN_model._get_unique_neighs_list`` and
``GNN_model.aggregate`` (agg_func 'MEAN') as unbound functions on a plain
namespace holding the attributes they read, on a small random weighted graph,
and stores inputs and outputs (plus the gradient of a fixed linear functional
of the output w.r.t. the embeddings) as plain .npz (no pickle).

    python tests/golden/make_golden_gnns.py
"""
from __future__ import annotations

import importlib.util
import os
import random
import sys
import types

import numpy as np
import scipy.sparse as sp
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/lib/gnns/GNNs_unsupervised.py"


def _ref_module():
    sys.dont_write_bytecode = True  # nothing is written into the reference tree
    spec = importlib.util.spec_from_file_location("_ref_gnns_unsup", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _graph(n, seed):
    rng = np.random.default_rng(seed)
    m = n * 4
    u = rng.integers(0, n - 3, m)
    v = rng.integers(0, n - 3, m)
    keep = u != v
    u, v = u[keep], v[keep]
    w = rng.integers(1, 5, len(u)).astype(np.float64)
    a = sp.coo_matrix((np.concatenate([w, w]), (np.concatenate([u, v]), np.concatenate([v, u]))),
                      shape=(n, n)).tocsr()
    a.sum_duplicates()
    # two self loops (gcn keeps the node itself in its set: its count is sqrt'ed too)
    a = a.tolil()
    a[0, 0] = 2.0
    a[5, 5] = 1.0
    a = a.tocsr()
    a.sort_indices()
    # the last 3 nodes are isolated (an empty mask row after the self node is removed)
    return a


def _case(mod, name, adj, nodes, gcn, num_sample, d, embeds_rows, seed, out):
    n = adj.shape[0]
    adj_list = {}
    for i in range(n):  # DataLoader.get_adj_list (GNNs_unsupervised.py:245-251)
        adj_list[i] = set(np.where(adj[i].toarray() != 0)[1])
    ns = types.SimpleNamespace(adj_lists=adj_list, adj_matrix=adj, gcn=gcn, gat=False, agg_func="MEAN")
    random.seed(seed)
    uniq, samp, uniq_map = mod.GNN_model._get_unique_neighs_list(ns, nodes, num_sample=num_sample)
    g = torch.Generator().manual_seed(seed)
    if embeds_rows == "unique":
        emb = torch.randn(len(uniq), d, generator=g)
    else:
        emb = torch.randn(n, d, generator=g)
    emb.requires_grad_(True)
    agg = mod.GNN_model.aggregate(ns, nodes, emb, (uniq, samp, uniq_map))
    G = torch.randn(agg.shape, generator=g)
    (agg * G).sum().backward()
    samp_ptr = np.zeros(len(samp) + 1, np.int64)
    np.cumsum([len(s) for s in samp], out=samp_ptr[1:])
    out[name] = dict(
        nodes=np.asarray(nodes, np.int64), gcn=np.int64(gcn), num_sample=np.int64(num_sample),
        seed=np.int64(seed), unique=np.asarray([int(x) for x in uniq], np.int64),
        samp_ptr=samp_ptr, samp=np.asarray([int(x) for s in samp for x in s], np.int64),
        emb=emb.detach().numpy(), G=G.numpy(), agg=agg.detach().numpy(), grad=emb.grad.numpy())


def main():
    mod = _ref_module()
    adj = _graph(300, 3)
    n = adj.shape[0]
    res = {}
    rng = np.random.default_rng(7)
    nodes = [int(x) for x in rng.choice(n - 3, 60, replace=False)] + [n - 1, n - 2, 0, 5]
    _case(mod, "sage", adj, nodes, False, 5, 48, "all", 11, res)
    _case(mod, "gcn", adj, nodes, True, 10, 64, "unique", 12, res)
    _case(mod, "sage_odd_d", adj, nodes[:20], False, 3, 30, "all", 13, res)
    flat = {"adj_indptr": adj.indptr.astype(np.int64), "adj_indices": adj.indices.astype(np.int64),
            "adj_data": adj.data.astype(np.float64), "n": np.int64(n)}
    for case, d in res.items():
        for k, v in d.items():
            flat[f"{case}__{k}"] = v
    np.savez_compressed(os.path.join(HERE, "gnns_mean.npz"), **flat)
    print("wrote gnns_mean.npz:", {k: res[k]["agg"].shape for k in res})


if __name__ == "__main__":
    main()
