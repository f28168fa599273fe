"""The GPU paths of the reference's evaluation side that sit next to the
PinSage train step: personalised-PageRank
neighbours (``PersPageRank``, baselines.py:106-151) on the walk + top-k
kernels, and cosine k-nearest neighbours over an embedding table
(``cosine_sim_ab`` / ``knn_from_emb``, baselines.py:69-103) with the
``save_knn`` / ``load_knn`` cache format of eval.py:112-149.

The reference's other baseline recommenders (node2vec, implicit ALS,
networkx similarities, lib/gnns) are out of scope; their libraries are not
part of this build.  Names, signatures, return types and RNG consumption
follow the reference; compute runs in HIP (no CPU fallback).
"""
from __future__ import annotations

import os
import time
from abc import ABC, abstractmethod

import torch

import _native as nat
import pinsage_model as psm

PRECOMP_K = 1000  # eval.py:31
# dot products of one batch of query rows live in this much device scratch
KNN_SCRATCH_BYTES = int(os.environ.get("PINSAGE_KNN_SCRATCH_MB", "2048")) << 20


class PredictionModel(ABC):
    """Base recommender class (baselines.py:33-46)."""

    @abstractmethod
    def __init__(self):
        pass

    @abstractmethod
    def train(self, g, ids, train_set, test_set, features):
        pass

    @abstractmethod
    def knn(self, nodeset, k):
        pass


class EmbeddingModel(PredictionModel):
    """An embedding-based recommender (baselines.py:48-53)."""

    @abstractmethod
    def embed(self, nodeset):
        pass


def cosine_sim_ab(a, b, eps=1e-16):
    """Pairwise cosine similarities [len(a), len(b)] (baselines.py:69-77), on the
    inputs' device with the reference's formula dot / (|a| |b|^T + eps)."""
    dot_prod = torch.mm(a, b.transpose(1, 0))
    lengths_mat = torch.mm(torch.norm(a, dim=1).unsqueeze(1), torch.norm(b, dim=1).unsqueeze(0))
    return dot_prod / (lengths_mat + eps)


def _knn_cosine(emb, q, k_total, eps=1e-16):
    """Top-k_total cosine neighbours of rows q of emb (HIP: MFMA dot products +
    per-row radix select), sorted descending: (w f32 [nq, k], n i64 [nq, k])."""
    nat.require_gpu()
    e = torch.as_tensor(emb)
    out_dev = e.device
    e = e.to(device="cuda", dtype=torch.float32).contiguous()
    qs = torch.as_tensor(q).reshape(-1).to(torch.int64).contiguous()
    n, d = int(e.shape[0]), int(e.shape[1])
    if qs.numel() and (int(qs.min()) < 0 or int(qs.max()) >= n):
        raise IndexError(f"knn: query ids out of range for {n} rows")
    if d % 4:  # the MFMA GEMM loads 16-byte row chunks: zero columns change no dot product
        e = torch.nn.functional.pad(e, (0, 4 - d % 4))
        d = int(e.shape[1])
    qd = qs.to("cuda")
    nq = int(qd.numel())
    w = torch.empty((nq, k_total), dtype=torch.float32, device="cuda")
    nb = torch.empty((nq, k_total), dtype=torch.int64, device="cuda")
    L = nat.lib()
    rows = max(1, min(nq, (KNN_SCRATCH_BYTES - 8 * n) // max(1, 4 * n)))
    nbytes = L.pinsage_knn_scratch_bytes(n, rows)
    scratch = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    nat.check(L.pinsage_knn_cosine(nat.ptr(e), n, d, d, nat.ptr(qd), nq, int(k_total), float(eps),
                                   nat.ptr(scratch), nbytes, nat.ptr(w), nat.ptr(nb),
                                   nat.stream_ptr()), "knn_cosine")
    return w.to(out_dev), nb.to(out_dev)


def knn_from_emb(emb, q, k, sim_func=None):
    """k nearest neighbours of the nodes q by cosine similarity of their
    embeddings (baselines.py:91-103): top k+1 per query, first column dropped
    (the reference assumes it is the query itself).  ``sim_func`` is accepted
    and ignored, as in the reference (cosine_sim_ab is always used)."""
    w, nb = _knn_cosine(emb, q, int(k) + 1)
    return w[:, 1:], nb[:, 1:]


class PersPageRank(PredictionModel):
    """Nearest graph neighbours via PPR aka random walks with restarts
    (baselines.py:106-151): 1000 hops, restart 0.85; the walk consumes torch's
    generator exactly like the reference loop (pinsage_model's MT19937 mode)."""

    def __init__(self):
        self.n_hops = 1000
        self.alpha = 0.85

    def visit_prob(self, g, nodeset, n_hops, alpha):
        """Dense f64 visit probabilities [len(nodeset), N_all], self column zeroed."""
        return psm.sample_neighborhood(g, None, nodeset, n_hops, alpha)

    def train(self, g, ids, train_set, test_set, features):
        self.g = g

    def knn(self, nodeset, k):
        """visit_prob(...).topk(k, 1) without the dense matrix (walk + top-k kernels)."""
        return psm.sample_neighborhood_topt(self.g, None, nodeset, self.n_hops, self.alpha, k)


class EmbeddingTable(EmbeddingModel):
    """kNN over a fixed embedding table (e.g. PinSage.embed output): the
    embed/knn pair of the reference's EmbeddingModel wrappers
    (baselines.py:324-328)."""

    def __init__(self, embedding=None):
        self.embedding = embedding

    def train(self, g, ids, train_set, test_set, features):
        pass

    def embed(self, nodeset):
        return self.embedding[nodeset, :]

    def knn(self, nodeset, k):
        return knn_from_emb(self.embedding, nodeset, k)


def save_knn(model, model_name, ids, save_dir, train_time=0, emb_time=0, b_size=1000):
    """eval.py:112-143: kNN lists of all nodes (k = PRECOMP_K) in batches, saved
    once as (w, n, train_time, emb_time, knn_time) to <save_dir>/knn/<name>.pt."""
    save_dir = os.path.join(save_dir, "knn")
    os.makedirs(save_dir, exist_ok=True)
    save_path = os.path.join(save_dir, model_name + ".pt")
    if os.path.isfile(save_path):
        return
    all_nodes = torch.arange(0, len(ids), dtype=torch.int64)
    n = len(all_nodes)
    knn_time = 0.0
    ws, ns = [], []
    for i in range(0, n, b_size):
        t0 = time.time()
        bw, bn = model.knn(all_nodes[i:min(i + b_size, n)], PRECOMP_K)
        ws.append(bw)
        ns.append(bn)
        knn_time += time.time() - t0
    torch.save((torch.cat(ws, dim=0), torch.cat(ns, dim=0), train_time, emb_time, knn_time),
               save_path)


def load_knn(model_name, ids, save_dir):
    """eval.py:146-149 (weights-only load: the file holds tensors and floats)."""
    return torch.load(os.path.join(save_dir, "knn", model_name + ".pt"), weights_only=True)


__all__ = ["PRECOMP_K", "PredictionModel", "EmbeddingModel", "cosine_sim_ab", "knn_from_emb",
           "PersPageRank", "EmbeddingTable", "save_knn", "load_knn"]
