"""Drop-in ``spotify_graph`` (reference ``spotify_graph.py:15-110``).

JSON dataset -> CSR graph (tracks first, then collections), z-scored node
features, positive pairs.  ``to_dgl_graph`` returns a :class:`graph.CSRGraph`
(the DGL subset the PinSage path uses) instead of a ``dgl.DGLGraph``.

Binary cache: parsing a 0.5-0.8 GB graph.json and
torch-loading one feature file per track dominate a cold start.  The first
``to_dgl_graph`` writes ``<dir>/pinsage_cache/graph.npz`` (CSR + the edge
list in file order) and ``features.npz`` (the z-scored matrix), each keyed by
the size and mtime of its sources; later loads read those and never parse
graph.json (``self.graph`` is loaded on first access).  Plain ``.npz`` (no
pickle); an unwritable dataset directory just skips the cache.
"""
from __future__ import annotations

import json
import os
from os import path

import numpy as np
import torch

from graph import CSRGraph


class SpotifyGraph:

    def __init__(self, dir, features_dir):
        self.base_dir = dir
        self.nbhds_path = os.path.join(self.base_dir, "neighborhoods.pt")
        self.tracks_pth = path.join(dir, "tracks.json")
        self.col_pth = path.join(dir, "collections.json")
        self.graph_pth = path.join(dir, "graph.json")
        self.img_dir = path.join(dir, "images")
        self.clip_dir = path.join(dir, "clips")

        print("Loading graph...")
        with open(self.tracks_pth, "r", encoding="utf-8") as f:
            self.tracks = json.load(f)
        with open(self.col_pth, "r", encoding="utf-8") as f:
            self.collections = json.load(f)
        self._graph = None  # graph.json: parsed on first access (the CSR cache avoids it)
        self.ft_dir = features_dir if (features_dir and os.path.isdir(features_dir)) else None
        self.features_dict = {}
        self.cache_dir = os.path.join(self.base_dir, CACHE_DIR)

    @property
    def graph(self):
        if self._graph is None:
            with open(self.graph_pth, "r", encoding="utf-8") as f:
                self._graph = json.load(f)
        return self._graph

    @graph.setter
    def graph(self, value):
        self._graph = value

    def to_dgl_graph(self):
        """(g, track_ids, col_ids, features); node ids = tracks.json order then
        collections.json order; edges in graph.json order (spotify_graph.py:41-85)."""
        track_ids = list(self.tracks)
        col_ids = list(self.collections)
        n_t = len(track_ids)
        n_all = n_t + len(col_ids)
        g = self._cached_graph(n_all)
        if g is None:
            index_map = {nid: i for i, nid in enumerate(track_ids)}
            for j, cid in enumerate(col_ids):
                index_map[cid] = n_t + j
            edges = self.graph["edges"]
            src = np.fromiter((index_map[e["from"]] for e in edges), np.int64, len(edges))
            dst = np.fromiter((index_map[e["to"]] for e in edges), np.int64, len(edges))
            g = CSRGraph(n_all, src, dst, base_dir=self.base_dir, nbhds_path=self.nbhds_path)
            self._store_graph(g)

        features = None
        if self.ft_dir:
            features = self._cached_features(n_t)
            if features is None:
                vecs = [torch.load(os.path.join(self.ft_dir, tid + ".pt"), weights_only=True)
                        for tid in track_ids]
                features = torch.stack(vecs, dim=0)
                mean = features.mean(dim=0)
                std = features.std(dim=0, unbiased=True) + 1e-12
                features = (features - mean) / std
                self._store_features(features)

        self.g, self.track_ids, self.col_ids, self.features = g, track_ids, col_ids, features
        return g, track_ids, col_ids, features

    # ---- binary cache
    def _graph_key(self):
        return _fingerprint([self.tracks_pth, self.col_pth, self.graph_pth])

    def _cached_graph(self, n_all):
        p = os.path.join(self.cache_dir, "graph.npz")
        try:
            with np.load(p, allow_pickle=False) as z:
                if bytes(z["key"]).decode() != self._graph_key() or int(z["n_all"]) != n_all:
                    return None
                g = CSRGraph.from_csr(z["indptr"], z["indices"], base_dir=self.base_dir,
                                      nbhds_path=self.nbhds_path)
                g._src = z["src"].astype(np.int64)
                g._dst = z["dst"].astype(np.int64)
                return g
        except (OSError, KeyError, ValueError):
            return None

    def _store_graph(self, g):
        src, dst = g._coo()
        _atomic_save(os.path.join(self.cache_dir, "graph.npz"), np.savez,
                     key=np.frombuffer(self._graph_key().encode(), np.uint8), n_all=np.int64(g._n),
                     indptr=g.indptr, indices=g.indices, src=src.astype(np.int32),
                     dst=dst.astype(np.int32))

    def _features_key(self):
        return _fingerprint([self.tracks_pth, self.ft_dir])

    def _cached_features(self, n_t):
        try:
            with np.load(os.path.join(self.cache_dir, "features.npz"), allow_pickle=False) as z:
                if bytes(z["key"]).decode() != self._features_key() or z["x"].shape[0] != n_t:
                    return None
                return torch.from_numpy(np.array(z["x"]))
        except (OSError, KeyError, ValueError):
            return None

    def _store_features(self, features):
        _atomic_save(os.path.join(self.cache_dir, "features.npz"), np.savez,
                     key=np.frombuffer(self._features_key().encode(), np.uint8),
                     x=features.detach().cpu().numpy())

    def load_positives(self, pos_pth):
        """[P, 2] int64 track-index pairs (spotify_graph.py:88-100).  Like the
        reference, draws one unused randperm(P) from the global generator."""
        with open(pos_pth, "r", encoding="utf-8") as f:
            positives = json.load(f)
        index_map = {nid: i for i, nid in enumerate(self.tracks)}
        a = torch.tensor([index_map[p["a"]] for p in positives], dtype=torch.int64)
        b = torch.tensor([index_map[p["b"]] for p in positives], dtype=torch.int64)
        _burn_randperm(a.shape[0])
        pos = torch.stack((a, b), dim=1)
        self.positives = pos
        return pos

    def load_positives_split(self, pos_pth, split=0.7, shuffle=True, random_seed=42):
        pos = self.load_positives(pos_pth)
        n = pos.shape[0]
        if shuffle:
            index = np.random.RandomState(random_seed).permutation(n)
            pos = pos[index, :]
        cut = int(split * n)
        return pos[:cut, :], pos[cut:, :]

    def load_batch_features(self, ids):
        return {nid: torch.load(os.path.join(self.ft_dir, nid + ".pt"), weights_only=True) for nid in ids}

    def song_info(self, index_id):
        track_ids = list(self.tracks)
        t = self.tracks[track_ids[index_id]]
        return f"{t['name']} - {t['artist']}"


CACHE_DIR = "pinsage_cache"


def _fingerprint(paths):
    """Size and mtime of each source (a directory's mtime moves when files are
    added or removed in it)."""
    parts = []
    for p in paths:
        try:
            st = os.stat(p)
            parts.append(f"{os.path.basename(p)}:{st.st_size}:{st.st_mtime_ns}")
        except (OSError, TypeError):
            parts.append(f"{p}:missing")
    return "|".join(parts)


def _atomic_save(target, saver, **arrays):
    """Write target via a temporary file and rename; a failure leaves no cache."""
    tmp = f"{target}.{os.getpid()}.tmp"
    try:
        os.makedirs(os.path.dirname(target), exist_ok=True)
        with open(tmp, "wb") as f:
            saver(f, **arrays)
        os.replace(tmp, target)
    except OSError:
        try:
            os.remove(tmp)
        except OSError:
            pass


def _burn_randperm(n):
    """Advance torch's CPU generator exactly as torch.randperm(n) would."""
    from _native import torch_rng
    with torch_rng() as mt:
        mt.skip(max(n - 1, 0))
