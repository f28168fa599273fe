"""Drop-in ``spotify_graph`` (reference ``spotify_graph.py:15-110``).

JSON dataset -> CSR graph (tracks first, then collections), z-scored node
features, positive pairs.  ``to_dgl_graph`` returns a :class:`graph.CSRGraph`
(the DGL subset the PinSage path uses) instead of a ``dgl.DGLGraph``.
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
        with open(self.graph_pth, "r", encoding="utf-8") as f:
            self.graph = json.load(f)
        self.ft_dir = features_dir if (features_dir and os.path.isdir(features_dir)) else None
        self.features_dict = {}

    def to_dgl_graph(self):
        """(g, track_ids, col_ids, features); node ids = tracks.json order then
        collections.json order; edges in graph.json order (spotify_graph.py:41-85)."""
        track_ids = list(self.tracks)
        col_ids = list(self.collections)
        index_map = {nid: i for i, nid in enumerate(track_ids)}
        n_t = len(track_ids)
        for j, cid in enumerate(col_ids):
            index_map[cid] = n_t + j
        edges = self.graph["edges"]
        src = np.fromiter((index_map[e["from"]] for e in edges), np.int64, len(edges))
        dst = np.fromiter((index_map[e["to"]] for e in edges), np.int64, len(edges))
        g = CSRGraph(n_t + len(col_ids), src, dst, base_dir=self.base_dir, nbhds_path=self.nbhds_path)

        if self.ft_dir:
            vecs = [torch.load(os.path.join(self.ft_dir, tid + ".pt"), weights_only=True)
                    for tid in track_ids]
            features = torch.stack(vecs, dim=0)
            mean = features.mean(dim=0)
            std = features.std(dim=0, unbiased=True) + 1e-12
            features = (features - mean) / std
        else:
            features = None

        self.g, self.track_ids, self.col_ids, self.features = g, track_ids, col_ids, features
        return g, track_ids, col_ids, features

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


def _burn_randperm(n):
    """Advance torch's CPU generator exactly as torch.randperm(n) would."""
    from _native import torch_rng
    with torch_rng() as mt:
        mt.skip(max(n - 1, 0))
