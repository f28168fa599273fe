"""Seeded synthetic track-collection ("playlist") graphs.

The reference trains on Spotify crawls whose large blobs are not available
(SURVEY.md section 8d), so every benchmark and most tests run on graphs built here.
The layout follows what the reference's loader produces:

* node ids: tracks ``0..n_tracks-1`` first, then collections
  (``spotify_graph.py:43-46``);
* edges: for each collection in order, for each member track, the pair
  ``collection -> track`` then ``track -> collection``
  (``dataset_creation/get_data.py:211-214``);
* ``successors(v)`` lists a node's out-edges in edge-insertion order (stable
  COO -> CSR), which is the order the walk indexes (``pinsage_model.py:41-46``).

Track popularity is Zipf(``zipf_a``); collection sizes are log-normal around
``n_memberships / n_cols``; every track belongs to at least one collection and
every collection has at least two distinct member tracks, so the walk never
meets a zero-degree node and no neighbourhood is all-zero.
"""
from __future__ import annotations

import json
import os
import string
from dataclasses import dataclass

import numpy as np


@dataclass
class PlaylistGraph:
    n_tracks: int
    n_cols: int
    # membership pairs in edge order: collection-major, member tracks ascending
    mem_col: np.ndarray     # int64 [M], collection index 0..n_cols-1
    mem_track: np.ndarray   # int64 [M], track index 0..n_tracks-1

    @property
    def n_all(self) -> int:
        return self.n_tracks + self.n_cols

    @property
    def n_edges(self) -> int:
        return 2 * int(self.mem_col.shape[0])

    def edge_arrays(self):
        """(src, dst) int64 in JSON edge order: c->t, t->c per membership."""
        m = self.mem_col.shape[0]
        src = np.empty(2 * m, dtype=np.int64)
        dst = np.empty(2 * m, dtype=np.int64)
        c = self.mem_col + self.n_tracks
        src[0::2] = c
        dst[0::2] = self.mem_track
        src[1::2] = self.mem_track
        dst[1::2] = c
        return src, dst

    def csr(self):
        """CSR (indptr int64 [N+1], indices int32 [E]) with rows in edge-insertion order."""
        n, m = self.n_tracks, self.mem_col.shape[0]
        n_all = self.n_all
        deg = np.zeros(n_all, dtype=np.int64)
        deg[:n] = np.bincount(self.mem_track, minlength=n)
        deg[n:] = np.bincount(self.mem_col, minlength=self.n_cols)
        indptr = np.zeros(n_all + 1, dtype=np.int64)
        np.cumsum(deg, out=indptr[1:])
        indices = np.empty(2 * m, dtype=np.int32)
        # collection rows: members in order (pairs are already collection-major)
        indices[indptr[n]:indptr[n_all]] = self.mem_track.astype(np.int32)
        # track rows: collections in order of first appearance in the edge list,
        # i.e. a stable sort of the pairs by track
        order = np.argsort(self.mem_track, kind="stable")
        indices[0:indptr[n]] = (self.mem_col[order] + n).astype(np.int32)
        return indptr, indices


def make_playlist_graph(n_tracks: int, n_cols: int, n_memberships: int,
                        seed: int = 0, zipf_a: float = 1.0,
                        size_sigma: float = 1.0) -> PlaylistGraph:
    """Build a seeded bipartite track-collection graph (see module docstring)."""
    if n_tracks < 2 or n_cols < 1:
        raise ValueError("need at least 2 tracks and 1 collection")
    n_memberships = max(int(n_memberships), n_tracks + n_cols)
    rng = np.random.default_rng(seed)
    # Zipf track popularity over a random rank permutation
    ranks = rng.permutation(n_tracks).astype(np.float64) + 1.0
    pop = ranks ** (-zipf_a)
    pop /= pop.sum()
    # log-normal collection sizes, mean ~ n_memberships / n_cols
    raw = rng.lognormal(mean=0.0, sigma=size_sigma, size=n_cols)
    sizes = np.maximum(2, np.round(raw / raw.mean() * (n_memberships / n_cols))).astype(np.int64)
    col_w = sizes / sizes.sum()
    # 1) every track joins one collection (degree >= 1)
    first_col = rng.choice(n_cols, size=n_tracks, p=col_w)
    # 2) fill remaining slots: collection by size, track by popularity
    extra = max(0, n_memberships - n_tracks)
    ex_col = rng.choice(n_cols, size=extra, p=col_w)
    ex_track = rng.choice(n_tracks, size=extra, p=pop)
    cols = np.concatenate([first_col, ex_col])
    tracks = np.concatenate([np.arange(n_tracks, dtype=np.int64), ex_track])
    key = np.unique(cols.astype(np.int64) * n_tracks + tracks)
    cols, tracks = key // n_tracks, key % n_tracks
    # 3) every collection gets >= 2 distinct tracks
    cnt = np.bincount(cols, minlength=n_cols)
    fix = np.nonzero(cnt < 2)[0]
    if fix.size:
        add_c, add_t = [], []
        lo = np.searchsorted(cols, fix, side="left")   # key is sorted: cols ascending
        hi = np.searchsorted(cols, fix, side="right")
        for c, a, b in zip(fix.tolist(), lo.tolist(), hi.tolist()):
            have = set(tracks[a:b].tolist())
            while len(have) < 2:
                t = int(rng.integers(n_tracks))
                if t not in have:
                    have.add(t)
                    add_c.append(c)
                    add_t.append(t)
        key = np.unique(np.concatenate([key, np.asarray(add_c, np.int64) * n_tracks
                                        + np.asarray(add_t, np.int64)]))
        cols, tracks = key // n_tracks, key % n_tracks
    return PlaylistGraph(n_tracks, n_cols, cols.astype(np.int64), tracks.astype(np.int64))


def make_features(n: int, d: int, seed: int = 1) -> np.ndarray:
    """N(0,1) features, z-scored per column as ``spotify_graph.py:77-79`` does."""
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((n, d)).astype(np.float32)
    mean = f.mean(axis=0, dtype=np.float64)
    std = f.std(axis=0, ddof=1, dtype=np.float64) + 1e-12
    return ((f - mean) / std).astype(np.float32)


def make_positives(g: PlaylistGraph, n_pairs: int, seed: int = 3, csr=None) -> np.ndarray:
    """Positive pairs (a, b) of distinct tracks sharing a collection ([P, 2] int64).

    Stands in for ``generate_positives.py:50`` ("auto" = 5 pairs per track)."""
    rng = np.random.default_rng(seed)
    indptr, indices = g.csr() if csr is None else csr
    n = g.n_tracks
    a = rng.integers(0, n, size=n_pairs)
    # pick one of a's collections, then one member of it
    da = indptr[a + 1] - indptr[a]
    c = indices[indptr[a] + (rng.random(n_pairs) * da).astype(np.int64)].astype(np.int64)
    dc = indptr[c + 1] - indptr[c]
    k = (rng.random(n_pairs) * dc).astype(np.int64)
    b = indices[indptr[c] + k].astype(np.int64)
    # collections have >= 2 distinct members: on a self-pair take the next member
    same = b == a
    k[same] = (k[same] + 1) % dc[same]
    b[same] = indices[indptr[c[same]] + k[same]]
    return np.stack([a, b], axis=1).astype(np.int64)


_ALPH = string.ascii_letters + string.digits


def random_ids(n: int, seed: int, length: int = 22) -> list:
    """Spotify-like base62 ids (unique)."""
    rng = np.random.default_rng(seed)
    out, seen = [], set()
    while len(out) < n:
        s = "".join(_ALPH[i] for i in rng.integers(0, 62, size=length))
        if s not in seen:
            seen.add(s)
            out.append(s)
    return out


def write_spotify_dataset(dirpath: str, g: PlaylistGraph, track_ids=None, col_ids=None,
                          seed: int = 5):
    """Write ``tracks.json`` / ``collections.json`` / ``graph.json`` in the crawler's
    schema (``get_data.py:107-123, 472-529``) for a synthetic graph."""
    os.makedirs(dirpath, exist_ok=True)
    track_ids = list(track_ids) if track_ids is not None else random_ids(g.n_tracks, seed)
    col_ids = list(col_ids) if col_ids is not None else random_ids(g.n_cols, seed + 1)
    assert len(track_ids) == g.n_tracks and len(col_ids) == g.n_cols
    tracks = {tid: {"name": f"track {i}", "artist": f"artist {i % 97}",
                    "album_id": f"album{i % 211}"} for i, tid in enumerate(track_ids)}
    members = [[] for _ in range(g.n_cols)]
    for c, t in zip(g.mem_col.tolist(), g.mem_track.tolist()):
        members[c].append(track_ids[t])
    cols = {cid: {"type": "playlist", "name": f"playlist {j}", "num_tracks": len(members[j]),
                  "ztracks": members[j]} for j, cid in enumerate(col_ids)}
    edges = []
    for j, cid in enumerate(col_ids):
        for tid in members[j]:
            edges.append({"from": cid, "to": tid})
            edges.append({"from": tid, "to": cid})
    graph = {"tracks": list(track_ids), "collections": list(col_ids), "edges": edges}
    for name, obj in (("tracks.json", tracks), ("collections.json", cols), ("graph.json", graph)):
        with open(os.path.join(dirpath, name), "w", encoding="utf-8") as f:
            json.dump(obj, f)
    return track_ids, col_ids


def make_playlist_graph_device(n_tracks: int, n_cols: int, n_memberships: int, seed: int = 0,
                               zipf_a: float = 1.0, size_sigma: float = 1.0, device="cuda",
                               chunk: int = 1 << 26):
    """make_playlist_graph's distribution drawn on the device (torch, seeded
    device generator), for graphs whose host build takes minutes (the C5 shape:
    100M nodes / 1B edges).  Same layout and guarantees -- tracks first, rows in
    edge-insertion order, every track in >= 1 collection, every collection with
    >= 2 distinct tracks -- but a different random stream than the host
    builder.  Returns (indptr int64 [N+1], indices int32 [E]) on the device."""
    import torch
    if n_tracks < 2 or n_cols < 1:
        raise ValueError("need at least 2 tracks and 1 collection")
    n_memberships = max(int(n_memberships), n_tracks + n_cols)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    f64 = torch.float64
    ranks = torch.randperm(n_tracks, generator=gen, device=device).to(f64) + 1.0
    cdf_t = torch.cumsum(ranks.pow_(-zipf_a), 0)
    del ranks
    cdf_t /= cdf_t[-1].clone()
    raw = torch.empty(n_cols, dtype=f64, device=device).log_normal_(0.0, size_sigma, generator=gen)
    sizes = torch.clamp(torch.round(raw / raw.mean() * (n_memberships / n_cols)), min=2)
    cdf_c = torch.cumsum(sizes, 0)
    cdf_c /= cdf_c[-1].clone()
    del raw, sizes

    def draw(cdf, n):
        u = torch.rand(n, dtype=f64, device=device, generator=gen)
        return torch.clamp(torch.searchsorted(cdf, u), max=cdf.shape[0] - 1)

    parts = [draw(cdf_c, n_tracks) * n_tracks + torch.arange(n_tracks, device=device)]
    extra = max(0, n_memberships - n_tracks)
    for i in range(0, extra, chunk):
        k = min(chunk, extra - i)
        parts.append(draw(cdf_c, k) * n_tracks + draw(cdf_t, k))
    key = torch.unique(torch.cat(parts))
    del parts, cdf_t, cdf_c
    # every collection gets >= 2 distinct tracks
    cnt = torch.bincount(key // n_tracks, minlength=n_cols)
    while bool((cnt < 2).any()):  # one random track more per short collection per round
        bad = torch.nonzero(cnt < 2).reshape(-1)
        add = torch.randint(0, n_tracks, (bad.numel(),), device=device, generator=gen)
        key = torch.unique(torch.cat([key, bad * n_tracks + add]))
        cnt = torch.bincount(key // n_tracks, minlength=n_cols)
    cols = key // n_tracks
    tracks = key - cols * n_tracks
    del key
    n_all = n_tracks + n_cols
    deg = torch.cat([torch.bincount(tracks, minlength=n_tracks), cnt])
    indptr = torch.zeros(n_all + 1, dtype=torch.int64, device=device)
    torch.cumsum(deg, 0, out=indptr[1:])
    del deg, cnt
    m = tracks.shape[0]
    indices = torch.empty(2 * m, dtype=torch.int32, device=device)
    # collection rows: members ascending (the pairs are collection-major)
    indices[m:] = tracks.to(torch.int32)
    # track rows: collections in edge order = a stable sort of the pairs by track
    _, order = torch.sort(tracks, stable=True)
    del tracks
    indices[:m] = (cols[order] + n_tracks).to(torch.int32)
    return indptr, indices


def make_positives_device(indptr, indices, n_tracks: int, n_pairs: int, seed: int = 3,
                          chunk: int = 1 << 26):
    """make_positives' co-membership pairs drawn on the device ([P, 2] int64 on
    the host, where the batch sampler reads them)."""
    import torch
    dev = indptr.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    out = torch.empty((n_pairs, 2), dtype=torch.int64)
    for i in range(0, n_pairs, chunk):
        k = min(chunk, n_pairs - i)
        a = torch.randint(0, n_tracks, (k,), device=dev, generator=gen)
        da = indptr[a + 1] - indptr[a]
        u = torch.rand(k, dtype=torch.float64, device=dev, generator=gen)
        c = indices[indptr[a] + (u * da).to(torch.int64)].to(torch.int64)
        dc = indptr[c + 1] - indptr[c]
        u = torch.rand(k, dtype=torch.float64, device=dev, generator=gen)
        kk = (u * dc).to(torch.int64)
        b = indices[indptr[c] + kk].to(torch.int64)
        same = b == a
        kk = torch.where(same, (kk + 1) % dc, kk)
        b = torch.where(same, indices[indptr[c] + kk].to(torch.int64), b)
        out[i:i + k, 0] = a.cpu()
        out[i:i + k, 1] = b.cpu()
    return out
