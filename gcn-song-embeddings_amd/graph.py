"""CSR track-collection graph: the subset of ``dgl.DGLGraph`` the PinSage path uses.

The reference builds a DGL graph (``spotify_graph.py:48-63``) and the sampler
only calls ``g.successors(v)`` (``pinsage_model.py:41,44``) and
``g.number_of_nodes()`` (``pinsage_model.py:93``); eval/baselines callers also
use ``in_degrees``, ``predecessors``, ``edges()`` and ``adj(scipy_fmt="csr")``.
Successor order is edge-insertion order (stable COO -> CSR), which decides the
``raw % deg`` neighbour choice of the walk.  The CSR is mirrored once to HBM
(``indptr`` int64, ``indices`` int32) for the walk kernels.
"""
from __future__ import annotations

import numpy as np
import torch


class CSRGraph:
    def __init__(self, n_nodes: int, src, dst, base_dir: str = ".", nbhds_path: str = "neighborhoods.pt"):
        src = np.asarray(src, np.int64)
        dst = np.asarray(dst, np.int64)
        if src.shape != dst.shape:
            raise ValueError("src and dst must have the same length")
        if src.size and (src.min() < 0 or dst.min() < 0 or max(src.max(), dst.max()) >= n_nodes):
            raise ValueError("edge endpoint out of range")
        self._n = int(n_nodes)
        self._src, self._dst = src, dst
        order = np.argsort(src, kind="stable")
        self.indptr = np.zeros(self._n + 1, np.int64)
        np.cumsum(np.bincount(src, minlength=self._n), out=self.indptr[1:])
        self.indices = dst[order].astype(np.int32)
        self._rev = None
        self._dev = None
        # attributes the reference attaches to its DGL graph (spotify_graph.py:53-54)
        self.base_dir = base_dir
        self.nbhds_path = nbhds_path

    @classmethod
    def from_csr(cls, indptr, indices, base_dir=".", nbhds_path="neighborhoods.pt"):
        """Wrap an existing CSR (rows in edge-insertion order) without a COO copy."""
        g = cls.__new__(cls)
        g.indptr = np.ascontiguousarray(indptr, np.int64)
        g.indices = np.ascontiguousarray(indices, np.int32)
        g._n = int(g.indptr.shape[0] - 1)
        g._src = None
        g._dst = None
        g._rev = None
        g._dev = None
        g.base_dir = base_dir
        g.nbhds_path = nbhds_path
        return g

    # ---- DGL-compatible API
    def number_of_nodes(self) -> int:
        return self._n

    num_nodes = number_of_nodes

    def number_of_edges(self) -> int:
        return int(self.indptr[-1])

    num_edges = number_of_edges

    def __len__(self):
        return self._n

    def successors(self, v):
        v = int(v)
        return torch.from_numpy(self.indices[self.indptr[v]:self.indptr[v + 1]].astype(np.int64))

    def out_degrees(self, v=None):
        deg = np.diff(self.indptr)
        return torch.from_numpy(deg if v is None else deg[np.asarray(v)])

    def _reverse(self):
        if self._rev is None:
            src, dst = self._coo()
            order = np.argsort(dst, kind="stable")
            ip = np.zeros(self._n + 1, np.int64)
            np.cumsum(np.bincount(dst, minlength=self._n), out=ip[1:])
            self._rev = (ip, src[order])
        return self._rev

    def predecessors(self, v):
        ip, ix = self._reverse()
        v = int(v)
        return torch.from_numpy(ix[ip[v]:ip[v + 1]].astype(np.int64))

    def in_degrees(self, v=None):
        ip, _ = self._reverse()
        deg = np.diff(ip)
        if v is None:
            return torch.from_numpy(deg)
        if np.ndim(v) == 0:
            return int(deg[int(v)])
        return torch.from_numpy(deg[np.asarray(v)])

    def _coo(self):
        if self._src is None:
            src = np.repeat(np.arange(self._n, dtype=np.int64), np.diff(self.indptr))
            return src, self.indices.astype(np.int64)
        return self._src, self._dst

    def edges(self, form="uv", order=None):
        src, dst = self._coo()
        return torch.from_numpy(src.copy()), torch.from_numpy(dst.copy())

    def adj(self, transpose=False, ctx=None, scipy_fmt=None, etype=None):
        import scipy.sparse as sp
        src, dst = self._coo()
        r, c = (dst, src) if transpose else (src, dst)
        m = sp.coo_matrix((np.ones(r.shape[0], np.float32), (r, c)), shape=(self._n, self._n))
        if scipy_fmt is None:
            idx = torch.from_numpy(np.stack([r, c]))
            return torch.sparse_coo_tensor(idx, torch.ones(r.shape[0]), (self._n, self._n))
        return m.asformat(scipy_fmt)

    # ---- device mirror for the HIP sampler
    def device_csr(self, dev):
        if self._dev is None or self._dev[0].device != dev:
            self._dev = (torch.from_numpy(self.indptr).to(dev), torch.from_numpy(self.indices).to(dev))
        return self._dev

    def max_degree(self) -> int:
        return int(np.diff(self.indptr).max()) if self._n else 0


class DeviceCSRGraph(CSRGraph):
    """A CSRGraph whose CSR was built on the device (synthetic.make_playlist_graph_device):
    the HBM mirror is the primary copy; ``indptr`` is kept on the host (degrees,
    max_degree) and ``indices`` crosses to the host only if a host-side caller
    (successors, edges, adj) asks for it."""

    def __init__(self, indptr_dev, indices_dev, base_dir=".", nbhds_path="neighborhoods.pt"):
        self._dev = (indptr_dev.to(torch.int64).contiguous(), indices_dev.to(torch.int32).contiguous())
        self.indptr = self._dev[0].cpu().numpy()
        self._indices = None
        self._n = int(self.indptr.shape[0] - 1)
        self._src = None
        self._dst = None
        self._rev = None
        self.base_dir = base_dir
        self.nbhds_path = nbhds_path

    @property
    def indices(self):
        if self._indices is None:
            self._indices = self._dev[1].cpu().numpy()
        return self._indices

    def device_csr(self, dev):
        if self._dev[0].device != dev:
            self._dev = (self._dev[0].to(dev), self._dev[1].to(dev))
        return self._dev
