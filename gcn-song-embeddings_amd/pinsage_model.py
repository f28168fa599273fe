"""Drop-in ``pinsage_model`` (reference ``pinsage_model.py``) on MI355X.

Same names, signatures, return types and RNG consumption as the reference; the
work runs in hand-written gfx950 kernels through ``libpinsage_hip.so``:

* ``do_random_walks`` / ``sample_neighborhood[_topt]`` /
  ``precompute_neighborhoods_topt`` -> walk + visit-count + libstdc++-exact
  top-k kernels.  RNG mode ``"mt19937"`` (default) consumes torch's global CPU
  generator draw-for-draw like the reference (bit-exact outputs); ``"philox"``
  is a counter-based stream for throughput (``set_rng_mode``).
* ``relevant_nodes_per_layer[_precomp]`` -> bitmap frontier kernels.
* ``PinSageModel.forward`` -> the fused engine (frontier, fp32-MFMA Q/W
  projections with fused epilogues, weighted aggregation, head), with a HIP
  backward for autograd.

Inputs may be CPU tensors (as the reference's callers pass); results come back
on the device of the input.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import time
import weakref

import numpy as np
import torch
import torch.nn as nn

import _native as nat

DEF_T_PRECOMP = 100
DEF_HOPS = 500
DEF_ALPHA = 0.85

_RNG_MODE = "mt19937"
_PHILOX_OFFSET = [0]


def set_rng_mode(mode: str):
    """'mt19937' (reference-exact, default) or 'philox' (counter-based, faster)."""
    global _RNG_MODE
    if mode not in ("mt19937", "philox"):
        raise ValueError("rng mode must be 'mt19937' or 'philox'")
    _RNG_MODE = mode


def get_rng_mode() -> str:
    return _RNG_MODE


# ----------------------------------------------------------------------------- embeddings
def get_embeddings(h, nodeset, d):
    """h[nodeset, :d] (pinsage_model.py:21-22)."""
    return h[nodeset, :d]


def put_embeddings(h, nodeset, nodeset_new_h):
    """Copy of h with rows ``nodeset`` replaced by zero-padded new rows
    (pinsage_model.py:24-30).  The fused forward never materialises this copy;
    the function is kept for API compatibility."""
    new_h = h.clone().detach()
    pad_cols = new_h.shape[1] - nodeset_new_h.shape[1]
    pad = torch.zeros(nodeset.shape[0], pad_cols, dtype=nodeset_new_h.dtype, device=nodeset_new_h.device)
    new_h[nodeset, :] = torch.cat([nodeset_new_h, pad], 1)
    return new_h


# ----------------------------------------------------------------------------- sampler
def _as_csr(g):
    if hasattr(g, "indptr") and hasattr(g, "indices"):
        return g
    raise TypeError("graph must be a graph.CSRGraph (spotify_graph.SpotifyGraph.to_dgl_graph())")


def _walk_device(g, nodeset, n_hops, alpha, philox=None):
    """int32 trace [n, n_hops] on the GPU; consumes RNG like the reference.
    philox=(seed, src_base): Philox mode with a given seed and absolute source
    position of nodeset[0] (draws nothing from torch's generator)."""
    g = _as_csr(g)
    dev = nat.device()
    indptr, indices = g.device_csr(dev)
    src = torch.as_tensor(nodeset).reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
    n = int(src.shape[0])
    n_all = g.number_of_nodes()
    trace = torch.empty((n, int(n_hops)), dtype=torch.int32, device=dev)
    if n == 0:
        return src, trace
    alpha32 = float(np.float32(alpha))
    L = nat.lib()
    if _RNG_MODE == "mt19937":
        if g.max_degree() >= (1 << 28):
            raise RuntimeError("degree >= 2^28: torch.randint switches to 64-bit draws; "
                               "use rng mode 'philox'")
        need = L.pinsage_walk_mt_workspace(n, int(n_hops))
        cap = 2 << 30  # <= 2 GiB of raw MT words per round
        ws = torch.empty(min(need, cap), dtype=torch.uint8, device=dev)
        with nat.torch_rng() as mt:
            nat.check(L.pinsage_walk_mt(nat.ptr(indptr), nat.ptr(indices), n_all, nat.ptr(src), n,
                                        int(n_hops), alpha32, mt.p, nat.ptr(ws), ws.numel(),
                                        nat.ptr(trace), nat.stream_ptr()), "walk")
    else:
        if philox is None:
            with nat.torch_rng() as mt:
                d = mt.draws(2)
            seed, base = (int(d[0]) << 32) | int(d[1]), 0
        else:
            seed, base = philox
        nat.check(L.pinsage_walk_philox(nat.ptr(indptr), nat.ptr(indices), n_all, nat.ptr(src), n,
                                        int(n_hops), alpha32, seed, 0, int(base), nat.ptr(trace),
                                        nat.stream_ptr()), "walk")
    return src, trace


def do_random_walks(g, nodeset, n_hops, alpha):
    """Random walks with restart; int64 trace [len(nodeset), n_hops]
    (pinsage_model.py:32-53)."""
    _, trace = _walk_device(g, nodeset, n_hops, alpha)
    out_dev = torch.as_tensor(nodeset).device
    return trace.to(torch.int64).to(out_dev)


def sample_neighborhood(g, n_items, nodeset, n_hops, alpha):
    """Dense normalised visit counts, self column zeroed: f64 [n, N_all]
    (pinsage_model.py:88-101)."""
    src, trace = _walk_device(g, nodeset, n_hops, alpha)
    n, n_all = int(src.shape[0]), g.number_of_nodes()
    dense = torch.empty((n, n_all), dtype=torch.float64, device=src.device)
    nat.check(nat.lib().pinsage_visit_dense(nat.ptr(trace), nat.ptr(src), n, int(n_hops), n_all,
                                            nat.ptr(dense), nat.stream_ptr()), "visit_dense")
    return dense.to(torch.as_tensor(nodeset).device)


def _topk_device(src, trace, n_all, n_hops, T, t_norm=0):
    dev = src.device
    n = int(src.shape[0])
    L = nat.lib()
    scratch_b = L.pinsage_visit_topk_scratch(n, n_all, T)
    scratch = torch.empty(max(scratch_b, 1), dtype=torch.uint8, device=dev)
    w = torch.empty((n, T), dtype=torch.float64, device=dev)
    nb = torch.empty((n, T), dtype=torch.int64, device=dev)
    wn = nb32 = None
    if t_norm:
        wn = torch.empty((n, t_norm), dtype=torch.float32, device=dev)
        nb32 = torch.empty((n, t_norm), dtype=torch.int32, device=dev)
    nat.check(L.pinsage_visit_topk(nat.ptr(trace), nat.ptr(src), n, int(n_hops), n_all, int(T),
                                   nat.ptr(scratch) if scratch_b else None, nat.ptr(w), nat.ptr(nb),
                                   nat.ptr(wn), nat.ptr(nb32), t_norm, nat.stream_ptr()), "visit_topk")
    return w, nb, wn, nb32


# fused walk + count + top-k (pinsage_ppr_topk): the trace never reaches HBM;
# at most this many bytes of device scratch per call (more sources run in rounds)
_PPR_WS_CAP = 1 << 30


def _ppr_topk_device(g, nodeset, n_hops, alpha, T, t_norm=0, philox=None, want_ref=True):
    """Top-T of visit_prob for each source (pinsage_model.py:32-53, 88-107) with
    the fused kernel; same draws as _walk_device (+ _topk_device).  Returns
    (w f64, nb i64, wn f32, nb32 i32) on the device (None where not asked).
    Tiny graphs (T * 64 > N_all: torch's nth_element regime) take the walk +
    visit_topk kernels."""
    g = _as_csr(g)
    n_all = g.number_of_nodes()
    T = int(T)
    if T * 64 > n_all or int(n_hops) + T >= 65536 or int(n_hops) > 8192:
        src, trace = _walk_device(g, nodeset, n_hops, alpha, philox)
        return _topk_device(src, trace, n_all, n_hops, T, t_norm=t_norm)
    dev = nat.device()
    indptr, indices = g.device_csr(dev)
    src = torch.as_tensor(nodeset).reshape(-1).to(device=dev, dtype=torch.int64).contiguous()
    n = int(src.shape[0])
    w = torch.empty((n, T), dtype=torch.float64, device=dev) if want_ref else None
    nb = torch.empty((n, T), dtype=torch.int64, device=dev) if want_ref else None
    wn = nb32 = None
    if t_norm:
        wn = torch.empty((n, t_norm), dtype=torch.float32, device=dev)
        nb32 = torch.empty((n, t_norm), dtype=torch.int32, device=dev)
    if n == 0:
        return w, nb, wn, nb32
    L = nat.lib()
    alpha32 = float(np.float32(alpha))
    mt_mode = _RNG_MODE == "mt19937" and philox is None
    if mt_mode and g.max_degree() >= (1 << 28):
        raise RuntimeError("degree >= 2^28: torch.randint switches to 64-bit draws; use rng mode 'philox'")
    need = L.pinsage_ppr_topk_workspace(n, int(n_hops), 1 if mt_mode else 0)
    ws = torch.empty(min(need, _PPR_WS_CAP), dtype=torch.uint8, device=dev)

    def run(mt_p, seed, base):
        nat.check(L.pinsage_ppr_topk(nat.ptr(indptr), nat.ptr(indices), n_all, nat.ptr(src), n,
                                     int(n_hops), alpha32, T, mt_p, seed, 0, base, nat.ptr(ws),
                                     ws.numel(), nat.ptr(w), nat.ptr(nb), nat.ptr(wn), nat.ptr(nb32),
                                     int(t_norm), nat.stream_ptr()), "ppr_topk")

    if mt_mode:
        with nat.torch_rng() as mt:
            run(mt.p, 0, 0)
    else:
        if philox is None:
            with nat.torch_rng() as mt:
                d = mt.draws(2)
            seed, base = (int(d[0]) << 32) | int(d[1]), 0
        else:
            seed, base = philox
        run(None, seed, int(base))
    return w, nb, wn, nb32


def sample_neighborhood_topt(g, n_items, nodeset, n_hops, alpha, T):
    """visit_prob.topk(T, 1) as a ``torch.return_types.topk`` (pinsage_model.py:103-107)."""
    w, nb, _, _ = _ppr_topk_device(g, nodeset, n_hops, alpha, int(T))
    out_dev = torch.as_tensor(nodeset).device
    return torch.return_types.topk((w.to(out_dev), nb.to(out_dev)))


def _shard():
    """(rank, world) of an initialised torch.distributed job (precompute is
    sharded by source over its ranks), else (0, 1).  PINSAGE_SHARD_PRECOMPUTE=0
    makes every rank compute the whole table."""
    d = torch.distributed
    if (os.environ.get("PINSAGE_SHARD_PRECOMPUTE", "1") != "0" and d.is_available()
            and d.is_initialized() and d.get_world_size() > 1):
        return d.get_rank(), d.get_world_size()
    return 0, 1


def _set_stream_position(st0, draws):
    """torch's CPU generator = state st0 advanced by `draws` MT19937 words
    (exact GF(2) jump-ahead for long skips)."""
    mt = nat.MT.from_state(st0)
    mt.skip(int(draws))
    mt.to_torch()


def _shard_range(n_items, rank, world):
    """Equal contiguous source shard of a rank: [rank*per, min((rank+1)*per, n))."""
    per = -(-n_items // world) if n_items else 0
    lo = min(rank * per, n_items)
    return lo, min(lo + per, n_items), per


def _gather_shards(w_sh, nb_sh, n_items, per, dev):
    """All-gather of the equal-sized (zero-padded) shards: ONE collective per
    table instead of reducing full-size tables."""
    d = torch.distributed
    world = d.get_world_size()
    out = []
    for t in (w_sh, nb_sh):
        if d.get_backend() == "nccl":  # RCCL over xGMI: device buffers
            x = t.to(dev)
            full = torch.empty((world * per,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            d.all_gather_into_tensor(full, x)
            out.append(full[:n_items].cpu())
        else:
            t = t.cpu()
            parts = [torch.empty_like(t) for _ in range(world)]
            d.all_gather(parts, t)
            out.append(torch.cat(parts, 0)[:n_items].contiguous())
    return out[0], out[1]


def precompute_neighborhoods_topt(g, n_items, n_hops, alpha, T, path):
    """Top-T PPR neighbourhoods of all items, cached at ``path`` as
    ``(weights f64 [n,T], nodes i64 [n,T])`` (pinsage_model.py:109-132).

    Sources are independent, so under torch.distributed each rank walks an
    equal contiguous shard of the sources and the shards are exchanged with
    one all-gather per table.  The RNG stream stays the
    single-process one: in MT19937 mode source s draws words
    [3*n_hops*s, 3*n_hops*(s+1)) of the reference's source-major stream, so a
    rank jumps its generator to its shard's start; in Philox mode one seed
    (two words) serves the whole table and each draw is keyed by the source's
    absolute position.  Afterwards every rank's generator is where the
    single-process run leaves it, and the table is bitwise the same."""
    if path and os.path.isfile(path):
        a, b = torch.load(path, weights_only=True)
        if b.shape[0] == n_items and b.shape[1] == T:
            return (a, b)
    t0 = time.time()
    dev = nat.device()
    rank, world = _shard()
    lo, hi, per = _shard_range(n_items, rank, world)
    rows = per if world > 1 else n_items
    # the shard is assembled on the device (zero padding rows of a short last
    # shard) and crosses to the host once
    sh_w = torch.zeros((rows, T), dtype=torch.float64, device=dev)
    sh_nb = torch.zeros((rows, T), dtype=torch.int64, device=dev)
    st0 = torch.get_rng_state().numpy().copy()
    mt_mode = _RNG_MODE == "mt19937"
    philox = None
    if not mt_mode:
        with nat.torch_rng() as mt:
            d = mt.draws(2)
        philox = (int(d[0]) << 32) | int(d[1])
    # sources in order; each chunk's draws are positioned absolutely, so the
    # chunking (and the rank that runs a chunk) does not change the result
    chunk = 1 << 18
    for i in range(lo, hi, chunk):
        if mt_mode:
            _set_stream_position(st0, 3 * int(n_hops) * i)
        ids = torch.arange(i, min(i + chunk, hi), dtype=torch.int64, device=dev)
        w, nb, _, _ = _ppr_topk_device(g, ids, n_hops, alpha, int(T), philox=None if mt_mode else (philox, i))
        sh_w[i - lo:i - lo + ids.shape[0]] = w
        sh_nb[i - lo:i - lo + ids.shape[0]] = nb
        print(f"{min(i + chunk, hi)}/{n_items} done.")
    if mt_mode:
        _set_stream_position(st0, 3 * int(n_hops) * n_items)
    if world > 1:
        all_w, all_nb = _gather_shards(sh_w, sh_nb, n_items, per, dev)
    else:
        all_w, all_nb = sh_w.cpu(), sh_nb.cpu()
    print(f"{time.time() - t0}s elapsed.")
    if path and rank == 0:
        torch.save((all_w, all_nb), path)
    return (all_w, all_nb)


def precompute_device_table(g, n_items, n_hops, alpha, T, T_precomp=DEF_T_PRECOMP, chunk=1 << 18):
    """The model's neighbourhood table built and kept on the device: for every
    item, the first T of its top-T_precomp PPR neighbours (the rows
    precompute_neighborhoods_topt returns, cut to [:, :T] as the model reads
    them, pinsage_model.py:164) with the weights normalised over those T
    (pinsage_model.py:202).  Same draws and positions as
    precompute_neighborhoods_topt (one process), but the [n, T_precomp] f64 + i64
    table never exists: at 80M items it would be 128 GB of host memory.  Returns
    a device table PinSageModel / PinSage accept as ``nbhds``."""
    dev = nat.device()
    T, T_precomp = int(T), int(T_precomp)
    if T > T_precomp:
        raise ValueError("T > T_precomp")
    nb32 = torch.empty((n_items, T), dtype=torch.int32, device=dev)
    wn = torch.empty((n_items, T), dtype=torch.float32, device=dev)
    st0 = torch.get_rng_state().numpy().copy()
    mt_mode = _RNG_MODE == "mt19937"
    philox = None
    if not mt_mode:
        with nat.torch_rng() as mt:
            d = mt.draws(2)
        philox = (int(d[0]) << 32) | int(d[1])
    for i in range(0, n_items, chunk):
        if mt_mode:
            _set_stream_position(st0, 3 * int(n_hops) * i)
        ids = torch.arange(i, min(i + chunk, n_items), dtype=torch.int64, device=dev)
        _, _, w_c, nb_c = _ppr_topk_device(g, ids, n_hops, alpha, T_precomp, t_norm=T,
                                           philox=None if mt_mode else (philox, i), want_ref=False)
        nb32[i:i + ids.shape[0]] = nb_c
        wn[i:i + ids.shape[0]] = w_c
    if mt_mode:
        _set_stream_position(st0, 3 * int(n_hops) * n_items)
    if n_items and int(nb32.max()) >= n_items:
        raise IndexError("neighbourhood table references ids >= n_items")
    return _DeviceTable.resident(nb32, wn)


def sample_hard_negatives(g, n_items, visit_prob, hn_per_query, min_rank, max_rank):
    """(NOT USED in the reference either; pinsage_model.py:135-140)"""
    rng = visit_prob.topk(max_rank, 1)[1][:, min_rank:]
    sample = torch.randint(0, rng.shape[1], (hn_per_query,))
    return rng[:, sample]


# ----------------------------------------------------------------------------- frontier
def _frontier_step(nodeset_dev, nb32, T, n_items):
    L = nat.lib()
    n = int(nodeset_dev.shape[0])
    cap = min(n_items, n * (T + 1))
    ws = torch.empty(L.pinsage_frontier_workspace(n_items), dtype=torch.uint8, device=nodeset_dev.device)
    out = torch.empty(max(cap, 1), dtype=torch.int32, device=nodeset_dev.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=nodeset_dev.device)
    nat.check(L.pinsage_frontier_step(nat.ptr(nodeset_dev), n, nat.ptr(nb32), nb32.shape[1], int(T),
                                      n_items, nat.ptr(ws), nat.ptr(out), nat.ptr(cnt),
                                      nat.stream_ptr()), "frontier")
    return out[:int(cnt.item())].to(torch.int64)


def relevant_nodes_per_layer(g, n_items, nodeset, n_layers, n_hops, alpha, T):
    """Computation graph with on-the-fly sampling (pinsage_model.py:142-154)."""
    out_dev = torch.as_tensor(nodeset).device
    dev = nat.device()
    S = []
    cur = torch.as_tensor(nodeset).to(dev, torch.int64)
    for _ in reversed(range(0, n_layers)):
        w, nb, _, nb32 = _ppr_topk_device(g, cur, n_hops, alpha, int(T), t_norm=int(T))
        S.insert(0, (cur.to(out_dev), w.to(out_dev), nb.to(out_dev)))
        # unique(cat(nb.flatten(), cur)): rows of nb belong to cur's positions
        table = torch.zeros((g.number_of_nodes(), int(T)), dtype=torch.int32, device=dev)
        table[cur] = nb32
        cur = _frontier_step(cur, table, int(T), g.number_of_nodes())
    return S


_FLY_CALLS = 3  # model calls per train step (q, pos, neg) that fly_calls runs as one


class _FlyDraws:
    """One model call's on-the-fly draws, laid out for the engine.

    ``tabs``: per-layer (nb int32 [rows][T], wn f32 [rows][T]) tables, index 0 =
    bottom, rows of each layer's nodes written.  A node repeated in the top
    nodeset keeps its LAST occurrence's row there: the reference's
    put_embeddings lets the last write win (pinsage_model.py:29), so the output
    rows of every repeat are the last one's.  ``uniq``/``inv``: the top
    nodeset's distinct ids and each position's index into them.  Every EARLIER
    occurrence of a repeated id walked its own neighbourhood, and index_put's
    backward hands its conv output the summed cotangent of its id
    (pinsage_model.py:257-265), so it is computed too: as a virtual node
    ``n_items + j`` (``ids_x[j]`` its real id, ``ui_x[j]`` its index into
    uniq) whose top-layer row holds that occurrence's draws and whose rows in
    the layers below (and feature row) are its real node's, so one engine
    call computes every occurrence (rows = n_items + len(ids_x))."""

    def __init__(self, tabs, uniq, inv, ids_x, ui_x, n_items):
        self.tabs, self.uniq, self.inv = tabs, uniq, inv
        self.ids_x, self.ui_x, self.n_items = ids_x, ui_x, int(n_items)

    @property
    def n_extra(self):
        return int(self.ids_x.shape[0])


def _fly_layer_tables(g, n_items, nodeset_dev, n_layers, n_hops, alpha, T):
    """relevant_nodes_per_layer (pinsage_model.py:142-154) for the engine: top
    layer first, each layer's nodeset is walked (the fused walk + top-k
    kernel: the same draws as the reference, in nodeset order) and its top-T
    rows land in that layer's own device table, indexed by node id.  The next
    layer's nodeset is unique(cat(nb.flatten(), cur)) over EVERY row drawn,
    repeated nodes' earlier rows included (:152), so the draws of the layers
    below follow the reference's stream.  Returns a _FlyDraws."""
    dev = nodeset_dev.device
    T = int(T)
    tabs = []
    cur = nodeset_dev
    rows = int(n_items)
    top_info = None
    for layer in range(n_layers):
        _, _, wn, nb32 = _ppr_topk_device(g, cur, n_hops, alpha, T, t_norm=T, want_ref=False)
        if layer == 0:
            # the top nodeset may repeat ids: occurrence rank of each position
            # counted from its id's last one; the earlier occurrences become
            # virtual nodes
            n = int(cur.shape[0])
            uniq, inv = torch.unique(cur, return_inverse=True)
            order = torch.argsort(inv, stable=True)
            ends = torch.cumsum(torch.bincount(inv, minlength=uniq.shape[0]), 0)
            rank = torch.empty(n, dtype=torch.int64, device=dev)
            rank[order] = ends[inv[order]] - 1 - torch.arange(n, device=dev)
            last = torch.empty(uniq.shape[0], dtype=torch.int64, device=dev)
            sel = rank == 0
            last[inv[sel]] = torch.arange(n, device=dev)[sel]
            pos_x = torch.nonzero(rank > 0).reshape(-1)
            rows = int(n_items) + int(pos_x.shape[0])
            top_info = (uniq, inv, pos_x)
        nbt = torch.empty((rows, T), dtype=torch.int32, device=dev)
        wnt = torch.empty((rows, T), dtype=torch.float32, device=dev)
        if layer == 0:
            nbt[uniq] = nb32[last]
            wnt[uniq] = wn[last]
            if rows > n_items:
                nbt[n_items:] = nb32[pos_x]
                wnt[n_items:] = wn[pos_x]
        else:  # lower nodesets are torch.unique outputs: one row per id already
            nbt[cur] = nb32
            wnt[cur] = wn
        tabs.insert(0, (nbt, wnt))
        cur = torch.unique(torch.cat([nb32.reshape(-1).to(torch.int64), cur]))
        # sorted: its last id is the largest drawn (before any table indexes it)
        if cur.numel() and int(cur[-1]) >= n_items:
            # the reference's h[nb] (features of tracks only) raises here
            raise IndexError("sampled neighbourhood reaches ids >= n_items (collection ids in the "
                             "zero-weight tail: the reference's h[nb] raises IndexError)")
    uniq, inv, pos_x = top_info
    ids_x = nodeset_dev[pos_x]
    if rows > n_items:
        # below the top, a virtual node is its real node (that node is in every
        # lower nodeset: each layer's nodeset contains the one above it)
        for l in range(n_layers - 1):
            nbt, wnt = tabs[l]
            nbt[n_items:] = nbt[ids_x]
            wnt[n_items:] = wnt[ids_x]
    return _FlyDraws(tabs, uniq, inv, ids_x, inv[pos_x], n_items)


def _fly_tables_merged(g, n_items, ids_c, n_layers, n_hops, alpha, T):
    """_fly_layer_tables for C model calls at once (Philox mode): the calls'
    seeds are drawn in the per-call order (call c, layer l: the (c * L + l)-th
    pair of words, as C sequential calls draw them), and each layer walks every
    call's nodeset in one pinsage_ppr_topk_segments call, so the tables are the
    per-call path's.  Call c's node v is c * n_items + v everywhere (rows and
    neighbour ids), earlier occurrences of repeated top ids are virtual nodes
    from C * n_items.  Returns (tabs, uniq, inv, ids_x, ui_x): uniq / inv over
    the concatenated nodesets, ids_x the virtual nodes' real ids."""
    L = nat.lib()
    gc = _as_csr(g)
    n_all = gc.number_of_nodes()
    indptr, indices = gc.device_csr(nat.device())
    C, n = len(ids_c), int(n_items)
    T = int(T)
    dev = ids_c[0].device
    with nat.torch_rng() as mt:
        d = [int(x) for x in mt.draws(2 * C * n_layers)]
    seed = [[(d[2 * (c * n_layers + l)] << 32) | d[2 * (c * n_layers + l) + 1] for l in range(n_layers)]
            for c in range(C)]
    alpha32 = float(np.float32(alpha))
    lens = [int(i.shape[0]) for i in ids_c]
    src = torch.cat(ids_c)
    off = torch.cat([torch.full((m,), c * n, dtype=torch.int64, device=dev) for c, m in enumerate(lens)])
    cur = src + off  # top layer: the nodesets as given (repeats included), offset per call
    tabs = []
    rows = C * n
    top = None
    for layer in range(n_layers):
        starts = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        n_src = int(starts[-1])
        wn = torch.empty((n_src, T), dtype=torch.float32, device=dev)
        nb32 = torch.empty((n_src, T), dtype=torch.int32, device=dev)
        need = L.pinsage_ppr_topk_workspace(n_src, int(n_hops), 0)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        seeds = np.array([seed[c][layer] for c in range(C)], dtype=np.uint64)
        bases = np.zeros(C, dtype=np.int64)
        nat.check(L.pinsage_ppr_topk_segments(
            nat.ptr(indptr), nat.ptr(indices), n_all, nat.ptr(src), C, starts.ctypes.data,
            seeds.ctypes.data, bases.ctypes.data, int(n_hops), alpha32, T, 0, nat.ptr(ws), ws.numel(),
            None, None, nat.ptr(wn), nat.ptr(nb32), T, nat.stream_ptr()), "ppr_topk_segments")
        nbo = nb32 + off[:, None].to(torch.int32)  # neighbour ids in their call's range
        if layer == 0:
            m = int(cur.shape[0])
            uniq, inv = torch.unique(cur, return_inverse=True)
            order = torch.argsort(inv, stable=True)
            ends = torch.cumsum(torch.bincount(inv, minlength=uniq.shape[0]), 0)
            rank = torch.empty(m, dtype=torch.int64, device=dev)
            rank[order] = ends[inv[order]] - 1 - torch.arange(m, device=dev)
            last = torch.empty(uniq.shape[0], dtype=torch.int64, device=dev)
            sel = rank == 0
            last[inv[sel]] = torch.arange(m, device=dev)[sel]
            pos_x = torch.nonzero(rank > 0).reshape(-1)
            rows = C * n + int(pos_x.shape[0])
            top = (uniq, inv, pos_x)
        nbt = torch.empty((rows, T), dtype=torch.int32, device=dev)
        wnt = torch.empty((rows, T), dtype=torch.float32, device=dev)
        if layer == 0:
            nbt[uniq] = nbo[last]
            wnt[uniq] = wn[last]
            if rows > C * n:
                nbt[C * n:] = nbo[pos_x]
                wnt[C * n:] = wn[pos_x]
        else:
            nbt[cur] = nbo
            wnt[cur] = wn
        tabs.insert(0, (nbt, wnt))
        nxt = torch.unique(torch.cat([nbo.reshape(-1).to(torch.int64), cur]))
        # one sync: the largest drawn id (before offsets) and the calls' boundaries
        bounds = torch.searchsorted(nxt, torch.arange(1, C, device=dev, dtype=torch.int64) * n)
        info = torch.cat([nb32.max().reshape(1).to(torch.int64), bounds]).tolist()
        if info[0] >= n_items:
            raise IndexError("sampled neighbourhood reaches ids >= n_items (collection ids in the "
                             "zero-weight tail: the reference's h[nb] raises IndexError)")
        edges = [0] + info[1:] + [int(nxt.shape[0])]
        lens = [edges[c + 1] - edges[c] for c in range(C)]
        cur = nxt
        off = torch.cat([torch.full((m,), c * n, dtype=torch.int64, device=dev) for c, m in enumerate(lens)])
        src = cur - off
    uniq, inv, pos_x = top
    top_ids = torch.cat(ids_c) + torch.cat([torch.full((m,), c * n, dtype=torch.int64, device=dev)
                                            for c, m in enumerate(int(i.shape[0]) for i in ids_c)])
    ids_xo = top_ids[pos_x]  # virtual nodes' ids in their call's range
    if rows > C * n:
        for l in range(n_layers - 1):
            nbt, wnt = tabs[l]
            nbt[C * n:] = nbt[ids_xo]
            wnt[C * n:] = wnt[ids_xo]
    return tabs, uniq, inv, ids_xo % n, inv[pos_x]


def _fly_seed_words(n_layers, C=_FLY_CALLS):
    """The Philox keys of C calls' walks, drawn from torch's generator as C
    sequential calls draw them (call c, layer l: the (c L + l)-th pair of
    words; _fly_tables_merged), as an int64 array [C * L] (bit patterns)."""
    with nat.torch_rng() as mt:
        d = [int(x) for x in mt.draws(2 * C * n_layers)]
    keys = [(d[2 * (c * n_layers + l)] << 32) | d[2 * (c * n_layers + l) + 1]
            for c in range(C) for l in range(n_layers)]
    return np.array(keys, dtype=np.uint64).view(np.int64)


class _FlyDevice:
    """Buffers of the device on-the-fly sampler (pinsage_fly_sample, fly.hip)
    for a train step's C = 3 calls of B ids each: per-layer tables [3 n + x_cap]
    [T] (engine layer order), the engine positions, the virtual nodes, the
    tiled feature rows (call c's copy of the table at c n, virtual rows after
    3 n) and the sampler's workspace.  sample() enqueues one step's sampling
    with no host synchronisation; its tables equal _fly_tables_merged's."""

    def __init__(self, model, B, feats, dev):
        L = nat.lib()
        self.model = model
        self.n = int(model.n_items)
        self.B = int(B)
        self.L = int(model.n_layers)
        self.T = int(model.T)
        self.n_hops = int(model.n_hops)
        self.alpha32 = float(np.float32(model.alpha))
        self.x_cap = _FLY_CALLS * self.B
        self.rows = _FLY_CALLS * self.n + self.x_cap
        gc = _as_csr(model.g)
        self.n_all = gc.number_of_nodes()
        self.indptr, self.indices = gc.device_csr(dev)
        self.tabs = [(torch.empty((self.rows, self.T), dtype=torch.int32, device=dev),
                      torch.empty((self.rows, self.T), dtype=torch.float32, device=dev)) for _ in range(self.L)]
        self.tab_ptrs = torch.tensor([nb.data_ptr() for nb, _ in self.tabs] + [wn.data_ptr() for _, wn in self.tabs],
                                     dtype=torch.int64, device=dev)
        self._nbt = (ctypes.c_void_p * self.L)(*[nb.data_ptr() for nb, _ in self.tabs])
        self._wnt = (ctypes.c_void_p * self.L)(*[wn.data_ptr() for _, wn in self.tabs])
        need = L.pinsage_fly_workspace_bytes(self.n, self.B, self.L, self.T, self.n_hops)
        if need < 0:
            raise ValueError("fly sampler: bad sizes")
        self.ws = torch.empty(int(need), dtype=torch.uint8, device=dev)
        nat.check(L.pinsage_fly_init_workspace(nat.ptr(self.ws), self.n, self.B, self.L, self.T, self.n_hops,
                                               nat.stream_ptr()), "fly_init_workspace")
        self.pos_ids = torch.empty(_FLY_CALLS * self.B, dtype=torch.int64, device=dev)
        self.n_x = torch.zeros(1, dtype=torch.int32, device=dev)
        self.ids_xo = torch.zeros(self.x_cap, dtype=torch.int64, device=dev)
        # [walk error, id error, halt]: halt is the captured step's sticky
        # refusal of its optimizer update (pinsage_fly_gate_adam)
        self.err = torch.zeros(3, dtype=torch.int32, device=dev)
        self.seeds = torch.zeros(_FLY_CALLS * self.L, dtype=torch.int64, device=dev)
        self.batch_dev = torch.zeros((self.B, _FLY_CALLS), dtype=torch.int64, device=dev)
        self.feats = feats
        d = int(feats.shape[1])
        self.fx = torch.empty((self.rows, d), dtype=torch.float32, device=dev)
        n_valid = min(int(feats.shape[0]), self.n)
        for c in range(_FLY_CALLS):
            self.fx[c * self.n:c * self.n + n_valid] = feats[:n_valid]

    def sample(self, batch_dev, pos_out=None):
        """Enqueue the sampling of batch_dev (int64 [B][3] on the device) with
        the keys in self.seeds; the engine positions go to pos_out (a device
        int64 [3 B] view, e.g. the engine workspace's ids) or self.pos_ids."""
        pos = self.pos_ids if pos_out is None else pos_out
        nat.check(nat.lib().pinsage_fly_sample(
            nat.ptr(self.indptr), nat.ptr(self.indices), self.n_all, nat.ptr(batch_dev), self.B, self.n, self.L,
            self.T, self.n_hops, self.alpha32, nat.ptr(self.seeds), nat.ptr(self.ws), self.ws.numel(), self._nbt,
            self._wnt, nat.ptr(self.tab_ptrs), self.rows, nat.ptr(pos), nat.ptr(self.n_x),
            nat.ptr(self.ids_xo), self.x_cap, nat.ptr(self.feats), self.feats.stride(0), int(self.feats.shape[1]),
            nat.ptr(self.fx), self.fx.stride(0), nat.ptr(self.err), nat.stream_ptr()), "fly_sample")

    def check_err(self):
        """Raise what the reference raises if the last sampled step met a
        zero-degree node or drew an id >= n (synchronises)."""
        e = self.err[:2].tolist()
        if e[0] != 0x7f7f7f7f:
            raise RuntimeError("walk: zero-degree node met (the reference's torch.randint(0) raises here)")
        if e[1]:
            raise IndexError("sampled neighbourhood reaches ids >= n_items (collection ids in the "
                             "zero-weight tail: the reference's h[nb] raises IndexError)")


class _DeviceTable:
    """Device mirror of a precomputed (weights, nodes) table: first T columns,
    nodes int32, weights f32 normalised by their f64 row sum."""

    @classmethod
    def resident(cls, nb32, wn, src=None):
        """A table already on the device (precompute_device_table): nb int32
        [n][T], wn f32 [n][T] normalised over the T columns."""
        t = cls.__new__(cls)
        t.src = src
        t.T = int(nb32.shape[1])
        t.nb32, t.wn = nb32, wn
        return t

    def __init__(self, nbhds, T, n_items, dev):
        w, nb = nbhds
        self.src = (w, nb)
        self.T = int(T)
        nb_t = torch.as_tensor(nb)[:, :T]
        w_t = torch.as_tensor(w)[:, :T].to(torch.float64)
        if nb_t.shape[0] < n_items:
            raise ValueError("neighbourhood table has fewer rows than n_items")
        if int(nb_t.min()) < 0 or int(nb_t.max()) >= n_items:
            # the reference's h[nb] raises IndexError for these (collection ids
            # in the zero-weight tail of a tiny graph)
            raise IndexError("neighbourhood table references ids >= n_items")
        self.nb32 = nb_t.to(torch.int32).contiguous().to(dev)
        self.wn = (w_t / w_t.sum(1, keepdim=True)).to(torch.float32).contiguous().to(dev)


def relevant_nodes_per_layer_precomp(nodeset, n_layers, T, nbhds):
    """Per-layer (nodeset, w[:, :T], nb[:, :T]) from the precomputed table;
    index 0 = bottom layer (pinsage_model.py:156-168)."""
    all_w, all_nb = nbhds
    n_items = int(all_nb.shape[0])
    out_dev = torch.as_tensor(nodeset).device
    dev = nat.device()
    nb32 = torch.as_tensor(all_nb)[:, :T].to(torch.int32).contiguous().to(dev)
    S = []
    cur = torch.as_tensor(nodeset).to(torch.int64)
    for _ in reversed(range(0, n_layers)):
        cur_c = cur.to(all_w.device)
        S.insert(0, (cur.to(out_dev), all_w[cur_c, :T].to(out_dev), all_nb[cur_c, :T].to(out_dev)))
        cur = _frontier_step(cur.to(dev), nb32, int(T), n_items)
    return S


# ----------------------------------------------------------------------------- modules
class ConvLayer(nn.Module):
    """A single PinSage convolution (pinsage_model.py:171-212).  Parameters and
    their initialisation (xavier_uniform_, bias 0.3) match the reference."""

    def __init__(self, in_dim, out_dim, hidden_dim):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.hidden_dim = hidden_dim
        self.Q = nn.Linear(in_dim, hidden_dim)
        torch.nn.init.xavier_uniform_(self.Q.weight)
        self.Q.bias.data.fill_(0.3)
        self.W = nn.Linear(in_dim + hidden_dim, out_dim)
        torch.nn.init.xavier_uniform_(self.W.weight)
        self.W.bias.data.fill_(0.3)

    def forward(self, h, nodeset, nb_nodes, nb_weights):
        """Standalone call (inside PinSageModel the fused engine runs all
        layers): the layer's rows for ``nodeset`` from the given neighbourhood
        rows on torch.ops.pinsage (pinsage_ops.conv_layer), differentiable in
        the parameters and in ``h``."""
        import pinsage_ops
        return pinsage_ops.conv_layer(h, nodeset, nb_nodes, nb_weights, self.Q.weight, self.Q.bias,
                                      self.W.weight, self.W.bias)


class PinSageModel(nn.Module):
    """PinSage model (pinsage_model.py:215-265): ``n_layers`` ConvLayers and the
    head G2(lrelu(G1 x)).  Same parameter names, init order and state_dict keys
    as the reference; forward runs the fused HIP engine."""

    def __init__(self, g, n_items, n_layers, dimensions, n_hops, alpha, T, nbhds):
        super().__init__()
        self.g = g
        self.n_items = n_items
        self.T = T
        self.n_hops = n_hops
        self.alpha = alpha
        self.nbhds = nbhds
        self.n_layers = n_layers
        self.in_dim = dimensions[0]
        self.hidden_dim = dimensions[1]
        self.out_dim = dimensions[2]
        self.in_dim_per_layer = [self.in_dim] + [self.out_dim for _ in range(n_layers - 1)]
        self.conv_layers = nn.ModuleList()
        for i in range(0, self.n_layers):
            self.conv_layers.append(ConvLayer(self.in_dim_per_layer[i], self.out_dim, self.hidden_dim))
        self.G1 = nn.Linear(self.out_dim, self.out_dim)
        torch.nn.init.xavier_uniform_(self.G1.weight)
        self.G1.bias.data.fill_(0.3)
        self.G2 = nn.Linear(self.out_dim, self.out_dim, bias=False)
        torch.nn.init.xavier_uniform_(self.G2.weight)
        # the reference's forward carries the on-the-fly sampler commented out
        # (pinsage_model.py:247-249): True samples every layer's neighbourhoods
        # per call (relevant_nodes_per_layer) instead of reading the table;
        # nbhds=None (no table) implies it
        self.sample_on_the_fly = nbhds is None
        self._runner = None
        if torch.cuda.is_available():
            self.to(nat.device())

    def runner(self):
        if self._runner is None:
            self._runner = _EngineRunner(self)
        return self._runner

    def forward(self, initial_h, nodeset):
        return self.runner()(initial_h, nodeset, self.nbhds)


# ----------------------------------------------------------------------------- engine glue
def _param_order(module_like_n_layers):
    names = []
    for i in range(module_like_n_layers):
        names += [f"conv_layers.{i}.Q.weight", f"conv_layers.{i}.Q.bias",
                  f"conv_layers.{i}.W.weight", f"conv_layers.{i}.W.bias"]
    return names + ["G1.weight", "G1.bias", "G2.weight"]


class _Engine:
    """Owns a native engine handle for one configuration."""

    def __init__(self, n_items, d_in, hid, out, n_layers, T, max_pos):
        self.cfg = nat.EngineConfig(n_items, d_in, hid, out, n_layers, T, max_pos)
        h = ctypes.c_void_p()
        nat.check(nat.lib().pinsage_engine_create(ctypes.byref(self.cfg), ctypes.byref(h)),
                  "engine_create")
        self.h = h
        self.ws_bytes = nat.lib().pinsage_engine_workspace_bytes(h)
        self.n_params = nat.lib().pinsage_engine_num_params(h)
        self.off = nat.EngineOffsets()
        nat.lib().pinsage_engine_offsets(h, ctypes.byref(self.off))

    def __del__(self):
        # capture-safe at the C-ABI (pinsage_engine_destroy makes no HIP call:
        # the engine's streams / events are retired for reuse), so a finaliser
        # the garbage collector runs inside a graph capture is harmless
        try:
            if getattr(self, "h", None):
                nat.lib().pinsage_engine_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def acquire_workspace(self, dev):
        """A workspace for an autograd call: one whose backward has run (its
        kernels left the zero-kept regions zero, so it needs no re-init), or a
        new one."""
        pool = self.__dict__.setdefault("_pool", [])
        return pool.pop() if pool else self.new_workspace(dev)

    def release_workspace(self, ws):
        """Back to the pool once the autograd node that used it is freed
        (stream order keeps the next call's kernels behind its backward); at
        most 4 kept."""
        pool = self.__dict__.setdefault("_pool", [])
        if len(pool) < 4:
            pool.append(ws)

    def new_workspace(self, dev):
        ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        nat.check(nat.lib().pinsage_engine_init_workspace(self.h, nat.ptr(ws), nat.stream_ptr()),
                  "init_workspace")
        return ws

    def counts(self, ws):
        """Frontier sizes (|S_l|, |N_l|) of the last forward in ws (synchronises)."""
        L = int(self.cfg.n_layers)
        S = (ctypes.c_int64 * L)()
        N = (ctypes.c_int64 * L)()
        nat.check(nat.lib().pinsage_engine_read_counts(self.h, nat.ptr(ws), S, N, nat.stream_ptr()),
                  "read_counts")
        return list(S), list(N)

    def tune(self, ws, margin=1.15):
        """Use the last forward's frontier sizes as GEMM tile hints (speed only)."""
        S, N = self.counts(ws)
        L = len(S)
        hs = (ctypes.c_int64 * L)(*[int(x * margin) + 1 for x in S])
        hn = (ctypes.c_int64 * L)(*[int(x * margin) + 1 for x in N])
        nat.lib().pinsage_engine_set_hints(self.h, hs, hn)
        return S, N

    def view(self, ws, off, dtype, n):
        nbytes = n * torch.empty((), dtype=dtype).element_size()
        return ws[off:off + nbytes].view(dtype)


class _EngineRunner:
    """Binds a PinSageModel's parameters (packed into one flat fp32 buffer in
    state_dict order), its features and its neighbourhood table to an engine."""

    def __init__(self, model):
        self.model = model
        self.dev = nat.device()
        self.engine = None
        self.flat = None
        self.grad_flat = None
        self._feat_key = None
        self._feat = None
        self._table_key = None
        self._table = None
        self._ws = None
        self.last_ws = None  # workspace of the last autograd forward

    # -- parameters
    def names(self):
        return _param_order(self.model.n_layers)

    def params(self):
        sd = dict(self.model.named_parameters())
        return [sd[n] for n in self.names()]

    def pack(self):
        """(Re)pack parameters into the flat device buffer if they are not
        already views of it (e.g. after .to() or assignment)."""
        ps = self.params()
        if self.flat is not None:
            ok = True
            off = 0
            base = self.flat.data_ptr()
            for p in ps:
                if p.data.data_ptr() != base + 4 * off or p.device != self.flat.device:
                    ok = False
                    break
                off += p.numel()
            if ok:
                return
        flat = torch.cat([p.detach().reshape(-1).to(self.dev, torch.float32) for p in ps])
        off = 0
        for p in ps:
            n = p.numel()
            p.data = flat[off:off + n].view(p.shape)
            off += n
        self.flat = flat

    # -- inputs
    def features(self, h):
        key = (id(h), h.data_ptr(), getattr(h, "_version", 0), tuple(h.shape))
        if key != self._feat_key:
            f = h.detach()
            if f.device != self.dev or f.dtype != torch.float32 or not f.is_contiguous():
                f = f.to(self.dev, torch.float32).contiguous()
            self._feat = f
            self._feat_key = key
        return self._feat

    def table(self, nbhds):
        m = self.model
        if m.sample_on_the_fly:
            return None
        if isinstance(nbhds, _DeviceTable):  # device-resident (precompute_device_table)
            if nbhds.T < int(m.T) or nbhds.nb32.shape[0] < m.n_items:
                raise ValueError("device table narrower than T or shorter than n_items")
            if nbhds.T == int(m.T):
                return nbhds
            key = (id(nbhds), int(m.T))
            if key != self._table_key:
                # the first T columns of a wider resident table, renormalised in f64
                w = nbhds.wn[:, :m.T].to(torch.float64)
                self._table = _DeviceTable.resident(nbhds.nb32[:, :m.T].contiguous(),
                                                    (w / w.sum(1, keepdim=True)).float().contiguous())
                self._table_key = key
            return self._table
        key = (id(nbhds[0]), id(nbhds[1]), int(m.T))
        if key != self._table_key:
            self._table = _DeviceTable(nbhds, m.T, m.n_items, self.dev)
            self._table_key = key
        return self._table

    def fly_tables(self, ids):
        """This call's on-the-fly draws as a _FlyDraws (None in table mode)."""
        m = self.model
        if not m.sample_on_the_fly:
            return None
        draws = _fly_layer_tables(m.g, m.n_items, ids, m.n_layers, m.n_hops, m.alpha, m.T)
        # (tests inspect the per-layer tables of the last calls)
        self.fly_history = (getattr(self, "fly_history", []) + [draws.tabs])[-3:]
        return draws

    def set_layer_tables(self, tabs):
        L = nat.lib()
        e = self.engine
        for l in range(self.model.n_layers):
            nb, wn = tabs[l] if tabs is not None else (None, None)
            nat.check(L.pinsage_engine_set_layer_table(e.h, l, nat.ptr(nb), nat.ptr(wn),
                                                       int(nb.shape[1]) if nb is not None else 0),
                      "set_layer_table")

    def ensure_engine(self, n_pos):
        m = self.model
        need = max(n_pos, 1)
        if self.engine is None or self.engine.cfg.max_pos < need:
            cap = max(need, self.engine.cfg.max_pos * 2 if self.engine else need)
            # on the fly, ids n_items .. n_items + cap - 1 are the earlier
            # occurrences of repeated ids (_FlyDraws)
            # (and fly_calls puts call c's nodes at c * n_items + id)
            n_eng = (_FLY_CALLS * m.n_items + cap) if m.sample_on_the_fly else m.n_items
            self.engine = _Engine(n_eng, m.in_dim, m.hidden_dim, m.out_dim, m.n_layers, m.T, cap)
            self._ws = None
        return self.engine

    def feature_planes(self, feats):
        """The feature table's hi / mid / lo bf16 planes [3, n, d] (pinsage_split_planes)
        for the layer-0 Q weight gradient on pre-split operands, re-split whenever
        the tensor changes (torch's version counter counts in-place writes); None
        unless enabled (PINSAGE_WGRAD_PLANES=1; off by default: measured no faster,
        DESIGN.md round 6), for shapes the kernel does not take,
        or when the planes would exceed PINSAGE_FPLANES_MAX_GB (default 32: C5's
        80M x 256 table stays on the in-register split)."""
        if os.environ.get("PINSAGE_WGRAD_PLANES", "0") != "1" or feats.dim() != 2:
            return None
        n, d = int(feats.shape[0]), int(feats.shape[1])
        limit = float(os.environ.get("PINSAGE_FPLANES_MAX_GB", "32")) * 2 ** 30
        if d % 64 or feats.stride(1) != 1 or feats.stride(0) % 4 or 6.0 * n * d > limit:
            return None
        key = (feats.data_ptr(), n, d, feats.stride(0), feats._version)
        if getattr(self, "_fpl_key", None) != key:
            pl = getattr(self, "_fpl", None)
            if pl is None or tuple(pl.shape) != (3, n, d) or pl.device != feats.device:
                pl = self._fpl = torch.empty((3, n, d), dtype=torch.int16, device=feats.device)
            nat.check(nat.lib().pinsage_split_planes(nat.ptr(feats), n, d, feats.stride(0), nat.ptr(pl),
                                                     nat.stream_ptr()), "split_planes")
            self._fpl_key = key
        return self._fpl

    def feature_ilv(self, feats):
        """The feature table's interleaved split-bf16 table [n, 3 d] (pinsage_split_ilv)
        for the layer-0 Q projection, re-split whenever the tensor changes (its
        version counter); None unless PINSAGE_Q0_ILV=1, for shapes the GEMM does not
        take (d % 16), or above PINSAGE_FPLANES_MAX_GB (default 32)."""
        if os.environ.get("PINSAGE_Q0_ILV", "0") != "1" or feats.dim() != 2:
            return None
        n, d = int(feats.shape[0]), int(feats.shape[1])
        limit = float(os.environ.get("PINSAGE_FPLANES_MAX_GB", "32")) * 2 ** 30
        if d % 16 or feats.stride(1) != 1 or feats.stride(0) % 4 or 6.0 * n * d > limit:
            return None
        key = (feats.data_ptr(), n, d, feats.stride(0), feats._version)
        if getattr(self, "_filv_key", None) != key:
            t = getattr(self, "_filv", None)
            if t is None or tuple(t.shape) != (n, 3 * d) or t.device != feats.device:
                t = self._filv = torch.empty((n, 3 * d), dtype=torch.int16, device=feats.device)
            nat.check(nat.lib().pinsage_split_ilv(nat.ptr(feats), feats.stride(0), n, d, nat.ptr(t), 3 * d,
                                                  nat.stream_ptr()), "split_ilv")
            self._filv_key = key
        return self._filv

    def bind(self, feats, table, grads=None, adam_m=None, adam_v=None, tabs=None):
        e = self.engine
        if table is not None:
            nb, wn = table.nb32, table.wn
        else:  # on-the-fly: the bottom layer's draws stand in as the engine-wide table
            nb, wn = tabs[0]
        nat.check(nat.lib().pinsage_engine_set_tensors(
            e.h, nat.ptr(feats), feats.stride(0), nat.ptr(nb), nat.ptr(wn),
            nb.shape[1], nat.ptr(self.flat), nat.ptr(grads), nat.ptr(adam_m),
            nat.ptr(adam_v)), "engine_set_tensors")
        pl = self.feature_planes(feats)
        nat.check(nat.lib().pinsage_engine_set_feature_planes(e.h, nat.ptr(pl), pl[0].numel() if pl is not None else 0),
                  "engine_set_feature_planes")
        ti = self.feature_ilv(feats)
        nat.check(nat.lib().pinsage_engine_set_feature_ilv(e.h, nat.ptr(ti), ti.shape[1] if ti is not None else 0),
                  "engine_set_feature_ilv")

    def run_forward(self, ws, ids_dev, inference=False):
        e = self.engine
        fn = nat.lib().pinsage_engine_forward_inference if inference else nat.lib().pinsage_engine_forward
        nat.check(fn(e.h, nat.ptr(ws), nat.ptr(ids_dev), ids_dev.shape[0], nat.stream_ptr()), "forward")

    def __call__(self, initial_h, nodeset, nbhds):
        m = self.model
        out_dev = initial_h.device
        feats = self.features(initial_h)
        if feats.shape[1] < m.in_dim:
            raise ValueError("features narrower than in_dim")
        if m.out_dim > feats.shape[1]:
            raise RuntimeError("zeros: Dimension size must be non-negative (out_dim > feature dim, "
                               "as the reference's put_embeddings)")
        table = self.table(nbhds)
        ids = torch.as_tensor(nodeset).reshape(-1).to(self.dev, torch.int64).contiguous()
        n = int(ids.shape[0])
        if n == 0:
            return torch.empty((0, m.out_dim), device=out_dev)
        n_valid = min(int(feats.shape[0]), int(m.n_items))
        lo, hi = (int(v) for v in torch.stack(torch.aminmax(ids)).tolist())
        if lo < 0 or hi >= n_valid:
            # the reference's features[nodeset] / all_w[nodeset] raise the same way
            raise IndexError(f"node ids out of range for {n_valid} items")
        self.pack()
        self.ensure_engine(n)
        draws = self.fly_tables(ids)
        tabs = draws.tabs if draws is not None else None
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.params())
        if need_grad and draws is not None and draws.n_extra:
            out = self._fly_with_repeats(feats, draws)
        elif need_grad:
            out = _EngineFn.apply(self, feats, table, ids, tabs, *self.params())
        else:
            if self._ws is None:
                self._ws = self.engine.new_workspace(self.dev)
            self.bind(feats, table, tabs=tabs)
            self.set_layer_tables(tabs)
            try:
                self.run_forward(self._ws, ids, inference=True)
            finally:
                self.set_layer_tables(None)
            out = torch.empty((n, m.out_dim), dtype=torch.float32, device=self.dev)
            nat.check(nat.lib().pinsage_engine_gather_output(self.engine.h, nat.ptr(self._ws), n,
                                                             nat.ptr(out), nat.stream_ptr()), "gather")
        return out.to(out_dev)


    def fly_calls(self, initial_h, nodesets):
        """The train step's model calls (q, pos, neg: pinsage_training.py:183-185)
        with on-the-fly sampling, in ONE engine call: each call draws its own
        layers' neighbourhoods in the reference's order (fly_tables), then call c's
        nodes become c * n_items + id (its tables' rows and neighbour ids moved by
        c * n_items, its repeated ids' earlier occurrences virtual nodes above
        len(nodesets) * n_items), so one forward / backward computes what the
        calls compute one by one.  Returns each call's output (autograd)."""
        m = self.model
        C = len(nodesets)
        if C > _FLY_CALLS or not m.sample_on_the_fly:
            return [self(initial_h, ns, None) for ns in nodesets]
        feats = self.features(initial_h)
        n_items = int(m.n_items)
        n_valid = min(int(feats.shape[0]), n_items)
        ids_c = [torch.as_tensor(ns).reshape(-1).to(self.dev, torch.int64).contiguous() for ns in nodesets]
        lohi = torch.stack([torch.stack(torch.aminmax(i)) for i in ids_c]).tolist()
        if any(lo < 0 or hi >= n_valid for lo, hi in lohi):
            raise IndexError(f"node ids out of range for {n_valid} items")
        self.pack()
        n_all = sum(int(i.shape[0]) for i in ids_c)
        self.ensure_engine(n_all)
        gc = _as_csr(m.g)
        if (_RNG_MODE != "mt19937" and os.environ.get("PINSAGE_FLY_MERGE", "1") != "0"
                and int(m.T) * 64 <= gc.number_of_nodes() and int(m.n_hops) <= 8192
                and int(m.n_hops) + int(m.T) < 65536):
            return self._fly_calls_merged(initial_h, feats, ids_c, n_items, n_valid)
        draws = [self.fly_tables(i) for i in ids_c]
        n_x = [d.n_extra for d in draws]
        base_x = C * n_items
        rows = base_x + sum(n_x)
        if rows > int(self.engine.cfg.n_items):
            raise RuntimeError("on-the-fly calls exceed the engine's node rows")
        T = int(m.T)
        tabs = []
        for l in range(m.n_layers):
            nbt = torch.empty((rows, T), dtype=torch.int32, device=self.dev)
            wnt = torch.empty((rows, T), dtype=torch.float32, device=self.dev)
            xo = base_x
            for c, d in enumerate(draws):
                nb, wn = d.tabs[l]
                torch.add(nb[:n_items], c * n_items, out=nbt[c * n_items:(c + 1) * n_items])
                wnt[c * n_items:(c + 1) * n_items] = wn[:n_items]
                if n_x[c]:
                    torch.add(nb[n_items:], c * n_items, out=nbt[xo:xo + n_x[c]])
                    wnt[xo:xo + n_x[c]] = wn[n_items:]
                xo += n_x[c]
            tabs.append((nbt, wnt))
        # feature rows: call c's copy of the table at c * n_items (made once per
        # feature tensor), the virtual rows written per call group
        fx = self._fly_feats(feats, C, n_items, n_valid, n_x=sum(n_x))
        parts, xo = [], base_x
        for c, d in enumerate(draws):
            parts.append(d.uniq + c * n_items)
            if n_x[c]:
                fx[xo:xo + n_x[c]] = feats[d.ids_x]
                parts.append(torch.arange(xo, xo + n_x[c], dtype=torch.int64, device=self.dev))
            xo += n_x[c]
        self._fly_mark_virtual(base_x, sum(n_x))
        ids = torch.cat(parts)
        out = _EngineFn.apply(self, fx, None, ids, tabs, *self.params())
        outs, o0 = [], 0
        for c, d in enumerate(draws):
            n_u = int(d.uniq.shape[0])
            out_u = out[o0:o0 + n_u]
            o0 += n_u
            if n_x[c]:
                o = out[o0:o0 + n_x[c]]
                o0 += n_x[c]
                out_u = out_u.index_add(0, d.ui_x, o - o.detach())
            outs.append(out_u[d.inv].to(initial_h.device))
        return outs

    def _fly_feats(self, feats, C, n_items, n_valid, n_x=0):
        """Feature rows of fly_calls' node ids: call c's copy of the table at
        c * n_items (made once per feature tensor); rows C * n_items .. + n_x
        are the virtual nodes', written per call group (_fly_mark_virtual).
        Every engine call over this buffer keeps a copy of its own virtual rows
        and puts them back before its backward if another call has overwritten
        them since (pending and retained-graph backwards)."""
        key = (id(feats), feats.data_ptr(), getattr(feats, "_version", 0), C, int(self.engine.cfg.n_items))
        if getattr(self, "_fly_feat_key", None) != key:
            fx = torch.empty((int(self.engine.cfg.n_items), feats.shape[1]), dtype=feats.dtype, device=self.dev)
            for c in range(C):
                fx[c * n_items:c * n_items + n_valid] = feats[:n_valid]
            self._fly_feat, self._fly_feat_key = fx, key
        return self._fly_feat

    def _fly_mark_virtual(self, base_x, n_x):
        """The virtual rows [base_x, base_x + n_x) of the shared buffer were just
        written: a new version (the next engine call records it with a copy)."""
        self._fly_ver = getattr(self, "_fly_ver", 0) + 1
        self._fly_cur = self._fly_ver
        self._fly_x = (base_x, n_x)

    def _fly_calls_merged(self, initial_h, feats, ids_c, n_items, n_valid):
        """fly_calls with the calls' walks merged per layer (_fly_tables_merged)."""
        m = self.model
        C = len(ids_c)
        tabs, uniq, inv, ids_x, ui_x = _fly_tables_merged(m.g, n_items, ids_c, m.n_layers, m.n_hops,
                                                          m.alpha, m.T)
        n_x = int(ids_x.shape[0])
        base_x = C * n_items
        if base_x + n_x > int(self.engine.cfg.n_items):
            raise RuntimeError("on-the-fly calls exceed the engine's node rows")
        fx = self._fly_feats(feats, C, n_items, n_valid, n_x=n_x)
        ids = uniq
        if n_x:
            fx[base_x:base_x + n_x] = feats[ids_x]
            ids = torch.cat([uniq, torch.arange(base_x, base_x + n_x, dtype=torch.int64, device=self.dev)])
        self._fly_mark_virtual(base_x, n_x)
        out = _EngineFn.apply(self, fx, None, ids, tabs, *self.params())
        n_u = int(uniq.shape[0])
        out_u = out[:n_u]
        if n_x:
            o = out[n_u:]
            out_u = out_u.index_add(0, ui_x, o - o.detach())
        full = out_u[inv]
        outs, p0 = [], 0
        for i in ids_c:
            outs.append(full[p0:p0 + int(i.shape[0])].to(initial_h.device))
            p0 += int(i.shape[0])
        return outs

    def _fly_with_repeats(self, feats, draws):
        """Autograd forward of an on-the-fly call whose nodeset repeats ids, in
        ONE engine call: the distinct ids (their last occurrence's draws: the
        output rows) and every earlier occurrence as a virtual node (its own
        top-layer draws, _FlyDraws).  An earlier occurrence enters the output as
        (o - o.detach()), an exact zero in the forward through which its conv
        output receives its id's summed cotangent -- index_put's backward
        (pinsage_model.py:257-265).  The virtual nodes' feature rows are copies
        of their real nodes' in this call's own feature buffer (the backward of
        every pending call reads its own)."""
        ps = self.params()
        n_u, n_x, n_items = int(draws.uniq.shape[0]), draws.n_extra, draws.n_items
        if n_items + n_x > int(self.engine.cfg.n_items):
            raise RuntimeError("on-the-fly repeats exceed the engine's virtual rows")
        fx = torch.empty((n_items + n_x, feats.shape[1]), dtype=feats.dtype, device=feats.device)
        nf = min(int(feats.shape[0]), n_items)
        fx[:nf] = feats[:nf]
        fx[n_items:] = feats[draws.ids_x]
        ids = torch.cat([draws.uniq, torch.arange(n_items, n_items + n_x, dtype=torch.int64,
                                                  device=draws.uniq.device)])
        out = _EngineFn.apply(self, fx, None, ids, draws.tabs, *ps)
        o = out[n_u:]
        out_u = out[:n_u].index_add(0, draws.ui_x, o - o.detach())
        return out_u[draws.inv]


class _EngineFn(torch.autograd.Function):
    """Forward + HIP backward of PinSageModel for autograd callers."""

    @staticmethod
    def forward(ctx, runner, feats, table, ids, tabs, *params):
        e = runner.engine
        ws = e.acquire_workspace(runner.dev)
        runner.bind(feats, table, tabs=tabs)
        runner.set_layer_tables(tabs)
        try:
            runner.run_forward(ws, ids)
        finally:
            runner.set_layer_tables(None)
        n = int(ids.shape[0])
        out = torch.empty((n, runner.model.out_dim), dtype=torch.float32, device=runner.dev)
        nat.check(nat.lib().pinsage_engine_gather_output(e.h, nat.ptr(ws), n, nat.ptr(out),
                                                         nat.stream_ptr()), "gather")
        ctx.runner, ctx.ws, ctx.feats, ctx.table, ctx.n = runner, ws, feats, table, n
        runner.last_ws = ws  # (bench.py reads frontier sizes from it: the last call to use it)
        ctx.tabs = tabs  # the frontier's tables stay alive with the workspace
        ctx.engine = e
        ctx.n_bwd = 0
        # the workspace holds this graph's activations: it goes back to the
        # pool when the autograd node is freed (after the last backward a
        # retained graph may still run), never earlier
        weakref.finalize(ctx, e.release_workspace, ws)
        fxr = getattr(runner, "_fly_x", None)
        if fxr is not None and fxr[1] and feats is getattr(runner, "_fly_feat", None):
            # this call's virtual-node rows of the shared on-the-fly feature
            # buffer (its backward reads them; a later call may overwrite them)
            b0, nx = fxr
            ctx.fly_x = (b0, nx, feats[b0:b0 + nx].clone(), runner._fly_cur)
        return out

    @staticmethod
    def backward(ctx, dout):
        runner, e, ws = ctx.runner, ctx.engine, ctx.ws
        grads = torch.zeros(e.n_params, dtype=torch.float32, device=runner.dev)
        runner.bind(ctx.feats, ctx.table, grads=grads, tabs=ctx.tabs)
        fx = getattr(ctx, "fly_x", None)
        if fx is not None and getattr(runner, "_fly_cur", None) != fx[3]:
            # another call wrote its virtual rows since this forward: put this
            # call's back (a retained graph's later backward)
            ctx.feats[fx[0]:fx[0] + fx[1]] = fx[2]
            runner._fly_cur = fx[3]
        dout = dout.contiguous().to(torch.float32)
        if ctx.n_bwd:  # a retained graph's next backward: re-zero what the last one accumulated into
            nat.check(nat.lib().pinsage_engine_reset_backward(e.h, nat.ptr(ws), nat.stream_ptr()),
                      "reset_backward")
        nat.check(nat.lib().pinsage_engine_set_output_grad(e.h, nat.ptr(ws), nat.ptr(dout), ctx.n,
                                                           nat.stream_ptr()), "set_output_grad")
        nat.check(nat.lib().pinsage_engine_backward(e.h, nat.ptr(ws), nat.stream_ptr()), "backward")
        ctx.n_bwd += 1
        out = []
        off = 0
        for p in runner.params():
            k = p.numel()
            out.append(grads[off:off + k].view(p.shape))
            off += k
        return (None, None, None, None, None, *out)
