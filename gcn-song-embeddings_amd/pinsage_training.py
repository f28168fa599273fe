"""Drop-in ``pinsage_training`` (reference ``pinsage_training.py:31-339``) on MI355X.

``PinSage.train_batch`` runs ONE fused device step: frontier of the union of
the query/positive/negative ids, fp32-MFMA convolutions, head, max-margin loss
with the reference's gradient semantics, HIP backward and a fused Adam update
on a flat parameter buffer -- no host synchronisation inside the step.  Batch
sampling reproduces the reference's torch RNG consumption exactly (native
Fisher-Yates prefix), so a seeded run draws the same batches.

Data parallel: when ``torch.distributed`` is initialised, every rank draws the
same global batch (world * batch_size triples, shared seed) and trains on its
slice; gradients are averaged with one RCCL all-reduce of the flat buffer.
"""
from __future__ import annotations

import ctypes
import gc
import os
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

import _native as nat
import pinsage_model as psm

BASE_RUN_DIR = "./runs"

TEST_TRACK_INFO = None
TEST_IDS = None


def max_margin_loss(h_q, h_pos, h_neg, margin):
    """Hinge on normalised dot products, batch mean (pinsage_training.py:31-41).
    Device tensors go through torch ops (small); the train step uses the fused kernel."""
    norm = torch.nn.functional.normalize
    h_q, h_pos, h_neg = norm(h_q, dim=1), norm(h_pos, dim=1), norm(h_neg, dim=1)
    dot = (h_q * h_neg).sum(1) - (h_q * h_pos).sum(1) + margin
    return torch.clamp(dot, min=0.0).mean()


def _triplet_loss(Z, margin):
    """max_margin_loss of outputs Z [3, B, d] and its cotangent [3, B, d] with
    the train step's own kernels and summation order (pinsage_triplet_loss):
    the micro-batched step then ends on the fused step's loss bits whenever
    its output rows are the same.  Outputs the kernel does not take (d > 256
    or not dividing 1024) go through torch.  Returns (loss, cotangent,
    variance or None)."""
    B, d = int(Z.shape[1]), int(Z.shape[2])
    if d > 256 or 1024 % d or not Z.is_cuda:
        Zr = Z.detach().requires_grad_()
        with torch.enable_grad():
            loss = max_margin_loss(Zr[0], Zr[1], Zr[2], margin)
            (g,) = torch.autograd.grad(loss, [Zr])
        return loss, g, None
    L = nat.lib()
    Zc = Z.detach().contiguous()
    G = torch.empty((3, 3, B, d), dtype=torch.float32, device=Z.device)
    scratch = torch.empty(int(L.pinsage_triplet_loss_scratch_bytes(B, d)), dtype=torch.uint8, device=Z.device)
    scal = torch.empty(4, dtype=torch.float32, device=Z.device)
    nat.check(L.pinsage_triplet_loss(nat.ptr(Zc), B, d, float(margin), nat.ptr(G), nat.ptr(scratch),
                                     nat.ptr(scal), nat.stream_ptr()), "triplet_loss")
    g = torch.stack([G[0, 0], G[1, 1], G[2, 2]])
    return scal[0], g, scal[3]


def cosine_dissimilarity(a, b):
    return 1 - F.cosine_similarity(a, b)


TRIPLET_LOSS = torch.nn.TripletMarginLoss(0.0001, reduction="mean")
COSINE_TRIPLET_LOSS = torch.nn.TripletMarginWithDistanceLoss(distance_function=cosine_dissimilarity,
                                                             margin=0.0001, reduction="mean")


# ----------------------------------------------------------------------------- batches
def sample_positives_with_rep(positives, batch_size):
    """positives[randperm(P)[:batch_size]] (pinsage_training.py:53-62)."""
    P = positives.shape[0]
    with nat.torch_rng() as mt:
        sel = mt.randperm_prefix(P, batch_size)
    return positives[torch.from_numpy(sel), :].to(torch.int64)


def sample_easy_negatives(all_ids, pos_batch):
    """One random non-batch id per pair (pinsage_training.py:64-77)."""
    n = all_ids.shape[0]
    members = pos_batch.flatten().unique()
    mask = torch.ones((n,)).bool()
    mask[members] = False
    possible_neg = all_ids[mask].to(torch.int64)
    with nat.torch_rng() as mt:
        sel = mt.randperm_prefix(possible_neg.shape[0], pos_batch.shape[0])
    negatives = possible_neg[torch.from_numpy(sel)]
    batch = torch.cat((pos_batch, negatives.unsqueeze(1)), dim=1)
    return batch, batch.flatten().unique().to(torch.int64)


def sample_hard_negatives(all_ids, pos_batch, nbhds, min_rank, max_rank):
    """pinsage_training.py:79-87, including its row-gather behaviour (the
    reference gathers rows 0..B-1 of the table, not the query rows)."""
    queries = pos_batch[:, 0]
    rnd_ranks = torch.randint(min_rank, max_rank, (queries.shape[0],))
    hard_neg = torch.gather(nbhds[1], 1, rnd_ranks.view(-1, 1)).squeeze()
    batch = torch.cat((pos_batch, hard_neg.unsqueeze(1)), dim=1)
    return batch, batch.flatten().unique().to(torch.int64)


def sample_batch(all_ids, positives, batch_size, nbhds, hard_negatives=True, hn_min=10, hn_max=100):
    """pinsage_training.py:89-97.  The easy-negative path runs natively
    (same draws as the reference, without materialising randperm(P))."""
    if hard_negatives:
        pos_batch = sample_positives_with_rep(positives, batch_size)
        return sample_hard_negatives(all_ids, pos_batch, nbhds, hn_min, hn_max)
    pos = positives if positives.dtype == torch.int64 else positives.to(torch.int64)
    pos = pos.contiguous()
    n_items = int(all_ids.shape[0])
    if not _all_ids_is_range(all_ids):
        batch, nodeset = sample_easy_negatives(all_ids, sample_positives_with_rep(positives, batch_size))
        return batch, nodeset
    return _PREFETCH.sample(pos, n_items, int(batch_size))


class _BatchPrefetcher:
    """Reference-exact easy batches through the native batch sampler
    (pinsage_batch_sampler_*, csrc/loader.hip).

    The reference draws every batch from torch's global CPU generator; its O(P)
    part is randperm(P) consuming P-1 draws.  After serving a batch, the native
    sampler draws the next one on its worker thread from a copy of the generator
    state it just handed back, and uses that draw only if the next request
    starts from a byte-identical state (nothing else touched torch's generator);
    otherwise it draws synchronously.  Batches and generator states are exactly
    the reference's either way.  PINSAGE_PREFETCH=0 disables the speculation."""

    def __init__(self):
        self.speculate = os.environ.get("PINSAGE_PREFETCH", "1") != "0"
        self.h = None
        self.key = None
        self.pos_np = None
        self.hits = 0

    def _sampler(self, pos, n_items, batch_size):
        key = (pos.data_ptr(), pos._version, tuple(pos.shape), n_items, batch_size)
        if key != self.key:
            self.close()
            self.pos_np = pos.numpy() if pos.device.type == "cpu" else pos.cpu().numpy()
            h = ctypes.c_void_p()
            nat.check(nat.lib().pinsage_batch_sampler_create(
                self.pos_np.ctypes.data_as(nat.vp), self.pos_np.shape[0], n_items, batch_size,
                ctypes.byref(h)), "batch_sampler_create")
            self.h, self.key = h, key
        return self.h

    def close(self):
        if self.h is not None:
            nat.lib().pinsage_batch_sampler_destroy(self.h)
            self.h = None
            self.key = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sample(self, pos, n_items, batch_size):
        h = self._sampler(pos, n_items, batch_size)
        B = min(batch_size, int(pos.shape[0]))
        state = torch.get_rng_state()
        st = state.numpy()
        after = torch.empty_like(state)
        out = np.empty((B, 3), np.int64)
        ns = np.empty(3 * B, np.int64)
        n_ns = ctypes.c_int64(0)
        rc = nat.lib().pinsage_batch_sampler_next(
            h, st.ctypes.data_as(nat.vp), st.nbytes, out.ctypes.data_as(nat.vp),
            ns.ctypes.data_as(nat.vp), ctypes.byref(n_ns), after.numpy().ctypes.data_as(nat.vp),
            1 if self.speculate else 0)
        nat.check(min(rc, 0), "sample_batch")
        self.hits += rc
        torch.set_rng_state(after)
        self.last = (B, torch.get_rng_state())
        return torch.from_numpy(out), torch.from_numpy(ns[:n_ns.value])

    def peek(self, batch_size):
        """The batch the next sample() of this size will return if nothing
        touches torch's generator before it ([B, 3] int64 numpy), or None.
        A hint only: whoever acts on it compares it with the batch it gets."""
        if not self.speculate or self.h is None or self.key is None or self.key[4] != batch_size:
            return None
        last = getattr(self, "last", None)
        if last is None or not torch.equal(last[1], torch.get_rng_state()):
            return None
        out = np.empty((last[0], 3), np.int64)
        rows = nat.lib().pinsage_batch_sampler_peek(self.h, out.ctypes.data_as(nat.vp), last[0])
        return out[:rows] if rows == last[0] else None


_PREFETCH = _BatchPrefetcher()


_RANGE_CACHE = {}


def _all_ids_is_range(all_ids):
    """all_ids == arange(n) (the reference's PinSage.all_ids); cached per tensor
    version so the per-batch check is free."""
    key = (id(all_ids), all_ids.data_ptr(), all_ids._version, tuple(all_ids.shape))
    hit = _RANGE_CACHE.get(key)
    if hit is None:
        n = int(all_ids.shape[0])
        hit = torch.equal(all_ids.cpu().to(torch.int64), torch.arange(n, dtype=torch.int64))
        _RANGE_CACHE.clear()
        _RANGE_CACHE[key] = hit
    return hit


def batch_variance(h):
    """Monitor of collapse to a constant (pinsage_training.py:99-103)."""
    mean = torch.mean(h, dim=0)
    var = torch.sum(torch.pow(h - mean, 2)) / (h.shape[0] - 1)
    return torch.prod(var)


# ----------------------------------------------------------------------------- data parallel
def _allreduce_start(flat):
    """Begin the mean of a flat gradient bucket over the process group, ordered
    after the current stream's work; returns a handle for _allreduce_finish.
    Both backends run it asynchronously (async_op=True), so the overlap and its
    stream ordering are the same code on RCCL (the 8-GPU run) and on gloo (the
    tests): RCCL averages in the collective; gloo sums (it has no AVG) and the
    finish scales."""
    d = torch.distributed
    if d.get_backend() == "nccl":
        return d.all_reduce(flat, op=d.ReduceOp.AVG, async_op=True), None
    return d.all_reduce(flat, async_op=True), flat


def _allreduce_finish(handle):
    """The current stream waits for a bucket started by _allreduce_start (and
    the gloo sum becomes the mean, on that stream)."""
    work, flat = handle
    work.wait()
    if flat is not None:
        flat.mul_(1.0 / torch.distributed.get_world_size())


def average_gradients(flat):
    """Mean of a flat gradient buffer over the process group: ONE all-reduce
    (RCCL over xGMI on MI355X nodes; gloo on CPU)."""
    d = torch.distributed
    if d.is_available() and d.is_initialized() and d.get_world_size() > 1:
        if d.get_backend() == "nccl":  # RCCL averages in the collective: no extra launch
            d.all_reduce(flat, op=d.ReduceOp.AVG)
        else:
            d.all_reduce(flat)
            flat.mul_(1.0 / d.get_world_size())
    return flat


# ----------------------------------------------------------------------------- trainer
# PINSAGE_HOST_TIMING=1: accumulate host seconds per section of the train step
_HOST_T = {} if os.environ.get("PINSAGE_HOST_TIMING") else None
_HOST_LAST = [0.0]


def _tick(name):
    if _HOST_T is not None:
        t = time.perf_counter()
        if name != "pre":
            _HOST_T[name] = _HOST_T.get(name, 0.0) + t - _HOST_LAST[0]
        _HOST_LAST[0] = t


class _FusedStep:
    """Device state of the fused train step: flat param/grad/Adam buffers, two
    engine workspaces (steps alternate between them), the host hand-off ring
    and the scalar outputs.

    One step is ONE graph launch and nothing else on the stream.  The host
    writes the step's ids and Adam coefficients into a slot of a pinned ring;
    the graph's first kernel stages them from the slot a device counter picks
    (pinsage_step_stage), its last kernel publishes (loss, node_feat_loss,
    variance) into the step's entry of a device ring and advances the counter
    (pinsage_step_publish); train_batch returns views of that entry, valid for
    ``OUT_RING`` steps.

    The frontier of a step (pinsage_engine_frontier) reads only its ids and the
    neighbourhood table.  So step i's graph also computes, on a branch beside
    its backward, the frontier of the batch the native sampler has already
    drawn for step i+1 (in the other workspace).  Step i+1 checks its batch is
    that one (it is whenever nothing else used torch's generator in between);
    otherwise it first launches its own frontier graph.  Results are the same
    either way.  PINSAGE_FRONTIER_AHEAD: "start" (default: the branch forks at
    the graph's start), "fwd" (forked by the engine after the layer-0 Q
    projection), "graph" (it forks before the backward) or "0" (no look-ahead);
    measured at C2 (ms/step, run-to-run noise ~4 %): 0.57-0.62 / 0.62 / 0.64 /
    0.70."""

    HOST_RING = 8
    OUT_RING = 1 << 16

    def __init__(self, trainer):
        self.tr = trainer
        model = trainer.model
        self.runner = model.runner()
        self.dev = self.runner.dev
        self.B = 0
        self.wss = None
        self.ws = None
        self.eng = None  # the engine the workspaces and staged views belong to
        self.m = self.v = None
        self.grads = None
        self._tuned = False
        self.dist = (torch.distributed.is_available() and torch.distributed.is_initialized()
                     and torch.distributed.get_world_size() > 1)
        # data parallel: the backward runs in two stages (head and layers L-1..1,
        # then layer 0) and the first stage's gradients are all-reduced while the
        # second runs (PINSAGE_DP_BUCKETS=0: one all-reduce after the backward)
        self.dp_buckets = os.environ.get("PINSAGE_DP_BUCKETS", "1") != "0"
        self.comm = None
        # the device step is captured into hipGraphs and replayed
        self.use_graph = os.environ.get("PINSAGE_HIPGRAPH", "1") != "0"
        # Adam fused into the gradient reductions (0: separate optimizer pass)
        self.fuse_adam = os.environ.get("PINSAGE_FUSED_ADAM", "1") != "0"
        mode = os.environ.get("PINSAGE_FRONTIER_AHEAD", "start")
        self.ahead = mode != "0"
        self.ahead_mode = mode
        self.graphs = None
        self.graph_B = None
        self.side = None
        self.gfr = None
        self.parity = 0
        self.ahead_hits = 0
        # in-context GEMM tuner (see _autotune); PINSAGE_AUTOTUNE=0 keeps the size model
        # (deterministic: the same choices, so the same summation orders, on every run)
        self.autotune = os.environ.get("PINSAGE_AUTOTUNE", "1") != "0"
        self.tuned_choices = None
        self.wait_s = 0.0  # host seconds blocked on ring slots (Python path)
        self.stepper = None

    def ring_wait_s(self):
        """Host seconds the steps spent blocked on ring slots, i.e. waiting for
        the device (both host paths)."""
        w = self.wait_s
        if self.stepper is not None:
            w += nat.lib().pinsage_stepper_wait_ns(self.stepper) * 1e-9
        return w

    def stepper_stats(self):
        """Host nanoseconds of the native step path so far (pinsage_stepper_stats):
        {wait_ns, launch_ns, call_ns, steps, hits}, or None without a stepper."""
        if self.stepper is None:
            return None
        v = (ctypes.c_int64 * 5)()
        nat.check(nat.lib().pinsage_stepper_stats(self.stepper, v, 5), "stepper_stats")
        return dict(zip(("wait_ns", "launch_ns", "call_ns", "steps", "hits"), (int(x) for x in v)))

    def ensure(self, B):
        r = self.runner
        r.pack()
        n_params = r.flat.numel()
        if self.grads is None or self.grads.numel() != n_params:
            self.grads = torch.zeros(n_params, dtype=torch.float32, device=self.dev)
            self.m = torch.zeros(n_params, dtype=torch.float32, device=self.dev)
            self.v = torch.zeros(n_params, dtype=torch.float32, device=self.dev)
            self.adopt_optimizer_state()
        # a forward over more ids (embed(), evaluation) may have replaced the
        # runner's engine: workspaces, staged views and graphs of the old one
        # are then stale and are rebuilt for the new one
        if (self.wss is None or r.engine is None or r.engine is not self.eng
                or r.engine.cfg.max_pos < 3 * B):
            r.ensure_engine(3 * B)
            self.eng = r.engine
            self.wss = [r.engine.new_workspace(self.dev) for _ in range(2)]
            self.B = B
            off = r.engine.off
            mp = r.engine.cfg.max_pos
            self.ids_view = [r.engine.view(w, int(off.ids), torch.int64, mp) for w in self.wss]
            # ids, and behind them the step's Adam coefficients (pinsage_engine_adam)
            self.stage_view = [w[int(off.ids):int(off.ids) + mp * 8 + 16] for w in self.wss]
            self.scal = [r.engine.view(w, int(off.scalars), torch.float32, 4) for w in self.wss]
            # pinned hand-off ring: slot = [ids of this step | ids of the next
            # (look-ahead) | Adam coefficients]
            self.slot_ids, self.slot_next, self.slot_coef = 0, mp * 8, 2 * mp * 8
            self.slot_bytes = 2 * mp * 8 + 16
            self.ring = torch.empty((self.HOST_RING, self.slot_bytes), dtype=torch.uint8).pin_memory()
            self.ring_ev = [None] * self.HOST_RING
            self.ctr = torch.zeros(1, dtype=torch.int64, device=self.dev)
            self.out_ring = torch.zeros((self.OUT_RING, 4), dtype=torch.float32, device=self.dev)
            self.nstep = 0
            self.pending = [None, None]  # ids whose frontier already sits in workspace q
            self.parity = 0
            self.ws = self.wss[0]
            self._tuned = False
            self.tuned_choices = None
            self.graphs = None
            self._drop_stepper()

    def adopt_optimizer_state(self):
        """Use the optimizer's Adam state (if any, e.g. after load_state_dict) as
        the initial flat m/v, then make the optimizer state views of them."""
        opt = self.tr.optimizer
        off = 0
        step = 0
        for p in self.runner.params():
            k = p.numel()
            st = opt.state.get(p)
            if st and "exp_avg" in st:
                self.m[off:off + k].copy_(st["exp_avg"].reshape(-1))
                self.v[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
                step = int(float(st["step"]))
            opt.state[p] = {"step": torch.tensor(float(step)),
                            "exp_avg": self.m[off:off + k].view(p.shape),
                            "exp_avg_sq": self.v[off:off + k].view(p.shape)}
            p.grad = self.grads[off:off + k].view(p.shape)
            off += k
        self.host_step = step

    def sync_optimizer_step(self):
        for p in self.runner.params():
            st = self.tr.optimizer.state.get(p)
            if st is not None:
                st["step"] = torch.tensor(float(self.host_step))

    def _adam_coef(self, step):
        """torch.optim.Adam's per-step scalars (_single_tensor_adam, computed in
        double as there): lr / (1 - beta1^t) and sqrt(1 - beta2^t)."""
        g = self.tr.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        lr = float(g["lr"])
        return lr / (1 - b1 ** step), (1 - b2 ** step) ** 0.5

    # ---- host side of the hand-off ring
    def _slot_write_ids(self, k, off, batch, B):
        ids = self.ring[k, off:off + 3 * B * 8].view(torch.int64)
        ids.copy_(torch.as_tensor(batch).reshape(-1).to(torch.int64))
        n_items = int(self.runner.engine.cfg.n_items)
        if int(ids.min()) < 0 or int(ids.max()) >= n_items:
            raise IndexError(f"batch ids out of range for {n_items} items")

    def _slot_write_coef(self, k):
        self.ring[k, self.slot_coef:self.slot_coef + 8].view(torch.float32).copy_(
            torch.tensor(self._adam_coef(self.host_step + 1), dtype=torch.float32))

    # ---- device phases
    def _stage(self, B, src_off, q_ids, p_coef):
        """Copy 3B ids at src_off of the counter's slot into workspace q_ids (if
        not None) and the coefficients into workspace p_coef (if not None)."""
        dst = self.ids_view[q_ids] if q_ids is not None else None
        coef = (ctypes.c_void_p(self.stage_view[p_coef].data_ptr() + 3 * B * 8)
                if p_coef is not None else None)
        nat.check(nat.lib().pinsage_step_stage(
            nat.ptr(self.ring), self.slot_bytes, self.HOST_RING, nat.ptr(self.ctr), src_off,
            3 * B * 8 if dst is not None else 0, nat.ptr(dst), self.slot_coef, coef,
            nat.stream_ptr()), "step_stage")

    def _publish(self, p):
        nat.check(nat.lib().pinsage_step_publish(nat.ptr(self.scal[p]), 4, nat.ptr(self.out_ring),
                                                 self.OUT_RING, nat.ptr(self.ctr), nat.stream_ptr()),
                  "step_publish")

    def _frontier(self, B, q):
        e = self.runner.engine
        nat.check(nat.lib().pinsage_engine_frontier(e.h, nat.ptr(self.wss[q]), nat.ptr(self.ids_view[q]),
                                                    3 * B, nat.stream_ptr()), "frontier")

    def _main(self, B, p, with_adam, before_backward=None, stage=None):
        """Layers, head, loss, backward (and Adam) of workspace p's frontier;
        before_backward() is called (to fork work) between loss and backward.
        stage=0: the backward's first stage only (_dp_tail runs the rest)."""
        tr = self.tr
        e = self.runner.engine
        st = nat.stream_ptr()
        L = nat.lib()
        nat.check(L.pinsage_engine_forward_layers(e.h, nat.ptr(self.wss[p]), st), "forward_layers")
        nat.check(L.pinsage_engine_loss(e.h, nat.ptr(self.wss[p]), B, float(tr.margin), 1, st), "loss")
        if not self._tuned:  # once: frontier sizes of a real batch pick the GEMM tiles
            e.tune(self.wss[p])
            self._tuned = True
        if before_backward is not None:
            before_backward()
        if stage == 0:
            nat.check(L.pinsage_engine_backward_stage(e.h, nat.ptr(self.wss[p]), 0, st), "backward_stage")
            return
        self._backward(p, with_adam)

    def _dp_split(self):
        """Flat offset of layer 1's first parameter: [0, split) are layer 0's
        gradients (the backward's last stage), [split, n) the rest."""
        return sum(p.numel() for p in self.runner.params()[:4])

    def _dp_tail(self, p, g2):
        """Data-parallel end of a step whose first backward stage is enqueued:
        all-reduce that stage's gradients (head and layers L-1..1) on a comm
        stream while layer 0's backward runs (graph g2, or eagerly), then layer
        0's bucket, then Adam on the averaged gradients (pinsage_training.py:
        188-191 with the gradients averaged over the ranks)."""
        cur = torch.cuda.current_stream()
        if self.comm is None:
            self.comm = torch.cuda.Stream()
        split = self._dp_split()
        bucket_a, bucket_b = self.grads[split:], self.grads[:split]
        self.comm.wait_stream(cur)
        with torch.cuda.stream(self.comm):
            wa = _allreduce_start(bucket_a)
        if g2 is not None:
            g2.replay()
        else:
            e = self.runner.engine
            nat.check(nat.lib().pinsage_engine_backward_stage(e.h, nat.ptr(self.wss[p]), 1, nat.stream_ptr()),
                      "backward_stage")
            self._publish(p)
        self.comm.wait_stream(cur)
        with torch.cuda.stream(self.comm):
            wb = _allreduce_start(bucket_b)
            _allreduce_finish(wa)
            _allreduce_finish(wb)
        cur.wait_stream(self.comm)
        self._adam(p)

    def _backward(self, p, with_adam):
        """Backward; with_adam: Adam fused into the gradient reductions
        (pinsage_engine_backward_adam, bitwise equal to backward + adam)."""
        e = self.runner.engine
        if with_adam and self.fuse_adam:
            g = self.tr.optimizer.param_groups[0]
            b1, b2 = g["betas"]
            nat.check(nat.lib().pinsage_engine_backward_adam(
                e.h, nat.ptr(self.wss[p]), self._coef_ptr(p), float(b1), float(b2), float(g["eps"]),
                nat.stream_ptr()), "backward_adam")
            return
        nat.check(nat.lib().pinsage_engine_backward(e.h, nat.ptr(self.wss[p]), nat.stream_ptr()),
                  "backward")
        if with_adam:
            self._adam(p)

    def _coef_ptr(self, p):
        return ctypes.c_void_p(self.stage_view[p].data_ptr() + 3 * self.B_cur * 8)

    def _adam(self, p):
        g = self.tr.optimizer.param_groups[0]
        b1, b2 = g["betas"]
        nat.check(nat.lib().pinsage_engine_adam(self.runner.engine.h, self._coef_ptr(p), float(b1),
                                                float(b2), float(g["eps"]), nat.stream_ptr()), "adam")

    # per-site candidates: (cfg, stream_k, splits); a GEMM site takes a block-tile
    # config with or without stream-K, a weight-gradient site a config and a split-K count
    # Candidates keep every site's fp32 summation order (the default tuner is
    # reproducible run to run): the block tile alone never changes an output
    # element's k order; stream-K (cut k ranges) and split-K counts do, so
    # stream-K stays off under the tuner and split counts stay the size model's
    # (splits 0).  PINSAGE_AUTOTUNE=wide also tries those (timing-picked, so
    # two runs may then differ at rounding level).
    _GEMM_OPTS = [(c, 0, 0) for c in (0, 1, 2, 3, 5)]
    _WGRAD_OPTS = [(c, -1, 0) for c in (0, 1, 2)]
    _GEMM_OPTS_WIDE = [(c, k, 0) for c in (0, 1, 2, 3) for k in (0, 1) if not (c == 0 and k == 1)]
    _WGRAD_OPTS_WIDE = [(c, -1, sp) for c in (0, 1, 2) for sp in (2, 4, 8, 16, 32, 64)]

    def _gemm_sites(self):
        wide = os.environ.get("PINSAGE_AUTOTUNE", "1") == "wide"
        G = self._GEMM_OPTS_WIDE if wide else self._GEMM_OPTS
        Wg = self._WGRAD_OPTS_WIDE if wide else self._WGRAD_OPTS
        sites = []
        for l in range(self.runner.model.n_layers):
            sites += [(f"fwd.q_gemm.l{l}", G), (f"fwd.w_gemm.l{l}", G),
                      (f"bwd.dcat.l{l}", G), (f"bwd.w_wgrad.l{l}", Wg),
                      (f"bwd.q_wgrad.l{l}", Wg)]
            if l > 0:
                sites.append((f"bwd.dh.l{l}", G))
        return sites + [("bwd.wgrad.g1", Wg), ("bwd.wgrad.g2", Wg)]

    def _autotune(self, B, p, reps=3):
        """In-context GEMM tuner: the size model picks tile configs from frontier
        sizes alone, and measured in the step it is off by up to 2x on the small
        projections (launch-latency bound, sensitive to the chip's state).  So on
        the first step's frontier, every GEMM site is timed under each candidate
        with HIP events on its launch stream (kernels back to back behind a
        stream hold), and the fastest is kept (pinsage_engine_set_gemm_choice).
        Probe k sets candidate k at every site at once (their interplay is second
        order).  The probes run before the step's own forward (the caller runs
        the real step afterwards, so its outputs, gradients and workspace are
        the step's): this step's frontier, layers, loss and backward WITHOUT
        the optimizer -- parameters and Adam state are untouched.

        Reproducibility: the candidates (_GEMM_OPTS / _WGRAD_OPTS) differ only
        in the block tile, which never changes an output element's summation
        order (a site the size model runs stream-K keeps the size model's
        schedule), so whichever wins, the step computes bitwise the same values
        (tests/test_gpu_parity.py::test_default_step_is_bitwise_reproducible).
        PINSAGE_AUTOTUNE=wide also tries stream-K and split-K counts, which
        change the order (two runs may then differ at rounding level).  The
        choices are recorded (``tuned_choices``; bench.py prints them as
        "gemm_choices"), PINSAGE_GEMM_CHOICES=<that json> replays them, and
        PINSAGE_AUTOTUNE=0 keeps the size model."""
        e = self.runner.engine
        L = nat.lib()
        sites = self._gemm_sites()
        if os.environ.get("PINSAGE_AUTOTUNE", "1") != "wide":
            # a site the size model runs stream-K keeps that schedule (its cut
            # points fix the summation order): probe the size model once, then
            # tune tile configs only where it runs whole-K tiles
            for site, _ in sites:
                nat.check(L.pinsage_engine_set_gemm_choice(e.h, site.encode(), -1, -1, 0), "set_gemm_choice")
            self._frontier(B, p)
            st = nat.stream_ptr()
            nat.check(L.pinsage_engine_forward_layers(e.h, nat.ptr(self.wss[p]), st), "forward_layers")
            nat.check(L.pinsage_engine_loss(e.h, nat.ptr(self.wss[p]), B, float(self.tr.margin), 1, st), "loss")
            nat.check(L.pinsage_engine_backward(e.h, nat.ptr(self.wss[p]), st), "backward")
            torch.cuda.synchronize()
            sites = [(site, [(-1, -1, 0)] if L.pinsage_engine_site_stream_k(e.h, site.encode()) == 1 else o)
                     for site, o in sites]
        n_probe = max(len(o) for _, o in sites)
        best = {name: (float("inf"), None) for name, _ in sites}
        hold = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        name = ctypes.create_string_buffer(128)
        ms = ctypes.c_double()
        calls = ctypes.c_int64()
        for k in range(n_probe):
            for site, opts in sites:
                o = opts[k % len(opts)]
                nat.check(L.pinsage_engine_set_gemm_choice(e.h, site.encode(), *o), "set_gemm_choice")
            nat.check(L.pinsage_engine_timing(e.h, 1), "timing")
            ok = True
            try:
                for _ in range(reps):
                    L.pinsage_stream_hold(2000, hold)
                    self._frontier(B, p)
                    st = nat.stream_ptr()
                    nat.check(L.pinsage_engine_forward_layers(e.h, nat.ptr(self.wss[p]), st), "forward_layers")
                    nat.check(L.pinsage_engine_loss(e.h, nat.ptr(self.wss[p]), B, float(self.tr.margin), 1, st),
                              "loss")
                    nat.check(L.pinsage_engine_backward(e.h, nat.ptr(self.wss[p]), st), "backward")
                torch.cuda.synchronize()
            except RuntimeError:  # e.g. a split count whose slabs do not fit: not a candidate
                ok = False
                torch.cuda.synchronize()
            L.pinsage_engine_timing_collect(e.h)
            i = 0
            while ok and L.pinsage_engine_timing_get(e.h, i, name, 128, ctypes.byref(ms), ctypes.byref(calls)) == 0:
                nm = name.value.decode()
                if nm in best and calls.value > 0:
                    opts = dict(sites)[nm]
                    t = ms.value / calls.value
                    if t < best[nm][0]:
                        best[nm] = (t, opts[k % len(opts)])
                i += 1
            L.pinsage_engine_timing(e.h, 0)
        for site, _ in sites:
            o = best[site][1]
            nat.check(L.pinsage_engine_set_gemm_choice(e.h, site.encode(), *(o if o else (-1, -1, 0))),
                      "set_gemm_choice")
        # a site that never launched (e.g. a Q GEMM fused into the layer below's
        # kernel) keeps the size model and is left out of the record
        self.tuned_choices = {k: {"us": v[0] * 1e3, "cfg": v[1]} for k, v in best.items() if v[1] is not None}

    def _load_choices(self, path):
        """Fixed per-site GEMM choices instead of the tuner (a bench line's
        "gemm_choices"): profiling passes re-run the configuration the timed run
        chose, so their counters belong to the same kernels."""
        import json
        L = nat.lib()
        e = self.runner.engine
        ch = json.load(open(path))
        for site, _ in self._gemm_sites():
            o = (ch.get(site) or {}).get("cfg")
            nat.check(L.pinsage_engine_set_gemm_choice(e.h, site.encode(), *(o if o else (-1, -1, 0))),
                      "set_gemm_choice")
        self.tuned_choices = {k: v for k, v in ch.items()}

    def _signature(self, feats, table):
        return (self.runner.flat.data_ptr(), self.grads.data_ptr(), self.m.data_ptr(),
                self.v.data_ptr(), feats.data_ptr(), table.nb32.data_ptr(), table.wn.data_ptr(),
                self.wss[0].data_ptr(), self.wss[1].data_ptr(), id(self.runner.engine))

    def _capture(self, B, sig):
        """Per workspace p: the frontier graph (stage this step's ids, frontier),
        the step graph (stage coefficients, layers ... Adam, publish), and the
        step graph whose branch stages the predicted next ids into workspace
        1-p and computes their frontier there.  The cyclic garbage collector is
        off while capturing (an engine finalised mid-capture once released HIP
        streams / events inside the capture and aborted the process; the C-ABI
        destroy is now capture-safe by itself, tests/test_gpu_trainer.py::
        test_engine_finalised_inside_a_capture, and this keeps unrelated
        finalisers out of the capture too)."""
        was = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            return self._capture_graphs(B, sig)
        finally:
            if was:
                gc.enable()

    def _capture_graphs(self, B, sig):
        # (PINSAGE_CAPTURE_MODE: torch.cuda.graph's capture_error_mode, "global"
        # by default; diagnostics of the forked-frontier capture)
        mode = os.environ.get("PINSAGE_CAPTURE_MODE", "global")

        def graph(g):
            return torch.cuda.graph(g, capture_error_mode=mode)
        adam = not self.dist
        staged = self.dist and self.dp_buckets  # DP: backward stage 1 in its own graph (g2)
        stage = 0 if staged else None
        # The look-ahead branch's stream is used once here, eagerly: torch's stream
        # pool creates a slot's HIP stream lazily, at its first use, and a stream
        # first created inside a capture -- then forking the engine's frontier
        # stream off it (PINSAGE_CSR_FORK) and joining it back -- sent
        # hipStreamEndCapture into unbounded recursion through its parallel
        # capture-stream lists (a stack overflow: the native backtrace is one
        # libamdhip64 frame repeated; tools/dbg/segv_bt.c).
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        split = self.ahead_mode == "split"
        if split:
            if self.side is None:
                self.side = torch.cuda.Stream()
            self.side.wait_stream(torch.cuda.current_stream())
            self.gfr = []
        graphs = []
        for p in (0, 1):
            gf, gm, ga, g2 = (torch.cuda.CUDAGraph() for _ in range(4))
            with graph(gf):
                self._stage(B, self.slot_ids, p, None)
                self._frontier(B, p)
            if split:  # the frontier alone: a linear graph, replayed on self.side
                gfr = torch.cuda.CUDAGraph()
                with graph(gfr):
                    self._frontier(B, p)
                self.gfr.append(gfr)
            with graph(gm):
                self._stage(B, 0, None, p)
                self._main(B, p, with_adam=adam, stage=stage)
                if not staged:
                    self._publish(p)
            if staged:
                with graph(g2):
                    e = self.runner.engine
                    nat.check(nat.lib().pinsage_engine_backward_stage(e.h, nat.ptr(self.wss[p]), 1,
                                                                      nat.stream_ptr()), "backward_stage")
                    self._publish(p)
            else:
                g2 = None
            with graph(ga):
                cur = torch.cuda.current_stream()

                def frontier_on_branch(q):
                    # the engine forks nothing off this branch (engine.hip
                    # frontier_fork_ok: a fork off a capture branch sent
                    # hipStreamEndCapture into unbounded recursion)
                    e = self.runner.engine
                    nat.check(nat.lib().pinsage_engine_set_frontier_fork(e.h, 0), "set_frontier_fork")
                    try:
                        self._frontier(B, q)
                    finally:
                        nat.lib().pinsage_engine_set_frontier_fork(e.h, 1)

                def fork_next_frontier():
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        frontier_on_branch(1 - p)

                # the next step's ids go to workspace 1-p, whose last user
                # (the previous step) is done: graph launches are stream-ordered
                # (split: _call stages them eagerly and forks the frontier)
                if not split:
                    self._stage(B, self.slot_next, 1 - p, p)
                if split:  # the step alone
                    self._main(B, p, with_adam=adam, stage=stage)
                elif self.ahead_mode == "late":
                    # forked at the start like "start", but captured after
                    # the main chain (the runtime dispatches a multi-stream
                    # graph's nodes in capture order)
                    fork_ev = torch.cuda.Event()
                    fork_ev.record(cur)
                    self._main(B, p, with_adam=adam, stage=stage)
                    side.wait_event(fork_ev)
                    with torch.cuda.stream(side):
                        frontier_on_branch(1 - p)
                elif self.ahead_mode == "start" or staged:
                    fork_next_frontier()
                    self._main(B, p, with_adam=adam, stage=stage)
                elif self.ahead_mode == "fwd":  # forked inside, after the layer-0 Q projection
                    side.wait_stream(cur)
                    e = self.runner.engine
                    nat.check(nat.lib().pinsage_engine_set_fork(
                        e.h, nat.ptr(self.wss[1 - p]), nat.ptr(self.ids_view[1 - p]), 3 * B,
                        ctypes.c_void_p(side.cuda_stream)), "set_fork")
                    try:
                        self._main(B, p, with_adam=adam)
                    finally:
                        nat.lib().pinsage_engine_set_fork(e.h, None, None, 0, None)
                else:  # beside the backward: a latency-bound chain with CUs to spare
                    self._main(B, p, with_adam=adam, before_backward=fork_next_frontier)
                if not split:
                    cur.wait_stream(side)
                if not staged:
                    self._publish(p)
            graphs.append((gf, gm, ga, g2))
        self.graphs = graphs
        self.graph_B = B
        self.graph_sig = sig
        self._make_stepper(B)

    # ---- the native per-step host path (pinsage_stepper_*)
    def _make_stepper(self, B):
        """After a capture: the host side of each step as one native call
        (ring slot wait, coefficients, ids / ahead check, graph launches) when
        the step is one stream's graphs (not data-parallel, not "split")."""
        self._drop_stepper(sync=False)
        if (self.dist or self.ahead_mode == "split" or os.environ.get("PINSAGE_NATIVE_STEP", "1") == "0"
                or not hasattr(torch.cuda.CUDAGraph, "raw_cuda_graph_exec")):
            return
        L = nat.lib()
        h = ctypes.c_void_p()
        nat.check(L.pinsage_stepper_create(nat.ptr(self.ring), self.HOST_RING, self.slot_bytes, self.slot_ids,
                                           self.slot_next, self.slot_coef, 3 * B,
                                           int(self.runner.engine.cfg.n_items), ctypes.byref(h)), "stepper_create")
        self.stepper = h
        for p, (gf, gm, ga, _) in enumerate(self.graphs):
            nat.check(L.pinsage_stepper_set_graphs(h, p, ctypes.c_void_p(gf.raw_cuda_graph_exec()),
                                                   ctypes.c_void_p(gm.raw_cuda_graph_exec()),
                                                   ctypes.c_void_p(ga.raw_cuda_graph_exec())), "stepper_set_graphs")
        # (called at the end of a capture, inside the eager step self.nstep: the
        # native path takes over from the next step, with every ring slot free)
        torch.cuda.current_stream().synchronize()
        nat.check(L.pinsage_stepper_sync_state(h, self.parity, self.nstep + 1), "stepper_sync_state")
        self._coef_np = np.zeros(2, np.float32)
        self._info = (ctypes.c_int64 * 2)()

    def _drop_stepper(self, sync=True):
        st = getattr(self, "stepper", None)
        if st is None:
            return
        if sync:  # its ring slots may still be read by launched steps
            torch.cuda.current_stream().synchronize()
        self.wait_s += nat.lib().pinsage_stepper_wait_ns(st) * 1e-9
        nat.lib().pinsage_stepper_destroy(st)
        self.stepper = None

    def _call_native(self, batch, B):
        """One captured step through pinsage_stepper_step (the graph path of
        _call below, in C)."""
        b = batch.numpy() if batch.device.type == "cpu" else batch.cpu().numpy()
        if b.dtype != np.int64 or not b.flags.c_contiguous:
            b = np.ascontiguousarray(b, dtype=np.int64)
        self._coef_np[:] = self._adam_coef(self.host_step + 1)
        nxt = self._predicted(B)
        if nxt is not None and (nxt.dtype != np.int64 or not nxt.flags.c_contiguous):
            nxt = np.ascontiguousarray(nxt, dtype=np.int64)
        _tick("peek")
        rc = nat.lib().pinsage_stepper_step(self.stepper, b.ctypes.data_as(nat.vp), 3 * B,
                                            self._coef_np.ctypes.data_as(nat.vp),
                                            nxt.ctypes.data_as(nat.vp) if nxt is not None else None,
                                            nat.stream_ptr(), self._info)
        if rc == -5:
            raise IndexError(f"batch ids out of range for {int(self.runner.engine.cfg.n_items)} items")
        nat.check(rc, "stepper_step")
        self.ahead_hits += int(self._info[0])
        self.parity ^= 1
        out = self.out_ring[self.nstep % self.OUT_RING]
        self.nstep += 1
        self.host_step += 1
        _tick("replay")
        return out[0], out[1], out[3]

    def _predicted(self, B):
        """This rank's slice of the batch the sampler drew ahead, or None."""
        if not self.ahead:
            return None
        rank, world = self.tr._dp()
        nxt = _PREFETCH.peek(self.tr.batch_size * world)
        if nxt is None or nxt.shape[0] != B * world:
            return None
        return nxt[rank * B:(rank + 1) * B]

    def __call__(self, batch):
        """One train step; for the caller it is optimizer.step(): the step's
        Adam update runs inside the graph, and around it the optimizer's (and
        the global) step pre- / post-hooks fire and torch's bookkeeping advances
        (``_opt_called``, so an LR scheduler sees optimizer.step() before its own
        step, as in pinsage_training.py:188-191, 256)."""
        from itertools import chain
        import torch.optim.optimizer as _topt
        opt = self.tr.optimizer
        pre = list(chain(_topt._global_optimizer_pre_hooks.values(), opt._optimizer_step_pre_hooks.values()))
        for hook in pre:
            if hook(opt, (opt,), {}) is not None:
                raise RuntimeError("the fused train step cannot apply an optimizer pre-hook's new arguments")
        if _HOST_T is not None:
            t0 = time.perf_counter()
            out = self._call(batch)
            _HOST_T["call"] = _HOST_T.get("call", 0.0) + time.perf_counter() - t0
        else:
            out = self._call(batch)
        opt._opt_called = True
        for hook in chain(opt._optimizer_step_post_hooks.values(), _topt._global_optimizer_post_hooks.values()):
            hook(opt, (opt,), {})
        return out

    def _call(self, batch):
        tr = self.tr
        batch = torch.as_tensor(batch)
        B = int(batch.shape[0])
        self.ensure(B)
        r = self.runner
        feats = r.features(tr.features)
        table = r.table(tr.nbhds)
        self.B_cur = B
        sig = self._signature(feats, table)
        if self.graphs is not None and (self.graph_B != B or self.graph_sig != sig or not self.use_graph):
            self.graphs = None  # buffers moved: the captured pointers are stale
            self._drop_stepper()
        if self.graphs is not None and getattr(self, "stepper", None) is not None:
            self.ws = self.wss[self.parity]
            # (the planes the graphs read: re-split in place if the features were
            # written in place since; a moved tensor changed the signature above)
            r.feature_planes(feats)
            r.feature_ilv(feats)
            _tick("pre")
            return self._call_native(batch, B)  # (the captured graphs hold every pointer: no bind)
        r.bind(feats, table, grads=self.grads, adam_m=self.m, adam_v=self.v)
        p = self.parity
        self.parity ^= 1
        self.ws = self.wss[p]
        _tick("pre")
        k = self.nstep % self.HOST_RING
        if self.ring_ev[k] is not None:  # the step that used this slot is done
            tw = time.perf_counter()
            self.ring_ev[k].synchronize()
            self.wait_s += time.perf_counter() - tw
        self._slot_write_coef(k)
        _tick("slot_wait")
        staged = self.dist and self.dp_buckets
        staged_done = False  # the eager path below runs its own staged tail
        join = None  # split look-ahead: the side stream's frontier
        if self.graphs is not None:
            gf, gm, ga, g2 = self.graphs[p]
            pend = self.pending[p]
            if pend is not None and np.array_equal(pend, batch.reshape(B, 3).cpu().numpy()):
                self.ahead_hits += 1
            else:
                self._slot_write_ids(k, self.slot_ids, batch, B)
                gf.replay()
            self.pending[p] = None
            nxt = self._predicted(B)
            _tick("peek")
            if nxt is not None:
                self._slot_write_ids(k, self.slot_next, nxt, B)
                if self.ahead_mode == "split":
                    # stage (next ids -> workspace 1-p, coefficients -> p),
                    # then the step's graph here and the next frontier's on
                    # the side stream; the next step waits for the latter
                    cur = torch.cuda.current_stream()
                    self._stage(B, self.slot_next, 1 - p, p)
                    fork = torch.cuda.Event()
                    fork.record(cur)
                    ga.replay()
                    self.side.wait_event(fork)
                    with torch.cuda.stream(self.side):
                        self.gfr[1 - p].replay()
                    join = torch.cuda.Event()
                    join.record(self.side)
                else:
                    ga.replay()
            else:
                gm.replay()
            self.pending[1 - p] = nxt
            _tick("replay")
        else:
            self._slot_write_ids(k, self.slot_ids, batch, B)
            self._stage(B, self.slot_ids, p, p)
            self._frontier(B, p)
            if self.autotune and self.tuned_choices is None:
                # the size hints come from this batch's frontier, then the
                # tuner's probes; the step itself runs after them
                if not self._tuned:
                    self.runner.engine.tune(self.wss[p])
                    self._tuned = True
                if os.environ.get("PINSAGE_GEMM_CHOICES"):
                    self._load_choices(os.environ["PINSAGE_GEMM_CHOICES"])
                else:
                    self._autotune(B, p)
                # the probes' backward scatter-added into this frontier's dY
                # targets, which only the frontier (layer_prep) zeroes: redo it
                self._frontier(B, p)
            self._main(B, p, with_adam=not self.dist, stage=0 if staged else None)
            if staged:
                self._dp_tail(p, None)
            else:
                self._publish(p)
            self.pending = [None, None]
            if self.use_graph and self._tuned:
                self._capture(B, sig)
            g2 = None
            staged_done = staged
        if self.dist and staged and not staged_done:
            self._dp_tail(p, g2)
        elif self.dist and not staged:
            average_gradients(self.grads)
            self._adam(p)
        if join is not None:  # the next step reads the look-ahead frontier
            torch.cuda.current_stream().wait_event(join)
        ev = torch.cuda.Event()
        ev.record()
        self.ring_ev[k] = ev
        out = self.out_ring[self.nstep % self.OUT_RING]
        self.nstep += 1
        self.host_step += 1
        _tick("tail")
        return out[0], out[1], out[3]


class _FusedFlyStep(_FusedStep):
    """The train step of an on-the-fly model (relevant_nodes_per_layer,
    pinsage_model.py:142-154; Philox draws) as ONE captured graph: stage the
    batch, Adam coefficients and the calls' walk keys from the host ring slot
    the device counter picks; sample every layer of the three calls on the
    device (pinsage_fly_sample: walks, top-T, next nodesets, virtual nodes for
    ids repeated inside a call -- the tables of _fly_tables_merged, bitwise);
    frontier, layers, loss (virtual nodes get their id's summed output
    gradient: pinsage_engine_set_fly), backward + Adam, publish.  The host's
    part of a step: the batch (native sampler), the 2 C L key words from
    torch's generator (where the per-call path draws them), one graph launch.

    A zero-degree node met by a walk, or a drawn id >= n_items, is reported
    through the ring slot and raised when the host next waits for that slot
    (up to HOST_RING steps late; the per-call path raises at the draw), or
    at the latest when the optimizer state is synchronised (save_model, the
    end of train(): sync_optimizer_step checks every outstanding slot).  The
    device refuses the optimizer update of that step and of every later one
    until the host has raised (pinsage_fly_gate_adam: a sticky halt word), so
    the parameters are the ones the reference holds when it raises."""

    def __init__(self, trainer):
        super().__init__(trainer)
        self.ahead = False
        self.ahead_mode = "0"
        self.autotune = False
        self.fd = None

    def ensure(self, B):
        super().ensure(B)
        m = self.tr.model
        feats = self.runner.features(self.tr.features)
        fkey = (id(feats), feats.data_ptr())
        if self.fd is None or self.fd.B != B or getattr(self, "_fkey", None) != fkey:
            self.fd = pm_fly_device(m, B, feats, self.dev)
            self._fkey = fkey
            self.graphs = None
            self._fly_ring = None
        if getattr(self, "_fly_ring", None) is not self.ring:  # (super().ensure may have rebuilt it)
            self.graphs = None
            L = int(m.n_layers)
            mp = int(self.runner.engine.cfg.max_pos)
            # slot: [ids | Adam coefficients | walk keys | error words]
            self.slot_ids, self.slot_coef = 0, mp * 8
            self.slot_seeds = self.slot_coef + 16
            self.slot_err = self.slot_seeds + 3 * L * 8
            self.slot_bytes = self.slot_err + 8
            self.ring = torch.zeros((self.HOST_RING, self.slot_bytes), dtype=torch.uint8).pin_memory()
            self.ring_ev = [None] * self.HOST_RING
            for k in range(self.HOST_RING):
                self.ring[k, self.slot_err:self.slot_err + 8].view(torch.int32)[0] = 0x7f7f7f7f
            self._fly_ring = self.ring

    def _slot_write_ids(self, k, off, batch, B):
        ids = self.ring[k, off:off + 3 * B * 8].view(torch.int64)
        ids.copy_(torch.as_tensor(batch).reshape(-1).to(torch.int64))
        n_valid = min(int(self.tr.model.n_items), int(self.fd.feats.shape[0]))
        if int(ids.min()) < 0 or int(ids.max()) >= n_valid:
            raise IndexError(f"node ids out of range for {n_valid} items")

    def _check_slot(self, k):
        e = self.ring[k, self.slot_err:self.slot_err + 8].view(torch.int32).tolist()
        self.ring[k, self.slot_err:self.slot_err + 8].view(torch.int32)[0] = 0x7f7f7f7f
        self.ring[k, self.slot_err:self.slot_err + 8].view(torch.int32)[1] = 0
        if e[0] != 0x7f7f7f7f or e[1]:
            # raising now: the steps after the failed one (already enqueued)
            # stay refused; steps enqueued from here on update again
            self.fd.err[2:3].zero_()
        if e[0] != 0x7f7f7f7f:
            raise RuntimeError("walk: zero-degree node met (the reference's torch.randint(0) raises here)")
        if e[1]:
            raise IndexError("sampled neighbourhood reaches ids >= n_items (collection ids in the "
                             "zero-weight tail: the reference's h[nb] raises IndexError)")

    def check_outstanding(self):
        """Wait for every step whose error words the host has not read yet and
        raise the first failure among them (in step order)."""
        R = self.HOST_RING
        for i in range(max(0, self.nstep - R), self.nstep):
            k = i % R
            ev = self.ring_ev[k]
            if ev is None:
                continue
            ev.synchronize()
            self.ring_ev[k] = None
            self._check_slot(k)

    def sync_optimizer_step(self):
        self.check_outstanding()
        super().sync_optimizer_step()

    def _fly_seq(self, B):
        """One step's device work (the captured graph's contents)."""
        L = nat.lib()
        e = self.runner.engine
        fd = self.fd
        st = nat.stream_ptr()
        ws = self.wss[0]
        coef = ctypes.c_void_p(self.stage_view[0].data_ptr() + 3 * B * 8)
        nat.check(L.pinsage_step_stage(nat.ptr(self.ring), self.slot_bytes, self.HOST_RING, nat.ptr(self.ctr),
                                       self.slot_ids, 3 * B * 8, nat.ptr(fd.batch_dev), self.slot_coef, coef, st),
                  "step_stage")
        nat.check(L.pinsage_step_stage(nat.ptr(self.ring), self.slot_bytes, self.HOST_RING, nat.ptr(self.ctr),
                                       self.slot_seeds, fd.seeds.numel() * 8, nat.ptr(fd.seeds), 0, None, st),
                  "step_stage")
        fd.sample(fd.batch_dev, pos_out=self.ids_view[0])
        # a failed sampling refuses this step's Adam update (and later ones)
        nat.check(L.pinsage_fly_gate_adam(nat.ptr(fd.err), coef, st), "fly_gate_adam")
        nat.check(L.pinsage_engine_frontier(e.h, nat.ptr(ws), nat.ptr(self.ids_view[0]), 3 * B, st), "frontier")
        nat.check(L.pinsage_engine_forward_layers(e.h, nat.ptr(ws), st), "forward_layers")
        nat.check(L.pinsage_engine_loss(e.h, nat.ptr(ws), B, float(self.tr.margin), 1, st), "loss")
        if not self._tuned:  # once: frontier sizes of a real batch pick the GEMM tiles
            e.tune(ws)
            self._tuned = True
        self._backward(0, True)
        nat.check(L.pinsage_fly_publish_err(nat.ptr(fd.err), nat.ptr(self.ring), self.slot_bytes, self.HOST_RING,
                                            nat.ptr(self.ctr), self.slot_err, st), "fly_publish_err")
        self._publish(0)

    def _bind_fly(self, on):
        r = self.runner
        e = r.engine
        fd = self.fd
        if on:
            r.bind(fd.fx, None, grads=self.grads, adam_m=self.m, adam_v=self.v, tabs=fd.tabs)
            r.set_layer_tables(fd.tabs)
            nat.check(nat.lib().pinsage_engine_set_fly(e.h, 3 * fd.n, nat.ptr(fd.n_x), nat.ptr(fd.ids_xo), fd.n,
                                                       fd.x_cap), "engine_set_fly")
        else:
            r.set_layer_tables(None)
            nat.lib().pinsage_engine_set_fly(e.h, 0, None, None, 1, 0)

    def _call(self, batch):
        batch = torch.as_tensor(batch)
        B = int(batch.shape[0])
        self.ensure(B)
        self.B_cur = B
        k = self.nstep % self.HOST_RING
        if self.ring_ev[k] is not None:  # the step that used this slot is done
            tw = time.perf_counter()
            self.ring_ev[k].synchronize()
            self.wait_s += time.perf_counter() - tw
            self._check_slot(k)
        self._slot_write_ids(k, self.slot_ids, batch, B)
        self._slot_write_coef(k)
        L = int(self.tr.model.n_layers)
        self.ring[k, self.slot_seeds:self.slot_seeds + 3 * L * 8].view(torch.int64).copy_(
            torch.from_numpy(pm_fly_seed_words(L)))
        sig = (B, id(self.fd), id(self.runner.engine))
        if self.graphs is not None and (self.graph_sig != sig or not self.use_graph):
            self.graphs = None
        if self.graphs is not None:
            self.graphs.replay()
        else:
            self._bind_fly(True)
            try:
                if self._tuned and self.use_graph:  # hints set: capture, then replay for this step
                    was = gc.isenabled()
                    gc.collect()
                    gc.disable()
                    try:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g):
                            self._fly_seq(B)
                    finally:
                        if was:
                            gc.enable()
                    self.graphs = g
                    self.graph_sig = sig
                    g.replay()
                else:
                    self._fly_seq(B)
            finally:
                self._bind_fly(False)
        ev = torch.cuda.Event()
        ev.record()
        self.ring_ev[k] = ev
        out = self.out_ring[self.nstep % self.OUT_RING]
        self.nstep += 1
        self.host_step += 1
        return out[0], out[1], out[3]


def pm_fly_device(model, B, feats, dev):
    import pinsage_model as pm
    return pm._FlyDevice(model, B, feats, dev)


def pm_fly_seed_words(L):
    import pinsage_model as pm
    return pm._fly_seed_words(L)


class PinSage:
    """The PinSage trainer (pinsage_training.py:108-295): same attributes,
    defaults and file formats; hyperparameters are bound at construction
    (T, n_layers, dims, lr, decay) exactly as in the reference."""

    def __init__(self, g, n_items, features, positives, log=True, load_save=True, nbhds=None):
        """``nbhds`` (an extension, default None = the reference's behaviour):
        a neighbourhood table to use instead of precompute_neighborhoods_topt,
        e.g. pinsage_model.precompute_device_table's device-resident one."""
        self.run_name = "pinsage_randomft_intersect"
        self.precomp_path = g.nbhds_path

        self.g = g
        self.n = n_items
        self.all_ids = torch.arange(0, n_items, 1, dtype=torch.int64)
        self.features = features
        self.positives = positives

        self.n_layers = 2
        self.in_dim = features.shape[1]
        self.hidden_dim = 512
        self.out_dim = 128
        self.dimensions = (self.in_dim, self.hidden_dim, self.out_dim)
        self.n_hops = 500
        self.alpha = 0.85
        self.T = 3
        self.hard_negatives = False
        self.hn_min = 10
        self.hn_max = 100

        self.nbhds = nbhds if nbhds is not None else psm.precompute_neighborhoods_topt(
            self.g, self.n, self.n_hops, self.alpha, psm.DEF_T_PRECOMP, self.precomp_path)
        self.model = psm.PinSageModel(self.g, self.n, self.n_layers, self.dimensions, self.n_hops,
                                      self.alpha, self.T, self.nbhds)
        self.lr = 1e-4
        self.decay = 0.95
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=self.lr)
        self.scheduler = torch.optim.lr_scheduler.ExponentialLR(self.optimizer, self.decay)
        self.margin = 1e-5
        self.epochs = 30
        self.batch_size = 128
        self.b_per_e = 500

        self.embeddings = None
        run_dir = os.path.join(BASE_RUN_DIR, self.run_name)
        os.makedirs(os.path.join(run_dir, "board"), exist_ok=True)
        self.e = 0
        self.b = 0

        self.log = log
        if self.log:
            try:
                import wandb
                wandb.config = {"learning_rate": self.lr, "epochs": self.epochs,
                                "batch_size": self.batch_size}
                wandb.init(project='gcn-song-embeddings', name=self.run_name)
                wandb.watch(self.model, log="all", log_freq=10, log_graph=True)
                self._wandb = wandb
            except Exception as ex:  # no network / not installed: keep training
                print(f"wandb unavailable ({ex}); logging disabled")
                self.log = False
        self._fused = None
        # micro-batched step (an extension): None = one fused step over the whole
        # batch; k = the batch in slices of k triples with recompute (see
        # _train_batch_micro), for frontiers that do not fit one workspace
        self.micro_batch = None
        self.load_save = load_save
        if self.load_save:
            self.load_model()

    # ---- the train step
    def _dp(self):
        d = torch.distributed
        if d.is_available() and d.is_initialized():
            return d.get_rank(), d.get_world_size()
        return 0, 1

    def _average_param_grads(self):
        """Data parallel: every rank's parameter gradients become their mean over
        the process group (ONE all-reduce of the flattened gradients), so the
        replicas take the same optimizer step."""
        rank, world = self._dp()
        if world <= 1:
            return
        params = [p for p in self.model.parameters() if p.grad is not None]
        flat_g = average_gradients(torch.cat([p.grad.reshape(-1) for p in params]))
        off = 0
        for p in params:
            p.grad.copy_(flat_g[off:off + p.numel()].view(p.shape))
            off += p.numel()

    def next_batch(self):
        """Sample this rank's slice of the global batch (same draws on every rank)."""
        rank, world = self._dp()
        batch, nodeset = sample_batch(self.all_ids, self.positives, self.batch_size * world, self.nbhds,
                                      hard_negatives=self.hard_negatives, hn_min=self.hn_min,
                                      hn_max=self.hn_max)
        if world > 1:
            B = batch.shape[0] // world
            batch = batch[rank * B:(rank + 1) * B]
            nodeset = batch.flatten().unique()
        return batch, nodeset

    def train_batch(self, batch):
        """Fetch and train one batch of (q, pos, neg) triples: returns
        (loss, node_feat_loss, variance) as device scalars (no host sync)."""
        if self.model.sample_on_the_fly:
            return self._train_batch_fly(batch)
        if self.micro_batch and int(torch.as_tensor(batch).shape[0]) > int(self.micro_batch):
            return self._train_batch_micro(batch)
        if self._fused is None:
            self._fused = _FusedStep(self)
        return self._fused(batch)

    def _fly_fused_ok(self, batch):
        """Whether the on-the-fly step runs as the captured device step
        (_FusedFlyStep): Philox draws with the merged calls, no model hooks,
        one process, the fused sampler's regime; PINSAGE_FLY_FUSED=0 keeps the
        host-orchestrated path."""
        import pinsage_model as pm
        from torch.nn.modules import module as _nnm
        model = self.model
        if (os.environ.get("PINSAGE_FLY_FUSED", "1") == "0" or pm.get_rng_mode() == "mt19937"
                or os.environ.get("PINSAGE_FLY_MERGE", "1") == "0" or self._dp()[1] > 1):
            return False
        if (model._forward_pre_hooks or model._forward_hooks or model._forward_hooks_with_kwargs
                or model._forward_hooks_always_called or model._backward_hooks or model._backward_pre_hooks
                or _nnm._global_forward_hooks or _nnm._global_forward_pre_hooks or _nnm._global_backward_hooks
                or _nnm._global_backward_pre_hooks):
            return False
        n_all = pm._as_csr(model.g).number_of_nodes()
        T, h = int(model.T), int(model.n_hops)
        return (torch.as_tensor(batch).dim() == 2 and int(torch.as_tensor(batch).shape[0]) >= 2 and T * 64 <= n_all
                and h <= 8192 and h + T < 65536)

    def _train_batch_fly(self, batch):
        """The reference's train_batch (pinsage_training.py:181-215) step for
        step when the model samples on the fly (relevant_nodes_per_layer,
        pinsage_model.py:142-154): three model calls -- each walks its own
        nodeset's neighbourhoods, in the order q, pos, neg, consuming torch's
        generator as the reference does -- max_margin_loss, the engine's HIP
        backward per call (autograd), torch's Adam."""
        batch = torch.as_tensor(batch)
        if self._fly_fused_ok(batch):
            if getattr(self, "_fused_fly", None) is None:
                self._fused_fly = _FusedFlyStep(self)
            return self._fused_fly(batch)
        model = self.model
        from torch.nn.modules import module as _nnm
        if (model._forward_pre_hooks or model._forward_hooks_with_kwargs or model._forward_hooks_always_called
                or model._backward_hooks or model._backward_pre_hooks or _nnm._global_forward_hooks
                or _nnm._global_forward_pre_hooks or _nnm._global_backward_hooks
                or _nnm._global_backward_pre_hooks):
            # hooks the merged call cannot replay per call (pre-hooks, global
            # and backward hooks): the reference's three model calls
            h_q = model(self.features, batch[:, 0])
            h_pos = model(self.features, batch[:, 1])
            h_neg = model(self.features, batch[:, 2])
        else:
            # the three calls' draws in the reference's order, then one engine
            # call for all of them (pinsage_model._EngineRunner.fly_calls); a
            # caller's forward hooks see each call as model(features, ids)
            calls = [batch[:, 0], batch[:, 1], batch[:, 2]]
            outs = model.runner().fly_calls(self.features, calls)
            for c, ids in enumerate(calls):
                for hook in list(model._forward_hooks.values()):
                    r = hook(model, (self.features, ids), outs[c])
                    if r is not None:
                        outs[c] = r
            h_q, h_pos, h_neg = outs
        loss = max_margin_loss(h_q, h_pos, h_neg, self.margin)
        self.optimizer.zero_grad()
        loss.backward()
        self._average_param_grads()
        self.optimizer.step()
        norm = torch.nn.functional.normalize
        f = self.features
        node_feat_loss = COSINE_TRIPLET_LOSS(norm(f[batch[:, 0]], dim=1), norm(f[batch[:, 1]], dim=1),
                                             norm(f[batch[:, 2]], dim=1))
        variance = batch_variance(h_q)
        return loss, node_feat_loss, variance

    def _train_batch_micro(self, batch):
        """The reference train step (pinsage_training.py:181-215) over slices of
        ``micro_batch`` triples, for frontiers too large for one workspace
        (3 layers at fanout 50 reach ~10^6 nodes at layer 0 per 512 triples).

        Every output row depends only on its own node's subtree, so:
        1. forward each slice (outputs only; nothing kept);
        2. the loss over the whole batch and its cotangent on every output row;
           with index_put's semantics (pinsage_model.py:257-265) a call's
           repeated id gets K x (its rows' summed cotangent), summed over the
           three calls into one cotangent per distinct id;
        3. per slice, forward again with activations and run the HIP backward
           with the cotangents of the ids this slice is the first to hold (each
           distinct id's cotangent enters exactly once); parameter gradients add
           up over slices as they would inside one backward.
        Then torch's Adam.  Costs one extra forward per step."""
        model = self.model
        dev = model.runner().dev
        out = model.out_dim
        batch = torch.as_tensor(batch).to(torch.int64)
        B = int(batch.shape[0])
        ids = batch.t().contiguous().to(dev)  # [3, B]: the q, pos and neg calls
        Z = self._micro_forward(ids)
        self.last_outputs = Z  # [3, B, out] rows the loss read (tests pin them)
        loss, g, variance = _triplet_loss(Z, self.margin)
        self._micro_backward(ids, g)
        self._average_param_grads()
        self.optimizer.step()
        norm = torch.nn.functional.normalize
        f = self.features
        bq = batch.to(f.device)
        node_feat_loss = COSINE_TRIPLET_LOSS(norm(f[bq[:, 0]], dim=1), norm(f[bq[:, 1]], dim=1),
                                             norm(f[bq[:, 2]], dim=1))
        if variance is None:
            variance = batch_variance(Z[0])
        return loss.detach(), node_feat_loss, variance

    def _micro_forward(self, ids):
        """Outputs [3, B, out] of the three calls over ids [3, B], slice by slice
        (nothing kept)."""
        m = int(self.micro_batch)
        model = self.model
        B = int(ids.shape[1])
        Z = torch.empty((3, B, model.out_dim), dtype=torch.float32, device=ids.device)
        with torch.no_grad():
            for j in range(0, B, m):
                part = ids[:, j:j + m]
                Z[:, j:j + m] = model(self.features, part.reshape(-1)).view(3, -1, model.out_dim)
        return Z

    def _micro_backward(self, ids, g):
        """Parameter gradients of the three calls over ids [3, B] under the
        cotangent g [3, B, out] of their outputs, slice by slice with recompute:
        a call's repeated id gets K x (its rows' summed cotangent) (index_put,
        pinsage_model.py:257-265), summed over the calls into one cotangent per
        distinct id, which enters with the first slice holding that id."""
        m = int(self.micro_batch)
        model = self.model
        runner = model.runner()
        dev = runner.dev
        out = model.out_dim
        B = int(ids.shape[1])
        n = int(self.n)
        g = g.reshape(3 * B, out)
        flat = ids.reshape(-1)
        call = torch.arange(3, device=dev).repeat_interleave(B)
        uk, inv = torch.unique(call * n + flat, return_inverse=True)
        G = torch.zeros((uk.shape[0], out), dtype=torch.float32, device=dev).index_add_(0, inv, g)
        K = torch.bincount(inv, minlength=uk.shape[0]).to(torch.float32)
        uv, inv2 = torch.unique(uk % n, return_inverse=True)
        D = torch.zeros((uv.shape[0], out), dtype=torch.float32, device=dev).index_add_(0, inv2, K[:, None] * G)
        slot = torch.searchsorted(uv, flat)
        first = torch.full((uv.shape[0],), B, dtype=torch.int64, device=dev)
        first.scatter_reduce_(0, slot, torch.arange(B, device=dev).repeat(3) // m, reduce="amin")
        params = runner.params()
        for p in params:
            p.grad = None
        for j in range(0, B, m):
            u = torch.unique(ids[:, j:j + m])
            su = torch.searchsorted(uv, u)
            d = torch.where((first[su] == j // m)[:, None], D[su], torch.zeros((), device=dev))
            y = model(self.features, u)
            torch.autograd.backward([y], [d])

    def train(self):
        from tqdm import tqdm
        print("\033[0;33mTraining PinSage...\033[0m")
        while self.e < self.epochs:
            print(f"Training epoch {self.e+1}/{self.epochs}...")
            cur_lr = self.optimizer.param_groups[0]["lr"]
            t1 = time.time()
            pbar = tqdm(total=self.b_per_e)
            pbar.update(1)
            while self.b < self.b_per_e:
                batch, nodeset = self.next_batch()
                loss, node_feat_loss, variance = self.train_batch(batch)
                pbar.update(1)
                if self.b % 50 == 0 or self.b == self.b_per_e - 1:
                    pbar.set_description(f"Loss = {float(loss)}, bathes done")
                if self.log:
                    self._wandb.log({'Train Loss': float(loss), 'Node Features Loss': float(node_feat_loss),
                                     'Batch Variance': float(variance), 'Learning Rate': cur_lr})
                if self.load_save:
                    self.save_model()
                self.b += 1
            print(f"{time.time() - t1}s elapsed.")
            pbar.close()
            self.b = 0
            self.e += 1
            self.scheduler.step()
        # the fused step's optimizer bookkeeping (and, sampling on the fly, the
        # error words of its last steps) before control returns to the caller
        self._sync_state()

    def embed(self, ids=None, bsize=None):
        """Node embeddings, optionally in bsize batches (pinsage_training.py:258-275,
        including its reset of ``ids`` to a range in the batched branch)."""
        if ids is None:
            ids = self.all_ids
        self.model.eval()
        n = len(ids)
        with torch.no_grad():
            if not bsize:
                self.embeddings = self.model(self.features, ids)
            else:
                self.embeddings = torch.zeros((n, self.out_dim))
                for i in range(0, n, bsize):
                    ids = torch.arange(i, min(i + bsize, n))
                    self.embeddings[ids, :] = self.model(self.features, ids).to(self.embeddings.device)
        return self.embeddings

    def _sync_state(self):
        for f in (self._fused, getattr(self, "_fused_fly", None)):
            if f is not None:
                f.sync_optimizer_step()

    def load_model(self):
        load_path = os.path.join(BASE_RUN_DIR, self.run_name, "state.pt")
        if os.path.isfile(load_path):
            prog = torch.load(load_path, map_location="cpu", weights_only=True)
            self.e = prog["epochs_done"]
            self.b = prog["batches_done"]
            self.model.load_state_dict(prog["model_state"])
            self.optimizer.load_state_dict(prog["optimizer_state"])
            if self._fused is not None and self._fused.grads is not None:
                self._fused.adopt_optimizer_state()
            print(f"Loaded existing model from {load_path}.")

    def save_model(self):
        self._sync_state()
        opt_sd = self.optimizer.state_dict()
        opt_sd = {"state": {k: {kk: (vv.detach().cpu().clone() if torch.is_tensor(vv) else vv)
                                for kk, vv in v.items()} for k, v in opt_sd["state"].items()},
                  "param_groups": opt_sd["param_groups"]}
        prog = {
            "epochs_done": self.e,
            "batches_done": self.b,
            "model_state": {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()},
            "optimizer_state": opt_sd,
        }
        torch.save(prog, os.path.join(BASE_RUN_DIR, self.run_name, "state.pt"))


def save_embeddings(trainer, dataset, base_run_dir=BASE_RUN_DIR, override_run_name=None):
    """One ``<track_id>.pt`` per track, skipping existing files
    (pinsage_training.py:297-327)."""
    track_ids = list(dataset.tracks)
    n = len(track_ids)
    bsize = 256
    run_name = override_run_name if override_run_name else trainer.run_name
    emb_dir = os.path.join(base_run_dir, run_name, "emb")
    os.makedirs(emb_dir, exist_ok=True)
    for i in range(0, n, bsize):
        ids = torch.arange(i, min(i + bsize, n))
        emb = trainer.embed(ids).detach().cpu()
        for j, tid in enumerate(ids.tolist()):
            save_path = os.path.join(emb_dir, track_ids[tid] + ".pt")
            if os.path.isfile(save_path):
                continue
            torch.save(emb[j, :].clone(), save_path)


def save_embeddings_tensor(trainer, dataset, base_run_dir=BASE_RUN_DIR, override_run_name=None,
                           bsize=1 << 16):
    """The embeddings of every track as ONE file (an extension beside the
    reference's per-track files): ``runs/<run>/emb.pt``
    holds ``{"ids": [track ids in dataset order], "emb": f32 [n, out]}``, the
    rows save_embeddings writes one file each, computed in ``bsize`` batches
    on the device.  Returns the path."""
    track_ids = list(dataset.tracks)
    n = len(track_ids)
    run_name = override_run_name if override_run_name else trainer.run_name
    run_dir = os.path.join(base_run_dir, run_name)
    os.makedirs(run_dir, exist_ok=True)
    emb = torch.empty((n, trainer.out_dim), dtype=torch.float32)
    trainer.model.eval()
    with torch.no_grad():
        for i in range(0, n, bsize):
            ids = torch.arange(i, min(i + bsize, n))
            emb[i:i + ids.shape[0]] = trainer.model(trainer.features, ids).cpu()
    path = os.path.join(run_dir, "emb.pt")
    torch.save({"ids": track_ids, "emb": emb}, path)
    return path


def load_embeddings_tensor(trainer, dataset=None, base_run_dir=BASE_RUN_DIR):
    """(ids, emb) of save_embeddings_tensor's file; rows reordered to
    ``dataset.tracks`` when a dataset is given."""
    d = torch.load(os.path.join(base_run_dir, trainer.run_name, "emb.pt"), weights_only=True)
    ids, emb = d["ids"], d["emb"]
    if dataset is not None:
        pos = {t: i for i, t in enumerate(ids)}
        order = torch.tensor([pos[t] for t in dataset.tracks], dtype=torch.int64)
        ids, emb = list(dataset.tracks), emb[order]
    return ids, emb


def load_embeddings(trainer, dataset, base_run_dir=BASE_RUN_DIR):
    emb_dir = os.path.join(base_run_dir, trainer.run_name, "emb")
    return torch.stack([torch.load(os.path.join(emb_dir, t + ".pt"), weights_only=True)
                        for t in dataset.tracks], dim=0)
