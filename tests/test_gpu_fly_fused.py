"""The on-the-fly step on the device (fly.hip: pinsage_fly_sample, and the
captured fused on-the-fly step of pinsage_training): relevant_nodes_per_layer
(pinsage_model.py:142-154) for the train step's three calls with every size
on the device.  Its per-layer tables, virtual nodes and engine positions are
bitwise those of the host-orchestrated merged path (_fly_tables_merged, whose
draws test_gpu_fly.py pins against the per-call walks and the oracle)."""
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, D_IN = 3000, 128


def _problem(tmp):
    import graph
    import synthetic
    pg = synthetic.make_playlist_graph(N, 750, 40000, seed=51)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(N, D_IN, seed=52))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * N, seed=53))
    return pg, g, feats, pos


def _batch(B, seed):
    rng = np.random.default_rng(seed)
    b = np.stack([rng.integers(0, N, B) for _ in range(3)], 1).astype(np.int64)
    b[3, 0] = b[10, 0] = b[20, 0]  # three occurrences in the query call
    b[7, 1] = b[8, 1]
    b[30, 2] = b[0, 0]  # (across calls: independent draws anyway)
    return torch.from_numpy(b)


@pytest.mark.parametrize("L,T,B", [(2, 5, 96), (2, 10, 64), (3, 3, 40), (1, 10, 32)])
def test_device_sampler_matches_merged_tables(L, T, B):
    import pinsage_model as pm
    pm.set_rng_mode("philox")
    try:
        with tempfile.TemporaryDirectory() as tmp:
            pg, g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            m = pm.PinSageModel(g, N, L, (D_IN, 512, 128), 200, 0.85, T, None)
            batch = _batch(B, L * 100 + T)
            ids_c = [batch[:, c].cuda() for c in range(3)]
            torch.manual_seed(99)
            tabs, uniq, inv, ids_x, ui_x = pm._fly_tables_merged(g, N, ids_c, L, 200, 0.85, T)
            st_ref = torch.get_rng_state()
            torch.manual_seed(99)
            keys = pm._fly_seed_words(L)
            assert torch.equal(torch.get_rng_state(), st_ref)
            fd = pm._FlyDevice(m, B, feats.cuda(), torch.device("cuda"))
            fd.seeds.copy_(torch.from_numpy(keys))
            bdev = batch.cuda()
            fd.sample(bdev)
            torch.cuda.synchronize()
            fd.check_err()
            n_x = int(fd.n_x.item())
            assert n_x == int(ids_x.shape[0]) and n_x >= 3
            assert torch.equal(fd.ids_xo[:n_x] % N, ids_x)
            assert torch.equal(fd.pos_ids.view(B, 3).cpu(), batch + torch.arange(3) * N)
            x0 = 3 * N
            rows = torch.cat([uniq, torch.arange(x0, x0 + n_x, device=uniq.device)])
            for k in range(L):  # fly layer k = engine layer L - 1 - k
                el = L - 1 - k
                nb_r, wn_r = tabs[el]
                nb_d, wn_d = fd.tabs[el]
                assert torch.equal(nb_d[rows], nb_r[rows]), (k, el)
                assert torch.equal(wn_d[rows], wn_r[rows]), (k, el)
                if k + 1 < L:  # the next layer's set: every drawn row and the set itself
                    nxt = torch.unique(torch.cat([nb_r[rows].reshape(-1).long(), rows[rows < x0]]))
                    rows = torch.cat([nxt, torch.arange(x0, x0 + n_x, device=nxt.device)])
            # virtual feature rows
            fr = fd.fx[x0:x0 + n_x]
            assert torch.equal(fr, feats.cuda()[ids_x])
            # a second step on the same buffers (the sampler's scratch is left clean)
            batch2 = _batch(B, 7)
            torch.manual_seed(5)
            tabs2, uniq2, _, ids_x2, _ = pm._fly_tables_merged(g, N, [batch2[:, c].cuda() for c in range(3)],
                                                               L, 200, 0.85, T)
            torch.manual_seed(5)
            fd.seeds.copy_(torch.from_numpy(pm._fly_seed_words(L)))
            fd.sample(batch2.cuda())
            torch.cuda.synchronize()
            n_x2 = int(fd.n_x.item())
            assert n_x2 == int(ids_x2.shape[0])
            rows2 = torch.cat([uniq2, torch.arange(x0, x0 + n_x2, device=uniq2.device)])
            assert torch.equal(fd.tabs[L - 1][0][rows2], tabs2[L - 1][0][rows2])
    finally:
        pm.set_rng_mode("mt19937")


@pytest.mark.parametrize("L,T", [(2, 5), (2, 10), (3, 3)])
def test_fused_fly_step_trains_like_the_per_call_path(L, T, monkeypatch):
    """PinSage.train_batch with an on-the-fly model (Philox): the captured
    device step (_FusedFlyStep: device sampler, engine loss with the virtual
    nodes' gradients, fused Adam) against the host-orchestrated merged path
    (PINSAGE_FLY_FUSED=0: the same draws, torch's loss, autograd and Adam) over
    four steps with ids repeated inside and across calls: the same generator
    state after every step, losses within 1e-5 and parameters within 1e-5
    (rounding: the loss and Adam are summed in a different order), and the
    graph path is the one that ran.  The caching allocator is first handed a
    block of random words, so workspace the step reads before writing (the
    position CSR's offsets of the virtual ranks, which no position names)
    shows up here instead of depending on what an earlier test left."""
    import pinsage_model as pm
    import pinsage_training as pt
    pm.set_rng_mode("philox")
    try:
        with tempfile.TemporaryDirectory() as tmp:
            cwd = os.getcwd()
            os.chdir(tmp)
            try:
                pg, g, feats, pos = _problem(tmp)
                batches = [_batch(64, 10 * L + T + i) for i in range(4)]

                def run(fused):
                    monkeypatch.setenv("PINSAGE_FLY_FUSED", fused)
                    torch.cuda.empty_cache()
                    junk = torch.randint(0, 1 << 20, (64 << 20,), dtype=torch.int32, device="cuda")
                    del junk  # (the block stays cached: the workspaces are carved from it)
                    torch.manual_seed(1)
                    tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
                    torch.manual_seed(2)
                    tr.model = pm.PinSageModel(g, N, L, tr.dimensions, 200, 0.85, T, None)
                    tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
                    tr.margin = 3.0
                    torch.manual_seed(99)
                    losses, states = [], []
                    for b in batches:
                        out = tr.train_batch(b)
                        losses.append([float(x) for x in out])
                        states.append(torch.get_rng_state())
                    torch.cuda.synchronize()
                    flat = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu()
                    return tr, losses, flat, states

                tr1, l1, p1, s1 = run("1")
                assert getattr(tr1, "_fused_fly", None) is not None and tr1._fused_fly.graphs is not None
                tr0, l0, p0, s0 = run("0")
                for a, b in zip(s1, s0):
                    assert torch.equal(a, b)
                for a, b in zip(l1, l0):
                    for x, y in zip(a, b):
                        assert abs(x - y) <= 1e-5 * abs(y) + 1e-7, (l1, l0)
                assert ((p1 - p0).norm() / p0.norm()).item() < 1e-5
            finally:
                os.chdir(cwd)
    finally:
        pm.set_rng_mode("mt19937")


def _drop_track(indptr, indices, z):
    """The CSR with every membership of track z removed (z keeps a zero-degree
    row): a walk from z meets a zero-degree node."""
    n_all = indptr.shape[0] - 1
    rows = np.repeat(np.arange(n_all), np.diff(indptr))
    keep = (rows != z) & (indices != z)
    cnt = np.bincount(rows[keep], minlength=n_all)
    ip = np.zeros(n_all + 1, np.int64)
    ip[1:] = np.cumsum(cnt)
    return ip, indices[keep].astype(np.int32)


@pytest.mark.parametrize("captured", [False, True])
def test_fused_fly_step_refuses_update_after_sampling_error(captured, monkeypatch):
    """A zero-degree node met by the captured on-the-fly step:
    the reference raises inside the model call, before optimizer.step().  The
    device step reports it through its ring slot; pinsage_fly_gate_adam
    refuses that step's Adam update and every later one until the host has
    raised, and the host raises at the latest when the optimizer state is
    synchronised (sync_optimizer_step checks every outstanding slot).  So after
    the error is raised, the parameters and Adam moments are exactly those
    after the last good step; once raised, training continues and updates."""
    import graph
    import pinsage_model as pm
    import pinsage_training as pt
    pm.set_rng_mode("philox")
    monkeypatch.setenv("PINSAGE_FLY_FUSED", "1")
    try:
        with tempfile.TemporaryDirectory() as tmp:
            cwd = os.getcwd()
            os.chdir(tmp)
            try:
                pg, g0, feats, pos = _problem(tmp)
                z = 17
                indptr, indices = _drop_track(*pg.csr(), z)
                g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb2.pt"))
                pos = pos[(pos != z).all(1)]
                torch.manual_seed(1)
                # (the trainer's precomputed table comes from the intact graph: the
                # reference's precompute would itself raise on the zero-degree track)
                tr = pt.PinSage(g0, N, feats, pos, log=False, load_save=False)
                torch.manual_seed(2)
                tr.model = pm.PinSageModel(g, N, 2, tr.dimensions, 200, 0.85, 5, None)
                tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
                good = [_batch(64, 300 + i) for i in range(4)]
                for b in good:
                    assert not (b == z).any()
                bad = _batch(64, 399)
                bad[5, 1] = z
                torch.manual_seed(99)
                n_good = 2 if captured else 0  # (the first two steps: eager tune, then the capture)
                for b in good[:n_good]:
                    tr.train_batch(b)
                torch.cuda.synchronize()
                fs = tr._fused_fly if n_good else None

                def state():
                    f = tr._fused_fly
                    return (torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu(),
                            f.m.detach().cpu().clone(), f.v.detach().cpu().clone())

                if n_good:
                    assert fs is not None and (fs.graphs is not None) == captured
                    before = state()
                else:
                    before = None
                    snap = [p.detach().cpu().clone() for p in tr.model.parameters()]
                tr.train_batch(bad)  # reported through the ring: no raise yet
                tr.train_batch(good[2])  # refused too (the halt word is sticky)
                with pytest.raises(RuntimeError, match="zero-degree"):
                    tr._sync_state()
                torch.cuda.synchronize()
                after = state()
                if before is not None:
                    for a, b in zip(before, after):
                        assert torch.equal(a, b)
                else:
                    now = [p.detach().cpu() for p in tr.model.parameters()]
                    for a, b in zip(snap, now):
                        assert torch.equal(a, b)
                    assert float(after[1].abs().max()) == 0.0 and float(after[2].abs().max()) == 0.0
                # raised: the next step updates again
                tr.train_batch(good[3])
                tr._sync_state()
                torch.cuda.synchronize()
                assert not torch.equal(state()[0], after[0])
            finally:
                os.chdir(cwd)
    finally:
        pm.set_rng_mode("mt19937")
