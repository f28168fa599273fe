"""Data-parallel train step on the GPU (pinsage_training.py:181-256 under
torch.distributed): two ranks train their halves of the same global batch and
average gradients with one all-reduce, then apply the same Adam step.  After
three steps the ranks agree with each other bitwise and with the oracle's
data-parallel restatement (RefTrainer.step_dp: per-rank forwards/backward, so
put_embeddings' repeated-id gradient semantics hold per rank as in any
torch.distributed run of the reference, averaged gradients, one Adam step):
losses within the north star's 1e-4 relative, parameters within 2 lr per step
element-wise (Adam's normalisation) and 1e-4 norm-relative.

The ranks share cuda:0 over gloo (one GPU per box here); the 8-GPU run uses
the same code over RCCL (nccl backend).  Each rank runs the captured step
graph without Adam, the all-reduce, and the separate Adam launch.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

N_TRACKS, D_IN, B_GLOBAL, STEPS = 3000, 128, 64, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(tmp):
    import graph
    import synthetic
    pg = synthetic.make_playlist_graph(N_TRACKS, 600, 20000, seed=1)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(N_TRACKS, D_IN, seed=2))
    pos = torch.from_numpy(synthetic.make_positives(pg, 15000, seed=3))
    return g, feats, pos


def _train(world, tmp):
    """STEPS train steps at batch B_GLOBAL / world; returns the initial and final
    state dicts, this rank's losses and the global batches drawn."""
    import pinsage_training as pt
    g, feats, pos = _problem(tmp)
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        torch.manual_seed(5)
        tr = pt.PinSage(g, N_TRACKS, feats.cuda(), pos, log=False, load_save=False)
        init = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
        tr.batch_size = B_GLOBAL // world
        torch.manual_seed(6)
        losses = []
        for _ in range(STEPS):
            batch, _ = tr.next_batch()
            losses.append(tr.train_batch(batch)[0])
        torch.cuda.synchronize()
        final = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
        return init, final, [float(x) for x in losses]
    finally:
        os.chdir(cwd)


def _worker(rank, world, port, tmp, out_q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out_q.put((rank,) + _train(world, tmp))
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_match_oracle_dp():
    tmp = tempfile.mkdtemp()
    # the neighbourhood table once, shared through the cache file (as the reference)
    import pinsage_model as pm
    g, _, _ = _problem(tmp)
    torch.manual_seed(0)
    pm.precompute_neighborhoods_topt(g, N_TRACKS, pm.DEF_HOPS, pm.DEF_ALPHA, pm.DEF_T_PRECOMP,
                                     g.nbhds_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, tmp, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, init, final, losses = q.get(timeout=100)
        res[r] = (init, final, losses)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for k in res[0][1]:  # replicas stay identical
        assert np.array_equal(res[0][1][k], res[1][1][k]), k
    # the oracle's data-parallel restatement on the same global batches
    from oracle import oracle as orc
    import pinsage_training as pt
    g2, feats, pos = _problem(tmp)
    w, nb = torch.load(g2.nbhds_path, weights_only=True)
    ref = orc.RefTrainer(res[0][0], feats, w.numpy(), nb.numpy(), n_layers=2, T=3)
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        torch.manual_seed(5)
        tr = pt.PinSage(g2, N_TRACKS, feats, pos, log=False, load_save=False)
        tr.batch_size = B_GLOBAL
        torch.manual_seed(6)
        batches = [tr.next_batch()[0].numpy() for _ in range(STEPS)]
    finally:
        os.chdir(cwd)
    lr = 1e-4
    for s, b in enumerate(batches):
        rl = ref.step_dp(b, 2)
        for r in range(2):
            assert abs(res[r][2][s] - rl[r]) <= 1e-4 * abs(rl[r]) + 1e-7, (s, r, res[r][2][s], rl[r])
    for k, v in res[0][1].items():
        rv = ref.p[k].detach().numpy().astype(np.float64)
        diff = np.abs(v.astype(np.float64) - rv)
        assert (diff <= 2 * lr * STEPS + 1e-6).all(), k
        assert np.linalg.norm(diff) <= 1e-4 * np.linalg.norm(rv), k


def _precompute_worker(rank, world, port, tmp, mode, out_q, n_items=N_TRACKS):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import pinsage_model as pm
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, _, _ = _problem(tmp)
        pm.set_rng_mode(mode)
        torch.manual_seed(0)
        w, nb = pm.precompute_neighborhoods_topt(g, n_items, 200, 0.85, 20, None)
        out_q.put((rank, w.numpy(), nb.numpy(), torch.get_rng_state().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,n_items", [("mt19937", N_TRACKS), ("philox", N_TRACKS),
                                          ("mt19937", N_TRACKS - 1), ("philox", N_TRACKS - 2)])
def test_precompute_sharded_over_ranks_matches_single_process(mode, n_items):
    """every rank walks an equal contiguous shard of the sources
    (the last one shorter when n is not divisible by the world size) and the
    shards are all-gathered; table and the generator state afterwards are bitwise those of one
    process computing everything (MT19937: exact jump-ahead to each chunk)."""
    import pinsage_model as pm
    tmp = tempfile.mkdtemp()
    g, _, _ = _problem(tmp)
    pm.set_rng_mode(mode)
    try:
        torch.manual_seed(0)
        w1, nb1 = pm.precompute_neighborhoods_topt(g, n_items, 200, 0.85, 20, None)
        st1 = torch.get_rng_state().numpy()
    finally:
        pm.set_rng_mode("mt19937")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_precompute_worker, args=(r, 3, port, tmp, mode, q, n_items)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for _, w, nb, st in res:
        assert np.array_equal(w, w1.numpy()) and np.array_equal(nb, nb1.numpy())
        assert np.array_equal(st, st1)


def _fly_worker(rank, world, port, tmp, out_q):
    """Two training steps with an on-the-fly model (pinsage_model.py:142-154):
    each rank samples and trains its own slice, so the replicas stay identical
    only if the gradients are averaged before the optimizer step."""
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pinsage_model as pm
        import pinsage_training as pt
        g, feats, pos = _problem(tmp)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            torch.manual_seed(5)
            tr = pt.PinSage(g, N_TRACKS, feats.cuda(), pos, log=False, load_save=False)
            torch.manual_seed(7)
            tr.model = pm.PinSageModel(g, N_TRACKS, 2, tr.dimensions, 200, 0.85, 3, None)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.batch_size = 8
            torch.manual_seed(11 + rank)  # the ranks' walks differ: different gradients
            for _ in range(2):
                batch, _ = tr.next_batch()
                tr.train_batch(batch)
            torch.cuda.synchronize()
            out_q.put((rank, {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}))
        finally:
            os.chdir(cwd)
    finally:
        dist.destroy_process_group()


def test_dp_on_the_fly_replicas_stay_identical():
    tmp = tempfile.mkdtemp()
    import pinsage_model as pm
    g, _, _ = _problem(tmp)
    torch.manual_seed(0)
    pm.precompute_neighborhoods_topt(g, N_TRACKS, pm.DEF_HOPS, pm.DEF_ALPHA, pm.DEF_T_PRECOMP,
                                     g.nbhds_path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fly_worker, args=(r, 2, port, tmp, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for k in res[0]:
        assert np.array_equal(res[0][k], res[1][k]), k
