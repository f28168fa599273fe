"""Data-parallel path on CPU (gloo, world_size 2): every rank draws the same
global batch from the shared-seed RNG and trains its slice; gradients are
averaged by one all-reduce.  (The GPU run uses the same code over RCCL.)"""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, out_q):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(2000, 400, 12000, seed=7)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(2000, 128, seed=1))
    pos = torch.from_numpy(synthetic.make_positives(pg, 10000, seed=2))
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        tr = pt.PinSage(g, 2000, feats, pos, log=False, load_save=False)
        tr.batch_size = 16
        torch.manual_seed(123)
        slices = [tr.next_batch()[0] for _ in range(3)]
        state = torch.get_rng_state()
        flat = torch.full((10,), float(rank + 1))
        pt.average_gradients(flat)
        # the staged step's bucket protocol (_dp_tail): two asynchronous starts,
        # work between them, then the finishes in start order -- the code the
        # RCCL path runs (gloo: async sum, the finish scales to the mean)
        ba, bb = torch.full((7,), 2.0 * (rank + 1)), torch.full((5,), -3.0 * (rank + 1))
        wa = pt._allreduce_start(ba)
        busy = torch.arange(1000.0).sum()
        wb = pt._allreduce_start(bb)
        pt._allreduce_finish(wa)
        pt._allreduce_finish(wb)
        buckets_ok = bool(torch.allclose(ba, torch.full((7,), 3.0)) and torch.allclose(bb, torch.full((5,), -4.5))
                          and float(busy) == 499500.0)
        # precompute exchange: equal contiguous shards (n not divisible by the
        # world size), one all-gather per table
        import pinsage_model as pm
        n = 2001
        lo, hi, per = pm._shard_range(n, rank, world)
        full_w = torch.arange(n * 3, dtype=torch.float64).reshape(n, 3) / 7
        full_nb = torch.arange(n * 3, dtype=torch.int64).reshape(n, 3) * 5
        sw = torch.zeros((per, 3), dtype=torch.float64)
        snb = torch.zeros((per, 3), dtype=torch.int64)
        sw[:hi - lo], snb[:hi - lo] = full_w[lo:hi], full_nb[lo:hi]
        gw, gnb = pm._gather_shards(sw, snb, n, per, None)
        gathered_ok = torch.equal(gw, full_w) and torch.equal(gnb, full_nb)
        out_q.put((rank, [s.numpy() for s in slices], state.numpy(), flat.numpy(), gathered_ok and buckets_ok))
    finally:
        os.chdir(cwd)
        dist.destroy_process_group()


def test_dp_batch_slices_and_grad_average():
    import graph
    import pinsage_training as pt
    import synthetic
    tmp = tempfile.mkdtemp()
    pg = synthetic.make_playlist_graph(2000, 400, 12000, seed=7)
    # a cached neighbourhood table, so the trainer needs no GPU to construct
    rng = np.random.default_rng(0)
    nb = torch.from_numpy(rng.integers(0, 2000, (2000, 100)).astype(np.int64))
    w = torch.from_numpy(rng.random((2000, 100)))
    torch.save((w, nb), os.path.join(tmp, "nb.pt"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, tmp, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (sl, st, fl, ok)) for r, sl, st, fl, ok in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: the global batch of 2 * 16 triples
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(2000, 128, seed=1))
    pos = torch.from_numpy(synthetic.make_positives(pg, 10000, seed=2))
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        tr = pt.PinSage(g, 2000, feats, pos, log=False, load_save=False)
        tr.batch_size = 32
        torch.manual_seed(123)
        ref = [tr.next_batch()[0].numpy() for _ in range(3)]
    finally:
        os.chdir(cwd)
    for s in range(3):
        got = np.concatenate([res[0][0][s], res[1][0][s]], 0)
        assert (got == ref[s]).all()
    assert (res[0][1] == res[1][1]).all()  # RNG stays in lock-step across ranks
    assert np.allclose(res[0][2], 1.5) and np.allclose(res[1][2], 1.5)
    assert res[0][3] and res[1][3]  # all-gathered precompute shards == the full table; async buckets averaged
