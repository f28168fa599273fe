"""CPU-side checks of the product: the C-ABI library loads and exports what
include/pinsage_hip.h declares, host RNG / batch sampling reproduce torch and
the reference draw for draw, the JSON loader and CSR graph match the reference,
and compute entry points fail loudly without a GPU (no CPU fallback)."""
import os
import re
import shutil
import tempfile

import numpy as np
import pytest
import torch

from conftest import REPO, golden


def _header_functions():
    txt = open(os.path.join(REPO, "include", "pinsage_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pinsage_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import _native
    L = _native.lib()
    names = _header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
    # the ctypes binding covers exactly the header
    assert sorted(_native.EXPORTED) == names


def test_library_loads_without_gpu():
    import _native
    assert _native.lib().pinsage_version() >= 100
    assert _native.lib().pinsage_device_count() >= 0


def test_native_mt_matches_torch_and_skip():
    import _native as nat
    torch.manual_seed(77)
    mt = nat.MT.from_torch()
    ref = [int(torch.randint(1000, ())) for _ in range(3000)]
    assert (mt.draws(3000) % 1000).tolist() == ref
    # skip == draw-and-discard, across twist boundaries
    for n in (0, 1, 623, 624, 625, 1247, 5000):
        a = nat.MT().seed(5)
        b = nat.MT().seed(5)
        a.draws(n)
        b.skip(n)
        assert (a.draws(700) == b.draws(700)).all(), n


def test_native_mt_state_roundtrip():
    import _native as nat
    torch.manual_seed(3)
    with nat.torch_rng() as mt:
        mt.draws(1234)
    x = int(torch.randint(1000, ()))
    torch.manual_seed(3)
    for _ in range(1234):
        torch.randint(1000, ())
    assert int(torch.randint(1000, ())) == x


@pytest.mark.parametrize("n,k", [(1, 1), (2, 2), (37, 37), (5000, 17), (100000, 512), (300, 0)])
def test_randperm_prefix_matches_torch(n, k):
    import _native as nat
    torch.manual_seed(n + k)
    with nat.torch_rng() as mt:
        got = mt.randperm_prefix(n, k)
    after = int(torch.randint(1000, ()))
    torch.manual_seed(n + k)
    ref = torch.randperm(n)[:k].numpy()
    assert (got == ref).all()
    assert int(torch.randint(1000, ())) == after


def test_sample_batch_matches_golden():
    import pinsage_training as pt
    d = golden("batch")
    pos = torch.from_numpy(d["positives"])
    all_ids = torch.arange(int(d["n_items"]))
    torch.manual_seed(5)
    for i in range(3):
        b, ns = pt.sample_batch(all_ids, pos, int(d[f"b{i}_bs"]), None, hard_negatives=False)
        assert (b.numpy() == d[f"b{i}_batch"]).all()
        assert (ns.numpy() == d[f"b{i}_nodeset"]).all()
    got = np.array([int(torch.randint(2 ** 31, ())) for _ in range(len(d["after"]))])
    assert (got == d["after"]).all()


def test_sample_batch_component_functions_match_torch():
    import pinsage_training as pt
    d = golden("batch")
    pos = torch.from_numpy(d["positives"])
    all_ids = torch.arange(int(d["n_items"]))
    torch.manual_seed(8)
    pb = pt.sample_positives_with_rep(pos, 64)
    b, ns = pt.sample_easy_negatives(all_ids, pb)
    torch.manual_seed(8)
    b2, ns2 = pt.sample_batch(all_ids, pos, 64, None, hard_negatives=False)
    assert torch.equal(b, b2) and torch.equal(ns, ns2)


def test_max_margin_loss_matches_golden():
    import pinsage_training as pt
    d = golden("loss")
    for i in range(3):
        hq, hp, hn = (torch.from_numpy(d[f"c{i}_{k}"]).requires_grad_() for k in ("hq", "hp", "hn"))
        loss = pt.max_margin_loss(hq, hp, hn, float(d[f"c{i}_margin"]))
        loss.backward()
        assert abs(loss.item() - float(d[f"c{i}_loss"])) <= 1e-6 * max(1.0, abs(float(d[f"c{i}_loss"])))
        np.testing.assert_allclose(hq.grad.numpy(), d[f"c{i}_gq"], rtol=1e-5, atol=1e-7)


def test_spotify_graph_matches_reference_loader():
    import spotify_graph
    import synthetic
    d = golden("dataset")
    ids = [str(x) for x in d["track_ids"]]
    pg = synthetic.make_playlist_graph(len(ids), int(d["n_cols"]), 9000, seed=int(d["graph_seed"]))
    tmp = tempfile.mkdtemp()
    try:
        ds_dir = os.path.join(tmp, "ds")
        synthetic.write_spotify_dataset(ds_dir, pg, track_ids=ids, seed=int(d["json_seed"]))
        fdir = os.path.join(ds_dir, "features_test")
        os.makedirs(fdir)
        raw = np.random.default_rng(int(d["feat_seed"])).standard_normal((len(ids), 8)).astype(np.float32) * 3 + 1
        for i, tid in enumerate(ids):
            torch.save(torch.from_numpy(raw[i].copy()), os.path.join(fdir, tid + ".pt"))
        # positives of the real dataset_micro ids, re-serialised from the fixture pairs
        import json
        pairs = [{"a": ids[a], "b": ids[b]} for a, b in d["positives"]]
        with open(os.path.join(ds_dir, "positives.json"), "w") as f:
            json.dump(pairs, f)
        ds = spotify_graph.SpotifyGraph(ds_dir, fdir)
        g, track_ids, col_ids, features = ds.to_dgl_graph()
        assert track_ids == ids and col_ids == [str(x) for x in d["col_ids"]]
        src, dst = g.edges()
        assert (src.numpy() == d["src"]).all() and (dst.numpy() == d["dst"]).all()
        assert (g.successors(69).numpy() == d["succ69"]).all()
        np.testing.assert_allclose(features.numpy(), d["features"], rtol=1e-6, atol=1e-6)
        torch.manual_seed(3)
        positives = ds.load_positives(os.path.join(ds_dir, "positives.json"))
        assert (positives.numpy() == d["positives"]).all()
        got = np.array([int(torch.randint(2 ** 31, ())) for _ in range(len(d["after"]))])
        assert (got == d["after"]).all()
        tr, te = ds.load_positives_split(os.path.join(ds_dir, "positives.json"))
        assert (tr.numpy() == d["split_train"]).all() and (te.numpy() == d["split_test"]).all()
    finally:
        shutil.rmtree(tmp)


def test_spotify_graph_binary_cache(monkeypatch):
    """Second load reads pinsage_cache/ (no graph.json parse, no per-track
    feature files) and returns the same graph, edge order and features; a
    changed graph.json invalidates the cache."""
    import json
    import spotify_graph
    import synthetic
    pg = synthetic.make_playlist_graph(500, 80, 3000, seed=4)
    ids = [f"t{i:05d}" for i in range(500)]
    tmp = tempfile.mkdtemp()
    try:
        ds_dir = os.path.join(tmp, "ds")
        synthetic.write_spotify_dataset(ds_dir, pg, track_ids=ids, seed=5)
        fdir = os.path.join(ds_dir, "features")
        os.makedirs(fdir)
        raw = np.random.default_rng(1).standard_normal((500, 6)).astype(np.float32)
        for i, tid in enumerate(ids):
            torch.save(torch.from_numpy(raw[i].copy()), os.path.join(fdir, tid + ".pt"))
        g1, t1, c1, f1 = spotify_graph.SpotifyGraph(ds_dir, fdir).to_dgl_graph()
        assert os.path.isfile(os.path.join(ds_dir, "pinsage_cache", "graph.npz"))
        assert os.path.isfile(os.path.join(ds_dir, "pinsage_cache", "features.npz"))
        parsed = []
        real_load = json.load

        def spy(f, *a, **k):
            parsed.append(os.path.basename(f.name))
            return real_load(f, *a, **k)

        monkeypatch.setattr(spotify_graph.json, "load", spy)
        monkeypatch.setattr(spotify_graph.torch, "load", None)  # per-track features unused
        g2, t2, c2, f2 = spotify_graph.SpotifyGraph(ds_dir, fdir).to_dgl_graph()
        assert "graph.json" not in parsed
        assert t2 == t1 and c2 == c1 and torch.equal(f1, f2)
        assert np.array_equal(g1.indptr, g2.indptr) and np.array_equal(g1.indices, g2.indices)
        for a, b in zip(g1.edges(), g2.edges()):
            assert torch.equal(a, b)
        # a changed graph.json (one edge dropped) is parsed again
        with open(os.path.join(ds_dir, "graph.json")) as f:
            gj = real_load(f)
        gj["edges"] = gj["edges"][:-1]
        with open(os.path.join(ds_dir, "graph.json"), "w") as f:
            json.dump(gj, f)
        parsed.clear()
        g3, *_ = spotify_graph.SpotifyGraph(ds_dir, fdir).to_dgl_graph()
        assert "graph.json" in parsed and g3.number_of_edges() == g1.number_of_edges() - 1
    finally:
        shutil.rmtree(tmp)


def test_csr_graph_api():
    import graph
    src = [5, 0, 0, 3, 5, 1, 0]
    dst = [1, 4, 2, 0, 0, 0, 1]
    g = graph.CSRGraph(6, src, dst)
    assert g.number_of_nodes() == 6 and g.num_edges() == 7 and len(g) == 6
    assert g.successors(0).tolist() == [4, 2, 1]      # edge-insertion order
    assert g.successors(5).tolist() == [1, 0]
    assert g.predecessors(0).tolist() == [3, 5, 1]
    assert g.in_degrees(0) == 3 and g.in_degrees().tolist() == [3, 2, 1, 0, 1, 0]
    s, d = g.edges()
    assert sorted(zip(s.tolist(), d.tolist())) == sorted(zip(src, dst))
    a = g.adj(scipy_fmt="csr")
    assert a.shape == (6, 6) and a[0, 4] == 1 and a[4, 0] == 0
    with pytest.raises(ValueError):
        graph.CSRGraph(3, [0, 7], [1, 1])


def test_synthetic_graph_invariants():
    import synthetic
    pg = synthetic.make_playlist_graph(2000, 300, 20000, seed=4)
    indptr, indices = pg.csr()
    deg = np.diff(indptr)
    assert deg[:2000].min() >= 1 and deg[2000:].min() >= 2
    # both directions present, in JSON edge order
    src, dst = pg.edge_arrays()
    assert (src[0::2] == dst[1::2]).all() and (dst[0::2] == src[1::2]).all()
    pos = synthetic.make_positives(pg, 5000, seed=1)
    assert (pos[:, 0] != pos[:, 1]).all()
    pg2 = synthetic.make_playlist_graph(2000, 300, 20000, seed=4)
    assert (pg2.mem_track == pg.mem_track).all()


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_compute_fails_loudly_without_gpu():
    import graph
    import pinsage_model as pm
    g = graph.CSRGraph(4, [0, 1, 2, 3], [2, 3, 0, 1])
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pm.do_random_walks(g, torch.tensor([0]), 3, 0.85)


def test_batch_sampler_speculation_is_exact():
    """The native sampler's speculative next batch is used only when torch's
    generator is untouched in between; batches, nodesets and the generator
    state after each call equal the synchronous reference-exact sampler's."""
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(3000, 500, 20000, seed=9)
    pos = torch.from_numpy(synthetic.make_positives(pg, 8000, seed=3))
    all_ids = torch.arange(3000)

    def run(speculate):
        pt._PREFETCH.close()
        pt._PREFETCH.speculate = speculate
        pt._PREFETCH.hits = 0
        torch.manual_seed(21)
        out = []
        for i in range(12):
            b, ns = pt.sample_batch(all_ids, pos, 64 + (i >= 8) * 16, None, hard_negatives=False)
            out.append((b, ns))
            if i % 4 == 1:
                torch.randint(1000, ())   # another generator user: speculation must miss
            if i == 6:
                torch.manual_seed(5)      # a reseed as well
        out.append(int(torch.randint(2 ** 31, ())))
        return out, pt._PREFETCH.hits

    ref, h0 = run(False)
    got, h1 = run(True)
    pt._PREFETCH.close()
    pt._PREFETCH.speculate = True
    assert h0 == 0 and h1 >= 4
    assert ref[-1] == got[-1]
    for (b1, n1), (b2, n2) in zip(ref[:-1], got[:-1]):
        assert torch.equal(b1, b2) and torch.equal(n1, n2)
        assert torch.equal(n2, b2.flatten().unique())


def test_batch_sampler_peek_is_the_next_batch():
    """peek() (the trainer computes that batch's frontier ahead) returns the
    batch the next sample() draws, and None once another generator user has
    moved torch's state; the chained speculation keeps hitting."""
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(3000, 500, 20000, seed=9)
    pos = torch.from_numpy(synthetic.make_positives(pg, 8000, seed=3))
    all_ids = torch.arange(3000)
    pt._PREFETCH.close()
    pt._PREFETCH.speculate = True
    pt._PREFETCH.hits = 0
    torch.manual_seed(3)
    pt.sample_batch(all_ids, pos, 64, None, hard_negatives=False)
    for _ in range(6):
        nxt = pt._PREFETCH.peek(64)
        b, _ = pt.sample_batch(all_ids, pos, 64, None, hard_negatives=False)
        assert nxt is not None and np.array_equal(nxt, b.numpy())
    assert pt._PREFETCH.hits >= 5
    torch.randint(10, ())
    assert pt._PREFETCH.peek(64) is None
    assert pt._PREFETCH.peek(32) is None
    pt._PREFETCH.close()


@pytest.mark.parametrize("n", [(1 << 21) + 7, 3_000_017, 12_345_678])
def test_mt_long_skip_jumps_exactly(n):
    """Skips of >= 2^21 draws use the GF(2) jump-ahead (mt_jump.h); the state
    must equal n sequential draws, from any position inside a block."""
    import _native as nat
    for pre in (0, 1, 311, 623, 624, 1000):
        a = nat.MT().seed(1234 + pre)
        b = nat.MT().seed(1234 + pre)
        a.draws(pre)
        b.draws(pre)
        a.skip(n)
        # reference: sequential twisting in bounded pieces (below the jump threshold)
        left = n
        while left:
            k = min(left, (1 << 21) - 1)
            b.skip(k)
            left -= k
        assert (a.draws(2000) == b.draws(2000)).all(), (n, pre)


def test_randperm_prefix_long_matches_torch():
    """torch.randperm(5M)[:512] and the generator state after it (jump path)."""
    import _native as nat
    n, k = 5_000_000, 512
    torch.manual_seed(99)
    with nat.torch_rng() as mt:
        got = mt.randperm_prefix(n, k)
    after = int(torch.randint(1000, ()))
    torch.manual_seed(99)
    ref = torch.randperm(n)[:k].numpy()
    assert (got == ref).all()
    assert int(torch.randint(1000, ())) == after


def test_device_graph_generator_properties():
    """synthetic.make_playlist_graph_device (the C5 bench's graph builder) on the
    CPU device: bipartite and symmetric, rows in edge-insertion order, every
    track in >= 1 collection and every collection with >= 2 distinct tracks;
    positives are co-members and never self-pairs."""
    import numpy as np
    import torch
    import synthetic
    n, nc = 3000, 700
    ip, ix = synthetic.make_playlist_graph_device(n, nc, 30000, seed=1, device="cpu")
    ip, ix = ip.numpy(), ix.numpy()
    deg = np.diff(ip)
    assert deg[:n].min() >= 1 and deg[n:].min() >= 2
    src = np.repeat(np.arange(n + nc), deg)
    assert ((src < n) != (ix < n)).all()
    fwd = set(zip(src.tolist(), ix.tolist()))
    assert fwd == set(zip(ix.tolist(), src.tolist())) and len(fwd) == ix.shape[0]
    for v in list(range(0, n, 97)) + list(range(n, n + nc, 13)):
        row = ix[ip[v]:ip[v + 1]]
        assert (np.diff(row) > 0).all()  # collection-major pairs: both row kinds ascend
    pos = synthetic.make_positives_device(torch.from_numpy(ip), torch.from_numpy(ix), n, 4000, seed=3).numpy()
    assert (pos[:, 0] != pos[:, 1]).all() and pos.max() < n
    cols_of = {v: set(ix[ip[v]:ip[v + 1]].tolist()) for v in np.unique(pos[:200]).tolist()}
    assert all(cols_of[a] & cols_of[b] for a, b in pos[:200].tolist())


def test_torch_operator_library_registers_every_op():
    """libpinsage_torch.so (csrc/torch_ops.cpp) loads and registers the
    torch.ops.pinsage schemas of SURVEY.md §8(b2), with autograd formulas for
    the differentiable ones; no compute (there is no CPU implementation)."""
    import torch
    import pinsage_ops
    pinsage_ops.load()
    for name in ("walk", "ppr_topk", "frontier", "gather_rows", "scatter_add_rows", "linear",
                 "concat_linear_lrelu_l2norm", "norm_lrelu_backward", "gemm", "weighted_agg",
                 "weighted_agg_backward", "segment_wmean"):
        assert hasattr(torch.ops.pinsage, name), name
    x = torch.zeros(4, 8)
    W = torch.zeros(4, 8)
    import pytest
    with pytest.raises(NotImplementedError, match="CPU"):  # HIP dispatch only: fails loudly
        torch.ops.pinsage.linear(x, None, W, None, True)


def test_bench_refuses_a_world_size_other_than_gpus():
    """bench.py started by a launcher with WORLD_SIZE != --gpus exits non-zero
    before touching the GPU (launch_ranks)."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in (r.stderr + r.stdout)
