"""Pin the CPU oracle against golden vectors produced by the real reference.

These run without a GPU.  Every fixture came from tests/golden/make_golden.py
(the reference imported with dgl/wandb/torchvision stubs).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import oracle as orc


def _csr(d):
    return d["indptr"], d["indices"], int(d["n_tracks"] + d["n_cols"])


def test_mt_matches_torch_stream():
    torch.manual_seed(123)
    mt = orc.MT.from_torch()
    # ranges < 2**28 take one 32-bit draw: value = raw % n
    ref = [int(torch.randint(1000, ())) for _ in range(2000)]
    assert (mt.draws(2000) % 1000).tolist() == ref


def test_mt_state_roundtrip_through_torch():
    torch.manual_seed(5)
    torch.randint(10, (7,))
    mt = orc.MT.from_torch()
    mt.draws(1000)
    mt.to_torch()
    a = int(torch.randint(1000, ()))
    torch.manual_seed(5)
    torch.randint(10, (7,))
    mt2 = orc.MT.from_torch()
    mt2.draws(1000)
    assert int(mt2.draws(1)[0]) % 1000 == a


def test_randperm_and_rand_semantics():
    d = golden("batch")
    mt = orc.MT(9)
    assert (mt.randperm(37) == d["randperm_37"]).all()
    assert (mt.randperm(5000) == d["randperm_5000"]).all()
    assert _after_ok(mt, d["randperm_after"])
    # randint(2**32) takes two draws (random64 = hi<<32 | lo) and keeps lo
    mt = orc.MT(10)
    raw = mt.draws(32)
    assert (raw[1::2].astype(np.int64) == d["raw_u32"]).all()
    u = (raw[:16] & 0xFFFFFF).astype(np.float32) * np.float32(2 ** -24)
    assert (u == d["rand_f32"]).all()


def _after_ok(mt, after):
    # torch.randint(2**31, ()): range >= 2**28 -> two draws, value = lo % 2**31
    d = mt.draws(2 * len(after)).astype(np.int64)
    return (d[1::2] % 2 ** 31 == after).all()


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_walk_trace_bit_exact(gname):
    d = golden(f"walk_{gname}")
    indptr, indices, _ = _csr(d)
    mt = orc.MT(int(d["seed"]))
    tr = orc.walk_mt(indptr, indices, d["nodeset"], 500, 0.85, mt)
    assert (tr == d["trace"]).all()
    assert _after_ok(mt, d["after"])
    tr1 = orc.walk_mt(indptr, indices, d["nodeset"][:8], 60, 1.0, orc.MT(int(d["seed"]) + 1))
    assert (tr1 == d["trace_a1"]).all()
    tr0 = orc.walk_mt(indptr, indices, d["nodeset"][:8], 60, 0.0, orc.MT(int(d["seed"]) + 2))
    assert (tr0 == d["trace_a0"]).all()


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_visit_prob_and_topk_bit_exact(gname):
    d = golden(f"topk_{gname}")
    indptr, indices, n_all = _csr(d)
    mt = orc.MT(int(d["seed"]))
    tr = orc.walk_mt(indptr, indices, d["nodeset"], int(d["n_hops"]), 0.85, mt)
    vp = orc.visit_prob(tr, d["nodeset"], n_all)
    ref = np.zeros(tuple(d["vp_shape"]))
    ref[d["vp_row"], d["vp_col"]] = d["vp_val"]
    assert (vp == ref).all()
    assert _after_ok(mt, d["after"])
    for k in d["ks"]:
        v, i = orc.topk(vp, int(k))
        assert (v == d[f"val_{k}"]).all(), k
        assert (i == d[f"idx_{k}"]).all(), k
    v, i = orc.sample_neighborhood_topt(indptr, indices, n_all, d["nodeset"], int(d["n_hops"]), 0.85,
                                        10, orc.MT(int(d["seed"])))
    assert (v == d["topt_val"]).all() and (i == d["topt_idx"]).all()


def test_topk_matches_torch_on_tie_heavy_rows():
    rng = np.random.default_rng(0)
    for n, k in [(1000, 3), (1000, 15), (640, 10), (7000, 100), (50, 50), (200, 1)]:
        m = (rng.integers(0, 4, size=(6, n)) / 500.0).astype(np.float64)
        v, i = orc.topk(m, k)
        tv, ti = torch.from_numpy(m).topk(k, 1)
        assert (v == tv.numpy()).all() and (i == ti.numpy()).all(), (n, k)


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_precompute_bit_exact(gname):
    d = golden(f"precompute_{gname}")
    indptr, indices, n_all = _csr(d)
    mt = orc.MT(int(d["seed"]))
    w, nb = orc.precompute_topt(indptr, indices, n_all, int(d["n_tracks"]), int(d["n_hops"]), 0.85,
                                100, mt)
    assert (w == d["weights"]).all()
    assert (nb == d["nodes"]).all()
    assert _after_ok(mt, d["after"])


def test_frontier_matches():
    d = golden("frontier")
    p = golden("precompute_mid")
    case = 0
    while f"c{case}_nodeset" in d:
        L, T = d[f"c{case}_LT"]
        S = orc.frontier(d[f"c{case}_nodeset"], int(L), int(T), p["weights"], p["nodes"])
        for l, (ns, w, nb) in enumerate(S):
            assert (ns == d[f"c{case}_l{l}_nodes"]).all()
            assert (w == d[f"c{case}_l{l}_w"]).all()
            assert (nb == d[f"c{case}_l{l}_nb"]).all()
        case += 1


def test_batch_sampler_matches():
    d = golden("batch")
    mt = orc.MT(5)
    for i in range(3):
        b, ns = orc.sample_batch_easy(mt, d["positives"], int(d["n_items"]), int(d[f"b{i}_bs"]))
        assert (b == d[f"b{i}_batch"]).all()
        assert (ns == d[f"b{i}_nodeset"]).all()
    assert _after_ok(mt, d["after"])


def test_loss_matches():
    d = golden("loss")
    for i in range(3):
        hq, hp, hn = (torch.from_numpy(d[f"c{i}_{k}"]).requires_grad_() for k in ("hq", "hp", "hn"))
        loss = orc.max_margin_loss(hq, hp, hn, float(d[f"c{i}_margin"]))
        loss.backward()
        assert abs(loss.item() - float(d[f"c{i}_loss"])) <= 1e-6 * max(1.0, abs(float(d[f"c{i}_loss"])))
        for t, k in ((hq, "gq"), (hp, "gp"), (hn, "gn")):
            np.testing.assert_allclose(t.grad.numpy(), d[f"c{i}_{k}"], rtol=1e-5, atol=1e-7)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def test_model_forward_backward_matches():
    import synthetic
    d = golden("model")
    p = golden("precompute_mid")
    feats = torch.from_numpy(synthetic.make_features(7000, 24, seed=5))
    assert abs(float(feats.double().sum()) - float(d["features_sum"])) < 1e-6
    for L in (1, 2, 3):
        state = {k[len(f"L{L}_p_"):]: d[k] for k in d if k.startswith(f"L{L}_p_")}
        P = {k: torch.from_numpy(v.copy()).requires_grad_() for k, v in state.items()}
        y = orc.model_forward(P, feats, d[f"L{L}_nodeset"], L, 5, p["weights"], p["nodes"], 16)
        assert _rel(y.detach().numpy(), d[f"L{L}_out"]) < 1e-6
        (y * torch.from_numpy(d[f"L{L}_cvec"])).sum().backward()
        for k, t in P.items():
            assert _rel(t.grad.numpy(), d[f"L{L}_g_{k}"]) < 1e-5, (L, k)


def test_train_step_matches():
    import synthetic
    d = golden("train")
    p = golden("precompute_mid")
    pg = synthetic.make_playlist_graph(7000, 1500, 40000, seed=12)
    feats = torch.from_numpy(synthetic.make_features(7000, 128, seed=6))
    assert abs(float(feats.double().sum()) - float(d["features_sum"])) < 1e-6
    pos = synthetic.make_positives(pg, 5 * 7000, seed=7)
    assert int(pos.sum()) == int(d["positives_sum"])
    init = {k[len("init_"):]: d[k] for k in d if k.startswith("init_")}
    tr = orc.RefTrainer(init, feats, p["weights"], p["nodes"], n_layers=2, T=3)
    mt = orc.MT(77)
    for s in range(2):
        b, _ = orc.sample_batch_easy(mt, pos, 7000, 128)
        assert (b == d[f"s{s}_batch"]).all()
        loss, nfl, var, grads = tr.step(b)
        assert abs(loss - float(d[f"s{s}_loss"])) <= 1e-5 * abs(float(d[f"s{s}_loss"])) + 1e-7
        assert abs(nfl - float(d[f"s{s}_nfl"])) <= 1e-5 * abs(float(d[f"s{s}_nfl"])) + 1e-7
        assert abs(var - float(d[f"s{s}_var"])) <= 1e-4 * abs(float(d[f"s{s}_var"]))
        if s == 0:
            for k, g in grads.items():
                assert _rel(g.numpy(), d[f"s0_g_{k}"]) < 1e-4, k
    for k in tr.order:
        assert _rel(tr.p[k].detach().numpy(), d[f"s1_p_{k}"]) < 1e-6, k


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_ppr_knn_bit_exact(gname):
    """PersPageRank.knn (baselines.py:106-151) fixtures from the reference."""
    d = golden(f"ppr_{gname}")
    indptr, indices, n_all = _csr(d)
    for k in d["ks"]:
        mt = orc.MT(int(d["seed"]) + int(k))
        w, nb = orc.ppr_knn(indptr, indices, n_all, d["nodeset"], int(k), mt, int(d["n_hops"]),
                            float(d["alpha"]))
        assert (w == d[f"val_{k}"]).all() and (nb == d[f"idx_{k}"]).all(), k
        assert _after_ok(mt, d[f"after_{k}"])


def test_knn_from_emb_matches_reference():
    """knn_from_emb / cosine_sim_ab (baselines.py:69-103) restated with the same
    torch CPU ops: bitwise equal to the reference's output."""
    d = golden("knn_emb")
    for k in (50, 1000):
        w, n = orc.knn_from_emb(d["emb"], d["q"], k)
        assert np.array_equal(w, d[f"w_{k}"]) and np.array_equal(n, d[f"n_{k}"]), k


def test_put_repeated_ids_last_write_and_index_put_backward():
    """The oracle's put_embeddings with repeated ids: the serial last write
    wins (torch-CPU's parallel index_put leaves the winner unspecified), and
    every occurrence's row gets the cotangent at its index (index_put's
    backward), pinsage_model.py:24-30."""
    import torch
    from oracle import oracle as orc
    h = torch.zeros(6, 3)
    idx = torch.tensor([4, 1, 4, 2, 4])
    rows = torch.arange(10, dtype=torch.float32).view(5, 2).requires_grad_()
    out = orc._put(h, idx, rows)
    assert out[4, :2].tolist() == [8.0, 9.0] and out[4, 2] == 0
    assert out[1, :2].tolist() == [2.0, 3.0] and out[2, :2].tolist() == [6.0, 7.0]
    g = torch.arange(18, dtype=torch.float32).view(6, 3)
    (out * g).sum().backward()
    assert torch.equal(rows.grad, g[idx, :2])
