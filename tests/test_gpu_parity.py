"""GPU parity: the HIP path (through the C-ABI) against the reference's golden
vectors and the CPU oracle.

Integer work (walks, visit counts, top-k indices, frontiers, batches) must be
bit-exact; f64 top-k weights are exact (count / n_hops); fp32 embeddings,
losses and gradients must agree within the north star's 1e-4 relative
tolerance (row/tensor-norm relative, since the reference aggregates in f64).
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

REL_TOL = 1e-4


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _graph(d):
    import graph
    return graph.CSRGraph.from_csr(d["indptr"], d["indices"])


def _after_ok(after):
    got = np.array([int(torch.randint(2 ** 31, ())) for _ in range(len(after))])
    return (got == after).all()


@pytest.fixture(autouse=True)
def _mt_mode():
    import pinsage_model as pm
    pm.set_rng_mode("mt19937")
    yield


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_walk_bit_exact(gname):
    import pinsage_model as pm
    d = golden(f"walk_{gname}")
    g = _graph(d)
    ns = torch.from_numpy(d["nodeset"])
    torch.manual_seed(int(d["seed"]))
    tr = pm.do_random_walks(g, ns, 500, 0.85)
    assert tr.dtype == torch.int64 and tr.device.type == "cpu"
    assert (tr.numpy() == d["trace"]).all()
    assert _after_ok(d["after"])
    torch.manual_seed(int(d["seed"]) + 1)
    assert (pm.do_random_walks(g, ns[:8], 60, 1.0).numpy() == d["trace_a1"]).all()
    torch.manual_seed(int(d["seed"]) + 2)
    assert (pm.do_random_walks(g, ns[:8], 60, 0.0).numpy() == d["trace_a0"]).all()


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_visit_dense_and_topk_bit_exact(gname):
    import pinsage_model as pm
    d = golden(f"topk_{gname}")
    g = _graph(d)
    ns = torch.from_numpy(d["nodeset"])
    n_hops = int(d["n_hops"])
    torch.manual_seed(int(d["seed"]))
    vp = pm.sample_neighborhood(g, int(d["n_tracks"]), ns, n_hops, 0.85)
    ref = np.zeros(tuple(d["vp_shape"]))
    ref[d["vp_row"], d["vp_col"]] = d["vp_val"]
    assert vp.dtype == torch.float64 and (vp.numpy() == ref).all()
    assert _after_ok(d["after"])
    for k in d["ks"]:
        torch.manual_seed(int(d["seed"]))
        tk = pm.sample_neighborhood_topt(g, int(d["n_tracks"]), ns, n_hops, 0.85, int(k))
        assert isinstance(tk, torch.return_types.topk)
        assert (tk.values.numpy() == d[f"val_{k}"]).all(), k
        assert (tk.indices.numpy() == d[f"idx_{k}"]).all(), k


@pytest.mark.parametrize("gname", ["small", "mid"])
def test_precompute_bit_exact(gname):
    import pinsage_model as pm
    d = golden(f"precompute_{gname}")
    g = _graph(d)
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "nb.pt")
        torch.manual_seed(int(d["seed"]))
        w, nb = pm.precompute_neighborhoods_topt(g, int(d["n_tracks"]), int(d["n_hops"]), 0.85, 100, path)
        assert _after_ok(d["after"])
        assert (w.numpy() == d["weights"]).all()
        assert (nb.numpy() == d["nodes"]).all()
        # cache hit returns the stored table without drawing
        st = torch.get_rng_state()
        w2, nb2 = pm.precompute_neighborhoods_topt(g, int(d["n_tracks"]), int(d["n_hops"]), 0.85, 100, path)
        assert torch.equal(st, torch.get_rng_state())
        assert torch.equal(w2, w) and torch.equal(nb2, nb)


def test_frontier_matches():
    import pinsage_model as pm
    d = golden("frontier")
    p = golden("precompute_mid")
    nbhds = (torch.from_numpy(p["weights"]), torch.from_numpy(p["nodes"]))
    case = 0
    while f"c{case}_nodeset" in d:
        L, T = (int(x) for x in d[f"c{case}_LT"])
        S = pm.relevant_nodes_per_layer_precomp(torch.from_numpy(d[f"c{case}_nodeset"]), L, T, nbhds)
        assert len(S) == L
        for l, (ns, w, nb) in enumerate(S):
            assert (ns.numpy() == d[f"c{case}_l{l}_nodes"]).all(), (case, l)
            assert (w.numpy() == d[f"c{case}_l{l}_w"]).all()
            assert (nb.numpy() == d[f"c{case}_l{l}_nb"]).all()
        case += 1
    s = golden("topk_small")
    g = _graph(s)
    torch.manual_seed(41)
    S = pm.relevant_nodes_per_layer(g, int(s["n_tracks"]), torch.from_numpy(d["fly_nodeset"]), 2, 100, 0.85, 3)
    assert _after_ok(d["fly_after"])
    for l, (ns, w, nb) in enumerate(S):
        assert (ns.numpy() == d[f"fly_l{l}_nodes"]).all()
        assert (w.numpy() == d[f"fly_l{l}_w"]).all()
        assert (nb.numpy() == d[f"fly_l{l}_nb"]).all()


def test_philox_walk_matches_cpu_twin():
    import pinsage_model as pm
    from oracle import oracle as orc
    d = golden("walk_mid")
    g = _graph(d)
    ns = torch.from_numpy(d["nodeset"])
    pm.set_rng_mode("philox")
    try:
        torch.manual_seed(3)
        tr = pm.do_random_walks(g, ns, 300, 0.85)
    finally:
        pm.set_rng_mode("mt19937")
    torch.manual_seed(3)
    mt = orc.MT.from_torch()
    dd = mt.draws(2)
    seed = (int(dd[0]) << 32) | int(dd[1])
    ref = orc.walk_philox(d["indptr"], d["indices"], d["nodeset"], 300, 0.85, seed)
    assert (tr.numpy() == ref).all()


def test_zero_degree_source_raises():
    import graph
    import pinsage_model as pm
    # node 2 has no out-edges
    g = graph.CSRGraph(4, [0, 3, 1, 3], [3, 0, 3, 1])
    with pytest.raises(RuntimeError):
        pm.do_random_walks(g, torch.tensor([2]), 5, 0.85)


def test_model_forward_backward_vs_golden():
    import pinsage_model as pm
    import synthetic
    d = golden("model")
    p = golden("precompute_mid")
    nbhds = (torch.from_numpy(p["weights"]), torch.from_numpy(p["nodes"]))
    feats = torch.from_numpy(synthetic.make_features(7000, 24, seed=5))
    for L in (1, 2, 3):
        torch.manual_seed(100 + L)
        m = pm.PinSageModel(None, 7000, L, (24, 32, 16), 500, 0.85, 5, nbhds)
        sd = {k[len(f"L{L}_p_"):]: torch.from_numpy(d[k]) for k in d if k.startswith(f"L{L}_p_")}
        # identical init under the same seed (same module construction order)
        for k, v in m.state_dict().items():
            assert torch.equal(v.cpu(), sd[k]), k
        y = m(feats, torch.from_numpy(d[f"L{L}_nodeset"]))
        assert y.device.type == "cpu"
        assert _rel(y.detach().numpy(), d[f"L{L}_out"]) < REL_TOL
        # row-wise too
        yy, rr = y.detach().numpy().astype(np.float64), d[f"L{L}_out"].astype(np.float64)
        assert (np.linalg.norm(yy - rr, axis=1) <= REL_TOL * np.linalg.norm(rr, axis=1) + 1e-7).all()
        (y * torch.from_numpy(d[f"L{L}_cvec"])).sum().backward()
        for k, prm in m.named_parameters():
            assert _rel(prm.grad.cpu().numpy(), d[f"L{L}_g_{k}"]) < REL_TOL, (L, k)


def test_conv_layer_standalone():
    import pinsage_model as pm
    import synthetic
    d = golden("model")
    p = golden("precompute_mid")
    feats = torch.from_numpy(synthetic.make_features(7000, 24, seed=5))
    conv = pm.ConvLayer(24, 16, 32)
    conv.load_state_dict({k[len("conv_p_"):]: torch.from_numpy(d[k]) for k in d if k.startswith("conv_p_")})
    ns = torch.from_numpy(d["conv_nodeset"])
    w = torch.from_numpy(p["weights"])[ns, :4]
    nb = torch.from_numpy(p["nodes"])[ns, :4]
    with torch.no_grad():
        y = conv(feats, ns, nb, w)
    assert _rel(y.numpy(), d["conv_out"]) < REL_TOL


def test_train_steps_vs_golden():
    """Two reference train_batch steps of the real trainer (default dims)."""
    import graph
    import pinsage_training as pt
    import synthetic
    d = golden("train")
    p = golden("precompute_mid")
    pg = synthetic.make_playlist_graph(7000, 1500, 40000, seed=12)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(7000, 128, seed=6))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * 7000, seed=7))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            torch.save((torch.from_numpy(p["weights"]), torch.from_numpy(p["nodes"])), g.nbhds_path)
            torch.manual_seed(2024)
            tr = pt.PinSage(g, 7000, feats, pos, log=False, load_save=False)
            for k, v in tr.model.state_dict().items():
                assert torch.equal(v.cpu(), torch.from_numpy(d[f"init_{k}"])), k
            torch.manual_seed(77)
            for s in range(2):
                batch, nodeset = pt.sample_batch(tr.all_ids, tr.positives, tr.batch_size, tr.nbhds,
                                                 hard_negatives=tr.hard_negatives)
                assert (batch.numpy() == d[f"s{s}_batch"]).all()
                loss, nfl, var = tr.train_batch(batch)
                assert abs(float(loss) - float(d[f"s{s}_loss"])) <= REL_TOL * abs(float(d[f"s{s}_loss"])) + 1e-7
                assert abs(float(nfl) - float(d[f"s{s}_nfl"])) <= REL_TOL * abs(float(d[f"s{s}_nfl"])) + 1e-7
                assert abs(float(var) - float(d[f"s{s}_var"])) <= 1e-3 * abs(float(d[f"s{s}_var"]))
                if s == 0:
                    for k, prm in tr.model.named_parameters():
                        assert _rel(prm.grad.cpu().numpy(), d[f"s0_g_{k}"]) < REL_TOL, k
            assert _after_ok(d["after"])
            for k, v in tr.model.state_dict().items():
                assert _rel(v.cpu().numpy(), d[f"s1_p_{k}"]) < 1e-6, k
        finally:
            os.chdir(cwd)


def test_train_step_vs_oracle_larger_graph():
    """Randomised parity at a C2-like shape (smaller n) against the CPU oracle."""
    import graph
    import pinsage_model as pm
    import pinsage_training as pt
    import synthetic
    from oracle import oracle as orc
    pg = synthetic.make_playlist_graph(20000, 5000, 200000, seed=3)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(20000, 256, seed=4))
    pos = torch.from_numpy(synthetic.make_positives(pg, 100000, seed=5))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            pm.set_rng_mode("philox")
            torch.manual_seed(0)
            w, nb = pm.precompute_neighborhoods_topt(g, 20000, 200, 0.85, 100, g.nbhds_path)
            pm.set_rng_mode("mt19937")
            torch.manual_seed(1)
            tr = pt.PinSage(g, 20000, feats, pos, log=False, load_save=False)
            tr.batch_size = 512
            init = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
            ref = orc.RefTrainer(init, feats, w.numpy(), nb.numpy(), n_layers=2, T=3)
            torch.manual_seed(2)
            for s in range(3):
                batch, _ = tr.next_batch()
                loss, nfl, var = tr.train_batch(batch)
                rl, rn, rv, rg = ref.step(batch.numpy())
                assert abs(float(loss) - rl) <= REL_TOL * abs(rl) + 1e-7
                assert abs(float(nfl) - rn) <= REL_TOL * abs(rn) + 1e-7
                if s == 0:
                    for k, prm in tr.model.named_parameters():
                        assert _rel(prm.grad.cpu().numpy(), rg[k].numpy()) < REL_TOL, k
            # Adam normalises each element by sqrt(v): where a gradient is ~0 a
            # 1-ulp difference can flip that element's update (+-lr per step),
            # so parameters are compared element-wise against 2*lr*steps.
            for k, v in tr.model.state_dict().items():
                diff = np.abs(v.cpu().numpy().astype(np.float64) - ref.p[k].detach().numpy())
                assert (diff <= 2 * 1e-4 * 3 + 1e-6).all(), k
                assert _rel(v.cpu().numpy(), ref.p[k].detach().numpy()) < 1e-4, k
        finally:
            os.chdir(cwd)


def test_fused_adam_matches_backward_plus_adam():
    """pinsage_engine_backward_adam (Adam inside the gradient reductions)
    against backward + adam, eager and as the captured step graph.  The
    arithmetic is the same, but a step is not bitwise repeatable run to run
    (the transposed-neighbour CSR is filled with atomics, which orders the dq
    sums; repeated ids' loss gradients are added with float atomics), and
    Adam's 1/sqrt(v) turns a rounding-level gradient change of a ~0 gradient
    into up to +-lr on that element, which later steps amplify.  So: three
    steps at lr = 0 (parameters fixed, the moments still accumulate) compare
    gradients and moments within 1e-5 relative; one step at the trainer's lr
    compares parameters element-wise within 2 * lr."""
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(6000, 1500, 40000, seed=21)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(6000, 128, seed=22))
    pos = torch.from_numpy(synthetic.make_positives(pg, 30000, seed=23))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp,
                                        nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)  # neighbourhoods on disk

            def run(fused, use_graph, steps, lr):
                torch.manual_seed(5)
                tr = pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)
                tr.batch_size = 256
                if lr is not None:
                    tr.optimizer.param_groups[0]["lr"] = lr
                tr._fused = f = pt._FusedStep(tr)
                f.fuse_adam = fused
                f.use_graph = use_graph
                torch.manual_seed(6)
                for _ in range(steps):
                    batch, _ = tr.next_batch()
                    tr.train_batch(batch)
                torch.cuda.synchronize()
                return ([t.detach().clone() for t in (f.runner.flat, f.grads, f.m, f.v)],
                        tr.optimizer.param_groups[0]["lr"])

            base, _ = run(False, False, 3, 0.0)
            for fused, use_graph in ((True, False), (True, True)):
                other, _ = run(fused, use_graph, 3, 0.0)
                assert torch.equal(base[0], other[0])
                for a, b in zip(base[1:], other[1:]):
                    assert ((a - b).norm() / a.norm()).item() < 1e-5
            p0, lr = run(False, False, 1, None)
            p1, _ = run(True, False, 1, None)
            assert ((p0[0] - p1[0]).abs() <= 2 * lr + 1e-7).all()
            assert ((p0[0] - p1[0]).norm() / p0[0].norm()).item() < 1e-5
        finally:
            os.chdir(cwd)


@pytest.mark.parametrize("mode", ["start", "split", "late"])
def test_frontier_ahead_matches_serial_step(mode):
    """The step graph that also computes the next batch's frontier (from the
    sampler's speculative draw; each PINSAGE_FRONTIER_AHEAD placement of that
    branch) trains exactly like the serial step: same
    losses and parameters (within rounding: the CSR fill order uses atomics),
    with look-ahead hits; a batch that is not the predicted one (here a
    caller-made batch) falls back to its own frontier first.  Parameters:
    Adam moves an element by at most lr per step, and an element whose
    gradient is at rounding level moves by +-lr with a sign the rounding
    picks, so the bound is 2 lr per step elementwise, and the relative norm of
    the difference (such elements included) stays below 2e-4 (measured
    0.9-1.2e-4 after six steps, differing between runs with the CSR order)."""
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(6000, 1500, 40000, seed=31)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(6000, 128, seed=32))
    pos = torch.from_numpy(synthetic.make_positives(pg, 30000, seed=33))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp,
                                        nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)

            def run(ahead):
                torch.manual_seed(5)
                tr = pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)
                tr.batch_size = 256
                tr._fused = f = pt._FusedStep(tr)
                f.ahead = ahead
                f.ahead_mode = mode
                f.autotune = False  # the same GEMM choices in both runs
                torch.manual_seed(6)
                losses = []
                for s in range(6):
                    batch, _ = tr.next_batch()
                    if s == 4:  # not what the sampler predicted
                        batch = batch.flip(0).contiguous()
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                return losses, f.runner.flat.detach().clone(), f.ahead_hits

            l0, p0, h0 = run(False)
            l1, p1, h1 = run(True)
            assert h0 == 0 and h1 >= 2
            for a, b in zip(l0, l1):
                assert abs(a - b) <= 1e-4 * abs(a) + 1e-7
            assert ((p0 - p1).abs() <= 2 * 1e-4 * 6 + 1e-7).all()
            assert ((p0 - p1).norm() / p0.norm()).item() < 2e-4
        finally:
            os.chdir(cwd)


@pytest.mark.parametrize("var,a,b", [("PINSAGE_DEFER_SIDE", "0", "3"), ("PINSAGE_DQ_CHUNK_ROWS", "0", "1"),
                                     ("PINSAGE_FUSED_NEXT_Q", "0", "1"), ("PINSAGE_HEAD_IN_AGGW", "0", "1"),
                                     ("PINSAGE_FORK_PLAN", "0", "7"), ("PINSAGE_FORK_PLAN", "0", "3"),
                                     ("PINSAGE_KW_SIDE_FORM", "0", "1"), ("PINSAGE_DQ_TREE", "0", "1"),
                                     ("PINSAGE_WGRAD_PLANES", "0", "1"), ("PINSAGE_Q0_ILV", "0", "1"),
                                     ("PINSAGE_KW_SIDE_WG", "128", "256")])
def test_engine_variants_train_alike(var, a, b, monkeypatch):
    """Engine variants that change only launch order or summation order train
    alike -- same published losses (the monitors' output) and parameters within
    rounding (CSR fill order), GEMM choices from the size model in both runs:
    PINSAGE_DEFER_SIDE (engine.hip fork_side / run_pend: when the backward's
    side launches and the loss monitors are enqueued, not what they wait for)
    and PINSAGE_DQ_CHUNK_ROWS (the bottom layer's Q weight gradient summed
    over masked dq chunk partials instead of combined dpq rows) and
    PINSAGE_FUSED_NEXT_Q (layer 1's Q projection inside layer 0's 32-row
    aggregation + W kernel, that form forced here) and PINSAGE_HEAD_IN_AGGW
    (the model head's forward inside the top layer's 16-row tile, exact fp32
    MFMAs in another k order than head_fwd_kernel's) and PINSAGE_FORK_PLAN
    (side launches merged into fewer forks: the same kernels on the same data,
    so bitwise) and PINSAGE_KW_SIDE_FORM (the side weight gradients as 4-wave
    workgroups: another wave-partial order) and PINSAGE_DQ_TREE (split dq rows
    summed by their chunk waves as a fan-in-8 tree instead of dq_combine's
    strided wave sums) and PINSAGE_WGRAD_PLANES (the layer-0 Q weight
    gradient on pre-split bf16 planes of dpq and of the features: the same
    products, 4-wave partial order) and PINSAGE_Q0_ILV (the layer-0 Q
    projection on the feature table's interleaved split, Q0 split per step:
    the same products, no stream-K) and PINSAGE_KW_SIDE_WG (the side weight
    gradients' grid target: other K-split counts, so other summation order)."""
    if var != "PINSAGE_HEAD_IN_AGGW":  # (the head is fused into the 16-row form only)
        monkeypatch.setenv("PINSAGE_AGGW32_MIN_ROWS", "0")
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(6000, 1500, 40000, seed=41)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(6000, 128, seed=42))
    pos = torch.from_numpy(synthetic.make_positives(pg, 30000, seed=43))
    old = {k: os.environ.get(k) for k in (var, "PINSAGE_AUTOTUNE")}
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp,
                                        nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)
            os.environ["PINSAGE_AUTOTUNE"] = "0"

            def run(mode):
                os.environ[var] = mode  # read when the engine is built
                torch.manual_seed(5)
                tr = pt.PinSage(g, 6000, feats, pos, log=False, load_save=False)
                tr.batch_size = 256
                torch.manual_seed(6)
                losses = []
                for _ in range(5):
                    batch, _ = tr.next_batch()
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                return losses, tr._fused.runner.flat.detach().clone()

            l0, p0 = run(a)
            l1, p1 = run(b)
            if var == "PINSAGE_FORK_PLAN":
                assert l0 == l1 and torch.equal(p0, p1)
            assert all(v > 0 for v in l0)
            for x, y in zip(l0, l1):
                assert abs(x - y) <= 1e-4 * abs(x) + 1e-7
            assert ((p0 - p1).norm() / p0.norm()).item() < 1e-4
        finally:
            os.chdir(cwd)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


def test_train_step_three_layers_fanout_50_vs_oracle():
    """The C5 shape (BASELINE.json configs[4]: 3 layers, fanout 50) at a size the
    CPU oracle finishes in seconds: 3000 tracks, d_in 128 (>= out, as put_embeddings needs), batch 32, so the bottom
    frontier covers the whole graph and popular tracks fill thousands of slots.
    Margin 3 keeps every triple on the hinge's linear side (at the reference's
    1e-5 a fresh model sits within rounding of the kink; test_gpu_fullsize.py).
    Loss and gradients within 1e-4 (measured ~4e-6)."""
    import graph
    import pinsage_model as pm
    import pinsage_training as pt
    import synthetic
    from oracle import oracle as orc
    n, T, L, d_in, B = 3000, 50, 3, 128, 32
    pg = synthetic.make_playlist_graph(n, 750, 40000, seed=7)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(n, d_in, seed=8))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * n, seed=9))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            pm.set_rng_mode("philox")
            torch.manual_seed(0)
            w, nb = pm.precompute_neighborhoods_topt(g, n, 200, 0.85, 100, g.nbhds_path)
            pm.set_rng_mode("mt19937")
            torch.manual_seed(1)
            tr = pt.PinSage(g, n, feats.cuda(), pos, log=False, load_save=False)
            tr.T, tr.n_layers = T, L
            torch.manual_seed(2)
            tr.model = pm.PinSageModel(g, tr.n, L, tr.dimensions, tr.n_hops, tr.alpha, T, tr.nbhds)
            # The reference init (biases 0.3) collapses a fresh 3-layer model: its outputs
            # agree to |q_hat - p_hat| ~ 3e-3, so the loss gradient (differences of nearly
            # equal unit vectors) is ill-conditioned and any fp32 reordering -- torch's own
            # autograd through this engine included -- moves it by ~1e-4
            # (tools/check_l3_trainer.py).  Zero biases and 3x weights spread the outputs
            # (|q_hat - p_hat| ~ 0.17), where the comparison measures the kernels.
            with torch.no_grad():
                for k, prm in tr.model.named_parameters():
                    prm.zero_() if k.endswith("bias") else prm.mul_(3.0)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.batch_size = B
            tr.margin = 3.0
            init = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
            assert len(init) == 4 * L + 3
            ref = orc.RefTrainer(init, feats, w.numpy(), nb.numpy(), n_layers=L, T=T, margin=3.0)
            torch.manual_seed(3)
            for s in range(2):
                batch, _ = tr.next_batch()
                loss, nfl, _ = tr.train_batch(batch)
                rl, rn, _, rg = ref.step(batch.numpy())
                assert abs(float(loss) - rl) <= REL_TOL * abs(rl) + 1e-7, (s, float(loss), rl)
                assert abs(float(nfl) - rn) <= REL_TOL * abs(rn) + 1e-7
                if s == 0:  # after an Adam step, ulp-level differences are lr-scaled (see above)
                    errs = {k: _rel(prm.grad.cpu().numpy(), rg[k].numpy())
                            for k, prm in tr.model.named_parameters()}
                    assert all(e < REL_TOL for e in errs.values()), errs
        finally:
            os.chdir(cwd)


@pytest.mark.parametrize("mode", ["mt19937", "philox"])
@pytest.mark.parametrize("k", [10, 100, 1000])
def test_fused_ppr_topk_matches_walk_plus_topk(mode, k):
    """pinsage_ppr_topk (walk + counts + heap replay in one pass, trace in LDS,
    one lane per source for the heap) against do_random_walks' trace fed to the
    visit_topk kernel and against the oracle: bit-exact, same RNG consumption,
    including the normalised device-table outputs (t_norm)."""
    import graph
    import pinsage_model as pm
    import synthetic
    from oracle import oracle as orc
    pg = synthetic.make_playlist_graph(70000, 10000, 300000, seed=31)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices)
    src = torch.from_numpy(np.random.default_rng(k).integers(0, 70000, 700).astype(np.int64))
    pm.set_rng_mode(mode)
    try:
        torch.manual_seed(99)
        w, nb, wn, nb32 = pm._ppr_topk_device(g, src, 500, 0.85, k, t_norm=min(k, 25))
        after_fused = torch.get_rng_state()
        torch.manual_seed(99)
        s2, trace = pm._walk_device(g, src, 500, 0.85)
        w2, nb2, wn2, nb322 = pm._topk_device(s2, trace, pg.n_all, 500, k, t_norm=min(k, 25))
        assert torch.equal(after_fused, torch.get_rng_state())
    finally:
        pm.set_rng_mode("mt19937")
    assert torch.equal(w, w2) and torch.equal(nb, nb2)
    assert torch.equal(wn, wn2) and torch.equal(nb32, nb322)
    if mode == "mt19937":
        rw, rn = orc.sample_neighborhood_topt(indptr, indices, pg.n_all, src.numpy()[:48], 500, 0.85, k,
                                              orc.MT(99))
        assert (w[:48].cpu().numpy() == rw).all() and (nb[:48].cpu().numpy() == rn).all()


@pytest.mark.parametrize("dims,T,n", [((24, 16, 32), 4, 300), ((128, 128, 512), 10, 700), ((256, 128, 512), 50, 200),
                                      # out_dim wider than the fused L2-norm epilogue: grid_search.py:130 and
                                      # dashboard.py:137 (out 256, hidden 1024), pinsage_model.py:285 (hidden
                                      # 1024, out 512)
                                      ((128, 256, 1024), 10, 300), ((96, 512, 1024), 3, 50)])
def test_conv_layer_autograd_vs_oracle(dims, T, n):
    """Standalone ConvLayer (pinsage_model.py:171-212) trained through autograd:
    output, every parameter gradient and the gradient of h (a wider h than
    in_dim; repeated nodeset rows) vs the oracle's ConvLayer under a fixed
    random cotangent, at the reference init (xavier, bias 0.3)."""
    import pinsage_model as pm
    from oracle import oracle as orc
    d_in, out, hid = dims
    rng = np.random.default_rng(d_in + T)
    n_items = 5000
    torch.manual_seed(d_in)
    conv = pm.ConvLayer(d_in, out, hid).cuda()
    h = torch.from_numpy(rng.standard_normal((n_items, d_in + 8)).astype(np.float32))
    ns = rng.integers(0, n_items, n)
    ns[3] = ns[7]
    nb = rng.integers(0, n_items, (n, T))
    w = rng.integers(1, 60, (n, T)).astype(np.float64) / 500.0
    c = torch.from_numpy(rng.standard_normal((n, out)).astype(np.float32))
    hg = h.cuda().requires_grad_()
    y = conv(hg, torch.from_numpy(ns), torch.from_numpy(nb), torch.from_numpy(w))
    (y * c.cuda()).sum().backward()
    p = {f"conv_layers.0.{k}": v.detach().cpu().clone().requires_grad_() for k, v in conv.state_dict().items()}
    hr = h.clone().requires_grad_()
    yr = orc.conv_layer(p, 0, hr, torch.from_numpy(ns), torch.from_numpy(nb), torch.from_numpy(w), d_in)
    (yr * c).sum().backward()
    assert _rel(y.detach().cpu().numpy(), yr.detach().numpy()) < REL_TOL
    for k, prm in conv.named_parameters():
        assert _rel(prm.grad.cpu().numpy(), p[f"conv_layers.0.{k}"].grad.numpy()) < REL_TOL, k
    assert _rel(hg.grad.cpu().numpy(), hr.grad.numpy()) < REL_TOL
    assert float(hg.grad[:, d_in:].abs().max()) == 0.0


def test_csr_transpose_ranges_match_atomic_path():
    """The backward's CSR transpose of the neighbour slots (conv.hip
    csr_count_kernel / csr_fill_kernel) beyond one LDS histogram (> 40960
    distinct layer-0 neighbours): the (range, slice) histogram path trains like
    the per-wave global-atomic path (PINSAGE_CSR_RANGES=0) -- same published
    losses and parameters within rounding (both fill rows in atomic order)."""
    import graph
    import pinsage_training as pt
    import synthetic
    n = 100000
    pg = synthetic.make_playlist_graph(n, 25000, 1000000, seed=51)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(n, 128, seed=52))
    pos = torch.from_numpy(synthetic.make_positives(pg, 400000, seed=53, csr=(indptr, indices)))
    old = os.environ.get("PINSAGE_CSR_RANGES")
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp,
                                        nbhds_path=os.path.join(tmp, "nb.pt"))
            import pinsage_model as pm
            pm.set_rng_mode("philox")
            try:
                pt.PinSage(g, n, feats, pos, log=False, load_save=False)
            finally:
                pm.set_rng_mode("mt19937")

            def run(mode):
                if mode is None:
                    os.environ.pop("PINSAGE_CSR_RANGES", None)
                else:
                    os.environ["PINSAGE_CSR_RANGES"] = mode
                torch.manual_seed(5)
                tr = pt.PinSage(g, n, feats, pos, log=False, load_save=False)
                # fanout 50 (C5's): top-T PPR neighbours concentrate on popular
                # tracks, so a wide T is what makes the layer-0 set this large
                tr.model = pm.PinSageModel(g, n, 2, tr.dimensions, tr.n_hops, tr.alpha, 50, tr.nbhds)
                tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
                tr.batch_size = 4096
                torch.manual_seed(6)
                losses = []
                for _ in range(3):
                    batch, _ = tr.next_batch()
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                f = tr._fused
                eng = f.runner.engine
                u0 = max(int(eng.view(ws, int(eng.off.count_N[0]), torch.int32, 1).item()) for ws in f.wss)
                return losses, f.runner.flat.detach().clone(), u0

            l0, p0, u0 = run("0")
            l1, p1, u1 = run(None)
            assert u0 > 40960 and u1 > 40960, (u0, u1)
            for a, b in zip(l0, l1):
                assert abs(a - b) <= 1e-4 * abs(a) + 1e-7
            assert ((p0 - p1).norm() / p0.norm()).item() < 1e-4
        finally:
            os.chdir(cwd)
            if old is None:
                os.environ.pop("PINSAGE_CSR_RANGES", None)
            else:
                os.environ["PINSAGE_CSR_RANGES"] = old


def test_default_step_is_bitwise_reproducible():
    """two fresh trainers with the default in-context GEMM
    tuner ON and the same seeds end 3 fused steps with bitwise-equal
    parameters and losses.  What makes it hold: the tuner's candidates keep
    every site's summation order (tile configs only; split-K counts and
    stream-K stay the size model's), the backward's CSR pairs are sorted by
    source row (canonical transposed-aggregation order), and a node repeated
    inside a call has its per-position loss gradients summed in position order
    by the last contributor (no float atomics).  The batch (512 triples over
    3000 tracks) repeats nodes three and more times per call, and popular
    tracks split over several CSR chunks."""
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(3000, 600, 20000, seed=61)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(3000, 256, seed=62))
    pos = torch.from_numpy(synthetic.make_positives(pg, 15000, seed=63))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        old = os.environ.pop("PINSAGE_AUTOTUNE", None)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)  # (precompute the table once)

            def run():
                torch.manual_seed(5)
                tr = pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)
                tr.batch_size = 512
                torch.manual_seed(6)
                losses, reps = [], 0
                for _ in range(3):
                    batch, _ = tr.next_batch()
                    for c in range(3):
                        reps = max(reps, int(torch.bincount(batch[:, c].reshape(-1)).max()))
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                assert tr._fused.tuned_choices is not None  # the tuner ran
                return losses, torch.cat([p.detach().flatten() for p in tr.model.parameters()]).cpu(), reps

            l0, p0, reps = run()
            l1, p1, _ = run()
            assert reps >= 3, reps
            assert l0 == l1, (l0, l1)
            assert torch.equal(p0, p1), (p0 - p1).abs().max().item()
        finally:
            os.chdir(cwd)
            if old is not None:
                os.environ["PINSAGE_AUTOTUNE"] = old


def test_head_sums_repeated_ranks_bitwise():
    """The fused head backward sums a repeated batch node's per-position loss
    rows itself (head.hip head_fetch_dz, from zero in position order) instead
    of a rep_sum_kernel launch between the loss and it (PINSAGE_HEAD_REP_SUM=0):
    the same additions in the same order, so three steps end with bitwise-equal
    parameters and losses.  GEMM choices from the size model in both runs; the
    batch repeats nodes three and more times per call."""
    import graph
    import pinsage_training as pt
    import synthetic
    pg = synthetic.make_playlist_graph(3000, 600, 20000, seed=61)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(3000, 256, seed=62))
    pos = torch.from_numpy(synthetic.make_positives(pg, 15000, seed=63))
    old = {k: os.environ.get(k) for k in ("PINSAGE_HEAD_REP_SUM", "PINSAGE_AUTOTUNE")}
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)
            os.environ["PINSAGE_AUTOTUNE"] = "0"

            def run(mode):
                os.environ["PINSAGE_HEAD_REP_SUM"] = mode  # read when the engine is built
                torch.manual_seed(5)
                tr = pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)
                tr.batch_size = 512
                torch.manual_seed(6)
                losses, reps = [], 0
                for _ in range(3):
                    batch, _ = tr.next_batch()
                    for c in range(3):
                        reps = max(reps, int(torch.bincount(batch[:, c].reshape(-1)).max()))
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                return losses, torch.cat([p.detach().flatten() for p in tr.model.parameters()]).cpu(), reps

            l0, p0, reps = run("0")
            l1, p1, _ = run("1")
            assert reps >= 3, reps
            assert l0 == l1, (l0, l1)
            assert torch.equal(p0, p1), (p0 - p1).abs().max().item()
        finally:
            os.chdir(cwd)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
