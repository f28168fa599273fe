"""On-the-fly sampling inside the model and the train step (SURVEY §8f row 1;
relevant_nodes_per_layer, pinsage_model.py:142-154, the sampler the reference's
forward carries commented out at :247-249): every model call walks its own
nodeset's neighbourhoods with the fused walk + top-k kernel, consuming torch's
generator exactly like the reference, and the engine reads per-layer tables of
those draws.  Checked against the oracle's restatement (whose walk and top-k are
pinned by the fly_* / topk_* fixtures): the draws of every call of a train step
bit-exact, forward rows and the step's loss and gradients within 1e-4."""
import os
import tempfile

import numpy as np
import pytest
import torch

import parity_util

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
    return pg, g, indptr, indices, feats, pos


def _rows_rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float((np.linalg.norm(a - b, axis=1) / np.linalg.norm(b, axis=1)).max())


@pytest.mark.parametrize("L,T", [(1, 3), (2, 3), (2, 10)])
def test_forward_on_the_fly_vs_oracle(L, T):
    """Forward with on-the-fly sampling, repeated ids included (the reference's
    output rows of a repeated id are its last occurrence's), vs the oracle; the
    generator ends where the reference's does."""
    import pinsage_model as pm
    from oracle import oracle as orc
    pm.set_rng_mode("mt19937")
    with tempfile.TemporaryDirectory() as tmp:
        pg, g, indptr, indices, feats, pos = _problem(tmp)
        torch.manual_seed(1)
        m = pm.PinSageModel(g, N, L, (D_IN, 512, 128), 200, 0.85, T, None)
        assert m.sample_on_the_fly
        params = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        ids = np.random.default_rng(L * 10 + T).integers(0, N, 64)
        ids[5] = ids[40]  # a repeated id
        torch.manual_seed(123)
        with torch.no_grad():
            y = m(feats.cuda(), torch.from_numpy(ids)).cpu().numpy()
        after = torch.get_rng_state()
        mt = orc.MT(123)
        lay = orc.relevant_nodes_fly(indptr, indices, pg.n_all, ids, L, 200, 0.85, T, mt)
        ref = orc.model_forward(params, feats, ids, L, T, None, None, 128, layers=lay).numpy()
        assert _rows_rel(y, ref) < 1e-4
        mt.to_torch()  # the oracle's generator, handed to torch: the same state
        assert torch.equal(torch.get_rng_state(), after)
        # the sampled tables of the call equal the oracle's draws (per node, last occurrence)
        tabs = m.runner().fly_history[-1]
        for l in range(L):
            ns, w, nb = lay[l]
            _check_last_rows(tabs[l][0].cpu().numpy(), ns, nb)


def _check_last_rows(tab_nb, ns, nb):
    """The engine's table rows equal the oracle's draws of each node's last
    occurrence in the layer's nodeset."""
    last = {}
    for i, v in enumerate(ns):
        last[int(v)] = i
    vs = np.fromiter(last.keys(), np.int64)
    rows = np.fromiter(last.values(), np.int64)
    assert np.array_equal(tab_nb[vs], nb[rows].astype(np.int32))


@pytest.mark.parametrize("margin,repeats", [(3.0, False), (1e-5, False), (3.0, True)])
def test_train_step_on_the_fly_vs_oracle(margin, repeats):
    """PinSage.train_batch with an on-the-fly model: three calls (q, pos, neg),
    each with its own draws -- bit-exact against the oracle's draws of the same
    calls -- then loss and every gradient vs the oracle's reference step
    (margin 3: every hinge active; the reference's 1e-5: loss within 1e-4 and
    gradients over the same active set, as parity_util explains).  With
    repeats, ids recur inside a call: every occurrence walks its own
    neighbourhood and its conv output gets its id's summed cotangent."""
    import pinsage_model as pm
    import pinsage_training as pt
    from oracle import oracle as orc
    pm.set_rng_mode("mt19937")
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            pg, g, indptr, indices, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            torch.manual_seed(2)
            tr.model = pm.PinSageModel(g, N, 2, tr.dimensions, 200, 0.85, 3, None)
            tr.n_hops = 200
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.margin = margin
            init = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
            ref = orc.RefTrainer(init, feats, None, None, n_layers=2, T=3, margin=margin)
            rng = np.random.default_rng(7)
            batch = np.stack([rng.permutation(N)[:32] for _ in range(3)], 1).astype(np.int64)
            if repeats:
                batch[3, 0] = batch[10, 0] = batch[20, 0]  # three occurrences in the query call
                batch[7, 1] = batch[8, 1]
                batch[30, 2] = batch[0, 0]  # (across calls: independent draws anyway)
            outs = []
            hook = tr.model.register_forward_hook(lambda mod, inp, out: outs.append(out.detach()))
            torch.manual_seed(99)
            loss, _, _ = tr.train_batch(torch.from_numpy(batch))
            hook.remove()
            gpu_grads = {k: p.grad.detach().cpu().numpy().astype(np.float64)
                         for k, p in tr.model.named_parameters()}
            after = torch.get_rng_state()
            mt = orc.MT(99)
            rl, rg, lays = ref.step_fly(batch, (indptr, indices, pg.n_all), 200, 0.85, mt)
            mt.to_torch()
            assert torch.equal(torch.get_rng_state(), after)  # the same draws consumed
            # the draws of each call (q, pos, neg): bit-exact
            for c, tabs in enumerate(tr.model.runner().fly_history):
                for l in range(2):
                    ns, w, nb = lays[c][l]
                    _check_last_rows(tabs[l][0].cpu().numpy(), ns, nb)
            assert abs(float(loss) - rl) <= 1e-4 * abs(rl) + 1e-7, (float(loss), rl)
            # forward rows of the three calls vs the oracle's, row-norm relative
            p = {k: torch.from_numpy(v).float().requires_grad_() for k, v in init.items()}
            with parity_util.taps() as rec_taps:
                hs = [orc.model_forward(p, feats, batch[:, c], 2, 3, None, None, 128, layers=lays[c])
                      for c in range(3)]
            Z = np.stack([o.cpu().double().numpy() for o in outs], 1)
            for c in range(3):
                assert _rows_rel(Z[:, c], hs[c].detach().numpy()) < 1e-4, c
            # gradients: the oracle's backward driven by the cotangent of the GPU's
            # own outputs over the GPU's active set (parity_util, part B) -- at the
            # reference init the loss derivative of nearly collapsed rows amplifies
            # rounding, so the kernels' backward is measured with it removed.  At
            # that init the head's bias gradient is a sum over rows whose result is
            # ~1e-3 of its terms, so every gradient is held componentwise: its error
            # over the sum of its terms' absolute values (parity_util.cond_rel)
            zt = torch.from_numpy(Z.copy()).requires_grad_()
            args = parity_util._hinge_args(zt[:, 0], zt[:, 1], zt[:, 2], margin)
            mask = (args.detach() >= 0).double()
            (dz,) = torch.autograd.grad((mask * args).sum() / batch.shape[0], [zt])
            lossB = sum((hs[c] * dz[:, c].float()).sum() for c in range(3))
            gB, sB = parity_util.cond_grads(lossB, p, list(init), rec_taps)
            for k in init:
                gb = np.zeros(init[k].shape) if gB[k] is None else gB[k].double().numpy()
                a = gpu_grads[k]
                assert np.linalg.norm(a - gb) <= 1e-4 * np.linalg.norm(sB[k]) + 1e-12, (
                    k, parity_util.cond_rel(a, gb, sB[k]), parity_util.rel(a, gb))
            # the same three calls' draws under a random cotangent (well conditioned),
            # at the parameters after the step
            init_after = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
            mt2 = orc.MT(99)
            states = []
            for c in range(3):
                mt2.to_torch()
                states.append(torch.get_rng_state())
                orc.relevant_nodes_fly(indptr, indices, pg.n_all, batch[:, c], 2, 200, 0.85, 3, mt2)
            rng_c = np.random.default_rng(3)
            for c in range(3):
                ct = torch.from_numpy(rng_c.standard_normal(Z[:, c].shape).astype(np.float32))
                for prm in tr.model.parameters():
                    prm.grad = None
                # replay call c with its own draws
                torch.set_rng_state(states[c])
                yc = tr.model(tr.features, torch.from_numpy(batch[:, c]))
                (yc * ct.to(yc.device)).sum().backward()
                pc = {k: torch.from_numpy(v).float().requires_grad_() for k, v in init_after.items()}
                hr = orc.model_forward(pc, feats, batch[:, c], 2, 3, None, None, 128, layers=lays[c])
                (hr * ct).sum().backward()
                for k, prm in tr.model.named_parameters():
                    assert parity_util.rel(prm.grad.cpu().numpy(), pc[k].grad.numpy()) <= 1e-4, (c, k)
        finally:
            os.chdir(cwd)


def test_philox_merged_calls_match_per_call_walks():
    """Philox mode: the train step's three calls walk each layer in ONE
    pinsage_ppr_topk_segments call (per-call seeds drawn in the per-call order,
    pinsage_model._fly_tables_merged) -- the same draws, losses and parameters
    as walking call by call (PINSAGE_FLY_MERGE=0), and the generator ends in
    the same state; repeated ids inside and across calls."""
    import pinsage_model as pm
    import pinsage_training as pt
    pm.set_rng_mode("philox")
    old = os.environ.get("PINSAGE_FLY_MERGE")
    try:
        with tempfile.TemporaryDirectory() as tmp:
            cwd = os.getcwd()
            os.chdir(tmp)
            try:
                pg, g, indptr, indices, feats, pos = _problem(tmp)
                rng = np.random.default_rng(17)
                batches = []
                for _ in range(3):
                    b = np.stack([rng.integers(0, N, 96) for _ in range(3)], 1).astype(np.int64)
                    b[3, 0] = b[10, 0] = b[20, 0]
                    b[7, 1] = b[8, 1]
                    b[30, 2] = b[0, 0]
                    batches.append(torch.from_numpy(b))

                def run(merge):
                    os.environ["PINSAGE_FLY_MERGE"] = merge
                    torch.manual_seed(1)
                    tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
                    torch.manual_seed(2)
                    tr.model = pm.PinSageModel(g, N, 2, tr.dimensions, 200, 0.85, 5, None)
                    tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
                    tr.margin = 3.0
                    torch.manual_seed(99)
                    losses = [float(tr.train_batch(b)[0]) for b in batches]
                    torch.cuda.synchronize()
                    flat = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu()
                    return losses, flat, torch.get_rng_state()

                l0, p0, s0 = run("0")
                l1, p1, s1 = run("1")
                assert torch.equal(s0, s1)
                for a, b in zip(l0, l1):
                    assert abs(a - b) <= 1e-6 * abs(a) + 1e-9, (l0, l1)
                assert ((p0 - p1).norm() / p0.norm()).item() < 1e-6
            finally:
                os.chdir(cwd)
    finally:
        pm.set_rng_mode("mt19937")
        if old is None:
            os.environ.pop("PINSAGE_FLY_MERGE", None)
        else:
            os.environ["PINSAGE_FLY_MERGE"] = old


def test_retained_fly_graph_backward_after_another_call_with_virtual_rows():
    """an on-the-fly call with repeated ids (virtual-node rows in the
    shared feature buffer), backward with retain_graph, then another such call
    that overwrites those rows (forward + backward), then the first graph's
    second backward: its gradients equal its first bitwise (each call keeps
    its virtual rows and puts them back before its backward if overwritten)."""
    import pinsage_model as pm
    pm.set_rng_mode("mt19937")
    with tempfile.TemporaryDirectory() as tmp:
        pg, g, indptr, indices, feats, pos = _problem(tmp)
        torch.manual_seed(1)
        m = pm.PinSageModel(g, N, 2, (D_IN, 512, 128), 200, 0.85, 5, None)
        params = list(m.parameters())
        fc = feats.cuda()
        ids_a = torch.tensor([3, 77, 3, 1500, 77, 12, 3, 640])
        ids_b = torch.tensor([9, 9, 2000, 11, 2000, 9, 5, 6])
        cot = torch.randn(len(ids_a), 128, generator=torch.Generator().manual_seed(5)).cuda()
        torch.manual_seed(11)
        out = m(fc, ids_a)
        loss = (out * cot).sum()
        g1 = torch.autograd.grad(loss, params, retain_graph=True)
        torch.manual_seed(12)
        out2 = m(fc, ids_b)
        (out2 * cot).sum().backward()
        for p in params:
            p.grad = None
        loss.backward()
        for a, p in zip(g1, params):
            assert torch.equal(a, p.grad), "a retained fly graph's second backward differs"
