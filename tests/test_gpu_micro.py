"""The C5 path pieces (100M nodes / 1B edges, d_in 256,
3 layers, fanout 50): the micro-batched train step with recompute
(PinSage.micro_batch), the device-resident neighbourhood table
(precompute_device_table) and the device-built synthetic graph, each pinned
against the oracle or against the paths the other tests pin."""
import os
import tempfile

import numpy as np
import pytest
import torch

import parity_util
from parity_util import check_record, make_trainer

pytestmark = pytest.mark.gpu


def _problem(tmp, n, n_cols, memb, d_in, seed, hops=300):
    import graph
    import pinsage_model as pm
    import synthetic
    pg = synthetic.make_playlist_graph(n, n_cols, memb, seed=seed)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(n, d_in, seed=seed + 1))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * n, seed=seed + 2, csr=(indptr, indices)))
    pm.set_rng_mode("philox")
    try:
        torch.manual_seed(seed + 3)
        w, nb = pm.precompute_neighborhoods_topt(g, n, hops, 0.85, 100, g.nbhds_path)
    finally:
        pm.set_rng_mode("mt19937")
    return g, feats, pos, w, nb


@pytest.fixture
def tmpdir_cwd():
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            yield tmp
        finally:
            os.chdir(cwd)


def _batch_with_repeats(tr, seed):
    torch.manual_seed(seed)
    batch, _ = tr.next_batch()
    b = batch.clone()
    b[1, 0] = b[2, 0]          # a repeated query inside the first slice
    b[40, 0] = b[2, 0]         # ... and in a later slice
    b[33, 2] = b[5, 1]         # one id in two calls and two slices
    return b


def _record(tr, b, run):
    init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
    loss, _, _ = run(b)
    grads = {k: p.grad.detach().cpu().numpy().astype(np.float64) for k, p in tr.model.named_parameters()}
    Zd = tr.last_outputs.permute(1, 0, 2)
    Z = Zd.cpu().double()
    # the arguments as the sliced step's loss evaluated them (torch fp32 on the device)
    hinge = parity_util._hinge_args(Zd[:, 0], Zd[:, 1], Zd[:, 2], tr.margin).double().cpu().numpy()
    return dict(init=init, batch=b.numpy(), grads=grads, loss=float(loss), Z=Z.numpy(), hinge=hinge,
                L=tr.n_layers, T=tr.T, margin=float(tr.margin), out_dim=tr.out_dim)


def test_micro_batched_step_c5_shape_vs_oracle(tmpdir_cwd):
    """3 layers, fanout 50, d_in 256, reference init and margin, in slices of
    16 triples with repeated ids inside and across slices: forward rows, hinge
    arguments, loss and gradients vs the oracle's full-batch reference step,
    with the tolerances of the unsliced C5-shape test (test_gpu_configs)."""
    n = 4000
    g, feats, pos, w, nb = _problem(tmpdir_cwd, n, 1000, 50000, 256, seed=21)
    tr = make_trainer(g, n, feats.cuda(), pos, 3, 50, 64, margin=1e-5, seed=7)
    tr.micro_batch = 16
    b = _batch_with_repeats(tr, 8)
    rec = _record(tr, b, tr.train_batch)
    res = check_record(rec, feats, w.numpy(), nb.numpy(), strict_a=False)
    assert res["grad_rel_A_max"] <= 1e-3, res


def test_micro_batched_backward_fixed_cotangent_c5_shape(tmpdir_cwd):
    """The micro-batched step's backward (PinSage._micro_backward: slices of 16
    triples with recompute, repeated ids inside and across slices) at the C5
    shape (3 layers, fanout 50, d_in 256) and the reference init, under a fixed
    random cotangent on the three calls' outputs: every parameter gradient
    within 1e-4 of the oracle's autograd (pinsage_model.py:246-265 per call,
    index_put's repeated-id semantics).  The random cotangent removes the
    hinge's conditioning (test_micro_batched_step_c5_shape_vs_oracle), so this
    pins the sliced kernels themselves at the north star's tolerance."""
    from oracle import oracle as orc
    n = 4000
    g, feats, pos, w, nb = _problem(tmpdir_cwd, n, 1000, 50000, 256, seed=21)
    tr = make_trainer(g, n, feats.cuda(), pos, 3, 50, 64, margin=1e-5, seed=7)
    tr.micro_batch = 16
    b = _batch_with_repeats(tr, 8)
    B = b.shape[0]
    init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
    c = torch.from_numpy(np.random.default_rng(5).standard_normal((3, B, tr.out_dim)).astype(np.float32))
    ids = b.t().contiguous().cuda()
    tr._micro_backward(ids, c.cuda())
    torch.cuda.synchronize()
    p = {k: v.float().requires_grad_() for k, v in init.items()}
    tot = 0.0
    for j in range(3):
        y = orc.model_forward(p, feats, b[:, j].numpy(), 3, 50, w.numpy(), nb.numpy(), tr.out_dim)
        tot = tot + (y * c[j]).sum()
    tot.backward()
    errs = {k: parity_util.rel(prm.grad.cpu().numpy(), p[k].grad.numpy())
            for k, prm in tr.model.named_parameters()}
    assert max(errs.values()) <= 1e-4, errs


@pytest.mark.parametrize("L,T,m", [(2, 10, 7), (3, 50, 16)])
def test_micro_batched_step_equals_fused_step(tmpdir_cwd, L, T, m):
    """The sliced step against the one-launch fused step on the same batch and
    parameters (spread init: well-conditioned outputs): loss, every gradient
    and the parameters after Adam agree to fp32 summation-order level."""
    n = 4000
    g, feats, pos, w, nb = _problem(tmpdir_cwd, n, 1000, 50000, 128, seed=31)
    trs = [make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
           for _ in range(2)]
    trs[0].micro_batch = m
    b = _batch_with_repeats(trs[0], 12)
    outs = [tr.train_batch(b) for tr in trs]
    torch.cuda.synchronize()
    l0, l1 = float(outs[0][0]), float(outs[1][0])
    # the sliced forward's rows are bitwise the whole batch's
    # (tools/dbg/micro_z.py) and its loss runs the step's own loss kernels
    # (pinsage_triplet_loss), so the loss agrees to the fused step's rounding
    assert abs(l0 - l1) <= 1e-5 * abs(l1) + 1e-8, (l0, l1)
    p0, p1 = dict(trs[0].model.named_parameters()), dict(trs[1].model.named_parameters())
    for k in p0:
        a, c = p0[k].grad.double().cpu().numpy(), p1[k].grad.double().cpu().numpy()
        assert parity_util.rel(a, c) <= 1e-5, (k, parity_util.rel(a, c))
        assert torch.allclose(p0[k].detach(), p1[k].detach(), rtol=0, atol=2.1e-4), k  # Adam: +-lr on ~0 gradients
    assert abs(float(outs[0][2]) - float(outs[1][2])) <= 1e-4 * abs(float(outs[1][2])) + 1e-9


@pytest.mark.parametrize("mode", ["philox", "mt19937"])
@pytest.mark.parametrize("T", [10, 50])
def test_device_table_equals_host_precompute(tmpdir_cwd, mode, T):
    """precompute_device_table = precompute_neighborhoods_topt(...)[:, :T]
    (nodes bit-exact, weights normalised over T within f32 rounding), the
    generator left where the host precompute leaves it."""
    import pinsage_model as pm
    n = 3000
    g, _, _, _, _ = _problem(tmpdir_cwd, n, 750, 40000, 16, seed=41)
    pm.set_rng_mode(mode)
    try:
        torch.manual_seed(5)
        w, nb = pm.precompute_neighborhoods_topt(g, n, 200, 0.85, 100, None)
        after = torch.get_rng_state()
        torch.manual_seed(5)
        tab = pm.precompute_device_table(g, n, 200, 0.85, T, chunk=1000)
        assert torch.equal(torch.get_rng_state(), after)
    finally:
        pm.set_rng_mode("mt19937")
    assert torch.equal(tab.nb32.cpu(), nb[:, :T].to(torch.int32))
    ref = (w[:, :T] / w[:, :T].sum(1, keepdim=True)).float()
    assert torch.allclose(tab.wn.cpu(), ref, rtol=1e-6, atol=0)


def test_resident_table_step_equals_host_table_step(tmpdir_cwd):
    """A trainer given the device-resident table (PinSage(..., nbhds=...))
    trains like one built from the host table."""
    import pinsage_model as pm
    import pinsage_training as pt
    n = 4000
    g, feats, pos, w, nb = _problem(tmpdir_cwd, n, 1000, 50000, 128, seed=51)
    tab = pm._DeviceTable.resident(nb[:, :10].to(torch.int32).cuda().contiguous(),
                                   (w[:, :10] / w[:, :10].sum(1, keepdim=True)).float().cuda().contiguous())
    out = []
    for nbhds in ((w, nb), tab):
        torch.manual_seed(3)
        tr = pt.PinSage(g, n, feats.cuda(), pos, log=False, load_save=False, nbhds=nbhds)
        tr.T = 10
        torch.manual_seed(4)
        tr.model = pm.PinSageModel(g, n, 2, tr.dimensions, tr.n_hops, tr.alpha, 10, tr.nbhds)
        tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
        tr.batch_size = 128
        torch.manual_seed(6)
        batch, _ = tr.next_batch()
        loss = float(tr.train_batch(batch)[0])
        out.append((loss, {k: p.grad.detach().cpu().clone() for k, p in tr.model.named_parameters()}))
    # same kernels, but each trainer's GEMM tuner may pick other split-K counts
    assert abs(out[0][0] - out[1][0]) <= 1e-6 * abs(out[1][0])
    for k in out[0][1]:
        assert parity_util.rel(out[0][1][k].numpy(), out[1][1][k].numpy()) <= 1e-5, k


def test_strided_nodeset_is_read_as_given(tmpdir_cwd):
    """A nodeset passed as a strided view (a column of a [B, 3] batch, or a row
    of its transpose reshaped) is the ids it shows, not the memory behind its
    first element (the runner hands the C-ABI a contiguous copy)."""
    n = 4000
    g, feats, pos, w, nb = _problem(tmpdir_cwd, n, 1000, 50000, 128, seed=61)
    tr = make_trainer(g, n, feats.cuda(), pos, 2, 10, 64, margin=1e-5, seed=3, spread=True)
    torch.manual_seed(2)
    b, _ = tr.next_batch()
    bt = b.t().cuda()
    with torch.no_grad():
        for view in (b[:, 1], bt[:, 5:6].reshape(-1), bt[1, ::2]):
            assert not view.is_contiguous() or view.dim() == 1
            y = tr.model(tr.features, view)
            y_ref = tr.model(tr.features, view.contiguous().clone())
            assert torch.equal(y, y_ref)


@pytest.mark.parametrize("B,d", [(1, 128), (5, 128), (64, 64), (512, 256)])
def test_triplet_loss_kernel_matches_torch(B, d):
    """pinsage_triplet_loss (the step's loss kernels on per-position rows,
    used by the micro-batched step) against torch's max_margin_loss and its
    autograd cotangent (pinsage_training.py:31-41): loss within 1e-6
    relative, cotangent within 1e-5, variance within 1e-5; hinge-inactive
    triples give zero rows."""
    import pinsage_training as pt
    g = torch.Generator(device="cuda").manual_seed(B + d)
    Z = torch.randn(3, B, d, device="cuda", generator=g)
    Z[2, ::3] = Z[1, ::3]  # some triples with the hinge exactly at the margin's side
    margin = 0.3
    loss, cot, var = pt._triplet_loss(Z, margin)
    Zr = Z.detach().requires_grad_()
    ref = pt.max_margin_loss(Zr[0], Zr[1], Zr[2], margin)
    (gref,) = torch.autograd.grad(ref, [Zr])
    torch.cuda.synchronize()
    ref = ref.detach()
    assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref)) + 1e-9, (float(loss), float(ref))
    assert ((cot - gref).norm() / gref.norm().clamp_min(1e-30)).item() <= 1e-5
    if B > 1:
        assert abs(float(var) - float(pt.batch_variance(Z[0]))) <= 1e-5 * abs(float(pt.batch_variance(Z[0])))
