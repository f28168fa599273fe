"""torch.ops.pinsage (the PyTorch-ROCm operator library, csrc/torch_ops.cpp)
against the paths the other tests pin: ppr_topk bit-exact against the
sampler's Philox path (whose MT19937 twin is pinned by the reference's
fixtures), frontier against relevant_nodes_per_layer_precomp, linear / gemm /
weighted_agg / segment_wmean and the registered autograd formulas against
float64 torch."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph():
    import graph
    import synthetic
    pg = synthetic.make_playlist_graph(3000, 750, 40000, seed=71)
    indptr, indices = pg.csr()
    return pg, graph.CSRGraph.from_csr(indptr, indices), indptr, indices


def test_ppr_topk_op_matches_sampler():
    import pinsage_model as pm
    import pinsage_ops
    pinsage_ops.load()
    pg, g, indptr, indices = _graph()
    src = torch.arange(0, 3000, 7, dtype=torch.int64, device="cuda")
    seed = 0x1234_5678_9abc
    w_ref, nb_ref, _, _ = pm._ppr_topk_device(g, src, 300, 0.85, 25, philox=(seed, 0))
    ip, ix = (torch.from_numpy(a).cuda() for a in (indptr, indices))
    w, nb = torch.ops.pinsage.ppr_topk(ip, ix, src, 300, 0.85, 25, seed, 0)
    assert torch.equal(nb, nb_ref) and torch.equal(w, w_ref)


def test_frontier_op_matches_precomp_frontier():
    import pinsage_model as pm
    import pinsage_ops
    pinsage_ops.load()
    rng = np.random.default_rng(5)
    n, T = 5000, 10
    nb = torch.from_numpy(rng.integers(0, n, (n, 100)))
    w = torch.from_numpy(rng.random((n, 100)))
    nodes = torch.from_numpy(rng.integers(0, n, 300))
    S = pm.relevant_nodes_per_layer_precomp(nodes, 2, T, (w, nb))
    out = torch.ops.pinsage.frontier(nodes.cuda(), nb[:, :T].to(torch.int32).contiguous().cuda(), T, n)
    assert torch.equal(out.cpu(), S[0][0].to(torch.int64))


def test_linear_and_agg_ops_with_autograd():
    import pinsage_ops
    pinsage_ops.load()
    ops = torch.ops.pinsage
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(700, 72, device="cuda", generator=g).requires_grad_()
    rows = torch.randint(0, 700, (333,), device="cuda", generator=g, dtype=torch.int32)
    W = torch.randn(48, 64, device="cuda", generator=g).requires_grad_()
    b = torch.randn(48, device="cuda", generator=g).requires_grad_()
    y = ops.linear(x, rows, W, b, True)
    loc = torch.randint(0, 333, (200, 7), device="cuda", generator=g, dtype=torch.int32)
    w = torch.rand(200, 7, device="cuda", generator=g) + 0.1
    w = w / w.sum(1, keepdim=True)
    agg = ops.weighted_agg(y, loc, w)
    c = torch.randn(200, 48, device="cuda", generator=g)
    (agg * c).sum().backward()
    # float64 torch reference of the same composition
    xd, Wd, bd = (t.detach().double().requires_grad_() for t in (x, W, b))
    yd = torch.nn.functional.leaky_relu(xd[rows.long(), :64] @ Wd.t() + bd, 0.01)
    aggd = (w.double()[:, :, None] * yd[loc.long()]).sum(1)
    (aggd * c.double()).sum().backward()

    def rel(a, r):
        return ((a.double() - r).norm() / r.norm()).item()
    assert rel(agg.detach(), aggd.detach()) < 1e-5
    assert rel(x.grad, xd.grad) < 1e-5 and float(x.grad[:, 64:].abs().max()) == 0.0
    assert rel(W.grad, Wd.grad) < 1e-5 and rel(b.grad, bd.grad) < 1e-5


def test_gemm_and_segment_ops():
    import pinsage_ops
    pinsage_ops.load()
    ops = torch.ops.pinsage
    g = torch.Generator(device="cuda").manual_seed(9)
    A = torch.randn(260, 128, device="cuda", generator=g)   # M-major A: [K][M]
    B = torch.randn(500, 96, device="cuda", generator=g)    # N-major B, k-rows gathered
    bi = torch.randint(0, 500, (260,), device="cuda", generator=g, dtype=torch.int32)
    C = ops.gemm(A, False, None, B, False, bi, 128, 96, 260)
    ref = A.double().t() @ B.double()[bi.long()]
    assert ((C.double() - ref).norm() / ref.norm()).item() < 1e-5
    h = torch.randn(50, 32, device="cuda", generator=g)
    seg = torch.tensor([0, 3, 3, 7], dtype=torch.int64, device="cuda")
    cols = torch.randint(0, 50, (7,), device="cuda", generator=g, dtype=torch.int32)
    w = torch.rand(7, device="cuda", generator=g)
    out = ops.segment_wmean(h, seg, cols, w, False)
    exp = torch.stack([(w[s:e, None].double() * h[cols[s:e].long()].double()).sum(0)
                       for s, e in ((0, 3), (3, 3), (3, 7))])
    assert torch.allclose(out.double(), exp, rtol=1e-6, atol=1e-6)
