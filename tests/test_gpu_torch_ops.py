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
    w, nb = torch.ops.pinsage.ppr_topk(ip, ix, src, 300, 0.85, 25, seed, 0, rng_mode="philox")
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
    # the reference's int64 table (its frontier step, pinsage_model.py:162-166) and an int32 one
    for tab in (nb.cuda(), nb[:, :T].to(torch.int32).contiguous().cuda()):
        for ns, nxt in ((nodes, S[0][0]), (S[0][0].to(torch.int64), None)):
            uniq, local_idx = torch.ops.pinsage.frontier(ns.cuda(), tab, T)
            ref = torch.cat([nb[ns, :T].flatten(), ns]).unique()
            if nxt is not None:
                assert torch.equal(ref, nxt.to(torch.int64))
            assert torch.equal(uniq.cpu(), ref)
            assert local_idx.dtype == torch.int32 and local_idx.shape == (len(ns), T)
            assert torch.equal(uniq.cpu()[local_idx.cpu().long()], nb[ns, :T])
    with pytest.raises(RuntimeError, match="T must be"):
        torch.ops.pinsage.frontier(nodes.cuda(), nb.cuda(), 101)


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


def test_walk_and_ppr_topk_ops_mt19937_match_reference_fixtures():
    """walk / ppr_topk with rng_mode="mt19937" draw from torch's global generator
    exactly as do_random_walks does (pinsage_model.py:32-53): traces and top-k
    (both libstdc++ regimes) bit-exact against the reference's own outputs, and
    the generator left where the reference leaves it."""
    import pinsage_ops
    from conftest import golden
    pinsage_ops.load()
    ops = torch.ops.pinsage
    for gname in ("small", "mid"):
        d = golden(f"walk_{gname}")
        ip, ix = torch.from_numpy(d["indptr"]).cuda(), torch.from_numpy(d["indices"]).cuda()
        ns = torch.from_numpy(d["nodeset"]).cuda()
        torch.manual_seed(int(d["seed"]))
        tr = ops.walk(ip, ix, ns, 500, 0.85, rng_mode="mt19937")
        assert tr.dtype == torch.int64 and (tr.cpu().numpy() == d["trace"]).all()
        got = np.array([int(torch.randint(2 ** 31, ())) for _ in range(len(d["after"]))])
        assert (got == d["after"]).all()
        d = golden(f"topk_{gname}")
        ip, ix = torch.from_numpy(d["indptr"]).cuda(), torch.from_numpy(d["indices"]).cuda()
        ns = torch.from_numpy(d["nodeset"]).cuda()
        for k in d["ks"]:
            torch.manual_seed(int(d["seed"]))
            w, nb = ops.ppr_topk(ip, ix, ns, int(d["n_hops"]), 0.85, int(k), rng_mode="mt19937")
            assert (w.cpu().numpy() == d[f"val_{k}"]).all(), (gname, k)
            assert (nb.cpu().numpy() == d[f"idx_{k}"]).all(), (gname, k)
        # the default rng_mode is the reference's stream
        torch.manual_seed(int(d["seed"]))
        w, nb = ops.ppr_topk(ip, ix, ns, int(d["n_hops"]), 0.85, int(d["ks"][0]))
        assert (nb.cpu().numpy() == d[f"idx_{d['ks'][0]}"]).all()
    d = golden("walk_small")
    torch.manual_seed(int(d["seed"]))
    tr = ops.walk(torch.from_numpy(d["indptr"]).cuda(), torch.from_numpy(d["indices"]).cuda(),
                  torch.from_numpy(d["nodeset"]).cuda(), 500, 0.85)
    assert (tr.cpu().numpy() == d["trace"]).all()
    with pytest.raises(RuntimeError, match="rng_mode"):
        ops.walk(ip, ix, ns, 5, 0.85, rng_mode="pcg")


def test_walk_and_ppr_topk_ops_philox_offset():
    """Philox mode keys every draw by (seed, hop, src_base + i, offset): the fused
    ppr_topk equals top-k over walk's trace at the same (seed, offset, src_base),
    a different offset gives different walks, and torch's generator is untouched."""
    import pinsage_model as pm
    import pinsage_ops
    pinsage_ops.load()
    ops = torch.ops.pinsage
    pg, g, indptr, indices = _graph()
    ip, ix = (torch.from_numpy(a).cuda() for a in (indptr, indices))
    src = torch.arange(5, 3000, 11, dtype=torch.int64, device="cuda")
    st = torch.get_rng_state()
    seed = 0xfeed_beef_1234
    tr3 = ops.walk(ip, ix, src, 200, 0.85, seed, 3, "philox", 40)
    tr0 = ops.walk(ip, ix, src, 200, 0.85, seed, 0, "philox", 40)
    assert not torch.equal(tr3, tr0)
    w, nb = ops.ppr_topk(ip, ix, src, 200, 0.85, 20, seed, 40, 3, "philox")
    w_ref, nb_ref, _, _ = pm._topk_device(src, tr3.to(torch.int32).contiguous(), g.number_of_nodes(), 200, 20)
    assert torch.equal(nb, nb_ref) and torch.equal(w, w_ref)
    assert torch.equal(st, torch.get_rng_state())


def test_gather_and_scatter_rows_ops_with_autograd():
    """gather_rows = get_embeddings' h[idx, :width] (pinsage_model.py:21-23) and its
    transpose scatter_add_rows (index_add: repeated ids summed), each the other's
    gradient, against float64 torch; out-of-range ids raise IndexError."""
    import pinsage_ops
    pinsage_ops.load()
    ops = torch.ops.pinsage
    g = torch.Generator(device="cuda").manual_seed(9)
    for n_h, d, width, n in ((500, 64, 48, 900), (37, 7, 7, 50), (1000, 130, -1, 1)):
        h = torch.randn(n_h, d, device="cuda", generator=g).requires_grad_()
        idx = torch.randint(0, n_h, (n,), device="cuda", generator=g)
        idx[0] = idx[-1]
        rows = ops.gather_rows(h, idx, width)
        w = d if width < 0 else width
        assert torch.equal(rows, h.detach()[idx, :w])
        c = torch.randn(n, w, device="cuda", generator=g)
        (rows * c).sum().backward()
        ref = torch.zeros(n_h, d, dtype=torch.float64, device="cuda")
        ref[:, :w].index_add_(0, idx, c.double())
        assert ((h.grad.double() - ref).norm() / ref.norm()).item() < 1e-6
        gr = torch.randn(n, w, device="cuda", generator=g).requires_grad_()
        s = ops.scatter_add_rows(gr, idx, n_h, d)
        (s * h.detach()).sum().backward()
        assert torch.equal(gr.grad, h.detach()[idx, :w])
    with pytest.raises(IndexError):
        ops.gather_rows(h.detach(), torch.tensor([0, n_h], device="cuda"))


def test_concat_linear_lrelu_l2norm_op_with_autograd():
    """concat_linear_lrelu_l2norm = ConvLayer's W projection (pinsage_model.py:208-210)
    with the concat read in place: y, the norms and every gradient (h rows
    repeated, h wider than d) against float64 torch."""
    import pinsage_ops
    pinsage_ops.load()
    ops = torch.ops.pinsage
    g = torch.Generator(device="cuda").manual_seed(4)
    for d, hid, out, n in ((128, 512, 128, 700), (24, 32, 16, 33), (512, 512, 128, 5)):
        h = torch.randn(900, d + 8, device="cuda", generator=g).requires_grad_()
        rows = torch.randint(0, 900, (n,), device="cuda", generator=g)
        rows[-1] = rows[0]
        agg = torch.randn(n, hid, device="cuda", generator=g).requires_grad_()
        W = (torch.randn(out, d + hid, device="cuda", generator=g) * 0.05).requires_grad_()
        b = torch.full((out,), 0.3, device="cuda").requires_grad_()
        y, nrm = ops.concat_linear_lrelu_l2norm(h, rows, agg, W, b)
        c = torch.randn(n, out, device="cuda", generator=g)
        (y * c).sum().backward()
        hd, aggd, Wd, bd = (t.detach().double().requires_grad_() for t in (h, agg, W, b))
        z = torch.nn.functional.leaky_relu(torch.cat([hd[rows, :d], aggd], 1) @ Wd.t() + bd, 0.01)
        yd = z / z.norm(dim=1, keepdim=True)
        (yd * c.double()).sum().backward()

        def rel(a, r):
            return ((a.double() - r).norm() / r.norm()).item()
        assert rel(y.detach(), yd.detach()) < 1e-5
        assert rel(nrm, z.detach().norm(dim=1)) < 1e-5
        for got, ref in ((h.grad, hd.grad), (agg.grad, aggd.grad), (W.grad, Wd.grad), (b.grad, bd.grad)):
            assert rel(got, ref) < 1e-5
        assert float(h.grad[:, d:].abs().max()) == 0.0
