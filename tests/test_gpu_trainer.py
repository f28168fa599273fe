"""The trainer API around the train step (pinsage_training.py:108-339) on the
GPU: the epoch loop with its per-epoch ExponentialLR decay and per-batch
checkpoint, resuming from that checkpoint (the reference's state.pt keys and
formats), and embedding export (embed, save_embeddings / load_embeddings).
"""
import os
import tempfile
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 3000


def _problem(tmp):
    import graph
    import synthetic
    pg = synthetic.make_playlist_graph(N, 600, 20000, seed=41)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(N, 128, seed=42))  # d_in >= out_dim (reference)
    pos = torch.from_numpy(synthetic.make_positives(pg, 12000, seed=43))
    return g, feats, pos


def test_train_loop_checkpoint_and_resume():
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=True)
            tr.epochs, tr.b_per_e, tr.batch_size = 2, 3, 32
            p0 = [p.detach().clone() for p in tr.model.parameters()]
            torch.manual_seed(2)
            tr.train()
            assert (tr.e, tr.b) == (2, 0)
            assert abs(tr.optimizer.param_groups[0]["lr"] - 1e-4 * 0.95 ** 2) < 1e-15
            assert all(not torch.equal(a, b.detach()) for a, b in zip(p0, tr.model.parameters()))
            path = os.path.join("runs", tr.run_name, "state.pt")
            prog = torch.load(path, weights_only=True)
            assert set(prog) == {"epochs_done", "batches_done", "model_state", "optimizer_state"}
            # the last checkpoint was written after the last batch of epoch 2
            assert (prog["epochs_done"], prog["batches_done"]) == (1, 2)
            assert set(prog["model_state"]) == set(tr.model.state_dict())
            st = prog["optimizer_state"]["state"]
            assert all(int(float(v["step"])) == 6 for v in st.values())  # 2 epochs x 3 batches
            for k, v in tr.model.state_dict().items():
                assert torch.equal(prog["model_state"][k], v.detach().cpu()), k
            # resume: the constructor loads state.pt (reference load_model semantics)
            torch.manual_seed(1)
            tr2 = pt.PinSage(g, N, feats, pos, log=False, load_save=True)
            assert (tr2.e, tr2.b) == (1, 2)
            for a, b in zip(tr.model.parameters(), tr2.model.parameters()):
                assert torch.equal(a.detach().cpu(), b.detach().cpu())
            sd1, sd2 = tr.optimizer.state_dict(), tr2.optimizer.state_dict()
            for k in sd1["state"]:
                for kk in ("exp_avg", "exp_avg_sq"):
                    assert torch.equal(sd1["state"][k][kk].cpu(), sd2["state"][k][kk].cpu())
            # and keeps training from there (one more batch through the fused step)
            tr2.batch_size = 32
            torch.manual_seed(3)
            batch, _ = tr2.next_batch()
            loss, _, _ = tr2.train_batch(batch)
            assert np.isfinite(float(loss))
            tr2._sync_state()  # (save_model syncs the optimizer's step counters)
            assert all(int(float(v["step"])) == 7 for v in tr2.optimizer.state_dict()["state"].values())
        finally:
            os.chdir(cwd)


def test_embed_and_embedding_files():
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            ids = torch.tensor([5, 17, 5, 2999, 0])
            e = tr.embed(ids)
            assert e.shape == (5, 128)
            ref = tr.model(tr.features, ids)
            assert torch.allclose(e.cpu(), ref.detach().cpu(), rtol=1e-5, atol=1e-6)
            assert torch.allclose(e[0], e[2])                     # a repeated id, same row
            # batched branch: the reference resets ids to range(len(ids)) (pinsage_training.py:270-273)
            eb = tr.embed(ids, bsize=2)
            rng = tr.model(tr.features, torch.arange(5)).detach().cpu()
            assert torch.allclose(eb.cpu(), rng, rtol=1e-5, atol=1e-6)
            ds = types.SimpleNamespace(tracks={f"track{i:05d}": {} for i in range(N)})
            pt.save_embeddings(tr, ds, base_run_dir=os.path.join(tmp, "runs"))
            emb_dir = os.path.join(tmp, "runs", tr.run_name, "emb")
            assert len(os.listdir(emb_dir)) == N
            one = torch.load(os.path.join(emb_dir, "track00017.pt"), weights_only=True)
            assert one.shape == (128,) and one.dtype == torch.float32
            allv = pt.load_embeddings(tr, ds, base_run_dir=os.path.join(tmp, "runs"))
            full = tr.embed().detach().cpu()
            assert torch.allclose(allv, full, rtol=1e-5, atol=1e-6)
            # the exported embeddings vs the oracle's reference forward over every track
            from oracle import oracle as orc
            params = {k: v.detach().cpu() for k, v in tr.model.state_dict().items()}
            w, nb = tr.nbhds
            ref = orc.model_forward(params, feats.cpu(), np.arange(N), tr.n_layers, tr.T, np.asarray(w),
                                    np.asarray(nb), tr.out_dim).detach().numpy()
            err = np.linalg.norm(allv.numpy() - ref, axis=1) / np.linalg.norm(ref, axis=1)
            assert err.max() < 1e-4, err.max()
            # one-tensor export: the same rows, dataset order
            path = pt.save_embeddings_tensor(tr, ds, base_run_dir=os.path.join(tmp, "runs"), bsize=1000)
            assert os.path.isfile(path)
            ids_t, emb_t = pt.load_embeddings_tensor(tr, ds, base_run_dir=os.path.join(tmp, "runs"))
            assert ids_t == list(ds.tracks)
            assert torch.allclose(emb_t, allv, rtol=1e-5, atol=1e-6)
        finally:
            os.chdir(cwd)


def test_train_after_large_forward_matches_oracle():
    """A forward over more ids than the fused step's engine holds (embed() of
    every track) replaces the runner's engine; the next train_batch must rebuild
    its workspaces for it and still match the oracle's step
    (parity_util.check_train_step, reference margin and init)."""
    import pinsage_training as pt
    from parity_util import check_train_step
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            tr.batch_size = 32
            torch.manual_seed(2)
            for it in range(3):
                batch, _ = tr.next_batch()
                # B = 32, ~14 active triples: the head's gradients are short signed sums
                # (cancelling q / pos / neg cotangents), so part A (oracle forward) is held
                # to 1e-3; part B (shared cotangent, componentwise) and forward rows, hinge
                # arguments and loss stay at 1e-4 / 1e-6 (parity_util)
                res = check_train_step(tr, feats, tr.nbhds[0].numpy(), tr.nbhds[1].numpy(), batch,
                                       strict_a=False)
                assert res["grad_rel_A_max"] <= 1e-3, res
                if it == 0:
                    e = tr.embed()  # all N ids: > 3 * batch_size, a larger engine
                    assert e.shape == (N, 128) and torch.isfinite(e).all()
                    tr.model.train()
        finally:
            os.chdir(cwd)


def test_fused_step_is_an_optimizer_step_for_hooks_and_scheduler():
    """The fused step (Adam inside the step graph) behaves like the reference's
    optimizer.step() (pinsage_training.py:188-191) to callers: step pre- and
    post-hooks fire once per step, in order, and the epoch's scheduler.step()
    (:256) does not warn that it ran before optimizer.step()."""
    import warnings
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            tr.epochs, tr.b_per_e, tr.batch_size = 1, 4, 32
            events = []
            tr.optimizer.register_step_pre_hook(lambda opt, a, k: events.append("pre"))
            tr.optimizer.register_step_post_hook(lambda opt, a, k: events.append("post"))
            torch.manual_seed(2)
            with warnings.catch_warnings(record=True) as caught:
                warnings.simplefilter("always")
                tr.train()
            assert not [w for w in caught if "lr_scheduler.step()" in str(w.message)]
            assert events == ["pre", "post"] * tr.b_per_e
        finally:
            os.chdir(cwd)


def test_retained_graph_backward_twice_and_interleaved_forward():
    """PinSageModel's autograd node keeps its engine
    workspace until the node is freed, and a retained graph's second backward
    re-arms it (pinsage_engine_reset_backward), so backward(retain_graph=True)
    followed by backward -- with another forward + backward in between that
    must not take the retained workspace -- gives the first gradients again
    (bitwise: same kernels, same inputs)."""
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            m = tr.model
            params = list(m.parameters())
            ids = torch.tensor([3, 77, 3, 1500, 2999, 12, 640, 77])
            cot = torch.randn(len(ids), 128, generator=torch.Generator().manual_seed(5))
            out = m(tr.features, ids)
            loss = (out * cot).sum()
            g1 = torch.autograd.grad(loss, params, retain_graph=True)
            # another forward / backward in between (the pool must not hand it this graph's workspace)
            out2 = m(tr.features, torch.tensor([9, 10, 11, 2000]))
            out2.sum().backward()
            for p in params:
                p.grad = None
            loss.backward()
            for a, p in zip(g1, params):
                assert torch.equal(a, p.grad), "second backward of a retained graph differs"
            # and the retained graph's node frees its workspace back to the pool
            eng = m.runner().engine
            del out, loss, out2
            import gc
            gc.collect()
            assert len(eng.__dict__.get("_pool", [])) >= 1
        finally:
            os.chdir(cwd)


def test_engine_finalised_inside_a_capture():
    """an engine the cyclic garbage collector finalises while a
    stream is being captured (torch.cuda.graph, global capture mode) must
    neither invalidate the capture nor abort: pinsage_engine_destroy makes no
    HIP call (its streams / events are retired for reuse).  The engine here has
    created its side streams (one forward + backward) and sits in a reference
    cycle; gc.collect() runs inside the capture; the graph then replays and the
    engine is gone."""
    import gc
    import _native as nat
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            out = tr.model(tr.features, torch.tensor([1, 2, 3, 40]))
            out.sum().backward()  # the engine's side streams and events exist now
            torch.cuda.synchronize()
            x = torch.randn(1 << 16, device="cuda")
            graph = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            gc.disable()  # (no automatic collection before the capture's own)
            try:
                runner = tr.model.runner()
                cyc = [runner.engine]
                cyc.append(cyc)  # only the cyclic collector can free it
                runner.engine = None
                tr.model._runner = None
                del tr, out, runner, cyc
                live = nat.lib().pinsage_engine_live_count()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(graph, stream=s):
                        y = x * 2.0 + 1.0
                        gc.collect()  # finalises the unreachable engine mid-capture
                        z = y.sum()
            finally:
                gc.enable()
            graph.replay()
            torch.cuda.synchronize()
            assert abs(float(z) - float((x * 2.0 + 1.0).sum())) <= 1e-3 * abs(float(z)) + 1e-3
            assert nat.lib().pinsage_engine_live_count() < live
            # a new engine reuses the retired streams and trains normally
            torch.manual_seed(1)
            tr2 = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            tr2.batch_size = 32
            torch.manual_seed(2)
            batch, _ = tr2.next_batch()
            loss, _, _ = tr2.train_batch(batch)
            assert np.isfinite(float(loss))
        finally:
            os.chdir(cwd)


def test_native_stepper_matches_python_step_path(monkeypatch):
    """the captured step's host side as one native call
    (pinsage_stepper_step, PINSAGE_NATIVE_STEP=1, the default) and in Python
    (=0) give bitwise-equal losses and parameters over steps that use the
    look-ahead frontier (equal ahead hits); after capture an out-of-range
    batch id raises IndexError on the native path and the trainer still takes
    a valid step afterwards."""
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            monkeypatch.setenv("PINSAGE_AUTOTUNE", "0")
            pt.PinSage(g, N, feats, pos, log=False, load_save=False)  # (precompute the table once)

            def run(mode):
                monkeypatch.setenv("PINSAGE_NATIVE_STEP", mode)
                torch.manual_seed(1)
                tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
                tr.batch_size = 64
                torch.manual_seed(2)
                losses = []
                for _ in range(8):
                    batch, _ = tr.next_batch()
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                flat = torch.cat([p.detach().flatten() for p in tr.model.parameters()]).cpu()
                return tr, losses, flat, tr._fused.ahead_hits

            tr1, l1, p1, h1 = run("1")
            assert tr1._fused.stepper is not None  # the native path ran
            tr0, l0, p0, h0 = run("0")
            assert tr0._fused.stepper is None
            assert l1 == l0, (l1, l0)
            assert torch.equal(p1, p0)
            assert h1 == h0 and h1 > 0, (h1, h0)
            bad = torch.tensor([[1, 2, 3]] * 63 + [[N + 5, 2, 3]], dtype=torch.int64)
            with pytest.raises(IndexError):
                tr1.train_batch(bad)
            batch, _ = tr1.next_batch()
            loss = float(tr1.train_batch(batch)[0])
            torch.cuda.synchronize()
            assert np.isfinite(loss)
        finally:
            os.chdir(cwd)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_engine_on_second_device_after_first_device_engine_destroyed():
    """streams and events of destroyed engines are pooled per
    device; an engine built on cuda:1 after one on cuda:0 was destroyed runs
    its forward and backward on cuda:1 streams."""
    import gc
    import pinsage_training as pt
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g, feats, pos = _problem(tmp)
            torch.manual_seed(1)
            tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
            out = tr.model(tr.features, torch.tensor([1, 2, 3, 40]))
            out.sum().backward()
            torch.cuda.synchronize()
            del tr, out
            gc.collect()
            with torch.cuda.device(1):
                torch.manual_seed(1)
                tr = pt.PinSage(g, N, feats.to("cuda:1"), pos, log=False, load_save=False)
                out = tr.model(tr.features, torch.tensor([1, 2, 3, 40]))
                out.sum().backward()
                torch.cuda.synchronize()
                assert out.device.index == 1
                assert all(torch.isfinite(p.grad).all() for p in tr.model.parameters())
        finally:
            os.chdir(cwd)


@pytest.mark.parametrize("fork", [2, 1])
def test_step_capture_with_forked_csr_branch(fork, monkeypatch):
    """the step graphs captured with a fork onto the
    engine's side stream inside the frontier (PINSAGE_CSR_FORK: 2 = an empty
    branch, 1 = layer 0's CSR transpose on side[0] beside the upper layers').
    The crash this reproduced (SIGSEGV in capture_end) was a stack overflow:
    hipStreamEndCapture recursing without end through its parallel
    capture-stream lists (tools/dbg/segv_bt.c: one libamdhip64 frame
    repeated) when the engine forked its stream off the look-ahead BRANCH of
    the step graph; the frontier graph's fork (off the capture's origin)
    captured fine.  The trainer now turns the engine's frontier fork off while
    it captures the frontier on a branch (pinsage_engine_set_frontier_fork),
    so the frontier graph carries the fork and the look-ahead branch none.
    The fork's wait binds to an event recorded on the frontier's stream, and
    the join is recorded on the side stream and waited on the frontier's
    stream before engine_frontier returns -- so every captured graph (the
    frontier graph, the step graph, and the step graph whose branch computes
    the look-ahead frontier) ends its capture with the side stream joined.
    Six steps (an eager first step, the capture, five replays with look-ahead
    hits) end bitwise equal to the unforked run, and the graphs were used.
    (tools/dbg/capture_fork_probe.cpp holds what hipStreamEndCapture does
    with the other shapes: an unjoined fork, work created inside a capture.)"""
    import graph
    import pinsage_training as pt
    import synthetic
    def segv_bt():  # (diagnostics: native backtrace of a host crash; installed once HIP is up)
        if os.environ.get("PINSAGE_SEGV_BT") == "1":
            import ctypes
            ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "dbg",
                                     "segv_bt.so")).install()
    pg = synthetic.make_playlist_graph(3000, 600, 20000, seed=71)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(3000, 128, seed=72))
    pos = torch.from_numpy(synthetic.make_positives(pg, 15000, seed=73))
    monkeypatch.setenv("PINSAGE_AUTOTUNE", "0")
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
            pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)  # (precompute the table once)

            def run(knob):
                monkeypatch.setenv("PINSAGE_CSR_FORK", str(knob))
                torch.manual_seed(5)
                tr = pt.PinSage(g, 3000, feats, pos, log=False, load_save=False)
                tr.batch_size = 256
                torch.manual_seed(6)
                losses = []
                for _ in range(6):
                    batch, _ = tr.next_batch()
                    losses.append(float(tr.train_batch(batch)[0]))
                torch.cuda.synchronize()
                f = tr._fused
                ahead = os.environ.get("PINSAGE_FRONTIER_AHEAD", "start") != "0"
                assert f.graphs is not None and (f.ahead_hits >= 3 or not ahead), (f.graphs, f.ahead_hits)
                return losses, torch.cat([p.detach().flatten() for p in tr.model.parameters()]).cpu()

            l0, p0 = run(0)
            segv_bt()
            l1, p1 = run(fork)
            assert l0 == l1, (l0, l1)
            assert torch.equal(p0, p1), (p0 - p1).abs().max().item()
        finally:
            os.chdir(cwd)
