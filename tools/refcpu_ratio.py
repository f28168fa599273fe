"""refcpu / reference time ratio: the real reference train
step (imported from /root/reference with the dgl / wandb / torchvision stubs
of tests/golden/make_golden.py) and the oracle's restatement of it
(oracle.RefTrainer, the `cpu_baseline` leg of bench.py) timed on the same
workload, the same host threads, in this (dev) container.

A step = sample_batch (easy negatives) + train_batch (3 forwards, hinge loss,
backward, Adam), the unit bench.py's cpu_baseline times.  The neighbourhood
table is a seeded stand-in (valid track ids, sorted weights): both sides read
the same one and neither's time depends on its values.

    python tools/refcpu_ratio.py [--n 100000] [--steps 6] [--threads 8]

Writes profiles/r02/refcpu_ratio.json.
"""
import argparse
import importlib.util
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "gcn-song-embeddings_amd"))
sys.path.insert(0, R)


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--T", type=int, default=10)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(R, "profiles", "r02", "refcpu_ratio.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    # the restatement's backward at the reference init produces denormals the
    # reference's op order does not (measured 1.6 -> 8 s/step growth without this);
    # flushed on both sides so the ratio compares the algorithms, not x87/SSE assists
    torch.set_flush_denormal(True)
    import synthetic
    from oracle import oracle as orc
    mg = _load("_make_golden", os.path.join(R, "tests", "golden", "make_golden.py"))
    ref_psm, ref_pt, _ = mg._import_reference()

    n = a.n
    pg = synthetic.make_playlist_graph(n, n // 4, 10 * n, seed=0)
    g = mg.stub_graph(pg)
    feats = torch.from_numpy(synthetic.make_features(n, a.d, seed=1))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * n, seed=2))
    rng = np.random.default_rng(3)
    nb = torch.from_numpy(rng.integers(0, n, (n, 100)).astype(np.int64))
    w = torch.from_numpy(-np.sort(-rng.integers(1, 50, (n, 100)) / 500.0, axis=1))
    res = {"workload": f"n={n} tracks, d_in={a.d}, 2 layers, T={a.T}, B={a.B}", "threads": a.threads}
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            g.nbhds_path = os.path.join(tmp, "nb.pt")
            g.base_dir = tmp
            os.mkdir("runs")  # the reference makes runs/<name> but not runs/
            torch.save((w, nb), g.nbhds_path)
            torch.manual_seed(0)
            tr = ref_pt.PinSage(g, n, feats, pos, log=False, load_save=False)
            tr.T, tr.n_layers, tr.batch_size = a.T, 2, a.B
            torch.manual_seed(0)
            tr.model = ref_psm.PinSageModel(g, n, 2, tr.dimensions, tr.n_hops, tr.alpha, a.T, tr.nbhds)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            init = {k: v.detach().numpy().copy() for k, v in tr.model.state_dict().items()}
            torch.manual_seed(1)
            ts = []
            for s in range(a.steps + 2):
                t0 = time.perf_counter()
                batch, _ = ref_pt.sample_batch(tr.all_ids, tr.positives, tr.batch_size, tr.nbhds,
                                               hard_negatives=False)
                tr.train_batch(batch)
                ts.append(time.perf_counter() - t0)
                print(f"reference step {s}: {ts[-1]*1e3:.0f} ms", flush=True)
            t_ref = float(np.median(ts[2:]))
            oc = orc.RefTrainer(init, feats, w.numpy(), nb.numpy(), n_layers=2, T=a.T)
            mt = orc.MT(1)
            ts = []
            for s in range(a.steps + 2):
                t0 = time.perf_counter()
                b, _ = orc.sample_batch_easy(mt, pos.numpy(), n, a.B)
                oc.step(b)
                ts.append(time.perf_counter() - t0)
                print(f"refcpu step {s}: {ts[-1]*1e3:.0f} ms", flush=True)
            t_port = float(np.median(ts[2:]))
        finally:
            os.chdir(cwd)
    res.update(reference_ms_per_step=t_ref * 1e3, refcpu_ms_per_step=t_port * 1e3,
               refcpu_over_reference=t_port / t_ref,
               reference_target_nodes_per_s=3 * a.B / t_ref, refcpu_target_nodes_per_s=3 * a.B / t_port,
               note="median of the timed steps after 2 warm-up steps; same batches' shape, "
                    "same table, same thread count, denormals flushed on both sides; dev container (no GPU)")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
