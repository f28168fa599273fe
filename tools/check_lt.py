"""Diagnostic: forward outputs and one train step's gradients of the HIP path
against the CPU oracle over layers x fanout (tests/ covers the chosen cases).

    python tools/check_lt.py
"""
import os
import sys
import tempfile

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "gcn-song-embeddings_amd"))
sys.path.insert(0, R)
import graph  # noqa: E402
import pinsage_model as pm  # noqa: E402
import pinsage_training as pt  # noqa: E402
import synthetic  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def main():
    n = 3000
    pg = synthetic.make_playlist_graph(n, 750, 40000, seed=7)
    indptr, indices = pg.csr()
    feats = torch.from_numpy(synthetic.make_features(n, 128, seed=8))
    pos = torch.from_numpy(synthetic.make_positives(pg, 5 * n, seed=9))
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
        pm.set_rng_mode("philox")
        torch.manual_seed(0)
        w, nb = pm.precompute_neighborhoods_topt(g, n, 200, 0.85, 100, g.nbhds_path)
        pm.set_rng_mode("mt19937")
        Ls = [int(x) for x in os.environ.get("CHECK_L", "2,3").split(",")]
        Ts = [int(x) for x in os.environ.get("CHECK_T", "10,50").split(",")]
        Bs = [int(x) for x in os.environ.get("CHECK_B", "32,128").split(",")]
        for L in Ls:
            for T in Ts:
                for B in Bs:
                    torch.manual_seed(1)
                    tr = pt.PinSage(g, n, feats.cuda(), pos, log=False, load_save=False)
                    tr.T, tr.n_layers = T, L
                    torch.manual_seed(2)
                    tr.model = pm.PinSageModel(g, tr.n, L, tr.dimensions, tr.n_hops, tr.alpha, T, tr.nbhds)
                    tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
                    tr.batch_size = B
                    tr.margin = 3.0
                    init = {k: v.detach().cpu().numpy().copy() for k, v in tr.model.state_dict().items()}
                    ref = orc.RefTrainer(init, feats, w.numpy(), nb.numpy(), n_layers=L, T=T, margin=3.0)
                    torch.manual_seed(3)
                    batch, _ = tr.next_batch()
                    loss, _, _ = tr.train_batch(batch)
                    rl, _, _, rg = ref.step(batch.numpy())
                    errs = [rel(p.grad.cpu().numpy(), rg[k].numpy()) for k, p in tr.model.named_parameters()]
                    b = batch.numpy()
                    dup = len(b.reshape(-1)) - len(np.unique(b.reshape(-1)))
                    print(f"L={L} T={T:3d} B={B:4d} dup_ids={dup:3d} loss_rel={abs(float(loss) - rl) / abs(rl):.2e} "
                          f"grad_rel max={max(errs):.2e} min={min(errs):.2e}", flush=True)


if __name__ == "__main__":
    main()
