"""Diagnostic: the fused train step's gradients vs torch autograd through the
engine's forward/backward (three model calls + max_margin_loss), L = 2, 3."""
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

n = 3000
pg = synthetic.make_playlist_graph(n, 750, 40000, seed=7)
indptr, indices = pg.csr()
feats = torch.from_numpy(synthetic.make_features(n, 128, seed=8)).cuda()
pos = torch.from_numpy(synthetic.make_positives(pg, 5 * n, seed=9))
with tempfile.TemporaryDirectory() as tmp:
    os.chdir(tmp)
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    pm.set_rng_mode("philox")
    torch.manual_seed(0)
    w, nb = pm.precompute_neighborhoods_topt(g, n, 200, 0.85, 100, g.nbhds_path)
    pm.set_rng_mode("mt19937")
    for L in (2, 3):
        for margin in (3.0, 1e-5):
            torch.manual_seed(1)
            tr = pt.PinSage(g, n, feats, pos, log=False, load_save=False)
            torch.manual_seed(2)
            tr.model = pm.PinSageModel(g, tr.n, L, tr.dimensions, tr.n_hops, tr.alpha, 10, tr.nbhds)
            if os.environ.get("ZERO_BIAS"):  # spread the outputs (0.3 biases collapse a fresh model)
                with torch.no_grad():
                    for k, p in tr.model.named_parameters():
                        if k.endswith("bias"):
                            p.zero_()
                        else:
                            p.mul_(3.0)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.batch_size, tr.margin, tr.T, tr.n_layers = 32, margin, 10, L
            torch.manual_seed(3)
            batch, _ = tr.next_batch()
            # autograd reference on a twin model with the same parameters
            torch.manual_seed(2)
            m2 = pm.PinSageModel(g, tr.n, L, tr.dimensions, tr.n_hops, tr.alpha, 10, tr.nbhds)
            m2.load_state_dict(tr.model.state_dict())
            hs = [m2(feats, batch[:, c]) for c in range(3)]
            loss2 = pt.max_margin_loss(*hs, margin)
            loss2.backward()
            loss, _, _ = tr.train_batch(batch)
            g2 = dict(m2.named_parameters())
            errs = {k: float((p.grad.double() - g2[k].grad.double()).norm() / g2[k].grad.double().norm())
                    for k, p in tr.model.named_parameters()}
            hq = torch.nn.functional.normalize(hs[0], dim=1)
            hp = torch.nn.functional.normalize(hs[1], dim=1)
            spread = float((hq - hp).norm(dim=1).mean())
            print(f"L={L} margin={margin} |q-p| {spread:.2e} loss {float(loss):.6f} vs {float(loss2):.6f}",
                  {k.replace('conv_layers.', 'c'): f"{v:.1e}" for k, v in errs.items()}, flush=True)
