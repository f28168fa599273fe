"""Diagnostic: autograd path (PinSageModel forward + backward) vs the oracle
for L = 2, 3 at the tools/check_lt.py graph; per-parameter gradient errors."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "gcn-song-embeddings_amd"))
sys.path.insert(0, R)
import graph  # noqa: E402
import pinsage_model as pm  # noqa: E402
import synthetic  # noqa: E402
from oracle import oracle as orc  # noqa: E402

n = 3000
pg = synthetic.make_playlist_graph(n, 750, 40000, seed=7)
indptr, indices = pg.csr()
feats = torch.from_numpy(synthetic.make_features(n, 128, seed=8))
g = graph.CSRGraph.from_csr(indptr, indices)
pm.set_rng_mode("philox")
torch.manual_seed(0)
w, nb = pm.precompute_neighborhoods_topt(g, n, 200, 0.85, 100, None)
rng = np.random.default_rng(0)
for L in (2, 3):
    for dup in (False, True):
        ids = rng.integers(0, n, 96)
        if dup:
            ids[10:20] = ids[0]
        torch.manual_seed(2)
        m = pm.PinSageModel(g, n, L, (128, 512, 128), 200, 0.85, 10, (w, nb))
        init = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
        ref = orc.RefTrainer(init, feats, w.numpy(), nb.numpy(), n_layers=L, T=10)
        c = torch.from_numpy(rng.standard_normal((96, 128)).astype(np.float32))
        y = m(feats.cuda(), torch.from_numpy(ids))
        (y * c.cuda()).sum().backward()
        yr = orc.model_forward(ref.p, ref.feats, ids, L, 10, ref.w, ref.nb, 128)
        (yr * c).sum().backward()
        errs = {k: float(np.linalg.norm(p.grad.cpu().numpy().astype(np.float64) - ref.p[k].grad.numpy())
                         / np.linalg.norm(ref.p[k].grad.numpy())) for k, p in m.named_parameters()}
        print(f"L={L} dup={dup} fwd={float((y.detach().cpu() - yr.detach()).norm() / yr.norm()):.2e}",
              {k.replace('conv_layers.', 'c'): f"{v:.1e}" for k, v in errs.items()}, flush=True)
