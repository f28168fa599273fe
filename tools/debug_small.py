"""Engine forward on tiny nodesets (1-6 ids) vs the oracle: per-row errors."""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gcn-song-embeddings_amd"), REPO, os.path.join(REPO, "tests")]

import parity_util  # noqa: E402
from test_gpu_micro import _problem  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        n = 4000
        g, feats, pos, w, nb = _problem(tmp, n, 1000, 50000, 128, seed=31)
        for L, T in ((1, 10), (2, 10)):
            tr = parity_util.make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
            init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
            p = {k: v.float() for k, v in init.items()}
            rng = np.random.default_rng(0)
            for mp, k in ((21, 21), (21, 3), (20, 3), (22, 3), (23, 3), (24, 3), (24, 24), (48, 3), (21, 5),
                          (7, 3), (6, 3), (5, 3)):
                r = tr.model.runner()
                r.engine = None
                r._ws = None
                r.pack()
                r.ensure_engine(mp)
                ids = rng.integers(0, n, k)
                with torch.no_grad():
                    y = tr.model(feats.cuda(), torch.from_numpy(ids)).cpu().double().numpy()
                ref = orc.model_forward(p, feats, ids, L, T, w.numpy(), nb.numpy(), 128).detach().double().numpy()
                e = np.linalg.norm(y - ref, axis=1) / np.linalg.norm(ref, axis=1)
                eng = tr.model.runner().engine
                print(f"L={L} T={T} k={k} max_pos={eng.cfg.max_pos} row errs {np.array2string(e, precision=2)}",
                      flush=True)


if __name__ == "__main__":
    main()
