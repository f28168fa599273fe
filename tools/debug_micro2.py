"""Replay of _train_batch_micro's first pass, row by row vs the oracle."""
import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gcn-song-embeddings_amd"), REPO, os.path.join(REPO, "tests")]

import parity_util  # noqa: E402
from test_gpu_micro import _problem, _batch_with_repeats  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        n = 4000
        g, feats, pos, w, nb = _problem(tmp, n, 1000, 50000, 128, seed=31)
        L, T = 2, 10
        tr = parity_util.make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
        b = _batch_with_repeats(tr, 12)
        init = {k: v.detach().cpu().clone() for k, v in tr.model.state_dict().items()}
        p = {k: v.float() for k, v in init.items()}
        hs = [orc.model_forward(p, feats, b.numpy()[:, c], L, T, w.numpy(), nb.numpy(), 128).detach().numpy()
              for c in range(3)]
        ids = b.t().contiguous().cuda()
        for m in (7, 1):
            for j in range(0, 64, m):
                part = ids[:, j:j + m].reshape(-1)
                with torch.no_grad():
                    y = tr.model(tr.features, part).cpu().numpy()
                ref = np.concatenate([hs[c][j:j + m] for c in range(3)])
                e = np.linalg.norm(y - ref, axis=1) / np.linalg.norm(ref, axis=1)
                if e.max() > 1e-5:
                    print(f"m={m} j={j} ids={part.tolist()} errs={np.array2string(e, precision=2)} "
                          f"norm ratio={np.linalg.norm(y, axis=1) / np.linalg.norm(ref, axis=1)} "
                          f"cos={(y * ref).sum(1) / np.linalg.norm(y, axis=1) / np.linalg.norm(ref, axis=1)}",
                          flush=True)
                    r = tr.model.runner()
                    for label in ("again", "fresh engine", "fresh ws"):
                        if label == "fresh engine":
                            r.engine = None
                            r._ws = None
                            r.pack()
                            r.ensure_engine(3)
                        if label == "fresh ws":
                            r._ws = None
                        with torch.no_grad():
                            y2 = tr.model(tr.features, part).cpu().numpy()
                        e2 = np.linalg.norm(y2 - ref, axis=1) / np.linalg.norm(ref, axis=1)
                        print(f"   {label}: errs={np.array2string(e2, precision=2)} max_pos={r.engine.cfg.max_pos}")
                    S, N = r.engine.counts(r._ws)
                    print("   counts S", S, "N", N, flush=True)
                    if m == 1 and j > 3:
                        break
        print("done")


if __name__ == "__main__":
    main()
