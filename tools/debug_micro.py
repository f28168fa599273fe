"""Diagnostics for the micro-batched step: loss of the sliced step at several
slice sizes vs the fused step and the oracle on one batch."""
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
        tr0 = parity_util.make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
        b = _batch_with_repeats(tr0, 12)
        init = {k: v.detach().cpu().clone() for k, v in tr0.model.state_dict().items()}
        p = {k: v.float() for k, v in init.items()}
        hs = [orc.model_forward(p, feats, b.numpy()[:, c], L, T, w.numpy(), nb.numpy(), 128) for c in range(3)]
        print("oracle loss", float(orc.max_margin_loss(*hs, 1e-5)))
        for m in (None, 64, 32, 16, 8, 7, 1):
            tr = parity_util.make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
            tr.micro_batch = m
            out = tr.train_batch(b)
            line = f"m={m} loss {float(out[0]):.9f}"
            if m and m < 64:
                Z = tr.last_outputs.cpu().double().numpy()
                errs = [parity_util.rel(Z[c], hs[c].detach().double().numpy()) for c in range(3)]
                rows = [np.nonzero(np.linalg.norm(Z[c] - hs[c].detach().double().numpy(), axis=1) > 1e-4)[0][:8]
                        for c in range(3)]
                line += f" Z rel {errs} bad rows {rows}"
            print(line, flush=True)


if __name__ == "__main__":
    main()
