"""Diagnostic: are the micro-batched (sliced) outputs bitwise the whole-batch
outputs?  Prints max |dZ| per env variant for the micro test's problem."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gcn-song-embeddings_amd"))
from parity_util import make_trainer  # noqa: E402
import test_gpu_micro as tm  # noqa: E402


def main():
    L, T, m = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        n = 4000
        g, feats, pos, w, nb = tm._problem(tmp, n, 1000, 50000, 128, seed=31)
        tr = make_trainer(g, n, feats.cuda(), pos, L, T, 64, margin=1e-5, seed=9, spread=True)
        tr.micro_batch = m
        b = tm._batch_with_repeats(tr, 12)
        ids = torch.as_tensor(b).to(torch.int64).t().contiguous().cuda()
        Zs = tr._micro_forward(ids)
        with torch.no_grad():
            Zf = tr.model(tr.features, ids.reshape(-1)).view(3, -1, tr.model.out_dim)
        torch.cuda.synchronize()
        d = (Zs - Zf).abs()
        print(os.environ.get("TAG", ""), "L T m", L, T, m, "max|dZ|", d.max().item(), "rows differing",
              int((d.amax(-1) > 0).sum().item()), "of", d.shape[0] * d.shape[1], flush=True)


if __name__ == "__main__":
    main()
