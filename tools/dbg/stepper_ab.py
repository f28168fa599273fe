"""Debug: native stepper vs Python step path, and native twice."""
import os, sys, tempfile
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "gcn-song-embeddings_amd")); sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import graph, synthetic
import pinsage_training as pt
N = 3000
os.environ["PINSAGE_AUTOTUNE"] = "0"
with tempfile.TemporaryDirectory() as tmp:
    os.chdir(tmp)
    pg = synthetic.make_playlist_graph(N, 600, 20000, seed=41)
    indptr, indices = pg.csr()
    g = graph.CSRGraph.from_csr(indptr, indices, base_dir=tmp, nbhds_path=os.path.join(tmp, "nb.pt"))
    feats = torch.from_numpy(synthetic.make_features(N, 128, seed=42))
    pos = torch.from_numpy(synthetic.make_positives(pg, 12000, seed=43))
    def run(mode):
        os.environ["PINSAGE_NATIVE_STEP"] = mode
        torch.manual_seed(1)
        tr = pt.PinSage(g, N, feats, pos, log=False, load_save=False)
        tr.batch_size = 64
        torch.manual_seed(2)
        losses, bs = [], []
        for _ in range(8):
            batch, _ = tr.next_batch()
            bs.append(batch.clone())
            losses.append(float(tr.train_batch(batch)[0]))
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().flatten() for p in tr.model.parameters()]).cpu()
        return losses, flat, tr._fused.ahead_hits, bs, tr._fused.stepper is not None
    r = {m: run(m) for m in ("1", "0", "1b")} if False else {}
    r["1"] = run("1"); r["0"] = run("0"); r["1b"] = run("1")
    for k, v in r.items():
        print(k, "stepper", v[4], "hits", v[2], [f"{x:.9e}" for x in v[0]])
    for a, b in (("1", "0"), ("1", "1b")):
        same_b = all(torch.equal(x, y) for x, y in zip(r[a][3], r[b][3]))
        print(a, b, "batches equal", same_b, "param maxdiff", (r[a][1] - r[b][1]).abs().max().item(),
              "first loss diff at", next((i for i, (x, y) in enumerate(zip(r[a][0], r[b][0])) if x != y), None))
