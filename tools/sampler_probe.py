"""Host batch-sampler throughput at a BASELINE config's sizes (no GPU work):
synchronous reference-exact draws, and the speculative chain as the trainer
drives it (sample + peek per step).  If the chain's rate is below the device
step rate, the train loop is host-bound.

    python tools/sampler_probe.py [--config c4] [--steps 30]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gcn-song-embeddings_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import pinsage_training as pt
    sizes = {"c2": (100_000, 512), "c3": (1_000_000, 2048), "c4": (8_000_000, 512)}
    n, B = sizes[a.config]
    pos = torch.from_numpy(np.random.default_rng(0).integers(0, n, (5 * n, 2)).astype(np.int64))
    all_ids = torch.arange(n)
    for spec in (False, True):
        pt._PREFETCH.close()
        pt._PREFETCH.speculate = spec
        torch.manual_seed(0)
        pt.sample_batch(all_ids, pos, B, None, hard_negatives=False)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            pt.sample_batch(all_ids, pos, B, None, hard_negatives=False)
            if spec:
                pt._PREFETCH.peek(B)
        dt = (time.perf_counter() - t0) / a.steps * 1e3
        print(f"{a.config} n={n} P={5 * n} B={B} speculate={spec}: {dt:.3f} ms per batch", flush=True)


if __name__ == "__main__":
    main()
