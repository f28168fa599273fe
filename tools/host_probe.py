"""Is the train loop host-bound?  Times a config's loop (argv[1], default
c2) as bench.py does, then
again with an extra GPU sleep kernel of known length per step: if the step
grows by the sleep, the GPU is the bottleneck (the host keeps ahead); if it
does not, the host's enqueue rate is."""
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gcn-song-embeddings_amd"))
import bench  # noqa: E402


def main():
    cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    import pinsage_training as pt
    pg, g, feats, pos = bench.build_problem(cfg)
    nbhds, _ = bench.precompute(g, cfg, "philox")
    # sleep calibration: cycles per microsecond
    x = torch.cuda._sleep
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); x(1_000_000); e1.record(); torch.cuda.synchronize()
    cyc_per_us = 1_000_000 / (e0.elapsed_time(e1) * 1e3)
    print(f"sleep: {cyc_per_us:.0f} cycles/us", flush=True)
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        g.nbhds_path = os.path.join(tmp, "nb.pt")
        torch.save(nbhds, g.nbhds_path)
        torch.manual_seed(0)
        tr = pt.PinSage(g, cfg["n_tracks"], feats.cuda(), pos, log=False, load_save=False)
        if tr.T != cfg["T"] or tr.n_layers != cfg["n_layers"]:  # as bench.py binds the config
            import pinsage_model as pm
            tr.T, tr.n_layers = cfg["T"], cfg["n_layers"]
            torch.manual_seed(0)
            tr.model = pm.PinSageModel(g, tr.n, tr.n_layers, tr.dimensions, tr.n_hops, tr.alpha, tr.T,
                                       tr.nbhds)
            tr.optimizer = torch.optim.Adam(tr.model.parameters(), lr=tr.lr)
            tr.scheduler = torch.optim.lr_scheduler.ExponentialLR(tr.optimizer, tr.decay)
        tr.batch_size = cfg["batch"]
        for sleep_us in (0, 100, 300, 0):
            for _ in range(10):
                b, _ = tr.next_batch()
                tr.train_batch(b)
            torch.cuda.synchronize()
            n = 200
            th = 0.0
            t0 = time.perf_counter()
            for _ in range(n):
                ta = time.perf_counter()
                b, _ = tr.next_batch()
                tr.train_batch(b)
                th += time.perf_counter() - ta
                if sleep_us:
                    x(int(sleep_us * cyc_per_us))
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n * 1e6
            print(f"extra GPU sleep {sleep_us:4d} us: {dt:7.1f} us/step (host in train loop {th / n * 1e6:.1f} us)",
                  flush=True)
        # the step graphs alone, back to back (no Python between replays):
        # what the device + graph dispatch sustain without the host loop
        f = tr._fused
        if f is not None and f.graphs is not None:
            torch.cuda.synchronize()
            n = 200
            t0 = time.perf_counter()
            for i in range(n):
                p = f.parity
                f.graphs[p][2].replay()
                f.parity ^= 1
            th = (time.perf_counter() - t0) / n * 1e6
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n * 1e6
            print(f"step graphs back to back: {dt:7.1f} us/step (host in replay {th:.1f} us)", flush=True)
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(200):
            b, _ = tr.next_batch()
            tr.train_batch(b)
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
