"""Host cost of replaying one captured graph back to back vs alternating two
identical graph instances (does a relaunch wait for the previous instance?)."""
import time

import torch

x = torch.zeros(1 << 20, device="cuda")
s = torch.cuda.Stream()


def work(nodes, spin):
    for _ in range(nodes):
        torch.cuda._sleep(spin)
        x.add_(1)


def capture(nodes, spin):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        work(nodes, spin)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            work(nodes, spin)
    torch.cuda.synchronize()
    return g


for nodes, spin in ((40, 2000), (40, 20000)):
    gs = [capture(nodes, spin), capture(nodes, spin)]
    for mode in ("same", "alternate"):
        for _ in range(5):
            gs[0].replay()
        torch.cuda.synchronize()
        n = 100
        th = 0.0
        t0 = time.perf_counter()
        for i in range(n):
            ta = time.perf_counter()
            (gs[0] if mode == "same" else gs[i & 1]).replay()
            th += time.perf_counter() - ta
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n * 1e6
        print(f"nodes={2*nodes} spin={spin}: {mode:9s} {dt:8.1f} us/replay, host in replay {th / n * 1e6:8.1f} us",
              flush=True)
    # GPU time of one replay alone
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gs[0].replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"  single replay GPU span {e0.elapsed_time(e1)*1e3:.1f} us", flush=True)
