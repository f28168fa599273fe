"""Per-launch cost of dependent kernels inside a replayed hipGraph
(torch.cuda.graph of N tiny in-place adds on one stream), vs eager launches."""
import torch

x = torch.zeros(1, device="cuda")
s = torch.cuda.Stream()
for n in (10, 100):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(n):
                x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                x.add_(1)
    torch.cuda.synchronize()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    per = e0.elapsed_time(e1) * 1e3 / 20 / n
    e0.record()
    for _ in range(20 * n):
        x.add_(1)
    e1.record()
    torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) * 1e3 / 20 / n
    print(f"n={n}: graph {per:.2f} us per dependent kernel, eager {eager:.2f} us", flush=True)
