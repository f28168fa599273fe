"""Replay cost of a captured graph with a forked branch, by capture order.

A linear chain of M tiny kernels (main) and a branch of N tiny kernels that
depends only on the graph's first kernel (side), joined at the end -- the
shape of a train step with its look-ahead frontier.  Prints µs per replay for:
  linear   main only (M nodes on one stream)
  serial   side then main on one stream (M + N nodes, no branch)
  side1st  branch captured before the main chain
  main1st  branch forked at the start but captured after the main chain
(GPU µs per replay between events, and the host's µs per replay call).
Run under different HIP runtime settings (one process each) to see how the
runtime dispatches multi-stream graphs."""
import sys
import time

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 40
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
a = torch.zeros(1, device="cuda")
b = torch.zeros(1, device="cuda")
s = torch.cuda.Stream()
side = torch.cuda.Stream()


def body(kind):
    cur = torch.cuda.current_stream()
    a.add_(1)  # the "stage" kernel both branches depend on
    if kind == "linear":
        for _ in range(M):
            a.add_(1)
    elif kind == "serial":
        for _ in range(N):
            b.add_(1)
        for _ in range(M):
            a.add_(1)
    elif kind == "side1st":
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(N):
                b.add_(1)
        for _ in range(M):
            a.add_(1)
        cur.wait_stream(side)
    elif kind == "main1st":
        ev = torch.cuda.Event()
        ev.record(cur)
        for _ in range(M):
            a.add_(1)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for _ in range(N):
                b.add_(1)
        cur.wait_stream(side)


def run(kind):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        body(kind)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            body(kind)
    torch.cuda.synchronize()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    th = (time.perf_counter() - t0) * 1e6 / reps
    e1.record()
    torch.cuda.synchronize()
    return f"{e0.elapsed_time(e1) * 1e3 / reps:.1f}us (host {th:.1f})"


out = {k: run(k) for k in ("linear", "serial", "side1st", "main1st")}
print({"M": M, "N": N, **out}, flush=True)
