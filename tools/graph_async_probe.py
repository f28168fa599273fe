"""Does replaying a multi-stream graph block the host?

Kernels are GPU sleeps of about US µs.  A main chain of M kernels and a side
chain of N kernels forked from the first, joined at the end, launched as:
  linear    one single-stream graph (side then main, serialised)
  branched  one captured graph with the side chain on a second stream
  two       two single-stream graphs on two streams, fork/join by events
  eager     the same launches without a graph, on two streams
Prints GPU µs per iteration (events around 30 back-to-back iterations) and
the host's µs per iteration: host ~ GPU means the launch call waited for the
device; host << GPU means it returned after enqueueing."""
import sys
import time

import torch

M = int(sys.argv[1]) if len(sys.argv) > 1 else 40
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
US = float(sys.argv[3]) if len(sys.argv) > 3 else 5.0
s = torch.cuda.Stream()
side = torch.cuda.Stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
torch.cuda._sleep(1_000_000)
e1.record()
torch.cuda.synchronize()
CYC = int(1_000_000 / (e0.elapsed_time(e1) * 1e3) * US)


def k():
    torch.cuda._sleep(CYC)


def chain(n):
    for _ in range(n):
        k()


def branched_body():
    cur = torch.cuda.current_stream()
    k()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        chain(N)
    chain(M)
    cur.wait_stream(side)


def capture(fn, stream):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            fn()
    torch.cuda.synchronize()
    return g


g_lin = capture(lambda: (k(), chain(N), chain(M)), s)
g_br = capture(branched_body, s)
g_main = capture(lambda: (k(), chain(M)), s)
g_side = capture(lambda: chain(N), side)


def it_linear():
    g_lin.replay()


def it_branched():
    g_br.replay()


def it_two():
    cur = torch.cuda.current_stream()
    g_main.replay()  # its first kernel stands in for the fork point
    ev = torch.cuda.Event()
    ev.record(cur)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        g_side.replay()
    cur.wait_stream(side)


def it_eager():
    branched_body()


def timeit(fn, reps=30):
    with torch.cuda.stream(s):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        th = (time.perf_counter() - t0) * 1e6 / reps
        b.record()
        torch.cuda.synchronize()
    return f"gpu {a.elapsed_time(b) * 1e3 / reps:.1f} host {th:.1f}"


print({"M": M, "N": N, "us": US,
       **{name: timeit(fn) for name, fn in (("linear", it_linear), ("branched", it_branched),
                                            ("two", it_two), ("eager", it_eager))}}, flush=True)
