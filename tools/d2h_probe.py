"""Device -> host copy rates for the precompute table's size (C2: 100k x 100
f64 + i64 = 160 MB): pageable .cpu(), into a preallocated pageable tensor,
into pinned memory (and the pinned allocation's own cost)."""
import time

import torch


def t(f, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def main():
    for n in (100_000, 1_000_000):
        x = torch.randn(n, 100, dtype=torch.float64, device="cuda")
        mb = x.numel() * 8 / 1e6
        print(f"{mb:.0f} MB f64: .cpu() {t(lambda: x.cpu()):.1f} ms", flush=True)
        h = torch.empty(x.shape, dtype=x.dtype)
        print(f"{mb:.0f} MB: copy_ into preallocated pageable {t(lambda: h.copy_(x)):.1f} ms", flush=True)
        ta = time.perf_counter()
        hp = torch.empty(x.shape, dtype=x.dtype, pin_memory=True)
        print(f"{mb:.0f} MB: pinned alloc {1e3 * (time.perf_counter() - ta):.1f} ms", flush=True)
        print(f"{mb:.0f} MB: copy_ into pinned {t(lambda: hp.copy_(x)):.1f} ms", flush=True)
        print(f"{mb:.0f} MB: torch.zeros host {t(lambda: torch.zeros(x.shape, dtype=x.dtype)):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
