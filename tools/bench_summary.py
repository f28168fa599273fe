"""Summarise bench lines: value, ms/step and selected kernel sites (µs)."""
import json
import sys

SITES = ("fwd.aggw.l0", "fwd.aggw.l1", "fwd.wsplit", "fwd.q_gemm.l0", "bwd.layer.l0", "bwd.layer.l1",
         "bwd.q_wgrad.l0", "fwd.frontier")
for p in sys.argv[1:]:
    try:
        d = json.load(open(p))
    except Exception as e:  # noqa: BLE001
        print(p, "unreadable", e)
        continue
    k = d.get("kernels", {})
    print(p, round(d["value"]), round(d["ms_per_step"], 4),
          {n: round(v["avg_ms"] * 1000, 1) for n, v in k.items() if n in SITES},
          "host", round(d.get("host_ms_per_step", {}).get("train_batch_enqueue", 0), 3))
