"""Does a timed region read slower when it starts right after its inputs were written?  Config 3 (1000 x
11,191,242 FedAvg) on one GPU: per-round HIP-event times of 10 rounds after each of
  fill+0 s, fill+2 s, fill+12 s, idle 12 s without a fill, and straight after 3 s of back-to-back rounds,
with the card's telemetry for each region.  bench.py's no-rest line read configs 3-5 about 3 % slower than its
rested line (two round-5 lines, since folded into DESIGN.md §5)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import synth  # noqa: E402
from fedscale_amd.cardstate import CardSampler  # noqa: E402
from fedscale_amd.state import ShardGroup  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cfg = bench.CONFIGS["c3"]
w = bench.Workload(cfg["policy"], cfg["clients"], cfg["params"], 0, 1, dev, 1, ShardGroup(0, 1), budget_fraction=bench.MEM_FRACTION)


def refill():
    with torch.cuda.stream(w.stream):
        for i, x in enumerate(w.xs):
            synth.fill(x, w.C, w.P, seed=11 + i)
    torch.cuda.synchronize(dev)


def region(tag, steps=10):
    s = CardSampler(dev, period_s=0.02)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize(dev)
    s.start()
    for e in evs:
        w.step(e)
    torch.cuda.synchronize(dev)
    card = s.stop().summary()
    ms = [a.elapsed_time(b) for a, b in evs]
    rec = {"region": tag, "round_ms": [round(m, 4) for m in ms], "mean_ms": sum(ms) / len(ms),
           "tb_s": w.alg_bytes / (sum(ms) / len(ms) * 1e-3) / 1e12,
           "card": {k: v["mean"] for k, v in card.items() if isinstance(v, dict)}}
    print(json.dumps(rec), flush=True)


torch.cuda.synchronize(dev)
region("after_construct_fill_0s")
for rep in range(2):
    refill()
    region(f"fill_0s_r{rep}")
    refill()
    time.sleep(2)
    region(f"fill_2s_r{rep}")
    refill()
    time.sleep(12)
    region(f"fill_12s_r{rep}")
    time.sleep(12)
    region(f"idle_12s_nofill_r{rep}")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 3:
        w.step()
        torch.cuda.synchronize(dev)
    region(f"after_3s_back_to_back_r{rep}")
w.free()
