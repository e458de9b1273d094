"""Does sampling the card's sysfs files (fedscale_amd/cardstate.py) slow the kernels it watches?  The headline
workload (FedAvg 1000 x 25 M, bench.Workload) after 1 s of warmup rounds, then regions of 20 rounds with one HIP
event pair per round (bench.py's timed region), alternating: no sampler, a 20 ms sampler (bench.py's timed region),
a 50 ms sampler (its sustained leg), and the 20 ms sampler reading only the clocks and temperatures (no power file).
Prints the mean ms per launch of each region."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd.cardstate import CardSampler  # noqa: E402
from fedscale_amd.state import ShardGroup  # noqa: E402


def region(w, dev, sampler, steps=20, launches=4):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize(dev)
    if sampler is not None:
        sampler.start()
    for e in evs:
        w.step(e)
    torch.cuda.synchronize(dev)
    if sampler is not None:
        sampler.stop()
    return float(np.mean([a.elapsed_time(b) for a, b in evs])) / launches


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.Workload("fedavg", 1000, 25_000_000, 0, 1, dev, 1, ShardGroup(0, 1), budget_fraction=0.6)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        w.step()
        torch.cuda.synchronize(dev)

    def no_power(period):
        s = CardSampler(dev, period_s=period)
        s.files.pop("power_w", None)
        s.samples.pop("power_w", None)
        return s

    kinds = {"none": lambda: None, "s20ms": lambda: CardSampler(dev, period_s=0.02),
             "s50ms": lambda: CardSampler(dev, period_s=0.05), "s20ms_no_power": lambda: no_power(0.02)}
    out = {k: [] for k in kinds}
    for rep in range(6):
        for k, mk in kinds.items():
            out[k].append(region(w, dev, mk()))
    print(json.dumps({k: {"ms_per_launch": [round(x, 4) for x in v], "mean": float(np.mean(v))}
                      for k, v in out.items()}), flush=True)
    w.free()


if __name__ == "__main__":
    main()
