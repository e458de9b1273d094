"""The N = 1 headline round two ways on one GPU, interleaved in blocks: bench.Workload (the line's `value`: fa_reduce
on the current stream over a resident [K, ld] chunk) and the drop-in's TorchModelAdapter round (begin_round /
adopt_resident / apply_round on the adapter's own stream, fedscale_amd.inproc_bench: the N > 1 line's methodology).
Prints the per-round kernel ms of each block (HIP events on the stream that ran it) and the block's wall ms."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import synth  # noqa: E402
from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter  # noqa: E402
from fedscale_amd.inproc_bench import _model  # noqa: E402
from fedscale_amd.state import ShardGroup  # noqa: E402


def main():
    K, P, rounds = 1000, 25_000_000, 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = bench.Workload("fedavg", K, P, 0, 1, dev, 2024, ShardGroup(0, 1), budget_fraction=0.3)
    ad = TorchModelAdapter(_model(P, 2024), device=dev, staging_capacity=K)
    rnd = ad.begin_round(K, "fedavg", capacity=K)
    with ad.dstream:
        synth.fill(rnd.staging.x, K, P, seed=2024)
    denom = float(np.float32(K))

    def wl(evs):
        w.step(evs)

    def dropin(evs):
        r = ad.begin_round(K, "fedavg", capacity=K)
        r.adopt_resident(K)
        evs[0].record(ad.dstream.stream)
        ad.apply_round(r, denom, float(K))
        evs[1].record(ad.dstream.stream)

    for name, fn in (("workload", wl), ("drop_in", dropin)):  # warm both
        for _ in range(30):
            fn((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
    torch.cuda.synchronize()
    for block in range(4):
        for name, fn in (("workload", wl), ("drop_in", dropin)):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for e in evs:
                fn(e)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3 / rounds
            ms = [a.elapsed_time(b) for a, b in evs]
            print(json.dumps({"block": block, "path": name, "wall_ms": round(wall, 4),
                              "kernel_ms_mean": round(float(np.mean(ms)), 4), "kernel_ms_min": round(min(ms), 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
