"""Does a 100 GB input buffer read slower when it is allocated into memory a freed 100 GB buffer held before?  The N = 1
line's drop-in figure (the headline round through TorchModelAdapter) read 3-4 % slower than the headline when its staging
was allocated after the headline's inputs were freed, while the two paths read the same when both were allocated fresh
(profiles/r06_dropin_vs_workload.log).  Sequence on one GPU, each step 30 warmup + 20 timed rounds (HIP events):
  A  bench.Workload (headline), fresh memory
  B  TorchModelAdapter round, fresh memory (A still allocated)
  C  free B, then the adapter again into B's freed memory
  D  free A and C, then bench.Workload into their freed memory
Prints the kernel ms per round of each."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import synth  # noqa: E402
from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter  # noqa: E402
from fedscale_amd.inproc_bench import _model  # noqa: E402
from fedscale_amd.state import ShardGroup  # noqa: E402

K, P = 1000, 25_000_000


def time_fn(fn, stream, rounds=20, warmup=30):
    for _ in range(warmup):
        fn(None)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(rounds)]
    for e in evs:
        fn(e)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs]
    return round(float(np.mean(ms)), 4), round(min(ms), 4)


def workload(dev):
    w = bench.Workload("fedavg", K, P, 0, 1, dev, 2024, ShardGroup(0, 1), chunk=K)
    return w, (lambda e: w.step(e))


def adapter(dev):
    ad = TorchModelAdapter(_model(P, 2024), device=dev, staging_capacity=K)
    rnd = ad.begin_round(K, "fedavg", capacity=K)
    with ad.dstream:
        synth.fill(rnd.staging.x, K, P, seed=2024)
    denom = float(np.float32(K))

    def fn(e):
        r = ad.begin_round(K, "fedavg", capacity=K)
        r.adopt_resident(K)
        if e is not None:
            e[0].record(ad.dstream.stream)
        ad.apply_round(r, denom, float(K))
        if e is not None:
            e[1].record(ad.dstream.stream)
    return ad, fn


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    a, fa = workload(dev)
    out["A_workload_fresh"] = time_fn(fa, None)
    b, fb = adapter(dev)
    out["B_adapter_fresh"] = time_fn(fb, None)
    del b, fb
    torch.cuda.empty_cache()
    c, fc = adapter(dev)
    out["C_adapter_into_freed"] = time_fn(fc, None)
    out["A_workload_again"] = time_fn(fa, None)
    a.free()
    del a, fa, c, fc
    torch.cuda.empty_cache()
    d, fd = workload(dev)
    out["D_workload_into_freed"] = time_fn(fd, None)
    print(json.dumps({"kernel_ms_mean_min": out}), flush=True)


if __name__ == "__main__":
    main()
