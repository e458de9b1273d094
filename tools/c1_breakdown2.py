"""Config 1's host round, function by function: wraps the calls of the drop-in's round (staging put, round add,
apply_round and its parts, get_weights and its parts) with perf_counter timers and reports the median
microseconds per round of each, over 300 rounds (after 20 untimed).  Nested timers include their children."""
import argparse
import collections
import functools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fedscale_amd import kernels as kx  # noqa: E402
from fedscale_amd import round as rd  # noqa: E402
from fedscale_amd import bucket, synth  # noqa: E402
from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator  # noqa: E402
from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer  # noqa: E402
from fedscale_amd.cloud.internal import torch_model_adapter as tma  # noqa: E402

ACC = collections.defaultdict(float)


def timed(owner, name, label=None):
    fn = getattr(owner, name)
    label = label or f"{getattr(owner, '__name__', owner)}.{name}"

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t0

    setattr(owner, name, w)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    job = bench.c1_job_conf()
    args = argparse.Namespace(**job["args"])
    K = args.num_participants
    names, shapes, base, ups = bench._c1_updates(1, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    ad = tma.TorchModelAdapter(model, optimizer=TorchServerOptimizer(args.gradient_policy, args, dev), device=dev)
    agg = DeviceAggregator(ad, args)
    for owner, name in [(bucket.ClientStaging, "put"), (rd.DeviceRound, "add"), (rd.DeviceRound, "finalize_mean"),
                        (tma.TorchModelAdapter, "begin_round"), (tma.TorchModelAdapter, "apply_round"),
                        (tma.TorchModelAdapter, "_commit_scratch"), (tma.TorchModelAdapter, "_acquire_host"),
                        (tma.TorchModelAdapter, "_clone_weights"), (tma.TorchModelAdapter, "round_mean_weights"),
                        (tma.TorchModelAdapter, "get_weights"), (kx, "reduce_mirror"), (kx, "reduce"),
                        (DeviceAggregator, "on_result"), (torch.cuda.Event, "synchronize")]:
        if hasattr(owner, name):
            timed(owner, name)
    rows = []
    for r in range(320):
        ACC.clear()
        t0 = time.perf_counter()
        agg.start_round(K)
        for k in range(K):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        agg.model_wrapper.get_weights()
        ACC["round"] = time.perf_counter() - t0
        if r >= 20:
            rows.append(dict(ACC))
    keys = sorted({k for r in rows for k in r})
    med = {k: round(float(np.median([r.get(k, 0.0) for r in rows])) * 1e6, 2) for k in keys}
    print(json.dumps(dict(sorted(med.items(), key=lambda kv: -kv[1]))), flush=True)


if __name__ == "__main__":
    main()
