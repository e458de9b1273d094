"""Where config 1's host round goes, function by function: wraps the drop-in's methods on the round's path
with inclusive timers (perf_counter_ns; each wrapper adds ~0.3 us) and runs bench.c1_host_round's loop.
Prints median-free means per round, in microseconds.  usage: python tools/c1_phases.py [rounds]"""
import functools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from fedscale_amd import _native, bucket, round as rnd_mod
    from fedscale_amd import kernels as kx
    from fedscale_amd.cloud.aggregation import aggregator as agg_mod
    from fedscale_amd.cloud.internal import torch_model_adapter as tma

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    acc = {}

    def wrap(owner, name, label=None):
        fn = getattr(owner, name)
        label = label or f"{getattr(owner, '__name__', owner)}.{name}"

        @functools.wraps(fn)
        def w(*a, **k):
            t0 = time.perf_counter_ns()
            try:
                return fn(*a, **k)
            finally:
                acc[label] = acc.get(label, 0) + time.perf_counter_ns() - t0
        setattr(owner, name, w)

    for owner, name in ((agg_mod.DeviceAggregatorMixin, "update_weight_aggregation"),
                        (rnd_mod.DeviceRound, "add"), (bucket.ClientStaging, "put"),
                        (bucket.ClientStaging, "_put_bulk_views"), (tma.TorchModelAdapter, "begin_round"),
                        (tma.TorchModelAdapter, "apply_round"), (rnd_mod.DeviceRound, "finalize_mean"),
                        (tma.TorchModelAdapter, "_mirror_target"), (tma.TorchModelAdapter, "_commit_scratch"),
                        (tma.TorchModelAdapter, "round_mean_weights"), (tma.TorchModelAdapter, "get_weights"),
                        (tma.TorchModelAdapter, "_acquire_host"), (tma.TorchModelAdapter, "_clone_weights"),
                        (bucket.ClientStaging, "host_rows"), (bucket.ClientStaging, "release_host_rows")):
        wrap(owner, name)
    real_call = _native.call

    def call(fn, *a):
        t0 = time.perf_counter_ns()
        try:
            return real_call(fn, *a)
        finally:
            acc["native." + fn] = acc.get("native." + fn, 0) + time.perf_counter_ns() - t0
    _native.call = kx.call = call
    real_rm = kx.reduce_mirror

    def rm(*a, **k):
        t0 = time.perf_counter_ns()
        try:
            return real_rm(*a, **k)
        finally:
            acc["kernels.reduce_mirror"] = acc.get("kernels.reduce_mirror", 0) + time.perf_counter_ns() - t0
    kx.reduce_mirror = rm
    dev = torch.device("cuda:0")
    bench.c1_host_round(dev, 0, rounds=20)
    acc.clear()
    t0 = time.perf_counter()
    r = bench.c1_host_round(dev, 0, rounds=rounds)
    wall = time.perf_counter() - t0
    n = rounds + 5
    out = {k: round(v / n / 1e3, 2) for k, v in sorted(acc.items(), key=lambda kv: -kv[1])}
    print(json.dumps({"round_ms_median": round(r["round_ms_incl_h2d_d2h"], 4), "wall_us_per_round": round(wall / n * 1e6, 1),
                      "us_per_round_inclusive": out}))


if __name__ == "__main__":
    main()
