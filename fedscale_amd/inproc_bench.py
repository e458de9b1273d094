"""Timed device-resident round of the drop-in a deployment runs on a multi-GPU node: ONE aggregator process
driving N GPUs through ``ShardedModelAdapter`` (FedScale's aggregator is a single process,
aggregator.py:177-192, uploads at :919-963), next to the single-device ``TorchModelAdapter`` on one of them.

    python -m fedscale_amd.inproc_bench --devices 0,1,2,3 [--clients 1000 --params 25000000]

``bench.py --gpus N`` runs it on rank 0, in a child process with a deadline, after the SPMD timed region (the
SPMD line times one process per GPU, which is not how FedScale's aggregator can be deployed).  The workload is
the headline's: FedAvg, K = 1000 updates of a 25M-fp32 model (10 tensors of 2.5M), HBM-resident — every part's
staging is filled on its own device before the timed region (``synth.fill``; ``DeviceRound.adopt_resident``
takes the K arrivals without host ingress, bench.py's SPMD convention).  A timed round is what the aggregator's
main thread does for the K-th arrival: ``begin_round`` + ``apply_round`` (every part's finishing reduce on its own
stream, then the version commit), from the first launch to every part's last kernel.  Egress of each new version
(``get_weights()``: per-part D2H into one pinned snapshot + the clones the reference API returns,
aggregator.py:788-804) is timed on its own (``egress_ms``) and together with the round (``round_ms_incl_egress``).
With a device listed more than once (a one-GPU rehearsal) the parts share that GPU (copy transport): the fields
are plumbing, not an N-GPU rate.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def _model(P: int, seed: int):
    import torch

    from . import synth

    n = 10 if P % 10 == 0 else 1
    names = [f"l{i}.weight" for i in range(n)]
    shapes = [(P // n,)] * n
    return synth.LayoutModule(names, shapes, [torch.float32] * n, seed=seed)


def _optimizer(policy: str, device):
    """The server optimizer of the round (None for FedAvg): FedYoGi is config 4's server step (optimizers.py:43-63)."""
    if policy == "fedavg":
        return None
    import argparse

    from .cloud.aggregation.optimizers import TorchServerOptimizer

    args = argparse.Namespace(gradient_policy=policy, yogi_eta=3e-3, yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99,
                              learning_rate=0.05, qfed_q=1.0)
    return TorchServerOptimizer(policy, args, device)


def _time_rounds(adapter, parts_streams, K: int, rounds: int, warmup: int) -> dict:
    """Warmup, then ``rounds`` timed rounds; per-part event pairs on each part's stream."""
    import numpy as np
    import torch

    denom32 = float(np.float32(K))
    devs = sorted({ds.index for ds in parts_streams})

    def sync():
        for d in devs:
            torch.cuda.synchronize(d)

    def one(evs=None):
        rnd = adapter.begin_round(K, "fedavg", capacity=K)
        rnd.adopt_resident(K)
        if evs is not None:
            for (e0, _), ds in zip(evs, parts_streams):
                e0.record(ds.stream)
        adapter.apply_round(rnd, denom32, float(K))
        if evs is not None:
            for (_, e1), ds in zip(evs, parts_streams):
                e1.record(ds.stream)

    for _ in range(warmup):
        one()
    sync()
    all_evs = []
    t0 = time.perf_counter()
    for _ in range(rounds):
        evs = []
        for ds in parts_streams:
            with torch.cuda.device(ds.index):
                evs.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        all_evs.append(evs)
        one(evs)
    sync()
    wall = (time.perf_counter() - t0) / rounds
    part_ms = [float(np.mean([evs[i][0].elapsed_time(evs[i][1]) for evs in all_evs]))
               for i in range(len(parts_streams))]
    # egress of each new version: one round, then get_weights() (D2H into the pinned snapshot + clones)
    eg, both = [], []
    for _ in range(max(2, rounds // 2)):
        sync()
        t0 = time.perf_counter()
        one()
        t1 = time.perf_counter()
        adapter.get_weights()
        t2 = time.perf_counter()
        both.append(t2 - t0)
        eg.append(t2 - t1)
    return {"round_ms": wall * 1e3, "part_kernel_ms": part_ms, "egress_ms": float(np.median(eg)) * 1e3,
            "round_ms_incl_egress": float(np.median(both)) * 1e3}


def _time_all_gather(group, ld: int, reps: int = 5) -> float:
    """ms of one RCCL all-gather of the model's N slices (ld fp32 each) to every GPU over xGMI (the device-side
    reassembly an egress could use; the drop-in's egress copies each part D2H instead)."""
    import torch

    parts, outs = [], []
    for ds in group.streams:
        with ds:
            parts.append(torch.zeros(ld, dtype=torch.float32, device=ds.device))
            outs.append(torch.empty(group.world * ld, dtype=torch.float32, device=ds.device))
    group.all_gather(parts, outs)  # warm
    for ds in group.streams:
        torch.cuda.synchronize(ds.device)
    t0 = time.perf_counter()
    for _ in range(reps):
        group.all_gather(parts, outs)
    for ds in group.streams:
        torch.cuda.synchronize(ds.device)
    return (time.perf_counter() - t0) * 1e3 / reps


def run(devices, K: int = 1000, P: int = 25_000_000, rounds: int = 6, warmup: int = 2, seed: int = 2024,
        one_gpu: bool = True, policy: str = "fedavg") -> dict:
    """``policy``: "fedavg" (the headline) or "fed-yogi" (config 4: the mean, then the YoGi step on every part).
    A round's arrivals are FedAvg arrivals either way; the server optimizer decides the finish."""
    import torch

    from . import synth
    from .cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from .cloud.internal.torch_model_adapter import TorchModelAdapter

    N = len(devices)
    out = {"devices": list(devices), "clients": K, "params": P, "policy": policy,
           "distinct_gpus": len(set(devices)) == N}
    alg = 4 * K * P + (4 * P if policy == "fedavg" else 24 * P)
    ad = ShardedModelAdapter(_model(P, seed), optimizer=_optimizer(policy, devices[0]), devices=list(devices),
                             staging_capacity=K)
    try:
        out["transport"] = ad.group.transport
        rnd = ad.begin_round(K, "fedavg", capacity=K)
        for i, (p, r) in enumerate(zip(ad.parts, rnd.rounds)):
            with p.dstream:  # the part's own device and stream
                synth.fill(r.staging.x, K, p.layout.P, seed=seed + 7919 * i)
        r = _time_rounds(ad, [p.dstream for p in ad.parts], K, rounds, warmup)
        from . import kernels as kx

        out.update({"inproc_round_ms": r["round_ms"], "part_kernel_ms": r["part_kernel_ms"], "rounds": rounds,
                    "warmup": warmup, "params_per_part": [p.layout.P for p in ad.parts],
                    "part_launches": [kx.reduce_launches(K, p.layout.P) + (1 if policy != "fedavg" else 0)
                                      for p in ad.parts],
                    "part_alg_bytes": [4 * K * p.layout.P + (4 if policy == "fedavg" else 24) * p.layout.P
                                       for p in ad.parts],
                    "client_updates_per_s": K / (r["round_ms"] * 1e-3),
                    "hbm_gbps_aggregate": alg / (r["round_ms"] * 1e-3) / 1e9,
                    "egress_ms": r["egress_ms"], "inproc_round_ms_incl_egress": r["round_ms_incl_egress"]})
        if policy == "fedavg":
            try:  # what RCCL itself reports for the group's communicator (reported; never discards the timing)
                out["rccl"] = ad.group.rccl_info()
                if ad.group.transport == "rccl":
                    out["rccl"]["all_gather_model_ms"] = _time_all_gather(ad.group,
                                                                          max(p.layout.ld for p in ad.parts))
            except Exception as e:
                out["rccl"] = {"error": f"{type(e).__name__}: {e}"}
    finally:
        ad.close()
        del ad
        for d in set(devices):
            with torch.cuda.device(d):
                torch.cuda.empty_cache()
    if one_gpu:
        d0 = devices[0]
        one = TorchModelAdapter(_model(P, seed), optimizer=_optimizer(policy, d0), device=d0, staging_capacity=K)
        rnd = one.begin_round(K, "fedavg", capacity=K)
        with one.dstream:
            synth.fill(rnd.staging.x, K, P, seed=seed)
        r1 = _time_rounds(one, [one.dstream], K, rounds, warmup)
        out["one_gpu"] = {"device": d0, "round_ms": r1["round_ms"], "kernel_ms": r1["part_kernel_ms"][0],
                          "client_updates_per_s": K / (r1["round_ms"] * 1e-3), "egress_ms": r1["egress_ms"],
                          "round_ms_incl_egress": r1["round_ms_incl_egress"]}
        out["speedup_vs_one_gpu"] = r1["round_ms"] / out["inproc_round_ms"]
        out["speedup_vs_one_gpu_incl_egress"] = r1["round_ms_incl_egress"] / out["inproc_round_ms_incl_egress"]
        del one, rnd
        with torch.cuda.device(d0):
            torch.cuda.empty_cache()
    return out


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--devices", required=True, help="comma-separated GPU ordinals, e.g. 0,1,2,3 (repeat one to "
                                                    "rehearse several parts on one GPU)")
    p.add_argument("--clients", type=int, default=1000)
    p.add_argument("--params", type=int, default=25_000_000)
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--no-one-gpu", action="store_true")
    p.add_argument("--policies", default="fedavg", help="comma-separated: fedavg, fed-yogi")
    a = p.parse_args(argv)
    devices = [int(d) for d in a.devices.split(",") if d.strip()]
    reps = {}
    for pol in [x.strip() for x in a.policies.split(",") if x.strip()]:
        try:
            r = run(devices, K=a.clients, P=a.params, rounds=a.rounds, warmup=a.warmup, one_gpu=not a.no_one_gpu,
                    policy=pol)
            r["ok"] = True
        except Exception as e:  # reported, not raised: bench.py records the failure
            r = {"devices": devices, "policy": pol, "ok": False, "error": f"{type(e).__name__}: {e}"}
        reps[pol] = r
    rep = reps[next(iter(reps))] if len(reps) == 1 else {"ok": all(r["ok"] for r in reps.values()), "policies": reps}
    print(json.dumps(rep), flush=True)
    return 0 if rep.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
