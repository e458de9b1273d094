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
        out["one_gpu"] = run_one(devices[0], K, P, rounds, warmup, seed, policy)
        out["speedup_vs_one_gpu"] = out["one_gpu"]["round_ms"] / out["inproc_round_ms"]
        out["speedup_vs_one_gpu_incl_egress"] = (out["one_gpu"]["round_ms_incl_egress"]
                                                 / out["inproc_round_ms_incl_egress"])
    return out


def run_one(device, K: int = 1000, P: int = 25_000_000, rounds: int = 6, warmup: int = 2, seed: int = 2024,
            policy: str = "fedavg") -> dict:
    """The same device-resident round through the single-device ``TorchModelAdapter`` on ``device``: the one-GPU
    figure of this methodology (the N > 1 line's ``scaling_vs_one_gpu`` divides by it; the N = 1 line reports it as
    ``value_drop_in``)."""
    import torch

    from . import synth
    from .cloud.internal.torch_model_adapter import TorchModelAdapter

    one = TorchModelAdapter(_model(P, seed), optimizer=_optimizer(policy, device), device=device, staging_capacity=K)
    try:
        rnd = one.begin_round(K, "fedavg", capacity=K)
        with one.dstream:
            synth.fill(rnd.staging.x, K, P, seed=seed)
        r1 = _time_rounds(one, [one.dstream], K, rounds, warmup)
    finally:
        del one
        with torch.cuda.device(device):
            torch.cuda.empty_cache()
    return {"device": device, "round_ms": r1["round_ms"], "kernel_ms": r1["part_kernel_ms"][0],
            "client_updates_per_s": K / (r1["round_ms"] * 1e-3), "egress_ms": r1["egress_ms"],
            "round_ms_incl_egress": r1["round_ms_incl_egress"], "rounds": rounds, "warmup": warmup}


# ------------------------------------------------------------------------------------------------
# the PCIe-inclusive round (SURVEY §8d's second figure): executors' pickled payloads -> host -> N GPUs -> model out
# ------------------------------------------------------------------------------------------------
def headline_model(seed: int = 0):
    """The headline's 25 M-fp32 model as the PCIe-inclusive round ships it: 10 tensors of 2.5 M (100 MB per upload)."""
    import torch

    from . import synth

    names, shapes = [f"l{i}.weight" for i in range(10)], [(2500, 1000)] * 10
    return synth.LayoutModule(names, shapes, [torch.float32] * 10, seed=seed)


def pcie_rounds(adapter, K: int = 64, rounds: int = 6, seed: int = 2024, n_payloads: int = 8) -> dict:
    """Rounds of the deployed path from the executors' pickled upload payloads (CLIENT_EXECUTE_COMPLETION,
    job_api.proto:31-39) to the new global model on the host: the mixin's zero-copy ``deserialize_response``
    (aggregator.py:704), the adapter's ingress (one GPU: pinned gather + H2D; ``ShardedModelAdapter``: the payload
    registered in place and every GPU's copy engine reading its slice over its own link), the reduce on every GPU,
    and ``get_weights()`` (D2H egress, torch_model_adapter.py:41-47).  ``n_payloads`` distinct payloads are reused
    round robin.  Median and min of ``rounds`` rounds after one warm-up round; synchronised on every GPU."""
    import pickle

    import numpy as np
    import torch

    from .cloud.aggregation.aggregator import DeviceAggregator

    model = adapter.model
    devs = sorted({d.index for d in getattr(getattr(adapter, "group", None), "devices", [adapter.device])})
    agg = DeviceAggregator(adapter)
    rng = np.random.default_rng(seed)
    payloads = []
    for i in range(n_payloads):
        up = {n: t.numpy() + rng.standard_normal(t.shape, dtype=np.float32) * np.float32(0.01)
              for n, t in model.state_dict().items()}
        payloads.append(pickle.dumps({"client_id": i, "moving_loss": 1.0, "trained_size": 200, "success": True,
                                      "utility": 1.0, "update_weight": up, "wall_duration": 0}))
        del up

    def sync():
        for d in devs:
            torch.cuda.synchronize(d)

    ts, t_in, t_fin, t_eg = [], [], [], []
    for r in range(rounds + 1):
        sync()
        t0 = time.perf_counter()
        agg.start_round(K)
        for k in range(K - 1):
            agg.on_result(agg.deserialize_response(payloads[k % n_payloads]))
        t1 = time.perf_counter()
        agg.on_result(agg.deserialize_response(payloads[(K - 1) % n_payloads]))  # the K-th: its H2D, then the reduce
        sync()
        t2 = time.perf_counter()
        adapter.get_weights()
        t3 = time.perf_counter()
        if r:
            ts.append(t3 - t0)
            t_in.append(t1 - t0)
            t_fin.append(t2 - t1)
            t_eg.append(t3 - t2)
    s, smin = float(np.median(ts)), float(np.min(ts))
    tin = float(np.median(t_in))
    P = adapter.layout.P_full
    out = {"clients": K, "params": P, "payload_bytes": len(payloads[0]), "round_ms": s * 1e3, "round_ms_min": smin * 1e3,
           "rounds_ms": [t * 1e3 for t in ts], "client_updates_per_s": K / s, "client_updates_per_s_best": K / smin,
           "host_to_device_GBps": 4 * K * P / s / 1e9, "host_to_device_GBps_best": 4 * K * P / smin / 1e9,
           "phases_ms": {"ingress_first_K_minus_1": tin * 1e3, "last_upload_and_reduce": float(np.median(t_fin)) * 1e3,
                         "egress_get_weights": float(np.median(t_eg)) * 1e3},
           "ingress_GBps": 4 * (K - 1) * P / tin / 1e9}
    if hasattr(adapter, "registered_uploads"):
        out["registered_uploads"] = adapter.registered_uploads
        out["registration_fallbacks"] = adapter.registration_fallbacks
    del agg, payloads
    return out, tin


def run_pcie(devices, K: int = 64, rounds: int = 6, seed: int = 2024) -> dict:
    """The PCIe-inclusive round of the headline model over ``devices``: one GPU through ``TorchModelAdapter``,
    several through ``ShardedModelAdapter`` (one part per GPU, each fed over its own link).  ``parts``: per GPU its
    slice, the host NUMA node its link hangs off (sysfs) and the rate its link carried over the ingress phase
    (its slice's bytes of the K - 1 uploads / that phase's wall: the parts copy concurrently)."""
    import torch

    from .cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from .cloud.internal.torch_model_adapter import TorchModelAdapter
    from .hostnuma import gpu_numa_node

    N = len(devices)
    model = headline_model()
    if N == 1:
        adapter = TorchModelAdapter(model, device=devices[0])
        parts = [(devices[0], adapter.layout.P_full)]
    else:
        adapter = ShardedModelAdapter(model, devices=list(devices))
        parts = [(p.device.index, p.layout.P) for p in adapter.parts]
    try:
        out, tin = pcie_rounds(adapter, K=K, rounds=rounds, seed=seed)
        out.update({"devices": list(devices), "n_gpus": N, "distinct_gpus": len(set(devices)) == N,
                    "transport": getattr(getattr(adapter, "group", None), "transport", "single device"),
                    "adapter": type(adapter).__name__})
        out["parts"] = [{"device": d, "params": n, "host_numa_node": gpu_numa_node(torch.device("cuda", d)),
                         "h2d_GBps_over_ingress": 4 * (K - 1) * n / tin / 1e9} for d, n in parts]
    finally:
        if hasattr(adapter, "close"):
            adapter.close()
        del adapter
        for d in set(devices):
            with torch.cuda.device(d):
                torch.cuda.empty_cache()
    out["note"] = ("from pickled executor payloads: zero-copy deserialize_response, ingress (one GPU: pinned gather + "
                   "H2D; N GPUs: the payload registered in place, each GPU's copy engine reading its slice over its own "
                   "link), reduce, get_weights() D2H; median and min of %d rounds after one warm-up round; never `value`"
                   % rounds)
    if not out["distinct_gpus"]:
        out["note"] += "; %d parts on %d GPU(s): plumbing, not an N-link rate" % (N, len(set(devices)))
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
    p.add_argument("--pcie", action="store_true", help="the PCIe-inclusive round from pickled payloads (run_pcie) "
                                                       "instead of the device-resident one; --clients defaults to 64")
    a = p.parse_args(argv)
    devices = [int(d) for d in a.devices.split(",") if d.strip()]
    if a.pcie:
        try:
            rep = run_pcie(devices, K=a.clients if a.clients != 1000 else 64, rounds=a.rounds)
            rep["ok"] = True
        except Exception as e:
            rep = {"devices": devices, "ok": False, "error": f"{type(e).__name__}: {e}"}
        print(json.dumps(rep), flush=True)
        return 0 if rep["ok"] else 1
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
