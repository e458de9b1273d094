"""Benchmark: device-resident FedAvg reduction of K x P fp32 client updates on MI355X.

Workload (BASELINE.json north_star target): K = 1000 clients x P = 25,000,000 fp32 parameters per GPU,
FedAvg (aggregator.py:489-511): out = (sum of the K updates in arrival order) / K, one fused HIP kernel
(fa_reduce, FA_FINALIZE).  Inputs are generated on the device before the timed region and stay in HBM.

A "step" is one aggregation round over the resident K x P batch.  With --gpus N (one process per GPU,
torchrun) every rank owns an equal 25M-parameter shard of an N x 25M-parameter model and reduces its
K client slices: weak scaling, no data-path collective.  ``value`` counts client updates of one 25M-fp32
(100 MB) slice across all ranks per second.  ``--shard clients`` is the other layout of SURVEY §8e: every
rank reduces its own K clients of a whole 25M-parameter model, then one RCCL all-reduce of the partial
sums (inside the timed step) and the replicated finish; ``value`` = N*K client updates per second.  --reassemble additionally times the RCCL all-gather that
rebuilds the global model for egress (reported as ``reassembly_ms``, not part of ``value``).

Extra objects on the JSON line:
  roofline     achieved algorithmic GB/s of the reduce kernel (4KP+4P bytes per launch / mean launch time
               from HIP events on the launch stream) vs the 8 TB/s HBM3E peak; ``traffic`` = HBM bytes
               per launch from the rocprofv3 PMC summary committed under profiles/ (null if absent)
  cpu_baseline the CPU oracle (numpy restatement of aggregator.py:497-507, bit-exact to the reference's
               golden vectors) timed on this host on a bounded sample of the same workload (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clients", type=int, default=1000)
    ap.add_argument("--params", type=int, default=25_000_000, help="fp32 parameters per GPU shard")
    ap.add_argument("--policy", default="fedavg", choices=["fedavg", "fedyogi", "fedbuff", "qfedavg"])
    ap.add_argument("--shard", default="params", choices=["params", "clients"],
                    help="params: each rank reduces its slice of the model for every client (no data-path "
                         "collective, bit-exact); clients: each rank reduces its own K clients over the whole "
                         "model, then one RCCL all-reduce of the partial sums (state.py)")
    ap.add_argument("--reassemble", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample (0 = skip)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the BASELINE configs 2/3 side measurements (reported under other_configs)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo only to rehearse ranks sharing a GPU")
    return ap.parse_args()


def cpu_baseline(K: int, P: int, budget_s: float, seed: int) -> dict:
    """Time the oracle's FedAvg restatement on host cores on a K-subsample, extrapolated to K."""
    import numpy as np

    from oracle.cpu_reference import fedavg_close, fedavg_step

    rng = np.random.default_rng(seed)
    pool_n = 8
    base = rng.standard_normal(P, dtype=np.float32) * np.float32(0.05)
    pool = [base + rng.standard_normal(P, dtype=np.float32) * np.float32(0.01) for _ in range(pool_n)]
    # per-client accumulate cost (aggregator.py:500-503: one numpy add per tensor, new array each time)
    acc = fedavg_step(None, [pool[0]], True)
    n = 0
    t0 = time.perf_counter()
    while True:
        acc = fedavg_step(acc, [pool[(n + 1) % pool_n]], False)
        n += 1
        if time.perf_counter() - t0 > budget_s * 0.8 or n >= K - 1:
            break
    t_acc = (time.perf_counter() - t0) / n
    t1 = time.perf_counter()
    fedavg_close(acc, K)
    t_fin = time.perf_counter() - t1
    t_round = t_acc * (K - 1) + t_fin
    return {"value": K / t_round, "unit": "client-updates/s", "cores": 1, "kind": "port",
            "sample": f"oracle FedAvg (numpy, single-threaded) over {n + 1} of the {K} x {P} fp32 client updates "
                      f"(pool of {pool_n} distinct 100 MB buffers), {t_acc * 1e3:.1f} ms/client + "
                      f"{t_fin * 1e3:.0f} ms finalize, extrapolated linearly to K={K}",
            "host": platform.processor() or platform.machine(), "host_cpus": os.cpu_count()}


def _c1_updates(seed: int, K: int):
    """Config 1's inputs: K FEMNIST small-CNN updates (P = 24,492) as the executor's result dicts hold
    them (torch_client.py:76-91: numpy arrays in host memory)."""
    import numpy as np

    from fedscale_amd import synth

    names, shapes, _ = synth.femnist_cnn_layout()
    rng = np.random.default_rng(seed)
    base = [rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in shapes]
    ups = [{n: b + rng.standard_normal(b.shape, dtype=np.float32) * np.float32(0.01) for n, b in zip(names, base)}
           for _ in range(K)]
    return names, shapes, base, ups


def c1_host_round(dev, seed: int, rounds: int = 50) -> dict:
    """BASELINE config 1 (FEMNIST small-CNN, K = 10) through the drop-in: start_round, K on_result calls
    with host dicts (pinned staging + H2D), the fused reduce, and get_weights() (D2H) — the whole round
    the reference runs on the CPU (aggregator.py:489-511, torch_model_adapter.py:23-47)."""
    import numpy as np
    import torch

    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    K = 10
    names, shapes, base, ups = _c1_updates(seed, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    agg = DeviceAggregator(TorchModelAdapter(model, device=dev))
    ts = []
    for r in range(rounds + 5):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        agg.start_round(K)
        for k in range(K):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        agg.model_wrapper.get_weights()
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts[5:])) * 1e3
    return {"clients": K, "params": sum(int(np.prod(s)) for s in shapes), "round_ms_incl_h2d_d2h": ms,
            "client_updates_per_s": K / (ms * 1e-3),
            "note": "host dicts in, global model out (get_weights); median of %d rounds" % rounds}


def cpu_baseline_c1(seed: int, rounds: int = 50) -> dict:
    """The oracle's restatement of the same config-1 round on one host core (cpu_baseline leg)."""
    import numpy as np

    from oracle.cpu_reference import fedavg_close, fedavg_step

    K = 10
    _, _, _, ups = _c1_updates(seed, K)
    ts = []
    for r in range(rounds + 5):
        t0 = time.perf_counter()
        acc = None
        for k in range(K):
            acc = fedavg_step(acc, ups[k], k == 0)
        fedavg_close(acc, K)
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts[5:])) * 1e3
    return {"round_ms": ms, "client_updates_per_s": K / (ms * 1e-3), "cores": 1, "kind": "port"}


def other_configs(dev, seed: int) -> dict:
    """BASELINE.json configs 2 and 3 on one GPU (FedAvg, device-resident), beside the headline line, plus
    one GPU's shard of configs 4 and 5 (``shard_configs``).
    Config 2 (400 MB) rotates two input sets so the 256 MiB Infinity Cache cannot serve repeats."""
    import numpy as np
    import torch

    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    out = {"c1_femnist_cnn_k10_host_round": c1_host_round(dev, seed)}
    for name, K, P, sets in (("c2_synthetic_k100_p1M", 100, 1_000_000, 2),
                             ("c3_resnet18_layout_k1000_p11191242", 1000, 11_191_242, 1)):
        ld = round_up(P, 64)
        xs = []
        for i in range(sets):
            x = torch.empty(K, ld, dtype=torch.float32, device=dev)
            synth.fill(x, K, P, seed=seed + 31 * i)
            xs.append(x)
        o = torch.empty(ld, dtype=torch.float32, device=dev)
        for i in range(4):
            kx.reduce(xs[i % sets], K, P, o, denom=float(np.float32(K)), finalize=True)
        torch.cuda.synchronize(dev)
        evs = []
        for i in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            kx.reduce(xs[i % sets], K, P, o, denom=float(np.float32(K)), finalize=True)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize(dev)
        ms = float(np.median([a.elapsed_time(b) for a, b in evs]))
        out[name] = {"clients": K, "params": P, "kernel_ms": ms, "client_updates_per_s": K / (ms * 1e-3),
                     "hbm_gbps": (4 * K * P + 4 * P) / (ms * 1e-3) / 1e9}
        del xs, o
        torch.cuda.empty_cache()
    out.update(shard_configs(dev, seed))
    return out


def _timed(fn, reps, stream):
    import numpy as np
    import torch

    evs = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def shard_configs(dev, seed: int) -> dict:
    """One GPU's share of the multi-GPU BASELINE configs (the 4- and 8-GPU runs are the driver's):
    config 4 = 1000 clients x 25M params FedYoGi over 4 GPUs -> a 6.25M-parameter shard per GPU, fused
    reduce + FedYoGi (fa_reduce_yogi, 4KP + 24P bytes); config 5 = 10000 clients x 100M params q-FedAvg over
    8 GPUs -> a 12.5M-parameter shard per GPU, the 10000 clients streamed through one 1000-client staging
    buffer (50 GB) as the device path does: 10 fa_qfed_accumulate launches continuing one delta chain,
    then hs + the step.  Refilling the staging buffer (on-device generator, standing in for the H2D
    ingress) is outside the timed launches; the timed region is every kernel of the round."""
    import numpy as np
    import torch

    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    stream = torch.cuda.current_stream(dev)
    out = {}
    # ---- config 4 shard: FedYoGi ------------------------------------------------------------------
    K, P = 1000, 25_000_000 // 4
    ld = round_up(P, 64)
    x = torch.empty(K, ld, dtype=torch.float32, device=dev)
    synth.fill(x, K, P, seed=seed + 4)
    st = {n: torch.zeros(ld, device=dev) for n in ("last", "m", "v", "out")}
    synth.fill(st["last"].view(1, -1), 1, P, seed=seed + 5, scale_noise=0.0)
    hp = dict(eta=float(np.float32(3e-3)), tau=float(np.float32(1e-8)), beta=float(np.float32(0.9)),
              omb=float(np.float32(1 - 0.9)), omb2=float(np.float32(1 - 0.99)))

    def yogi_round(init=False):
        kx.reduce_yogi(x, K, P, last=st["last"], m=st["m"], v=st["v"], out=st["out"], denom=float(np.float32(K)),
                       init=init, **hp)

    yogi_round(True)
    ms = float(np.median(_timed(yogi_round, 10, stream)))
    out["c4_fedyogi_shard_k1000_p6250000"] = {
        "clients": K, "params_per_gpu": P, "of": "1000 x 25M FedYoGi over 4 GPUs", "round_ms": ms,
        "client_updates_per_s": K / (ms * 1e-3), "hbm_gbps": (4 * K * P + 24 * P) / (ms * 1e-3) / 1e9}
    del x, st
    torch.cuda.empty_cache()
    # ---- config 5 shard: q-FedAvg, streamed -------------------------------------------------------
    Ktot, C, P = 10_000, min(1000, kx.qfed_max_chunk()), 100_000_000 // 8
    ld = round_up(P, 64)
    x = torch.empty(C, ld, dtype=torch.float32, device=dev)
    last = torch.empty(1, ld, dtype=torch.float32, device=dev)
    synth.fill(last, 1, P, seed=seed + 6, scale_noise=0.0)
    last = last[0]
    rng = np.random.default_rng(seed)
    losses = rng.uniform(0.5, 2.0, size=Ktot)
    lr, q = 0.05, 1.0
    alpha = torch.tensor([np.float32(np.float_power(l + 1e-10, q)) for l in losses], device=dev)
    c1 = torch.tensor([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses], device=dev)
    c2 = torch.tensor([np.float32((1 / lr) * np.float_power(l + 1e-10, q)) for l in losses], device=dev)
    delta = torch.zeros(ld, device=dev)
    sq = torch.zeros(Ktot, dtype=torch.float64, device=dev)
    ws = kx.qfed_workspace(C, dev)
    hs = torch.zeros(2, device=dev)
    new = torch.zeros(ld, device=dev)
    kern = []
    for rep in range(2):  # the first pass warms up; the second is reported
        sq.zero_()
        kern = []
        for c0 in range(0, Ktot, C):
            synth.fill(x, C, P, seed=seed + 7, k0=c0)  # refill = ingress stand-in, not timed
            kern += _timed(lambda: kx.qfed_accumulate(x, C, P, last=last, alpha=alpha[c0:c0 + C], lr=lr,
                                                      delta=delta, sqnorm=sq[c0:c0 + C], workspace=ws,
                                                      accumulate=c0 > 0), 1, stream)

        def finish():
            kx.qfed_hs(sq, c1, c2, Ktot, hs)
            kx.qfed_finalize(last, delta, hs, new, P)

        kern += _timed(finish, 1, stream)
    ms = float(sum(kern))
    alg = 4 * Ktot * P + 8 * P + 8 * Ktot  # SURVEY §8d q-FedAvg: 4KP + 4P (last) + 4P (new) + 8K
    out["c5_qfedavg_shard_k10000_p12500000_streamed"] = {
        "clients": Ktot, "params_per_gpu": P, "chunk": C, "of": "10000 x 100M q-FedAvg over 8 GPUs",
        "round_kernel_ms": ms, "client_updates_per_s": Ktot / (ms * 1e-3), "hbm_gbps": alg / (ms * 1e-3) / 1e9,
        "note": "staging refills (ingress stand-in) excluded; all round kernels timed with HIP events"}
    del x
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local_dev = local if args.dist_backend == "nccl" else local % max(1, ndev)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from fedscale_amd.state import ShardGroup

    shards = ShardGroup(rank, world, mode=args.shard)
    cmode = shards.shards_clients

    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    K, P = args.clients, args.params
    ld = round_up(P, 64)
    x = torch.empty(K, ld, dtype=torch.float32, device=dev)
    synth.fill(x, K, P, seed=args.seed + 7919 * rank)
    out = torch.zeros(ld, dtype=torch.float32, device=dev)
    acc = torch.zeros(ld, dtype=torch.float32, device=dev) if cmode else None  # client mode: partial chain
    Kg = K * world if cmode else K  # clients in the round (client mode: every rank brings K)
    denom = float(np.float32(Kg))
    yogi = None
    if args.policy == "fedyogi":
        yogi = dict(last=torch.zeros(ld, device=dev), m=torch.zeros(ld, device=dev), v=torch.zeros(ld, device=dev),
                    eta=float(np.float32(3e-3)), tau=float(np.float32(1e-8)), beta=float(np.float32(0.9)),
                    omb=float(np.float32(1 - 0.9)), omb2=float(np.float32(1 - 0.99)), init=False)
        synth.fill(yogi["last"].view(1, -1), 1, P, seed=args.seed + 1)
    a = None
    if args.policy == "fedbuff":
        s = [1 / (1 + (k % 6)) ** 0.5 for k in range(Kg)]
        a = torch.tensor(np.asarray(s[rank * K:(rank + 1) * K] if cmode else s, dtype=np.float32), device=dev)
        denom = float(np.float32(sum(s)))
    gathered = None
    qf = None
    if args.policy == "qfedavg":
        if K > kx.qfed_max_chunk():
            raise SystemExit(f"--policy qfedavg: K <= {kx.qfed_max_chunk()} per chunk in this bench")
        rng = np.random.default_rng(args.seed)
        losses = rng.uniform(0.5, 2.0, size=Kg)
        lr, q = 0.05, 1.0
        mine = losses[rank * K:(rank + 1) * K] if cmode else losses
        qf = dict(last=torch.empty(1, ld, device=dev), delta=torch.zeros(ld, device=dev),
                  sq=torch.zeros(Kg, dtype=torch.float64, device=dev), ws=kx.qfed_workspace(K, dev),
                  hs=torch.zeros(2, device=dev), lr=lr,
                  alpha=torch.tensor([np.float32(np.float_power(l + 1e-10, q)) for l in mine], device=dev),
                  c1=torch.tensor([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses], device=dev),
                  c2=torch.tensor([np.float32((1 / lr) * np.float_power(l + 1e-10, q)) for l in losses], device=dev))
        synth.fill(qf["last"], 1, P, seed=args.seed + (0 if cmode else 7919 * rank), scale_noise=0.0)
        qf["last"] = qf["last"][0]

    stream = torch.cuda.current_stream(dev)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        if qf is not None:  # optimizers.py:73-104: phase 1 (timed as the dominant kernel), hs, phase 2
            qf["sq"].zero_()
            k0 = rank * K if cmode else 0
            kx.qfed_accumulate(x, K, P, last=qf["last"], alpha=qf["alpha"], lr=qf["lr"], delta=qf["delta"],
                               sqnorm=qf["sq"][k0:k0 + K], workspace=qf["ws"], accumulate=False)
            if ev is not None:
                ev[1].record(stream)
            if cmode:  # per-rank partial delta chains + each client's norm from its owner rank
                shards.all_reduce_sum(qf["delta"])
                shards.all_reduce_sum(qf["sq"])
            elif world > 1:
                shards.all_reduce_sum(qf["sq"])
            kx.qfed_hs(qf["sq"], qf["c1"], qf["c2"], Kg, qf["hs"])
            kx.qfed_finalize(qf["last"], qf["delta"], qf["hs"], out, P)
            return
        if cmode:  # partial chain of this rank's clients, RCCL all-reduce, finish on the summed vector
            kx.reduce(x, K, P, acc, a=a)
            if ev is not None:
                ev[1].record(stream)
            shards.all_reduce_sum(acc)
            if yogi is None:
                kx.reduce(acc.view(1, ld), 1, P, out, denom=denom, finalize=True)
            else:
                kx.reduce_yogi(acc.view(1, ld), 1, P, out=out, denom=denom, **yogi)
            return
        if yogi is None:
            kx.reduce(x, K, P, out, a=a, denom=denom, finalize=True)
        else:
            kx.reduce_yogi(x, K, P, out=out, denom=denom, **yogi)
        if ev is not None:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))

    reassembly_ms = None
    if args.reassemble and world > 1:
        shards.all_gather(out)  # warm the communicator
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0r = time.perf_counter()
        for _ in range(5):
            gathered = shards.all_gather(out)
        torch.cuda.synchronize(dev)
        reassembly_ms = (time.perf_counter() - t0r) * 1e3 / 5

    t = torch.tensor([wall, kern_ms], dtype=torch.float64)
    if world > 1:
        if args.dist_backend == "nccl":
            t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_ms_max = float(t[0]), float(t[1])

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        value = world * K * args.steps / wall
        extra = {"fedavg": 0, "fedbuff": 4 * K, "fedyogi": 0 if cmode else 20 * P,
                 "qfedavg": 4 * P + 8 * K}[args.policy]
        alg_bytes = 4 * K * P + 4 * P + extra  # SURVEY §8d algorithmic bytes per launch (per GPU)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(PMC_FILE):
            try:
                pmc = json.load(open(PMC_FILE))
                key = f"{args.policy}_k{K}_p{P}"
                if key in pmc:
                    traffic = pmc[key]["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
        res = {
            "metric": ("client-updates/sec + HBM GB/s, device-resident FedAvg reduce of KxP fp32"
                       if args.policy == "fedavg" else
                       f"client-updates/sec + HBM GB/s, device-resident {args.policy} round of KxP fp32"),
            "value": value, "unit": "client-updates/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic full-weight client updates (base + noise, hash-generated on device), HBM-resident",
            "config": ({"workload": f"{args.policy}_k{K}_p{P}_per_gpu", "clients": K, "params_per_gpu": P,
                        "model_params_total": P * world, "policy": args.policy,
                        "parallelism": f"param-shard x{world} (one process per GPU)"} if not cmode else
                       {"workload": f"{args.policy}_k{K}_per_gpu_p{P}_clientshard", "clients": Kg,
                        "clients_per_gpu": K, "params": P, "model_params_total": P, "policy": args.policy,
                        "parallelism": f"client-shard x{world} + RCCL all-reduce (one process per GPU)"}),
            "hbm_gbps": achieved,
            "kernel_ms": kern_ms,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": ("k_qfed_accum + k_qfed_gather (fa_qfed_accumulate)" if args.policy == "qfedavg"
                                    else "k_reduce (fa_reduce, this rank's partial chain)" if cmode else
                                    {"fedavg": "k_reduce (fa_reduce FA_FINALIZE)",
                                     "fedbuff": "k_reduce weighted (fa_reduce FA_FINALIZE)",
                                     "fedyogi": "k_reduce EPI_YOGI (fa_reduce_yogi)"}[args.policy]),
                         "alg_bytes_per_launch": alg_bytes},
        }
        if reassembly_ms is not None:
            res["reassembly_ms"] = reassembly_ms
        if world == 1 and not args.no_other_configs:
            del x
            torch.cuda.empty_cache()
            res["other_configs"] = other_configs(dev, args.seed)
        if world == 1 and args.cpu_seconds > 0:
            x = None
            torch.cuda.empty_cache()
            res["cpu_baseline"] = cpu_baseline(K, P, args.cpu_seconds, args.seed)
            if "other_configs" in res:  # the oracle on config 1's round, beside the device round
                res["other_configs"]["c1_femnist_cnn_k10_host_round"]["cpu_baseline"] = cpu_baseline_c1(args.seed)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
