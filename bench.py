"""Benchmark: device-resident reduction of K x P fp32 client updates on MI355X (FedScale's aggregator hot
path, aggregator.py:489-511 + the server step, optimizers.py:31-108).

Headline workload (BASELINE.json north_star target): FedAvg, K = 1000 clients x P = 25,000,000 fp32
parameters, one fused HIP kernel (fa_reduce, FA_FINALIZE): out = (sum of the K updates in arrival order)/K.
Inputs are generated on the device before the timed region and stay in HBM.

A "step" is one aggregation round over the resident K x P batch.

--gpus N (one process per GPU, torchrun; RCCL over xGMI) shards THE SAME model over the ranks (strong
scaling, the north star's "1000 x 25M ... >= 3.5x at 8 GPUs"): rank r owns the 64-aligned parameter slice
[b_r, b_r+1), b_r = r*P/N rounded to a multiple of 64 (every slice within 64 floats of P/N), and
reduces its slice of every client update — no
data-path collective (each output element depends only on its own column).  ``value`` = K * steps / wall
(max over ranks): client updates of the whole model per second.  The RCCL all-gather that reassembles the
global model for egress is timed separately (``reassembly_ms``), outside ``value``.
``--scaling weak`` keeps round 1's alternative (every rank a 25M shard of an N x 25M model, value = N*K*steps
/ wall); ``--shard clients`` is SURVEY §8e's other layout (every rank reduces K clients of the whole model,
then one RCCL all-reduce of the partial chains inside the step; value = N*K*steps/wall).

--config c2 | c3 | c4 | c5 runs a BASELINE config as the headline line instead (c4 = 1000 x 25M FedYoGi,
c5 = 10000 x 100M q-FedAvg streamed through a resident chunk of <= 1000 clients); at N>1 they are sharded
the same way.  The default run also reports configs 4 and 5 sharded over the N ranks under
``other_configs`` (so the driver's 4- and 8-GPU runs measure them at their BASELINE GPU counts), and at
N=1 configs 1-3 plus each config's CPU leg.

Extra objects on the JSON line:
  roofline     achieved algorithmic GB/s of the dominant kernel on one GPU (algorithmic bytes per launch,
               SURVEY §8d, over this rank's slice / mean launch time from HIP events on the launch stream)
               vs the 8 TB/s HBM3E peak; ``traffic`` = HBM bytes per launch from the rocprofv3 PMC summary
               committed under profiles/ (null if absent)
  cpu_baseline the CPU oracle (restatement of aggregator.py:497-507, bit-exact to the reference's golden
               vectors) timed on this host on a bounded sample of the same workload (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")

# BASELINE.json configs as device workloads (config 1 is the host round, measured separately)
CONFIGS = {
    "headline": dict(policy="fedavg", clients=1000, params=25_000_000),
    "c2": dict(policy="fedavg", clients=100, params=1_000_000),
    "c3": dict(policy="fedavg", clients=1000, params=11_191_242),
    "c4": dict(policy="fedyogi", clients=1000, params=25_000_000),
    "c5": dict(policy="qfedavg", clients=10_000, params=100_000_000),
}
EXTRA_BYTES = {  # SURVEY §8d algorithmic bytes beyond the 4KP client read + 4P model write, per GPU slice
    "fedavg": lambda K, P: 0, "fedbuff": lambda K, P: 4 * K, "fedyogi": lambda K, P: 20 * P,
    "qfedavg": lambda K, P: 4 * P + 8 * K}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=-1,
                    help="untimed warmup rounds; -1 (default): at least 3 and, at N = 1, at least 1 s of them, so the "
                         "timed region starts with the card's clocks settled (the line reports the count)")
    ap.add_argument("--config", default="headline", choices=sorted(CONFIGS))
    ap.add_argument("--clients", type=int, default=None, help="override the config's K")
    ap.add_argument("--params", type=int, default=None,
                    help="override the config's P (the whole model; per GPU with --scaling weak)")
    ap.add_argument("--policy", default=None, choices=["fedavg", "fedyogi", "fedbuff", "qfedavg"])
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"])
    ap.add_argument("--shard", default="params", choices=["params", "clients"],
                    help="params: each rank reduces its slice of the model for every client (no data-path "
                         "collective, bit-exact); clients: each rank reduces its own K clients over the whole "
                         "model, then one RCCL all-reduce of the partial sums (state.py)")
    ap.add_argument("--no-reassemble", action="store_true", help="skip the egress all-gather timing at N>1")
    ap.add_argument("--rest", type=float, default=None,
                    help="seconds the card idles before each heavy timed region (default %g; 0 = off)" % REST_S)
    ap.add_argument("--mean-chain", default="auto", choices=["auto", "on", "off"],
                    help="q-FedAvg: carry the FedAvg chain in phase 1 (auto: as the drop-in, when the round spans "
                         "several resident chunks)")
    ap.add_argument("--sustain", type=float, default=10.0,
                    help="N = 1: seconds of back-to-back headline rounds after the rested timed region (the sustained "
                         "rate and the card's state; 0 = skip)")
    ap.add_argument("--config-sustain", type=float, default=None,
                    help="seconds of back-to-back rounds after each heavy config's rested region (default %g; 0 = off)"
                         % 3.0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the headline CPU sample (0 = skip "
                                                                     "every CPU leg)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-other-configs", action="store_true", help="skip the side measurements (other_configs)")
    ap.add_argument("--no-pcie", action="store_true",
                    help="N > 1: skip the PCIe-inclusive N-link round (pcie_inclusive) rank 0 runs after the timed region")
    ap.add_argument("--no-selfcheck", action="store_true",
                    help="N > 1: skip the in-process multi-GPU drop-in check (fedscale_amd.selfcheck) rank 0 runs "
                         "over all N GPUs after the timed region")
    ap.add_argument("--mem-fraction", type=float, default=0.6,
                    help="share of the free HBM a workload's resident client chunk may take (lower it when several "
                         "ranks share one GPU in a rehearsal)")
    ap.add_argument("--sets", type=int, default=None,
                    help="rotating resident input sets (default 1; 2 for --config c2, whose 400 MB would otherwise "
                         "be served partly by the 256 MiB Infinity Cache)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo only to rehearse ranks sharing a GPU")
    a = ap.parse_args()
    cfg = dict(CONFIGS[a.config])
    for k in ("clients", "params", "policy"):
        if getattr(a, k) is not None:
            cfg[k] = getattr(a, k)
    a.cfg = cfg
    return a


# ------------------------------------------------------------------------------------------------
# CPU baseline legs (the oracle on this host: bench.py is the one product-side file allowed to call it)
# ------------------------------------------------------------------------------------------------
def _host_info() -> dict:
    import torch

    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"host_cpu": model, "host_cpus": os.cpu_count(), "torch_threads": torch.get_num_threads()}


def _pool(P: int, n: int, seed: int):
    """n distinct fp32 client buffers of P elements (> LLC each for the large configs): one normal draw,
    then cheap distinct scalings (values only need to be ordinary floats for the timing)."""
    import numpy as np

    rng = np.random.default_rng(seed)
    base = rng.standard_normal(P, dtype=np.float32) * np.float32(0.05)
    return [base * np.float32(1.0 + 1e-3 * i) for i in range(n)]


def _cpu_accumulate(pool, K: int, budget_s: float):
    """Per-client accumulate cost of aggregator.py:497-503 (numpy add, a new array per client) on a
    rotating pool; returns (s per client, clients timed, last accumulator)."""
    from oracle.cpu_reference import fedavg_step

    acc = fedavg_step(None, [pool[0]], True)
    n, t0 = 0, time.perf_counter()
    while True:
        acc = fedavg_step(acc, [pool[(n + 1) % len(pool)]], False)
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= K - 1:
            break
    return (time.perf_counter() - t0) / n, n + 1, acc


def cpu_leg(policy: str, K: int, P: int, budget_s: float, seed: int, pool_n: int = 16) -> dict:
    """The oracle's round for one config on this host: accumulate (per client, extrapolated to K) and
    finalize timed separately; q-FedAvg's finalize loop over the K retained results is
    timed on a subsample at two sizes (per-client slope + fixed part) and extrapolated."""
    import argparse as _ap
    import copy

    import numpy as np
    import torch

    from oracle.cpu_reference import (OracleModel, OracleModelAdapter, OracleServerOptimizer, fedavg_close)

    pool = _pool(P, pool_n, seed)
    t_acc, n_acc, acc = _cpu_accumulate(pool, K, budget_s * (0.5 if policy != "fedavg" else 0.9))
    out = {"policy": policy, "clients": K, "params": P, "accumulate_ms_per_client": t_acc * 1e3,
           "accumulate_clients_timed": n_acc, "pool_buffers": pool_n, "kind": "port"}
    t1 = time.perf_counter()
    mean = fedavg_close(acc, K)
    t_div = time.perf_counter() - t1
    args = _ap.Namespace(gradient_policy=None, yogi_eta=3e-3, yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99,
                         learning_rate=0.05, qfed_q=1.0)
    if policy == "fedavg":
        t_fin = t_div
    elif policy == "fedyogi":
        args.gradient_policy = "fed-yogi"
        ad = OracleModelAdapter(OracleModel(["w"], [torch.from_numpy(pool[1].copy())]),
                                OracleServerOptimizer("fed-yogi", args))
        ad.set_weights(copy.deepcopy(mean))  # lazy YoGi state init (yogi.py:17-19) outside the timing
        t1 = time.perf_counter()
        ad.set_weights(copy.deepcopy(mean))  # torch_model_adapter.py:23-39 -> optimizers.py:43-63
        t_fin = t_div + time.perf_counter() - t1
    else:
        args.gradient_policy = "q-fedavg"
        rng = np.random.default_rng(seed)
        ts = []
        for n in (2, 4):
            res = [{"update_weight": [pool[(i + 2) % pool_n]], "moving_loss": float(rng.uniform(0.5, 2.0))}
                   for i in range(n)]
            ad = OracleModelAdapter(OracleModel(["w"], [torch.from_numpy(pool[1].copy())]),
                                    OracleServerOptimizer("q-fedavg", args))
            t1 = time.perf_counter()
            ad.set_weights(copy.deepcopy(mean), client_training_results=res)  # optimizers.py:65-104
            ts.append(time.perf_counter() - t1)
        per = max(1e-9, (ts[1] - ts[0]) / 2)
        fixed = max(0.0, ts[0] - 2 * per)
        out["finalize_ms_per_retained_client"] = per * 1e3
        t_fin = t_div + fixed + per * K
    t_round = t_acc * (K - 1) + t_fin
    out.update({"finalize_ms": t_fin * 1e3, "round_s": t_round, "client_updates_per_s": K / t_round,
                "hbm_equiv_gbps": (4 * K * P + 4 * P + EXTRA_BYTES[policy](K, P)) / t_round / 1e9,
                "cores": 1 if policy == "fedavg" else torch.get_num_threads(),
                "sample": f"{n_acc} of {K} client adds timed on a {pool_n}-buffer pool, extrapolated linearly"})
    del pool
    return out


def cpu_baseline(K: int, P: int, budget_s: float, seed: int, policy: str = "fedavg") -> dict:
    """The line's CPU leg: the oracle's round of the line's policy on a K-subsample, extrapolated to K (the whole
    model, at every N: the reference aggregator is one CPU process whatever the GPU count)."""
    leg = cpu_leg(policy, K, P, budget_s, seed)
    name = {"fedavg": "FedAvg (numpy, single-threaded)", "fedbuff": "FedAvg accumulate (numpy, single-threaded)",
            "fedyogi": "FedYoGi (numpy accumulate + torch CPU YoGi step)",
            "qfedavg": "q-FedAvg (numpy accumulate + torch CPU q-FedAvg step)"}[policy]
    return dict({"value": leg["client_updates_per_s"], "unit": "client-updates/s", "cores": leg["cores"],
                 "kind": "port",
                 "sample": (f"oracle {name} over {leg['accumulate_clients_timed']} of the "
                            f"{K} x {P} fp32 client updates (pool of {leg['pool_buffers']} distinct "
                            f"{4 * P / 1e6:.0f} MB buffers), {leg['accumulate_ms_per_client']:.1f} ms/client + "
                            f"{leg['finalize_ms']:.0f} ms finalize, extrapolated linearly to K={K}")},
                **_host_info())


# ------------------------------------------------------------------------------------------------
# config 1: the whole host round through the drop-in
# ------------------------------------------------------------------------------------------------
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


C1_JOB_CONF = os.path.join(ROOT, "tests", "golden", "c1_femnist_job_conf.json")


def c1_job_conf() -> dict:
    """Config 1's flags: benchmark/configs/femnist/conf.yml's job_conf converted as docker/driver.py:81-95 and
    parsed by config_parser.py, num_participants 50 -> 10 (tests/golden/gen_golden_r3.py, from the reference)."""
    with open(C1_JOB_CONF) as f:
        return json.load(f)


def c1_host_round(dev, seed: int, rounds: int = 300) -> dict:
    """BASELINE config 1 (FEMNIST small-CNN, K = num_participants of the job config = 10) through the drop-in:
    start_round, K on_result calls with host dicts (pinned staging + H2D), the fused reduce, and get_weights()
    (D2H) — the whole round the reference runs on the CPU (aggregator.py:489-511, torch_model_adapter.py:23-47)."""
    import argparse

    import numpy as np
    import torch

    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    job = c1_job_conf()
    args = argparse.Namespace(**job["args"])
    K = args.num_participants
    names, shapes, base, ups = _c1_updates(seed, K)
    model = synth.LayoutModule(names, shapes, [torch.float32] * len(names))
    on = args.cuda_device or dev  # aggregator.py:47: --cuda_device, else the current GPU
    agg = DeviceAggregator(TorchModelAdapter(model, optimizer=TorchServerOptimizer(args.gradient_policy, args, on),
                                             device=on), args)
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
            "job_config": {"file": "benchmark/configs/femnist/conf.yml (job_conf)",
                           "num_participants": f"{job['job_conf_num_participants']} -> {K}",
                           "gradient_policy": args.gradient_policy, "learning_rate": args.learning_rate,
                           "local_steps": args.local_steps, "data_set": args.data_set,
                           "model": (f"the job config names {args.model!r} (conf.yml:40); this line uses BASELINE "
                                     "config 1's FEMNIST small-CNN layout (MnistCNN with a 62-way head, P = 24,492, "
                                     "SURVEY §8) as BASELINE.json names it — the ResNet-18 layout is config 3")},
            "note": "host dicts in, global model out (get_weights); median of %d rounds" % rounds}


def pcie_inclusive_leg(dev, seed: int, K: int = 64, rounds: int = 6) -> dict:
    """SURVEY §8d's second figure: the headline model's round as a deployment sees it, from the executors'
    pickled upload payloads (CLIENT_EXECUTE_COMPLETION) through the mixin's zero-copy deserialize_response
    (aggregator.py:704), the pinned gather + H2D and the reduce, to get_weights() (D2H egress,
    torch_model_adapter.py:41-47).  25 M fp32 as 10 tensors of 2.5 M (100 MB per update); 8 distinct payloads
    reused.  Never `value`: it is bound by one PCIe link (PCIe-inclusive rate).  The same rounds as
    the N > 1 line's ``pcie_inclusive`` (fedscale_amd.inproc_bench.pcie_rounds), on one GPU."""
    import torch

    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from fedscale_amd.inproc_bench import headline_model, pcie_rounds

    adapter = TorchModelAdapter(headline_model(), device=dev)
    out, _ = pcie_rounds(adapter, K=K, rounds=rounds, seed=seed)
    del adapter
    torch.cuda.empty_cache()
    out["note"] = ("from pickled executor payloads: zero-copy deserialize_response, pinned gather + H2D, reduce, "
                   "get_weights() D2H; median and min of %d rounds after one warm-up round; bound by one PCIe "
                   "link, never `value`" % rounds)
    return out


def cpu_baseline_c1(seed: int, rounds: int = 300) -> dict:
    """The oracle's restatement of the same config-1 round on one host core (cpu_baseline leg)."""
    import numpy as np

    from oracle.cpu_reference import fedavg_close, fedavg_step

    K = c1_job_conf()["args"]["num_participants"]
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
    # the same round through the oracle's restatement of the reference loop: client_completion_handler's
    # lines, update_weight_aggregation, set_weights (deepcopy + load_state_dict + update_round_gradient)
    # and get_weights() — what the device leg's round covers (aggregator.py:454-511,
    # torch_model_adapter.py:23-47)
    import argparse

    import torch

    from oracle.cpu_reference import OracleAggregator, OracleModel, OracleModelAdapter, OracleServerOptimizer

    names, shapes, base, _ = _c1_updates(seed, K)
    args = argparse.Namespace(gradient_policy="fed-avg")
    agg = OracleAggregator(OracleModelAdapter(OracleModel(names, [torch.from_numpy(b) for b in base]),
                                              OracleServerOptimizer("fed-avg", args)), args)
    th = []
    for r in range(rounds + 5):
        t0 = time.perf_counter()
        agg.start_round(K)
        for k in range(K):
            agg.on_result({"client_id": k, "update_weight": ups[k], "moving_loss": 1.0})
        agg.model_wrapper.get_weights()
        th.append(time.perf_counter() - t0)
    hms = float(np.median(th[5:])) * 1e3
    return {"round_ms": ms, "client_updates_per_s": K / (ms * 1e-3), "cores": 1, "kind": "port",
            "note": "round_ms: the reduction arithmetic alone (fedavg_step x K + fedavg_close)",
            "handler_round_ms": hms,
            "handler_note": "the reference loop's whole round as the device leg runs it: handler lines, "
                            "update_weight_aggregation, set_weights, get_weights (oracle restatement)"}


# ------------------------------------------------------------------------------------------------
# device workloads
# ------------------------------------------------------------------------------------------------
class Workload:
    """One aggregation round of ``policy`` over K clients of a P-parameter model, on this rank's slice
    (parameter sharding over ``world`` ranks; the whole model when world == 1 or client mode).

    The client updates are resident in HBM: C <= K rows; a round with K > C streams K/C passes over the
    resident chunk (each pass reads its full 4*C*P bytes from HBM — the refill that ingress would do is
    not part of the device throughput), continuing one chain / delta across the passes exactly as the
    device path's chunk folding does."""

    def __init__(self, policy, K, P_total, rank, world, dev, seed, shards, *, weak=False, chunk=None,
                 budget_fraction=0.6, sets=1, mean_chain="auto", share_inputs=None):
        """``mean_chain`` (q-FedAvg): carry the plain FedAvg chain in the phase-1 kernel (fa_qfed_accumulate's
        ``chain``, the reference's model_weights, aggregator.py:497-507).  "auto" does what the drop-in does:
        fuse it whenever the round spans several resident chunks (DeviceRound, device_keep_mean=True)."""
        import numpy as np
        import torch

        from fedscale_amd import kernels as kx
        from fedscale_amd import synth
        from fedscale_amd.bucket import round_up, shard_bounds, shard_ld

        self.policy, self.K, self.world, self.dev, self.shards = policy, K, world, dev, shards
        self.cmode = shards.shards_clients
        if weak or self.cmode or world == 1:
            self.P, self.P_total = P_total, P_total * (world if weak else 1)
            ld = round_up(P_total, 64)
        else:
            b = shard_bounds(P_total, world)  # the drop-in's balanced 64-aligned slices (BucketLayout)
            self.P, self.P_total = b[rank + 1] - b[rank], P_total
            ld = shard_ld(P_total, world)
        self.ld = ld
        if share_inputs is not None:  # the resident uploads of another workload of the same shape (paired timing)
            cap = share_inputs.C
        else:
            free, _ = torch.cuda.mem_get_info(dev)
            cap = max(1, int(free * budget_fraction) // (4 * ld * sets))
            if policy == "qfedavg":
                cap = min(cap, kx.qfed_max_chunk())
        self.C = min(K, cap, chunk or K)
        self.passes = [(k0, min(self.C, K - k0)) for k0 in range(0, K, self.C)]
        self.mean_chain = (len(self.passes) > 1) if mean_chain == "auto" else bool(mean_chain)
        self.xs = []
        for i in range(sets):  # sets > 1: rotate input sets so the 256 MiB Infinity Cache cannot serve repeats
            if share_inputs is not None:
                if share_inputs.xs[i].shape != (self.C, ld):
                    raise ValueError("share_inputs: another shape")
                self.xs.append(share_inputs.xs[i])
                continue
            x = torch.empty(self.C, ld, dtype=torch.float32, device=dev)
            synth.fill(x, self.C, self.P, seed=seed + 7919 * rank + 31 * i)
            self.xs.append(x)
        self.it = 0
        self.rest_s = 0.0  # the card's idle before this workload's timed region (time_workload)
        self.out = torch.zeros(ld, dtype=torch.float32, device=dev)
        self.acc = torch.zeros(ld, dtype=torch.float32, device=dev) if (self.cmode or len(self.passes) > 1) else None
        self.Kg = K * world if self.cmode else K  # clients in the round (client mode: every rank brings K)
        self.denom = float(np.float32(self.Kg))
        self.a = None
        if policy == "fedbuff":
            s = [1 / (1 + (k % 6)) ** 0.5 for k in range(self.Kg)]
            self.a = torch.tensor(np.asarray(s[rank * K:(rank + 1) * K] if self.cmode else s, dtype=np.float32),
                                  device=dev)
            self.denom = float(np.float32(sum(s)))
        self.yogi = None
        if policy == "fedyogi":
            self.yogi = dict(last=torch.zeros(ld, device=dev), m=torch.zeros(ld, device=dev),
                             v=torch.zeros(ld, device=dev), eta=float(np.float32(3e-3)), tau=float(np.float32(1e-8)),
                             beta=float(np.float32(0.9)), omb=float(np.float32(1 - 0.9)),
                             omb2=float(np.float32(1 - 0.99)), init=False)
            synth.fill(self.yogi["last"].view(1, -1), 1, self.P, seed=seed + 1)
            self.mean = torch.zeros(ld, device=dev)  # the round's FedAvg mean (model_weights)
        self.qf = None
        if policy == "qfedavg":
            rng = np.random.default_rng(seed)
            losses = rng.uniform(0.5, 2.0, size=self.Kg)
            lr, q = 0.05, 1.0
            mine = losses[rank * K:(rank + 1) * K] if self.cmode else losses
            self.qf = dict(last=torch.empty(1, ld, device=dev), delta=torch.zeros(ld, device=dev),
                           sq=torch.zeros(self.Kg, dtype=torch.float64, device=dev),
                           ws=kx.qfed_workspace(self.C, dev, ld, self.P), hs=torch.zeros(2, device=dev), lr=lr,
                           alpha=torch.tensor([np.float32(np.float_power(l + 1e-10, q)) for l in mine], device=dev),
                           c1=torch.tensor([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses],
                                           device=dev),
                           c2=torch.tensor([np.float32((1 / lr) * np.float_power(l + 1e-10, q)) for l in losses],
                                           device=dev))
            synth.fill(self.qf["last"], 1, self.P, seed=seed + (0 if self.cmode else 7919 * rank), scale_noise=0.0)
            self.qf["last"] = self.qf["last"][0]
            self.qf["chain"] = torch.zeros(ld, device=dev) if (self.mean_chain and not self.cmode) else None
        self.stream = torch.cuda.current_stream(dev)

    @property
    def alg_bytes(self) -> int:
        """SURVEY §8d algorithmic bytes of this rank's dominant kernel(s) per round.  q-FedAvg over several
        passes re-reads last and reads back delta (and the chain) on every pass after the first."""
        b = 4 * self.K * self.P + 4 * self.P + EXTRA_BYTES[self.policy](self.K, self.P)
        if self.policy == "qfedavg":
            n = len(self.passes)
            b += 12 * self.P * (n - 1)  # passes 2..n: last re-read, delta read back and written again
            if self.qf is not None and self.qf["chain"] is not None:
                b += 4 * self.P * (2 * n - 1)  # chain written every pass, read back on passes 2..n
        return b

    def step(self, ev=None):
        from fedscale_amd import kernels as kx

        x = self.xs[self.it % len(self.xs)]
        self.it += 1
        K, P, st = self.K, self.P, self.stream
        if ev is not None:
            ev[0].record(st)
        if self.qf is not None:  # optimizers.py:73-104: phase 1 (timed as the dominant kernel), hs, phase 2
            qf = self.qf
            qf["sq"].zero_()
            kb = self.shards.rank * K if self.cmode else 0
            for i, (k0, n) in enumerate(self.passes):
                kx.qfed_accumulate(x, n, P, last=qf["last"], alpha=qf["alpha"][k0:k0 + n], lr=qf["lr"],
                                   delta=qf["delta"], sqnorm=qf["sq"][kb + k0:kb + k0 + n], workspace=qf["ws"],
                                   accumulate=i > 0, chain=qf["chain"])
            if ev is not None:
                ev[1].record(st)
            if self.cmode:  # per-rank partial delta chains + each client's norm from its owner rank
                self.shards.all_reduce_sum(qf["delta"])
                self.shards.all_reduce_sum(qf["sq"])
            elif self.world > 1:  # the one exchange of parameter sharding: per-client norms over the shards
                self.shards.sum_partials(qf["sq"])
            kx.qfed_hs(qf["sq"], qf["c1"], qf["c2"], self.Kg, qf["hs"])
            kx.qfed_finalize(qf["last"], qf["delta"], qf["hs"], self.out, P)
            return
        last = len(self.passes) - 1
        for i, (k0, n) in enumerate(self.passes):
            a = self.a[k0:k0 + n] if self.a is not None else None
            acc_in = self.acc if i > 0 else None
            if i < last or self.cmode:  # chain only: a middle pass, or this rank's partial (client mode)
                kx.reduce(x, n, P, self.acc, a=a, acc_in=acc_in)
            elif self.yogi is None:
                kx.reduce(x, n, P, self.out, a=a, acc_in=acc_in, denom=self.denom, finalize=True)
            else:  # as the drop-in runs FedYoGi: the mean, then the YoGi step over it (TorchModelAdapter)
                kx.reduce(x, n, P, self.mean, a=a, acc_in=acc_in, denom=self.denom, finalize=True)
                if ev is not None and len(ev) > 2:  # between the two kernels: each one's time on its own
                    ev[2].record(st)
                y = self.yogi
                kx.yogi_step(self.mean, y["last"], y["m"], y["v"], self.out, P, init=y["init"],
                             **{k: y[k] for k in ("eta", "tau", "beta", "omb", "omb2")})
        if ev is not None:
            ev[1].record(st)
        if self.cmode:  # partial chain of this rank's clients, RCCL all-reduce, finish on the summed vector
            self.shards.all_reduce_sum(self.acc)
            x1 = self.acc.view(1, self.ld)
            if self.yogi is None:
                kx.reduce(x1, 1, P, self.out, denom=self.denom, finalize=True)
            else:
                kx.reduce(x1, 1, P, self.mean, denom=self.denom, finalize=True)
                y = self.yogi
                kx.yogi_step(self.mean, y["last"], y["m"], y["v"], self.out, P, init=y["init"],
                             **{k: y[k] for k in ("eta", "tau", "beta", "omb", "omb2")})

    def free(self):
        import torch

        self.xs = []
        self.acc = self.out = self.qf = self.yogi = self.mean = None
        torch.cuda.empty_cache()


def _sync_all(dev, world):
    import torch
    import torch.distributed as dist

    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize(dev)


def _max_over_ranks(vals, dev, world, backend):
    import torch
    import torch.distributed as dist

    t = torch.tensor(vals, dtype=torch.float64)
    if world > 1:
        if backend == "nccl":
            t = t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def _all_ranks(val: float, dev, world, backend) -> list:
    """[value of rank 0, rank 1, ...] (an all-gather of one float per rank)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [float(val)]
    t = torch.tensor([float(val)], dtype=torch.float64)
    if backend == "nccl":
        t = t.to(dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o.cpu()[0]) for o in out]


def pmc_traffic(workload: str, resident: int, launches: int, build_id: str, path: str = None):
    """roofline.traffic: HBM bytes per launch of THIS run's shape and library, from profiles/pmc_traffic.json
    (tools/pmc_parse.py keys every entry by workload, resident clients per pass, launches per round and the build
    id of the library the profiled command loaded).  None when no entry has all four."""
    path = path or PMC_FILE
    try:
        with open(path) as f:
            db = json.load(f)
    except (OSError, ValueError):
        return None
    e = db.get("entries", {}).get(f"{workload}|C{resident}|L{launches}|{build_id}")
    return None if e is None else float(e["hbm_bytes_per_launch"])


#: seconds the card idles before each heavy timed region of ``other_configs`` (--rest; the headline's region, the first
#: of the line, takes no rest unless --rest is given).  100 s of back-to-back headline rounds showed no decay
#: (profiles/r05_sustain100.json), but the configs timed one after another do: without a rest config 5 on one GPU ran
#: at the board's 1400 W cap (1384 W mean) with the shader clock down to 2150 MHz, and the shard of 8 timed after it at
#: 1810 MHz, 3 % slower (a round-5 no-rest line).  An aggregator's GPU works in bursts (one round,
#: then idle while the clients train), so each config is timed from a rested card and ALSO back to back right after
#: (``sustained`` on each config line), both with the card's telemetry.  Outside the timed region.
REST_S = 12.0
HEADLINE_REST_S = 0.0  # --rest sets both


def _rest(w, steps, dev, rest_s=None):
    import torch

    REST_S_ = REST_S if rest_s is None else rest_s
    if REST_S_ > 0 and w.alg_bytes * max(1, steps) > 20e9:  # heavy regions only (c2's 0.4 GB rounds need none)
        torch.cuda.synchronize(dev)
        time.sleep(REST_S_)
        return REST_S_
    return 0.0


def time_workload(w: Workload, steps: int, warmup: int, dev, world, backend, rest_s=None):
    """Warmup, then exactly ``steps`` rounds between barrier + synchronize; (wall s, mean dominant-kernel
    ms), both max over ranks.  With ``--rest`` > 0 heavy regions start after that idle (every rank rests alike)."""
    import numpy as np
    import torch

    w.rest_s = _rest(w, steps, dev, rest_s)
    if warmup < 0:  # auto: at least 3 rounds and, on one GPU, at least WARMUP_S seconds of them (clocks settled)
        import torch

        n, t0 = 0, time.perf_counter()
        while n < 3 or (world == 1 and time.perf_counter() - t0 < WARMUP_S):
            for _ in range(4):  # batches of 4 rounds queued back to back, as the timed rounds are
                w.step()
                n += 1
            torch.cuda.synchronize(dev)
        warmup = n
    else:
        for _ in range(warmup):
            w.step()
    w.warmup_rounds = warmup
    split = w.yogi is not None and not w.cmode  # FedYoGi: a third event between the mean and the YoGi step
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3 if split else 2)) for _ in range(steps)]
    from fedscale_amd.cardstate import CardSampler

    w.card_before = CardSampler(dev).read_once()
    sampler = CardSampler(dev, period_s=0.02, process=True)  # a child process: no GIL contention with the launches
    _sync_all(dev, world)
    sampler.start()
    t0 = time.perf_counter()
    for i in range(steps):
        w.step(evs[i])
    _sync_all(dev, world)
    wall = time.perf_counter() - t0
    w.card = sampler.stop().summary()
    w.step_ms = [e[0].elapsed_time(e[1]) for e in evs]  # each timed round's dominant-kernel ms (this rank)
    kern_ms = float(np.mean(w.step_ms))
    w.split_ms = None
    if split:  # (mean of k_reduce's launches, mean of k_yogi_step) per step, max over ranks
        w.split_ms = _max_over_ranks([float(np.mean([e[0].elapsed_time(e[2]) for e in evs])),
                                      float(np.mean([e[2].elapsed_time(e[1]) for e in evs]))], dev, world, backend)
    return _max_over_ranks([wall, kern_ms], dev, world, backend), kern_ms, _all_ranks(kern_ms, dev, world, backend)


MEM_FRACTION = 0.6
CONFIG_SUSTAIN_S = 3.0  # back-to-back seconds after each heavy config's rested region (--config-sustain)
PAIR_S = 3.0  # seconds of each form in config 5's paired chain / chain-free region
WARMUP_S = 1.0  # --warmup -1: seconds of untimed rounds before the headline's timed region (one GPU)


def time_paired(wa: "Workload", wb: "Workload", steps: int, dev, world, backend):
    """Rounds of ``wa`` and ``wb`` alternating in one region (after one rest and one warmup round each); (mean ms of
    wa's rounds, mean ms of wb's rounds), each from its own HIP event pairs on the launch stream, max over ranks."""
    import numpy as np
    import torch

    _rest(wa, steps, dev)
    wa.step()
    wb.step()
    ea = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    eb = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    _sync_all(dev, world)
    for i in range(steps):
        wa.step(ea[i])
        wb.step(eb[i])
    _sync_all(dev, world)
    a = float(np.mean([e[0].elapsed_time(e[1]) for e in ea]))
    b = float(np.mean([e[0].elapsed_time(e[1]) for e in eb]))
    return _max_over_ranks([a, b], dev, world, backend)


def config_line(name, cfg, dev, rank, world, shards, seed, backend, steps=5, warmup=2, **kw) -> dict:
    """A BASELINE config on all ranks (parameter-sharded over them), for other_configs."""
    kw.setdefault("budget_fraction", MEM_FRACTION)
    w = Workload(cfg["policy"], cfg["clients"], cfg["params"], rank, world, dev, seed, shards, **kw)
    (wall, kern_max), _, _ = time_workload(w, steps, warmup, dev, world, backend)
    ms = wall * 1e3 / steps
    out = {"policy": cfg["policy"], "clients": cfg["clients"], "params": cfg["params"], "n_gpus": world,
           "params_per_gpu": w.P, "resident_clients": w.C, "passes": len(w.passes), "round_ms": ms,
           "client_updates_per_s": cfg["clients"] / (ms * 1e-3),
           "hbm_gbps_per_gpu": w.alg_bytes / (ms * 1e-3) / 1e9, "dominant_kernel_ms": kern_max,
           "hbm_gbps_kernel": w.alg_bytes / (kern_max * 1e-3) / 1e9, "card_rest_s": w.rest_s,
           "card": {k: (v["mean"] if isinstance(v, dict) else v) for k, v in (getattr(w, "card", None) or {}).items()
                    if k in ("power_w", "temp_junction_c", "temp_mem_c", "sclk_mhz", "mclk_mhz", "samples")}}
    if CONFIG_SUSTAIN_S > 0 and world == 1 and w.alg_bytes * max(1, steps) > 20e9:
        # the same rounds back to back right after the rested region (no rest): the rate this config settles at
        # (one GPU only: the ranks' rounds would not stay in step through a time-bounded loop's collectives)
        sus = sustained_leg(w, dev, CONFIG_SUSTAIN_S, 1, ms, window_s=CONFIG_SUSTAIN_S, chunk_s=0.5)
        out["sustained"] = {"round_ms": sus["ms_per_step"], "hbm_gbps_kernel": sus["hbm_gbps"],
                            "seconds": sus["seconds"], "rounds": sus["steps"],
                            "card": {k: v["mean"] for k, v in sus["card_window"].items() if isinstance(v, dict)}}
    if getattr(w, "split_ms", None):
        from fedscale_amd import kernels as kx

        red_ms, yogi_ms = w.split_ms
        K_, P_ = w.K, w.P
        out["kernels"] = {
            "k_reduce (fa_reduce FA_FINALIZE, the mean)": {
                "ms": red_ms, "launches": len(w.passes) * kx.reduce_launches(w.C if len(w.passes) > 1 else K_, P_),
                "alg_bytes": 4 * K_ * P_ + 4 * P_, "hbm_gbps": (4 * K_ * P_ + 4 * P_) / (red_ms * 1e-3) / 1e9},
            "k_yogi_step (fa_yogi_step)": {
                "ms": yogi_ms, "launches": 1, "alg_bytes": 28 * P_, "hbm_gbps": 28 * P_ / (yogi_ms * 1e-3) / 1e9,
                "note": "reads mean, last, m, v; writes m, v, new (16P + 12P)"},
            "note": "one HIP event pair per kernel, on the launch stream; rocprofv3 of the same round: "
                    "profiles/r04_c4_fedyogi_unfused_kernel_stats.csv"}
    if cfg["policy"] == "qfedavg":
        out["mean_chain"] = w.mean_chain
        if w.mean_chain:
            out["mean_chain_note"] = ("timed as the drop-in runs this round: it spans several chunks, so the FedAvg "
                                      "chain (the reference's model_weights) is fused into phase 1; the chain-free "
                                      "kernel is beside it (no_chain)")
            # the chain-free kernel over the SAME resident uploads, its rounds alternating with the chain form's
            # in one region (one event pair per round): the card's drift over a region hits both alike, so the
            # pair gives the chain's cost where two separately timed regions differed by up to +-2 % (round 5)
            kw2 = dict(kw, mean_chain=False)
            w2 = Workload(cfg["policy"], cfg["clients"], cfg["params"], rank, world, dev, seed, shards,
                          share_inputs=w, **kw2)
            # about PAIR_S seconds of each form (config 5 on one GPU: 6 rounds each; its shard of 8: ~40): the
            # chain cost is 1-2 % of a round, and 3 rounds each read 1.5-6 % on one box (profiles/r05_budget*_paired.log)
            n_pair = max(steps, 3, int(math.ceil(PAIR_S / max(kern_max * 1e-3, 1e-6))))
            pair = time_paired(w, w2, n_pair, dev, world, backend)
            out["no_chain"] = {"round_ms_paired": pair[1], "dominant_kernel_ms": pair[1],
                               "hbm_gbps_kernel": w2.alg_bytes / (pair[1] * 1e-3) / 1e9,
                               "chain_round_ms_paired": pair[0],
                               "chain_cost_pct": 100.0 * (pair[0] / pair[1] - 1.0),
                               "chain_cost_pct_unpaired_note": "the chain form's timed region above against this "
                                                               "pair's chain-free rounds: %.2f %%" % (
                                                                   100.0 * (kern_max / pair[1] - 1.0)),
                               "rounds_each": n_pair,
                               "note": "rounds alternate chain / chain-free over the same resident uploads in one "
                                       "region; one HIP event pair per round on the launch stream"}
            w2.xs = []
            w2.free()
    if kern_max < 1.0:  # short kernels: a HIP event pair per launch adds µs; also time back-to-back launches
        import torch

        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = max(steps, 50)
        _sync_all(dev, world)
        e0.record(w.stream)
        for _ in range(n):
            w.step()
        e1.record(w.stream)
        torch.cuda.synchronize(dev)
        chained = _max_over_ranks([e0.elapsed_time(e1) / n], dev, world, backend)[0]
        out["kernel_ms_back_to_back"] = chained
        out["hbm_gbps_back_to_back"] = w.alg_bytes / (chained * 1e-3) / 1e9
        out["timing_note"] = ("dominant_kernel_ms: a HIP event pair around each launch (adds a few µs to a ~60 µs "
                              "kernel); kernel_ms_back_to_back: one event pair around %d back-to-back launches "
                              "(launch gaps included); rocprofv3's kernel duration is in DESIGN.md §5" % n)
    if len(w.passes) > 1:
        out["note"] = ("K > resident chunk: each round streams %d passes over the resident %d clients (every pass "
                       "reads its 4*C*P bytes from HBM; the ingress refill is not part of this device rate)"
                       % (len(w.passes), w.C))
    w.free()
    return out


def single_gpu_configs(dev, seed, shards, backend, cpu_budget) -> dict:
    """N = 1: BASELINE configs 1-5 on this GPU, each beside its CPU leg (the oracle on this host)."""
    out = {"c1_femnist_cnn_k10_host_round": c1_host_round(dev, seed)}
    c2 = config_line("c2", CONFIGS["c2"], dev, 0, 1, shards, seed, backend, steps=20, warmup=4, sets=2)
    c2["note"] = "two rotating input sets (400 MB each): the 256 MiB Infinity Cache cannot serve repeats"
    out["c2_synthetic_k100_p1M"] = c2
    out["c3_resnet18_layout_k1000_p11191242"] = config_line("c3", CONFIGS["c3"], dev, 0, 1, shards, seed, backend,
                                                            steps=10, warmup=2)
    out["c4_fedyogi_k1000_p25M"] = config_line("c4", CONFIGS["c4"], dev, 0, 1, shards, seed, backend)
    out["c5_qfedavg_k10000_p100M"] = config_line("c5", CONFIGS["c5"], dev, 0, 1, shards, seed, backend, steps=2,
                                                 warmup=1)
    # one GPU's share of the multi-GPU configs at their BASELINE GPU counts
    out["c4_fedyogi_shard_of_4"] = config_line(
        "c4s", dict(CONFIGS["c4"], params=25_000_000 // 4), dev, 0, 1, shards, seed, backend, steps=10)
    out["c5_qfedavg_shard_of_8"] = config_line(
        "c5s", dict(CONFIGS["c5"], params=100_000_000 // 8), dev, 0, 1, shards, seed, backend, steps=3, warmup=1)
    out["headline_model_pcie_inclusive"] = pcie_inclusive_leg(dev, seed)
    if cpu_budget > 0:
        out["c1_femnist_cnn_k10_host_round"]["cpu_baseline"] = cpu_baseline_c1(seed)
        for key, name, share in (("c2_synthetic_k100_p1M", "c2", 0.1), ("c3_resnet18_layout_k1000_p11191242", "c3", 0.4),
                                 ("c4_fedyogi_k1000_p25M", "c4", 0.8), ("c5_qfedavg_k10000_p100M", "c5", 1.0)):
            c = CONFIGS[name]
            leg = cpu_leg(c["policy"], c["clients"], c["params"], cpu_budget * share, seed)
            leg["device_speedup"] = out[key]["client_updates_per_s"] / leg["client_updates_per_s"]
            out[key]["cpu_baseline"] = leg
    return out


def run_selfcheck(world: int, timeout_s: int = 150) -> dict:
    """fedscale_amd.selfcheck over GPUs 0..N-1 in a child process (rank 0, N > 1): the sharded drop-in against
    one GPU, bit for bit, with every launch checked against its part's stream.  Summarised for the JSON line."""
    import subprocess

    import torch

    n = min(world, torch.cuda.device_count())
    if n < 2:
        return {"skipped": f"{n} GPU(s) visible to rank 0"}
    cmd = [sys.executable, "-m", "fedscale_amd.selfcheck", "--devices", ",".join(str(i) for i in range(n))]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"devices": n, "ok": False, "error": f"no result within {timeout_s} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        return {"devices": n, "ok": False, "rc": r.returncode, "error": r.stderr[-400:]}
    rep = json.loads(lines[-1])
    out = {"devices": n, "ok": bool(rep.get("ok")), "seconds": round(time.perf_counter() - t0, 1)}
    if "error" in rep:
        out["error"] = rep["error"]
    for pol, v in rep.get("policies", {}).items():
        out[pol] = {k: v[k] for k in ("ok", "transport", "native_calls", "calls_off_their_stream",
                                      "buffers_on_their_device", "mismatch") if k in v}
    return out


def promote_inproc(res: dict, inproc: dict, K: int, steps: int) -> None:
    """N > 1: the line's ``value`` is the in-process drop-in's round (one aggregator process driving the N GPUs,
    ShardedModelAdapter: what a FedScale deployment runs, aggregator.py:177-192 / 919-963), timed over the same
    ``steps`` after the same warmup, every part's launches included, from the first launch to every part's last
    kernel.  The SPMD figure (one process per GPU) stays beside it as ``value_spmd``.  If the in-process run failed,
    ``value`` stays the SPMD one and ``value_source`` says why."""
    fa = inproc.get("policies", {}).get("fedavg") if "policies" in inproc else inproc
    if not fa or not fa.get("ok") or "inproc_round_ms" not in fa:
        res["value_source"] = "spmd (the in-process drop-in run failed: %s)" % ((fa or inproc).get("error"),)
        return
    if fa.get("distinct_gpus") is False:  # parts sharing a GPU (a rehearsal): plumbing, never the line's value
        res["value_source"] = "spmd (the in-process parts share %s GPU(s): plumbing, not promoted)" % (
            len(set(fa.get("devices", []))) or "one")
        return
    res["value_spmd"], res["ms_per_step_spmd"] = res["value"], res["ms_per_step"]
    for k in ("scaling_vs_one_gpu", "scaling_vs_one_gpu_incl_reassembly", "value_incl_reassembly",
              "round_ms_incl_reassembly"):
        if k in res:
            res[k + "_spmd"] = res.pop(k)
    if fa.get("part_kernel_ms") and fa.get("part_alg_bytes"):
        # the per-GPU roofline of the promoted round: every part's bytes over its own kernel time, the slowest part
        rates = [b / (ms * 1e-3) / 1e9 for b, ms in zip(fa["part_alg_bytes"], fa["part_kernel_ms"])]
        i = min(range(len(rates)), key=rates.__getitem__)
        L = fa.get("part_launches", [1] * len(rates))[i]
        res["roofline_spmd"] = res["roofline"]
        res["roofline"] = dict(res["roofline"], achieved=rates[i], frac=rates[i] / HBM_PEAK_GBS,
                               alg_bytes_per_launch=fa["part_alg_bytes"][i] / L, launches_per_step=L,
                               kernel_ms_per_launch=fa["part_kernel_ms"][i] / L, traffic=None,
                               source="inproc_drop_in.fedavg: the slowest part (its bytes over its own kernel events)")
        res["hbm_gbps"], res["kernel_ms"] = rates[i], fa["part_kernel_ms"][i]
    ms = fa["inproc_round_ms"]
    res["ms_per_step"] = ms
    res["value"] = K / (ms * 1e-3)
    res["value_source"] = ("inproc_drop_in.fedavg: one process, ShardedModelAdapter over the N GPUs, %d timed rounds "
                           "after the same warmup (synchronize on every GPU both sides)" % fa.get("rounds", steps))
    if fa.get("egress_ms") is not None:
        res["round_ms_incl_egress"] = fa.get("inproc_round_ms_incl_egress")
    if "speedup_vs_one_gpu" in fa:
        res["scaling_vs_one_gpu"] = fa["speedup_vs_one_gpu"]
    res["config"]["parallelism"] = (f"param-shard x{len(fa['devices'])} in ONE aggregator process "
                                    f"(ShardedModelAdapter, transport {fa.get('transport')}); value_spmd: one process "
                                    "per GPU")


def run_inproc_bench(world: int, K: int, P: int, backend: str, steps: int = 6, warmup: int = 2,
                     timeout_s: int = 300) -> dict:
    """fedscale_amd.inproc_bench in a child process (rank 0, N > 1): a timed device-resident round of the
    in-process drop-in (ShardedModelAdapter over GPUs 0..N-1, the way FedScale's single-process aggregator is
    deployed on a node) beside the single-device adapter.  With fewer GPUs than ranks (a gloo rehearsal on one
    card) the parts share the visible GPUs (copy transport): plumbing only."""
    import subprocess

    import torch

    nd = torch.cuda.device_count()
    devs = [i % max(1, nd) for i in range(world)]
    cmd = [sys.executable, "-m", "fedscale_amd.inproc_bench", "--devices", ",".join(map(str, devs)),
           "--clients", str(K), "--params", str(P), "--policies", "fedavg,fed-yogi", "--rounds", str(steps),
           "--warmup", str(warmup)]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"devices": devs, "ok": False, "error": f"no result within {timeout_s} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        return {"devices": devs, "ok": False, "rc": r.returncode, "error": r.stderr[-400:]}
    rep = json.loads(lines[-1])
    rep["seconds"] = round(time.perf_counter() - t0, 1)
    rep["workloads"] = "fedavg: the headline round; fed-yogi: config 4's (1000 x 25 M, mean then YoGi step per part)"
    if len(set(devs)) < len(devs):
        rep["note"] = (f"{world} parts on {len(set(devs))} GPU(s) (backend {backend} rehearsal): plumbing only, "
                       "not an N-GPU rate")
    return rep


#: one PCIe link's rate for the PCIe-inclusive round of the headline model on one GPU (BENCH_r05.json
#: other_configs.headline_model_pcie_inclusive: 53.8 GB/s end to end, the copy engine's 56-57 GB/s, r01_h2d_probe.json): the
#: basis of the N-link prediction each N > 1 line carries
PCIE_LINK_GBPS = 54.0


def pcie_prediction(world: int) -> dict:
    """What the N-GPU PCIe-inclusive round should reach if every GPU's link carries what one link carries alone:
    N x one link.  The registered ingress reads each payload byte once from host DRAM, so up to
    8 links (~430 GB/s) stays inside the host's memory bandwidth (2 sockets x 12 channels of DDR5); below
    N x 54 GB/s, the bound is elsewhere (a shared PCIe switch, one socket's DRAM, the Python ingress loop)."""
    return {"host_to_device_GBps": world * PCIE_LINK_GBPS, "client_updates_per_s": world * PCIE_LINK_GBPS * 1e9 / 100e6,
            "basis": "N x %g GB/s (one link's PCIe-inclusive rate at N = 1, DESIGN.md §5/§6)" % PCIE_LINK_GBPS}


def run_inproc_pcie(world: int, backend: str, K: int = 64, rounds: int = 6, timeout_s: int = 300) -> dict:
    """The PCIe-inclusive round over GPUs 0..N-1 in a child process (rank 0, N > 1; fedscale_amd.inproc_bench
    --pcie): one aggregator process, the executors' pickled payloads registered in place and sliced over the N links
    (ShardedModelAdapter), reduce on every GPU, get_weights() D2H.  With fewer GPUs than ranks (a gloo rehearsal on
    one card) the parts share the visible GPUs: plumbing only."""
    import subprocess

    import torch

    nd = torch.cuda.device_count()
    devs = [i % max(1, nd) for i in range(world)]
    cmd = [sys.executable, "-m", "fedscale_amd.inproc_bench", "--devices", ",".join(map(str, devs)), "--pcie",
           "--clients", str(K), "--rounds", str(rounds)]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"devices": devs, "ok": False, "error": f"no result within {timeout_s} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if not lines:
        return {"devices": devs, "ok": False, "rc": r.returncode, "error": r.stderr[-400:]}
    rep = json.loads(lines[-1])
    rep["seconds"] = round(time.perf_counter() - t0, 1)
    rep["prediction"] = pcie_prediction(world)
    if rep.get("ok") and rep.get("distinct_gpus"):
        rep["vs_prediction"] = rep["host_to_device_GBps"] / rep["prediction"]["host_to_device_GBps"]
    elif rep.get("ok"):
        rep["note_backend"] = (f"{world} parts on {len(set(devs))} GPU(s) (backend {backend} rehearsal): plumbing only, "
                               "not an N-link rate")
    return rep


#: fields every line carries (the contract), and what an N > 1 line must carry on top (the north
#: star's CPU baseline beside the 1/2/4/8-GPU figures, and the rate including H2D and D2H copies)
LINE_FIELDS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
               "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
ROOFLINE_FIELDS = ("bound", "achieved", "peak", "unit", "frac", "traffic")
CPU_BASELINE_FIELDS = ("value", "unit", "cores", "kind", "sample")
PCIE_FIELDS = ("round_ms", "client_updates_per_s", "host_to_device_GBps", "phases_ms", "parts", "prediction")
PART_FIELDS = ("device", "params", "host_numa_node", "h2d_GBps_over_ingress")


def check_line(res: dict) -> list:
    """Missing north-star quantities of a bench line ([] = complete).  N = 1: the contract's fields with a non-null
    cpu_baseline (unless its CPU legs were switched off).  N > 1: also ``cpu_baseline`` (the oracle on rank 0's host
    cores, same run) and ``pcie_inclusive`` (the N-link round from pickled payloads, every part's link rate and NUMA
    node, and the prediction it is checked against)."""
    miss = [k for k in LINE_FIELDS if k not in res]
    miss += ["roofline." + k for k in ROOFLINE_FIELDS if k not in (res.get("roofline") or {})]
    cb = res.get("cpu_baseline")
    if cb is None:
        if res.get("n_gpus", 1) > 1 or not res.get("cpu_legs_off"):
            miss.append("cpu_baseline (null)")
    else:
        miss += ["cpu_baseline." + k for k in CPU_BASELINE_FIELDS if k not in cb]
    if res.get("n_gpus", 1) > 1:
        pc = res.get("pcie_inclusive")
        if not pc:
            miss.append("pcie_inclusive")
        elif not pc.get("ok", True):
            miss.append("pcie_inclusive (failed: %s)" % pc.get("error"))
        else:
            miss += ["pcie_inclusive." + k for k in PCIE_FIELDS if k not in pc]
            parts = pc.get("parts") or []
            if len(parts) != res["n_gpus"]:
                miss.append("pcie_inclusive.parts (%d for %d GPUs)" % (len(parts), res["n_gpus"]))
            for i, p in enumerate(parts):
                miss += ["pcie_inclusive.parts[%d].%s" % (i, k) for k in PART_FIELDS if k not in p]
    return miss


def one_gpu_reference(policy, K, P, dev, seed, steps=5, warmup=2) -> dict:
    """The same round on ONE GPU over the whole model, in the same run (rank 0, after the N-rank timed region):
    the reference the scaling figures below divide by."""
    from fedscale_amd.state import ShardGroup

    w = Workload(policy, K, P, 0, 1, dev, seed, ShardGroup(0, 1), budget_fraction=MEM_FRACTION)
    _rest(w, steps, dev)  # from the same card state as the N-rank region it is compared with
    for _ in range(warmup):
        w.step()
    import torch

    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        w.step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / steps
    w.free()
    return {"ms_per_step": ms, "client_updates_per_s": K / (ms * 1e-3), "steps": steps}


def sustained_leg(w: "Workload", dev, seconds: float, launches: int, est_ms: float, window_s: float = 3.0,
                  chunk_s: float = 1.0) -> dict:
    """Back-to-back rounds of the headline workload for ``seconds`` right after its rested timed region, no rest:
    the rate a card streaming without pause settles at, beside the card's power, temperatures and clocks (sysfs,
    fedscale_amd/cardstate.py).  Chunks of ~1 s, each timed by one HIP event pair on the launch stream;
    ``sustained`` = the chunks of the last ``window_s`` seconds."""
    import numpy as np
    import torch

    from fedscale_amd.cardstate import CardSampler

    per_chunk = max(1, int(round(1000.0 * chunk_s / max(est_ms, 1e-3))))
    sampler = CardSampler(dev, period_s=0.05)
    torch.cuda.synchronize(dev)
    sampler.start()
    t_start = time.perf_counter()
    chunks = []
    while time.perf_counter() - t_start < seconds:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(w.stream)
        for _ in range(per_chunk):
            w.step()
        e1.record(w.stream)
        torch.cuda.synchronize(dev)
        chunks.append((t0, time.perf_counter(), per_chunk, e0.elapsed_time(e1) / per_chunk))
    sampler.stop()
    alg = w.alg_bytes
    keys = ("power_w", "temp_junction_c", "temp_mem_c", "sclk_mhz", "mclk_mhz")
    series = []
    for t0, t1, n, ms in chunks:
        card = sampler.summary(t0, t1)
        series.append(dict({"t_s": round(t0 - t_start, 2), "steps": n, "ms_per_step": ms,
                            "hbm_gbps": alg / (ms * 1e-3) / 1e9},
                           **{k: card[k]["mean"] for k in keys if k in card}))
    t_end = chunks[-1][1]
    last = [c for c in chunks if c[0] >= t_end - window_s] or chunks[-1:]
    ms = float(np.sum([c[2] * c[3] for c in last]) / np.sum([c[2] for c in last]))
    gbps = alg / (ms * 1e-3) / 1e9
    return {"seconds": round(t_end - t_start, 2), "window_s": window_s, "steps": int(sum(c[2] for c in chunks)),
            "ms_per_step": ms, "ms_per_launch": ms / launches, "hbm_gbps": gbps, "frac": gbps / HBM_PEAK_GBS,
            "card_window": sampler.summary(last[0][0], t_end), "series": series,
            "note": ("back-to-back headline rounds right after the rested timed region, no rest: the last %g s of "
                     "%g s; one HIP event pair per ~1 s chunk on the launch stream" % (window_s, round(t_end - t_start, 1)))}


def main():
    global REST_S
    args = parse()
    global HEADLINE_REST_S, CONFIG_SUSTAIN_S
    if args.config_sustain is not None:
        CONFIG_SUSTAIN_S = max(0.0, args.config_sustain)
    if args.rest is not None:
        REST_S = HEADLINE_REST_S = max(0.0, args.rest)
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
    # as the drop-in's init_model does (DeviceAggregatorMixin.device_numa_bind): the thread that stages uploads
    # in pinned memory runs on the GPU's NUMA node (fedscale_amd/hostnuma.py)
    from fedscale_amd.hostnuma import bind_to_gpu

    numa_node = bind_to_gpu(dev)
    cpu_group = None
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            cpu_group = dist.new_group(backend="gloo")  # host-side waits (no kernel parked on the GPUs)
        else:
            dist.init_process_group("gloo")
    from fedscale_amd import _native

    _native.load()  # refuses a library not built from this tree's sources (fedscale_amd/buildinfo.py)
    from fedscale_amd.state import ShardGroup

    shards = ShardGroup(rank, world, mode=args.shard)
    cfg = args.cfg
    policy, K, P = cfg["policy"], cfg["clients"], cfg["params"]
    weak = args.scaling == "weak"
    global MEM_FRACTION
    MEM_FRACTION = args.mem_fraction
    sets = args.sets if args.sets is not None else (2 if args.config == "c2" else 1)
    w = Workload(policy, K, P, rank, world, dev, args.seed, shards, weak=weak, budget_fraction=args.mem_fraction,
                 sets=sets, mean_chain={"auto": "auto", "on": True, "off": False}[args.mean_chain])
    (wall, kern_ms_max), kern_ms, kern_ms_ranks = time_workload(w, args.steps, args.warmup, dev, world,
                                                                 args.dist_backend, rest_s=HEADLINE_REST_S)
    warmup_used = w.warmup_rounds  # --warmup -1: the count the auto warmup ran
    step_ms = list(w.step_ms)
    pg_world = dist.get_world_size() if world > 1 else 1
    strong = not weak and not w.cmode
    card_state = {"before_timed_region": w.card_before, "timed_region": w.card, "rest_s": w.rest_s}
    from fedscale_amd import kernels as kx
    if policy == "qfedavg":
        launches = len(w.passes) * kx.qfed_launches(w.ld, w.P, chain=bool(w.qf.get("chain") is not None))
    else:
        launches = len(w.passes) * kx.reduce_launches(w.C if len(w.passes) > 1 else K, w.P,
                                                      weighted=policy == "fedbuff")
        if policy == "fedyogi":
            launches += 1  # k_yogi_step after the mean
    sustained = None
    if world == 1 and args.sustain > 0:
        sustained = sustained_leg(w, dev, args.sustain, launches, wall * 1e3 / args.steps)

    reassembly_ms = None
    if world > 1 and not args.no_reassemble and not w.cmode:  # egress: rebuild the global model (RCCL)
        shards.collective_all_gather(w.out)  # warm the communicator
        _sync_all(dev, world)
        t0r = time.perf_counter()
        for _ in range(5):
            shards.collective_all_gather(w.out)
        torch.cuda.synchronize(dev)
        reassembly_ms = _max_over_ranks([(time.perf_counter() - t0r) * 1e3 / 5], dev, world, args.dist_backend)[0]
    rccl_probe = None
    if world > 1:  # what RCCL itself sees over the ranks (its own communicator; ranks sharing a GPU cannot open one)
        if args.dist_backend == "nccl":
            from fedscale_amd.state import spmd_rccl_probe

            try:
                rccl_probe = spmd_rccl_probe(local_dev, group=cpu_group)
            except Exception as e:  # reported, never fatal
                rccl_probe = {"error": f"{type(e).__name__}: {e}"}
        else:
            rccl_probe = {"skipped": "gloo rehearsal: the ranks share one GPU, RCCL takes one rank per GPU"}
    alg_bytes = w.alg_bytes
    P_local, n_passes = w.P, len(w.passes)
    resident = w.C
    split_ms = getattr(w, "split_ms", None)  # FedYoGi: (k_reduce ms, k_yogi_step ms) per step
    # (launches: of the dominant kernel per step; fa_reduce runs long buckets as column windows (fedagg.hip
    # FA_WINDOWS), so the per-launch figures rocprof reports are the step's divided by it)
    one_gpu = inproc = None
    if world > 1 and strong and not args.no_selfcheck:
        # outside the timed region, the other ranks waiting at a host-side barrier (gloo: an RCCL barrier would park
        # a spinning kernel on their GPUs while rank 0's child uses them): (1) the same round on one GPU over the
        # whole model, so the line carries its own scaling reference; (2) the in-process drop-in timed over the
        # node's GPUs — what a FedScale deployment runs (one aggregator process), and the N > 1 line's `value`.
        # Both run before any rank frees its inputs: a 100 GB buffer allocated into memory freed buffers held reads
        # 3-4 % slower than one allocated fresh, whichever path reads it (profiles/r06_alloc_reuse_probe.log), and
        # the headline's own inputs were allocated fresh
        _sync_all(dev, world)
        dist.barrier(group=cpu_group)
        if rank == 0:
            one_gpu = one_gpu_reference(policy, K, P, dev, args.seed)
            if policy == "fedavg":
                inproc = run_inproc_bench(world, K, P, args.dist_backend, steps=args.steps, warmup=warmup_used)
        dist.barrier(group=cpu_group)

    drop_in = None
    if world == 1 and policy == "fedavg" and not weak and not args.no_other_configs:
        # the same round through the drop-in (TorchModelAdapter begin_round / apply_round, every launch on the part's
        # stream) with the N > 1 line's in-process timing (fedscale_amd.inproc_bench): value(N) / value_drop_in(1)
        # then compares one methodology; outside the timed region, never `value`.  Run while the headline's
        # inputs are still allocated, so its staging is fresh memory as the headline's was (allocated after the
        # headline's 100 GB were freed it read 3-4 % slower, r06_bench_default_n1.json / the verification line)
        from fedscale_amd.inproc_bench import run_one

        try:
            # (at least 30 warmup rounds: with 8 the adapter's rounds read ~3 % slow on a card still ramping its clocks,
            # while 4 x 20 interleaved rounds of both paths read the same, profiles/r06_dropin_vs_workload.log)
            drop_in = run_one(local_dev, K, P, rounds=args.steps, warmup=max(30, warmup_used), seed=args.seed)
        except Exception as e:  # reported, never fatal
            drop_in = {"error": f"{type(e).__name__}: {e}"}

    w.free()
    del w

    other = None
    if not args.no_other_configs and args.config == "headline":
        if world == 1:
            other = single_gpu_configs(dev, args.seed, shards, args.dist_backend, args.cpu_seconds)
        elif not shards.shards_clients:  # configs 4 and 5 at N GPUs (the driver's 4- and 8-GPU runs)
            other = {
                f"c4_fedyogi_k1000_p25M_x{world}": config_line(
                    "c4", CONFIGS["c4"], dev, rank, world, shards, args.seed, args.dist_backend),
                f"c5_qfedavg_k10000_p100M_x{world}": config_line(
                    "c5", CONFIGS["c5"], dev, rank, world, shards, args.seed, args.dist_backend, steps=2, warmup=1)}

    selfcheck = None
    if world > 1 and not args.no_selfcheck and args.dist_backend == "nccl":
        # the in-process drop-in (ShardedModelAdapter) over the node's N distinct GPUs, RCCL between them: what a
        # one-GPU box cannot run.  A child process with a deadline, after every rank has freed its workloads;
        # the other ranks wait at the barrier.  Outside the timed region; reported, never fatal.
        _sync_all(dev, world)
        dist.barrier(group=cpu_group)
        if rank == 0:
            selfcheck = run_selfcheck(world)
        dist.barrier(group=cpu_group)

    pcie = cpu_base = None
    if world > 1 and not args.no_pcie:
        # the north star's two other figures beside the N-GPU one, outside the timed region, the other ranks waiting at
        # a host-side barrier: the rate including H2D and D2H copies over the N links (one aggregator process, pickled
        # payloads -> N GPUs -> get_weights), and the reference CPU aggregator (the oracle) on rank 0's host cores
        _sync_all(dev, world)
        dist.barrier(group=cpu_group)
        if rank == 0:
            pcie = run_inproc_pcie(world, args.dist_backend)
            if args.cpu_seconds > 0:
                cpu_base = cpu_baseline(K, P, args.cpu_seconds, args.seed, policy)
        dist.barrier(group=cpu_group)

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        value = (K if strong else world * K) * args.steps / wall
        # the slowest rank's kernel sets the job's pace: roofline from the max over ranks (rank 0's slice is the
        # largest, so bytes / max time is the conservative per-GPU rate); N = 1: the same number
        achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
        w_cmode = shards.shards_clients
        if w_cmode:
            config = {"workload": f"{policy}_k{K}_per_gpu_p{P}_clientshard", "clients": K * world,
                      "clients_per_gpu": K, "params": P, "model_params_total": P, "policy": policy,
                      "parallelism": f"client-shard x{world} + RCCL all-reduce (one process per GPU)"}
        elif world == 1 or weak:
            config = {"workload": f"{policy}_k{K}_p{P}_per_gpu", "clients": K, "params_per_gpu": P,
                      "model_params_total": P * world, "policy": policy,
                      "parallelism": f"param-shard x{world} (one process per GPU)"}
        else:
            config = {"workload": f"{policy}_k{K}_p{P}_sharded_x{world}", "clients": K, "params_per_gpu": P_local,
                      "model_params_total": P, "policy": policy,
                      "parallelism": f"param-shard x{world} (one process per GPU, no data-path collective)"}
        if n_passes > 1:
            config["streamed_passes"] = n_passes
        build_id = _native.build_info()["build_id"]
        res = {
            "metric": ("client-updates/sec + HBM GB/s, device-resident FedAvg reduce of KxP fp32"
                       if policy == "fedavg" else
                       f"client-updates/sec + HBM GB/s, device-resident {policy} round of KxP fp32"),
            "value": value, "unit": "client-updates/s", "n_gpus": world, "steps": args.steps,
            "warmup": warmup_used, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic full-weight client updates (base + noise, hash-generated on device), HBM-resident",
            "host_numa_node": numa_node,
            "card_rest_s": HEADLINE_REST_S, "other_configs_card_rest_s": REST_S,
            "build_id": build_id,
            "config": config,
            "hbm_gbps": achieved,
            "kernel_ms": kern_ms_max,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc_traffic(config["workload"], resident, launches, build_id),
                         "kernel": ("k_qfed_accum + k_qfed_gather (fa_qfed_accumulate)" if policy == "qfedavg"
                                    else "k_reduce (fa_reduce, this rank's partial chain)" if w_cmode else
                                    {"fedavg": "k_reduce (fa_reduce FA_FINALIZE)",
                                     "fedbuff": "k_reduce weighted (fa_reduce FA_FINALIZE)",
                                     "fedyogi": "k_reduce (fa_reduce FA_FINALIZE) + k_yogi_step"}[policy]),
                         "alg_bytes_per_launch": alg_bytes / launches, "launches_per_step": launches,
                         "resident_clients": resident, "kernel_ms_per_launch": kern_ms_max / launches,
                         "kernel_ms_per_launch_by_round": [round(x / launches, 4) for x in step_ms],
                         "traffic_key": "profiles/pmc_traffic.json entries[workload|C<resident_clients>|"
                                        "L<launches_per_step>|<build_id>] (null: no PMC pass of this shape and build)"},
            "card_state": card_state,
        }
        if sustained is not None:
            res["sustained"] = sustained
        if drop_in is not None:
            res["drop_in_one_gpu"] = drop_in
            if "round_ms" in drop_in:
                res["value_drop_in"] = drop_in["client_updates_per_s"]
                drop_in["note"] = ("the same round through TorchModelAdapter, timed as the N > 1 line's in-process value "
                                   "(fedscale_amd.inproc_bench): value(N) / value_drop_in(1) is one methodology")
        if split_ms:
            res["roofline"]["kernel_ms_split"] = {"k_reduce": split_ms[0], "k_yogi_step": split_ms[1],
                                                  "k_reduce_launches": launches - 1}
        if world > 1:  # self-checking SCALE records: every rank's kernel time and the process group's size
            res["ranks"] = {"world_process_group": pg_world, "backend": args.dist_backend,
                            "kernel_ms_per_rank": kern_ms_ranks, "kernel_ms_max": kern_ms_max,
                            "kernel_ms_rank0": kern_ms, "rccl": rccl_probe,
                            "roofline_from": "max over ranks of the dominant kernel's mean time per step"}
            n_visible = torch.cuda.device_count()
            if args.dist_backend != "nccl" or n_visible < world:
                # a rehearsal: ranks (and the in-process parts) share the visible GPU(s), so no rate on this line is
                # an N-GPU rate (SCALE-shaped JSON must not read as scaling data)
                res["plumbing_only"] = (f"{world} ranks on {min(n_visible, world)} GPU(s), backend {args.dist_backend}: "
                                        "every rate on this line is plumbing, not an N-GPU measurement")
        if reassembly_ms is not None:
            # every round ends in egress (aggregator.py:788-804): the model reassembled from the shards
            res["reassembly_ms"] = reassembly_ms
            res["round_ms_incl_reassembly"] = ms_per_step + reassembly_ms
            res["value_incl_reassembly"] = K / ((ms_per_step + reassembly_ms) * 1e-3)
        if one_gpu is not None:
            res["one_gpu_reference"] = one_gpu
            res["scaling_vs_one_gpu"] = one_gpu["ms_per_step"] / ms_per_step
            if reassembly_ms is not None:
                res["scaling_vs_one_gpu_incl_reassembly"] = one_gpu["ms_per_step"] / (ms_per_step + reassembly_ms)
        if inproc is not None:
            res["inproc_drop_in"] = inproc
            promote_inproc(res, inproc, K, args.steps)
        if selfcheck is not None:
            res["inproc_multi_gpu_check"] = selfcheck
        if other is not None:
            res["other_configs"] = other
        if world == 1 and args.cpu_seconds > 0:
            res["cpu_baseline"] = cpu_baseline(K, P, args.cpu_seconds, args.seed, policy)
        else:
            res["cpu_baseline"] = cpu_base
            if world == 1 or args.cpu_seconds <= 0:
                res["cpu_legs_off"] = True
        if world == 1 and other is not None and "headline_model_pcie_inclusive" in other:
            res["pcie_inclusive"] = dict(other["headline_model_pcie_inclusive"], n_gpus=1)
        elif pcie is not None:
            res["pcie_inclusive"] = pcie
        missing = check_line(res)
        res["schema"] = {"complete": not missing, "missing": missing}
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier(group=cpu_group)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
