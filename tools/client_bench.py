"""Client-side handlers on a ResNet-18 / CIFAR-10 model layout: device kernels vs the
reference's own torch code run per tensor on the same GPU, and on the host CPU.

usage: python tools/client_bench.py [reps]

* FedProx (optimizers.py:6-10, once per local step): ``fa_prox_update`` (one multi-tensor launch over the
  62 parameter tensors, 12 B per parameter) vs the reference loop ``param.data += lr*mu*(param.data - g)``.
* Local DP (customized_client.py:51-63, once per round): ``privatize_update`` (norm pass + recover/noise
  pass, 8 + 16 B per parameter and 8 B per buffer element) vs the reference's delta / clip_grad_norm_ /
  recover / torch.normal sequence.
Prints one JSON line per measurement.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fedscale_amd import kernels as kx  # noqa: E402
from fedscale_amd import synth  # noqa: E402
from fedscale_amd.cloud.execution.local_dp import privatize_update  # noqa: E402

BUFFERS = ("running_mean", "running_var", "num_batches_tracked")


class LayoutNet(torch.nn.Module):
    def __init__(self, names, shapes, dtypes, seed=0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        for n, s, d in zip(names, shapes, dtypes):
            mod = self
            *path, leaf = n.split(".")
            for part in path:
                if not hasattr(mod, part):
                    mod.add_module(part, torch.nn.Module())
                mod = getattr(mod, part)
            t = (torch.randn(s, generator=g) * 0.05).to(d) if d.is_floating_point else torch.zeros(s, dtype=d)
            if leaf in BUFFERS:
                mod.register_buffer(leaf, t)
            else:
                mod.register_parameter(leaf, torch.nn.Parameter(t, requires_grad=False))


def timed_events(fn, reps, stream):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def timed_wall(fn, reps, sync=True):
    fn()
    if sync:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    if sync:
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / reps


def ref_prox(params, glob, lr, mu):  # optimizers.py:9-10, literally
    for idx, param in enumerate(params):
        param.data += lr * mu * (param.data - glob[idx])


def ref_dp(model, last, clip, noise_factor):  # customized_client.py:51-63 with clip_norm.py:32-52
    delta = [p.data - last[i] for i, p in enumerate(model.parameters())]
    total = torch.norm(torch.stack([torch.norm(d, 2.0) for d in delta]), 2.0)
    coef = clip / (total + 1e-6)
    if coef < 1:
        for d in delta:
            d.mul_(coef)
    for i, p in enumerate(model.parameters()):
        p.data = last[i] + delta[i]
    sigma = noise_factor * clip
    sd = model.state_dict()
    return {n: (t.data + torch.normal(mean=0, std=sigma, size=t.shape, device=t.device)) for n, t in sd.items()}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    names, shapes, dtypes = synth.resnet18_layout()
    net = LayoutNet(names, shapes, dtypes).to(dev)
    params = [p.data for p in net.parameters()]
    P = sum(p.numel() for p in params)
    nbuf = sum(b.numel() for b in net.buffers())
    glob = [p.clone() for p in params]
    lr, mu = 0.05, 0.1
    out = []

    # ---- FedProx -----------------------------------------------------------------------------
    ms = timed_events(lambda: kx.prox_update(params, glob, float(lr * mu)), reps, stream)
    wall = timed_wall(lambda: kx.prox_update(params, glob, float(lr * mu)), reps)
    ms_ref = timed_events(lambda: ref_prox(params, glob, lr, mu), reps, stream)
    cpu_params = [p.cpu() for p in params]
    cpu_glob = [g.cpu() for g in glob]
    ms_cpu = timed_wall(lambda: ref_prox(cpu_params, cpu_glob, lr, mu), max(3, reps // 10), sync=False)
    out.append({"handler": "fedprox_step", "layout": "resnet18_cifar10", "tensors": len(params), "params": P,
                "device_ms": ms, "device_wall_ms_incl_host": wall, "alg_bytes": 12 * P,
                "device_gbps": 12 * P / (ms * 1e-3) / 1e9, "hbm_frac": 12 * P / (ms * 1e-3) / 8e12,
                "torch_per_tensor_gpu_ms": ms_ref, "speedup_vs_torch_gpu": ms_ref / ms,
                "reference_cpu_ms": ms_cpu, "cpu_threads": torch.get_num_threads()})

    # ---- local SGD step + FedProx (torch_client.py:236-240) ------------------------------------
    import argparse

    from fedscale_amd.cloud.execution.optimizers import ClientOptimizer

    conf = argparse.Namespace(gradient_policy="fed-prox", learning_rate=lr, proxy_mu=mu)
    for p in net.parameters():
        p.grad = torch.randn_like(p) * 0.01
    sgd_kw = dict(lr=lr, momentum=0.9, weight_decay=5e-4)  # get_optimizer's default (:127-128)
    opt_ref = torch.optim.SGD(net.parameters(), **sgd_kw)

    def ref_step():
        opt_ref.step()
        ref_prox(params, glob, lr, mu)

    ms_sgd_ref = timed_events(ref_step, reps, stream)
    opt_dev = torch.optim.SGD(net.parameters(), **sgd_kw)
    co = ClientOptimizer()
    ms_sgd = timed_events(lambda: co.step_and_update(opt_dev, conf, net, glob), reps, stream)
    wall_sgd = timed_wall(lambda: co.step_and_update(opt_dev, conf, net, glob), reps)
    alg = 24 * P  # read param, grad, momentum buffer, global model; write param, momentum buffer
    out.append({"handler": "sgd_fedprox_step", "layout": "resnet18_cifar10", "params": P,
                "device_ms": ms_sgd, "device_wall_ms_incl_host": wall_sgd, "alg_bytes": alg,
                "device_gbps": alg / (ms_sgd * 1e-3) / 1e9,
                "torch_sgd_plus_prox_gpu_ms": ms_sgd_ref, "speedup_vs_torch_gpu": ms_sgd_ref / ms_sgd})

    # the detection task's optimizer: one param group per parameter (torch_client.py:100-108)
    groups = [dict(params=[p], lr=lr * (1 + 0.01 * i), weight_decay=5e-4 if i % 2 else 0.0, momentum=0.9)
              for i, p in enumerate(net.parameters())]
    opt_g_ref, opt_g = torch.optim.SGD(groups, lr=lr), torch.optim.SGD(
        [dict(g, params=list(g["params"])) for g in groups], lr=lr)

    def ref_step_g():
        opt_g_ref.step()
        ref_prox(params, glob, lr, mu)

    ms_g_ref = timed_events(ref_step_g, reps, stream)
    co_g = ClientOptimizer()
    ms_g = timed_events(lambda: co_g.step_and_update(opt_g, conf, net, glob), reps, stream)
    wall_g = timed_wall(lambda: co_g.step_and_update(opt_g, conf, net, glob), reps)
    out.append({"handler": "sgd_fedprox_step_one_group_per_param", "layout": "resnet18_cifar10", "params": P,
                "groups": len(groups), "device_ms": ms_g, "device_wall_ms_incl_host": wall_g,
                "device_gbps": alg / (ms_g * 1e-3) / 1e9, "torch_sgd_plus_prox_gpu_ms": ms_g_ref,
                "speedup_vs_torch_gpu": ms_g_ref / ms_g})

    # ---- local DP ----------------------------------------------------------------------------
    last = [p.clone() for p in params]
    with torch.no_grad():
        for p in params:
            p.add_(0.01)
    state = [p.clone() for p in params]

    def dev_dp(as_numpy):
        for p, s in zip(params, state):
            p.copy_(s)
        return privatize_update(net, last, 3.0, 0.1, seed=7, as_numpy=as_numpy)

    def restore():
        for p, s in zip(params, state):
            p.copy_(s)

    ms_restore = timed_events(restore, reps, stream)
    ms_dp = timed_events(lambda: dev_dp(False), reps, stream) - ms_restore
    wall_np = timed_wall(lambda: dev_dp(True), max(3, reps // 5))
    ms_dp_ref = timed_events(lambda: (restore(), ref_dp(net, last, 3.0, 0.1)), reps, stream) - ms_restore
    net_cpu = LayoutNet(names, shapes, dtypes)
    last_cpu = [p.data.clone() for p in net_cpu.parameters()]
    ms_dp_cpu = timed_wall(lambda: ref_dp(net_cpu, last_cpu, 3.0, 0.1), 3, sync=False)
    alg = 8 * P + 16 * P + 8 * nbuf  # norm pass (p, last) + apply (p, last read; p, upload write) + buffers
    out.append({"handler": "local_dp_privatize", "layout": "resnet18_cifar10", "params": P, "buffer_elems": nbuf,
                "device_ms": ms_dp, "device_gbps": alg / (ms_dp * 1e-3) / 1e9,
                "device_wall_ms_incl_d2h_numpy": wall_np, "alg_bytes": alg,
                "torch_reference_gpu_ms": ms_dp_ref, "speedup_vs_torch_gpu": ms_dp_ref / ms_dp,
                "reference_cpu_ms": ms_dp_cpu, "cpu_threads": torch.get_num_threads()})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
