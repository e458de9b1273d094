"""Generate golden vectors for the client-side element-wise handlers from the REAL FedScale reference.

Run ONLY in the build container (it needs /root/reference, which never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_client.py

What it drives (paths relative to /root/reference):

* ``ClientOptimizer.update_client_weight``  fedscale/cloud/execution/optimizers.py:6-10 (fed-prox), imported
  and called as torch_client.py:238-240 does after each local step (here: several consecutive steps, the
  parameters perturbed in between as an optimizer step would).
* ``clip_grad_norm_``                        examples/differential_privacy/clip_norm.py:12-52, imported from
  the example directory.  clip_norm.py imports ``inf`` from ``torch._six``, a module removed from torch
  2.x; a ``sys.modules`` placeholder exposing ``inf = math.inf`` (what torch._six.inf was) stands in for it.
  The lines of customized_client.py:51-63 that wrap it (delta = p - last; clip; p = last + delta;
  upload = state_dict + torch.normal(0, sigma)) are three tensor expressions restated below, because
  the module itself imports the whole executor stack.

Outputs (data only): tests/golden/client_<scenario>.npz / .json.  The DP fixtures also store the noise
the reference drew (upload - recovered state), so the oracle can be checked bit-exactly on them.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import types

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True

import numpy as np
import torch
import torch.nn as nn

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "examples", "differential_privacy"))
    six = types.ModuleType("torch._six")
    six.inf = math.inf
    sys.modules["torch._six"] = six
    from clip_norm import clip_grad_norm_
    from fedscale.cloud.execution.optimizers import ClientOptimizer

    return ClientOptimizer, clip_grad_norm_


class BNNet(nn.Module):
    """conv + BN (fp32 running stats + int64 num_batches_tracked) + odd-sized linear layers."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3)
        self.bn = nn.BatchNorm2d(8)
        self.fc1 = nn.Linear(8 * 4 * 4, 37)
        self.fc2 = nn.Linear(37, 10)


class BigNet(nn.Module):
    """Tensors spanning several 4096-element workgroups plus tiny ones (multi-tensor tiling)."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(150, 97)     # 14,550 + 97
        self.b = nn.Linear(97, 3)       # 291 + 3
        self.c = nn.Linear(3, 5001)     # 15,003 + 5,001


def _perturb(model, rng, scale):
    with torch.no_grad():
        for p in model.parameters():
            p.add_(torch.from_numpy(rng.normal(0, scale, size=tuple(p.shape)).astype(np.float32)))


def _save(name, meta, arrays):
    np.savez(os.path.join(OUT, f"client_{name}.npz"), **arrays)
    with open(os.path.join(OUT, f"client_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f"  client_{name}: {os.path.getsize(os.path.join(OUT, f'client_{name}.npz')) / 1024:.1f} KiB")


def gen_prox(ClientOptimizer, name, cls, seed, lr, mu, steps):
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    model = cls()
    global_model = [p.data.clone() for p in model.parameters()]  # torch_client.py:58-60
    conf = argparse.Namespace(gradient_policy="fed-prox", learning_rate=lr, proxy_mu=mu)
    opt = ClientOptimizer()
    arrays = {f"global/{i}": g.numpy().copy() for i, g in enumerate(global_model)}
    for s in range(steps):
        _perturb(model, rng, 0.02)  # stands in for optimizer.step()
        for i, p in enumerate(model.parameters()):
            arrays[f"in/{s}/{i}"] = p.data.numpy().copy()
        opt.update_client_weight(conf, model, global_model)  # optimizers.py:6-10
        for i, p in enumerate(model.parameters()):
            arrays[f"out/{s}/{i}"] = p.data.numpy().copy()
    meta = {"kind": "prox", "lr": lr, "mu": mu, "steps": steps,
            "shapes": [list(p.shape) for p in model.parameters()]}
    _save(name, meta, arrays)


def gen_dp(clip_grad_norm_, name, cls, seed, clip, noise_factor, norm_type=2.0, train_scale=0.05):
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    model = cls()
    with torch.no_grad():  # non-trivial BN buffers
        for n, b in model.named_buffers():
            if b.dtype == torch.float32:
                b.add_(torch.from_numpy(rng.normal(0, 0.1, size=tuple(b.shape)).astype(np.float32)))
            else:
                b.fill_(int(rng.integers(1, 50)))
    last_model_params = [p.data.clone() for p in model.parameters()]  # customized_client.py:27
    _perturb(model, rng, train_scale)                                   # local training
    arrays = {}
    names = list(model.state_dict().keys())
    param_ids = {id(p) for p in model.parameters()}
    sd0 = model.state_dict(keep_vars=True)
    is_param = [id(sd0[n]) in param_ids for n in names]
    for i, t in enumerate(last_model_params):
        arrays[f"last/{i}"] = t.numpy().copy()
    for j, n in enumerate(names):
        arrays[f"in/{j}"] = model.state_dict()[n].numpy().copy()
    # customized_client.py:51-55
    delta_weight = []
    for param in model.parameters():
        delta_weight.append((param.data.cpu() - last_model_params[len(delta_weight)]))
    total = clip_grad_norm_(delta_weight, max_norm=clip, norm_type=norm_type)
    # :57-61
    idx = 0
    for param in model.parameters():
        param.data = last_model_params[idx] + delta_weight[idx]
        idx += 1
    # :62-64
    sigma = noise_factor * clip
    state_dicts = model.state_dict()
    recovered = {p: state_dicts[p].data.cpu().numpy().copy() for p in state_dicts}
    noise = {p: torch.normal(mean=0, std=sigma, size=state_dicts[p].data.shape).cpu().numpy() for p in state_dicts}
    model_param = {p: np.asarray(state_dicts[p].data.cpu().numpy() + noise[p]) for p in state_dicts}
    for j, n in enumerate(names):
        arrays[f"recovered/{j}"] = recovered[n]
        if sigma != 0:  # with sigma = 0 the drawn noise is +0.0 everywhere
            arrays[f"noise/{j}"] = noise[n]
        arrays[f"upload/{j}"] = model_param[n]
    meta = {"kind": "dp", "clip": clip, "noise_factor": noise_factor, "norm_type": norm_type,
            "names": names, "is_param": is_param, "total_norm": float(total),
            "shapes": [list(model.state_dict()[n].shape) for n in names],
            "dtypes": [str(model.state_dict()[n].dtype).replace("torch.", "") for n in names]}
    _save(name, meta, arrays)


def main():
    ClientOptimizer, clip_grad_norm_ = _import_reference()
    gen_prox(ClientOptimizer, "prox_bnnet", BNNet, 11, lr=0.05, mu=0.1, steps=3)
    gen_prox(ClientOptimizer, "prox_bignet", BigNet, 12, lr=0.04, mu=0.01, steps=1)
    gen_dp(clip_grad_norm_, "dp_bnnet_clipped", BNNet, 21, clip=0.5, noise_factor=0.0)
    gen_dp(clip_grad_norm_, "dp_bnnet_unclipped", BNNet, 22, clip=1e4, noise_factor=0.0)
    gen_dp(clip_grad_norm_, "dp_bignet_clipped", BigNet, 23, clip=3.0, noise_factor=0.0)
    gen_dp(clip_grad_norm_, "dp_bnnet_inf", BNNet, 24, clip=0.05, noise_factor=0.0, norm_type=math.inf)
    gen_dp(clip_grad_norm_, "dp_bnnet_noise", BNNet, 25, clip=3.0, noise_factor=0.1)


if __name__ == "__main__":
    main()
