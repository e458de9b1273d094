"""CPU ORACLE for the FedScale aggregator update-reduction path — TEST INFRASTRUCTURE ONLY.

This module is a from-scratch CPU restatement of the reference algorithm, op for op, so that the
HIP product path (``fedscale_amd``) can be checked against it. It is imported only by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg — as the checker / the timed CPU
baseline, never as something the product calls. The product path never imports ``oracle``.

Parity of this restatement is PINNED: ``tests/test_oracle_golden.py`` checks it bit-exact against
the golden vectors in ``tests/golden/`` that ``tests/golden/gen_golden.py`` produced by running the real
reference (/root/reference, FedScale v0.5) in the build container.

Reference anchors (paths relative to /root/reference):

* FedAvg accumulate/finalize ........ fedscale/cloud/aggregation/aggregator.py:489-511 (+ :430-434)
* FedBuff staleness accumulate ...... fedscale/cloud/aggregation/async_aggregator.py:115-137
* model adapter set/get ............. fedscale/cloud/internal/torch_model_adapter.py:23-47
* server optimizer dispatch ......... fedscale/cloud/aggregation/optimizers.py:16-108
* YoGi .............................. fedscale/utils/optimizer/yogi.py:5-36
* Auxo per-cohort FedAvg ............ examples/auxo/aggregator.py:451-472
* HeteroFL combine_models ........... examples/heterofl/customized_aggregator.py:78-119
* FedProx client step ............... fedscale/cloud/execution/optimizers.py:6-10
* local-DP clip + recover + noise ... examples/differential_privacy/customized_client.py:51-63,
                                      clip_norm.py:12-52 (pinned by tests/golden/gen_golden_client.py)

Numerics notes (each reproduced deliberately):
* accumulation is numpy, fp32, strictly in arrival order, allocating a new array each add;
* ``np.divide(x, K)`` is true division; int64 tensors sum in int64 and divide to float64;
* Python-float scalars are *weak* (NEP 50): fp32 arrays stay fp32, int arrays promote to float64;
* torch CPU ops with Python scalars round the scalar to the tensor dtype first;
* ``eta / t`` on a tensor is ``t.reciprocal() * eta`` (torch ``__rtruediv__``);
* ``load_state_dict`` copies with dtype conversion (float -> int64 truncates toward zero).
"""
from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


def _as_list(update_weight):
    """dict name->array  or  list  ->  list in state_dict order (aggregator.py:494-496)."""
    if type(update_weight) is dict:
        return list(update_weight.values())
    return update_weight


# ------------------------------------------------------------------------------------------------
# A2 / A3: streaming accumulators
# ------------------------------------------------------------------------------------------------
def fedavg_step(acc: Optional[list], update_weight, first: bool) -> list:
    """One arrival of aggregator.py:497-503: alias on the first result, else a fresh ``w + u``."""
    u = _as_list(update_weight)
    if first:
        return u
    return [acc[i] + u[i] for i in range(len(acc))]


def fedavg_close(acc: list, tasks_round: int) -> list:
    """aggregator.py:505-507: true division of every accumulated tensor by K."""
    return [np.divide(w, tasks_round) for w in acc]


def fedbuff_weight(cur_round: int, model_version: int) -> float:
    """async_aggregator.py:125: 1/sqrt(1 + staleness) as a Python float."""
    return 1 / (1 + cur_round - model_version) ** 0.5


def fedbuff_step(acc: Optional[list], update_weight, s: float, first: bool) -> list:
    """async_aggregator.py:129-133: first ``u*s``, else ``acc + s*u``."""
    u = _as_list(update_weight)
    if first:
        return [x * s for x in u]
    return [acc[i] + s * u[i] for i in range(len(acc))]


def fedbuff_close(acc: list, denominator: float) -> list:
    """async_aggregator.py:134-135."""
    return [np.divide(w, denominator) for w in acc]


# ------------------------------------------------------------------------------------------------
# A6: YoGi (yogi.py:5-36)
# ------------------------------------------------------------------------------------------------
class OracleYoGi:
    def __init__(self, eta=1e-2, tau=1e-3, beta=0.9, beta2=0.99):
        self.eta, self.tau, self.beta, self.beta2 = eta, tau, beta, beta2
        self.m_t: List[torch.Tensor] = []
        self.v_t: List[torch.Tensor] = []

    def update(self, gradients: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        if len(self.v_t) == 0:  # lazy state init, yogi.py:17-19
            self.v_t = [torch.full_like(g, self.tau) for g in gradients]
            self.m_t = [torch.full_like(g, 0.0) for g in gradients]
        steps = []
        for i, g in enumerate(gradients):
            g2 = g ** 2
            self.m_t[i] = self.beta * self.m_t[i] + (1.0 - self.beta) * g
            self.v_t[i] = self.v_t[i] - (1.0 - self.beta2) * g2 * torch.sign(self.v_t[i] - g2)
            # ``eta / tensor`` is Tensor.__rtruediv__ == reciprocal() * eta
            lr = self.eta / (torch.sqrt(self.v_t[i]) + self.tau)
            steps.append(lr * self.m_t[i])
        return steps if steps else list(gradients)


# ------------------------------------------------------------------------------------------------
# A4 model state + A5 dispatch + A8 q-FedAvg
# ------------------------------------------------------------------------------------------------
class OracleModel:
    """Stands in for the torch nn.Module whose state_dict TorchModelAdapter drives."""

    def __init__(self, names: Sequence[str], tensors: Sequence[torch.Tensor]):
        self.sd: "OrderedDict[str, torch.Tensor]" = OrderedDict(
            (n, t.detach().clone()) for n, t in zip(names, tensors))

    def state_dict(self):
        return self.sd

    def load_state_dict(self, new: Dict[str, torch.Tensor]):
        # nn.Module.load_state_dict: param.copy_(input) under no_grad (dtype-converting copy)
        for n, dst in self.sd.items():
            dst.copy_(new[n])



def _as_numpy(x):
    """np.array(x) of the reference without numpy's __array__(copy=...) deprecation path for tensors."""
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else x

class OracleServerOptimizer:
    """optimizers.py:16-108 with ``device=None`` (the reference aggregator runs on CPU)."""

    def __init__(self, mode, args, device=None, sample_seed=233):
        self.mode, self.args, self.device = mode, args, device
        if mode == "fed-yogi":
            self.gradient_controller = OracleYoGi(eta=args.yogi_eta, tau=args.yogi_tau,
                                                  beta=args.yogi_beta, beta2=args.yogi_beta2)

    def update_round_gradient(self, last_model, current_model, target_model, client_training_results=None):
        names = list(target_model.state_dict().keys())
        if self.mode == "fed-yogi":
            steps = self.gradient_controller.update([c - l for l, c in zip(last_model, current_model)])
            target_model.load_state_dict({
                n: torch.from_numpy(np.array(_as_numpy(last_model[i] + steps[i]), dtype=np.float32))
                for i, n in enumerate(names)})
        elif self.mode == "q-fedavg":
            lr, q = self.args.learning_rate, self.args.qfed_q
            delta, hs = None, 0.0
            for res in client_training_results:
                w_k = [torch.tensor(x) for x in _as_list(res["update_weight"])]
                g_k = [(L - W) * 1.0 / lr for L, W in zip(last_model, w_k)]
                base = res["moving_loss"] + 1e-10
                a_k = np.float_power(base, q)
                if delta is None:
                    delta = [a_k * g for g in g_k]
                else:
                    for i in range(len(delta)):
                        delta[i] += a_k * g_k[i]
                sq = torch.sum(torch.stack([torch.square(g).sum() for g in g_k]))
                hs += q * np.float_power(base, q - 1) * sq + (1.0 / lr) * a_k
            target_model.load_state_dict({
                n: last_model[i] - delta[i] / (hs + 1e-10) for i, n in enumerate(names)})
        # any other mode: FedAvg was already applied by the aggregator (optimizers.py:106-108)


class OracleModelAdapter:
    """torch_model_adapter.py:10-53."""

    def __init__(self, model: OracleModel, optimizer: Optional[OracleServerOptimizer] = None):
        self.model, self.optimizer = model, optimizer

    def set_weights(self, weights, is_aggregator=True, client_training_results=None):
        names = list(self.model.state_dict().keys())
        last = [t.clone() for t in self.model.state_dict().values()]
        self.model.load_state_dict({n: torch.from_numpy(np.asarray(weights[i], dtype=np.float32))
                                    for i, n in enumerate(names)})
        if self.optimizer and is_aggregator:
            current = [torch.tensor(x) for x in copy.deepcopy(weights)]
            self.optimizer.update_round_gradient(last, current, self.model, client_training_results)

    def get_weights(self):
        return [t.clone() for t in self.model.state_dict().values()]

    def get_model(self):
        return self.model


class OracleAggregator:
    """The reduction state of ``Aggregator`` (MockAggregator contract, test_aggregator.py:11-17)
    plus the per-arrival lines of ``client_completion_handler`` (aggregator.py:466-467, 484-485)."""

    def __init__(self, model_wrapper: OracleModelAdapter, args, asynchronous: bool = False):
        self.model_wrapper, self.args, self.asynchronous = model_wrapper, args, asynchronous
        self.model_weights = []
        self.model_in_update = 0
        self.tasks_round = 0
        self.client_training_results = []
        # FedBuff state (async_aggregator.py:103-112)
        self.round = 0
        self.client_task_model_version = {}
        self.aggregation_denominator = 0

    def start_round(self, tasks_round: int):
        self.tasks_round = tasks_round  # aggregator.py:609
        self.model_in_update = 0  # :620
        self.client_training_results = []  # :622

    def on_result(self, results):
        if self.args.gradient_policy in ["q-fedavg"]:
            self.client_training_results.append(results)
        self.model_in_update += 1
        self.update_weight_aggregation(results)

    def update_weight_aggregation(self, results):
        first = self.model_in_update == 1
        last = self.model_in_update == self.tasks_round
        if self.asynchronous:
            s = fedbuff_weight(self.round, self.client_task_model_version[results["client_id"]])
            self.aggregation_denominator += s
            self.model_weights = fedbuff_step(self.model_weights, results["update_weight"], s, first)
            if last:
                self.model_weights = fedbuff_close(self.model_weights, self.aggregation_denominator)
                self.model_wrapper.set_weights(copy.deepcopy(self.model_weights))
                self.aggregation_denominator = 0
            return
        self.model_weights = fedavg_step(self.model_weights, results["update_weight"], first)
        if last:
            self.model_weights = fedavg_close(self.model_weights, self.tasks_round)
            self.model_wrapper.set_weights(copy.deepcopy(self.model_weights),
                                           client_training_results=self.client_training_results)


class OracleCohortAggregator:
    """Auxo's per-cohort FedAvg (examples/auxo/aggregator.py:451-472): every reduction field is a list
    indexed by cohort; set_weights is called without client_training_results (:472)."""

    def __init__(self, wrappers, tasks_round):
        self.model_wrapper = list(wrappers)
        self.tasks_round = list(tasks_round)
        self.model_in_update = [0] * len(self.model_wrapper)
        self.model_weights = [[] for _ in self.model_wrapper]

    def on_result(self, results, cohort_id):
        self.model_in_update[cohort_id] += 1  # auxo/aggregator.py:307
        first = self.model_in_update[cohort_id] == 1
        last = self.model_in_update[cohort_id] == self.tasks_round[cohort_id]
        self.model_weights[cohort_id] = fedavg_step(self.model_weights[cohort_id], results["update_weight"], first)
        if last:
            self.model_weights[cohort_id] = fedavg_close(self.model_weights[cohort_id], self.tasks_round[cohort_id])
            self.model_wrapper[cohort_id].set_weights(copy.deepcopy(self.model_weights[cohort_id]))


def heterofl_combine(global_sd, local_states):
    """Restatement of Customized_Aggregator.combine_models (examples/heterofl/customized_aggregator.py:78-119)
    for prefix index sets (customized_fllibs.py:25-70 builds only prefixes): per tensor an fp32 zero sum
    and count, clients scatter-added in order, then sum/count where count > 0 (in place on global_sd)."""
    for name, v in global_sd.items():
        tmp = torch.zeros(v.shape, dtype=torch.float32)
        cnt = torch.zeros(v.shape, dtype=torch.float32)
        for loc in local_states:
            lv = torch.as_tensor(np.asarray(loc[name]))
            box = tuple(slice(0, n) for n in lv.shape[:2])
            tmp[box] += lv
            cnt[box] += 1
        mask = cnt > 0
        tmp[mask] = tmp[mask].div_(cnt[mask])
        v[mask] = tmp[mask].to(v.dtype)


# ------------------------------------------------------------------------------------------------
# flat-bucket helpers used by tests / bench for large synthetic cases (same arithmetic, no lists)
# ------------------------------------------------------------------------------------------------
def fedavg_flat(x: np.ndarray) -> np.ndarray:
    """x: [K, P] fp32 client-major.  Sequential fp32 sum in row order, then true division by K."""
    acc = x[0]
    for k in range(1, x.shape[0]):
        acc = acc + x[k]
    return np.divide(acc, x.shape[0])


def fedbuff_flat(x: np.ndarray, s: Sequence[float]) -> np.ndarray:
    acc = x[0] * s[0]
    den = s[0]
    for k in range(1, x.shape[0]):
        acc = acc + s[k] * x[k]
        den += s[k]
    return np.divide(acc, den)


# ------------------------------------------------------------------------------------------------
# client-side element-wise handlers
# ------------------------------------------------------------------------------------------------
def fedprox_update(params: Sequence[np.ndarray], global_model: Sequence[np.ndarray], lr: float,
                   mu: float) -> list:
    """optimizers.py:10 ``param.data += conf.learning_rate * conf.proxy_mu * (param.data - global_model[idx])``:
    the Python-double product lr*mu multiplies an fp32 tensor, so it is rounded to fp32 first; every op
    rounds in fp32."""
    c = np.float32(lr * mu)
    return [np.asarray(p, np.float32) + c * (np.asarray(p, np.float32) - np.asarray(g, np.float32))
            for p, g in zip(params, global_model)]


def dp_clip_coef(deltas: Sequence[np.ndarray], max_norm: float, norm_type: float = 2.0):
    """clip_norm.py:32-52 on CPU tensors, op for op (torch CPU norm, as the reference computes it).
    Returns (total_norm, clip_coef, apply) as fp32 / bool."""
    ts = [torch.from_numpy(np.ascontiguousarray(d, dtype=np.float32)) for d in deltas]
    if len(ts) == 0:
        return np.float32(0.0), None, False
    if norm_type == float("inf"):
        norms = [t.detach().abs().max() for t in ts]
        total = norms[0] if len(norms) == 1 else torch.max(torch.stack(norms))
    else:
        total = torch.norm(torch.stack([torch.norm(t.detach(), norm_type) for t in ts]), norm_type)
    coef = float(max_norm) / (total + 1e-6)
    return np.float32(total.item()), np.float32(coef.item()), bool(coef < 1)


def dp_privatize(state: "OrderedDict[str, np.ndarray]", is_param: Sequence[bool], last: Sequence[np.ndarray],
                 max_norm: float, noise_factor: float, noise: Optional[Dict[str, np.ndarray]] = None,
                 norm_type: float = 2.0):
    """customized_client.py:51-63: delta = p - last (parameters only); clip_grad_norm_(delta); p = last + delta;
    upload = state_dict + torch.normal(0, sigma) (numpy add: fp32 + fp32 -> fp32, int64 + fp32 -> fp64).

    ``noise`` (name -> fp32 array of the entry's shape) replaces the reference's torch.normal draws so the
    device's own stream can be checked; None with noise_factor == 0 means +0.0 noise.
    Returns (recovered state, upload, total_norm)."""
    names = list(state.keys())
    pidx = [i for i, f in enumerate(is_param) if f]
    deltas = [np.asarray(state[names[i]], np.float32) - np.asarray(l, np.float32) for i, l in zip(pidx, last)]
    total, coef, apply = dp_clip_coef(deltas, max_norm, norm_type)
    if apply:
        deltas = [d * coef for d in deltas]
    rec = OrderedDict((n, np.array(state[n])) for n in names)
    for i, l, d in zip(pidx, last, deltas):
        rec[names[i]] = np.asarray(l, np.float32) + d
    sigma = noise_factor * max_norm
    upload = OrderedDict()
    for n in names:
        z = (noise[n] if noise is not None else
             np.zeros(np.shape(rec[n]), np.float32) if sigma == 0 else None)
        if z is None:
            raise ValueError("dp_privatize: sigma > 0 needs the noise draws")
        upload[n] = np.asarray(rec[n] + np.asarray(z, np.float32))
    return rec, upload, total
