"""Multi-GPU self-check of the in-process drop-in: ``ShardedModelAdapter`` over distinct GPUs (RCCL) against one
GPU, on the same uploads.

    python -m fedscale_amd.selfcheck --devices 0,1,2,3

``bench.py --gpus N`` runs it (rank 0, in a child process with a deadline, after the timed region) so that a
node with N GPUs exercises the part of the drop-in a one-GPU box cannot: every part's kernels, copies and
events on its own device's stream, and the q-FedAvg norm exchange as an RCCL all-gather between distinct
GPUs.  Checks, per server step (FedAvg, FedBuff, fused FedYoGi, q-FedAvg with the fused FedAvg chain), over two
rounds with chunk folds (staging capacity < K):
  * the sharded model equals the one-GPU model: FedAvg / FedBuff / FedYoGi bit for bit (the per-element
    chains are the same), q-FedAvg within 1e-6 relative (the fp64 norm sum re-associates over the shards);
  * the FedAvg mean (``model_weights``) equals the one-GPU mean bit for bit;
  * every native launch carried the non-null stream of the part whose device it targeted, and every part's
    buffers live on that part's device.
Prints one JSON line; exit status 0 only when every check passed.  No oracle is involved (the one-GPU adapter
is the product's own path, itself pinned to the reference by the test suite).
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def _model(seed: int):
    import torch

    g = torch.Generator().manual_seed(seed)
    names = ["conv.weight", "conv.bias", "bn.running_mean", "bn.num_batches_tracked", "fc.weight", "fc.bias"]
    tensors = [torch.randn(64, 32, 3, 3, generator=g) * 0.05, torch.randn(64, generator=g) * 0.05,
               torch.randn(64, generator=g) * 0.05, torch.tensor(7), torch.randn(1000, 1153, generator=g) * 0.05,
               torch.randn(1000, generator=g) * 0.05]
    return names, tensors


class _Module:
    """The smallest state_dict holder the adapters need (an nn.Module stand-in)."""

    def __init__(self, names, tensors):
        from collections import OrderedDict

        self._sd = OrderedDict((n, t.clone()) for n, t in zip(names, tensors))

    def state_dict(self, *a, **k):
        return self._sd

    def load_state_dict(self, new, strict=True):
        for n, t in self._sd.items():
            t.copy_(new[n])


def _uploads(names, tensors, K, seed):
    import numpy as np

    rng = np.random.default_rng(seed)
    out = []
    for k in range(K):
        u = {}
        for n, t in zip(names, tensors):
            a = t.numpy()
            if a.dtype == np.int64:
                u[n] = np.asarray(a + int(rng.integers(0, 9)), dtype=np.int64)
            else:
                u[n] = (a + rng.standard_normal(a.shape).astype(np.float32) * np.float32(0.01)).astype(np.float32)
        out.append({"client_id": k + 1, "update_weight": u, "moving_loss": float(rng.uniform(0.5, 2.0))})
    return out


def run(devices, K=24, capacity=7, rounds=2) -> dict:
    import argparse as ap

    import numpy as np
    import torch

    from . import _native
    from . import kernels as kx
    from .cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from .cloud.aggregation.optimizers import TorchServerOptimizer
    from .cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from .cloud.internal.torch_model_adapter import TorchModelAdapter
    from .state import DeviceStream

    calls, real = [], _native.call

    def spy(fn, *args):
        calls.append((fn, args[-1] if args else None, DeviceStream.current()))
        return real(fn, *args)

    _native.call = kx.call = spy
    names, tensors = _model(5)
    report = {"devices": list(devices), "ok": True, "policies": {}}
    try:
        for policy in ("fedavg", "fedbuff", "fed-yogi", "q-fedavg"):
            t0 = time.perf_counter()
            args = ap.Namespace(gradient_policy=None if policy in ("fedavg", "fedbuff") else policy, yogi_eta=3e-3,
                                yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99, learning_rate=0.05, qfed_q=1.0)
            opt_s = TorchServerOptimizer(args.gradient_policy, args, devices[0])
            opt_1 = TorchServerOptimizer(args.gradient_policy, args, devices[0])
            sharded = ShardedModelAdapter(_Module(names, tensors), optimizer=opt_s, devices=list(devices),
                                          staging_capacity=capacity)
            single = TorchModelAdapter(_Module(names, tensors), optimizer=opt_1, device=devices[0],
                                       staging_capacity=capacity)
            cls = DeviceAsyncAggregator if policy == "fedbuff" else DeviceAggregator
            aggs = [cls(sharded, args), cls(single, args)]
            for a in aggs:
                a.device_keep_mean = True
            del calls[:]
            res = {"transport": sharded.group.transport}
            for r in range(rounds):
                ups = _uploads(names, tensors, K, 100 * r + len(policy))
                for a in aggs:
                    if policy == "fedbuff":
                        a.round = 10 + r
                        for k in range(K):
                            a.client_task_model_version[k + 1] = a.round - k % 6
                    a.start_round(K)
                    for u in ups:
                        a.on_result(dict(u))
                got, want = sharded.get_weights(), single.get_weights()
                for i, (x, y) in enumerate(zip(got, want)):
                    if policy == "q-fedavg" and x.dtype == torch.float32:
                        xd, yd = x.double(), y.double()
                        scale = torch.maximum(yd.abs(), yd.pow(2).mean().sqrt())
                        ok = bool(((xd - yd).abs() <= 1e-6 * scale).all())
                    elif policy == "q-fedavg":
                        ok = bool(((x - y).abs() <= 1).all())
                    else:
                        ok = torch.equal(x, y)
                    if not ok:
                        res.setdefault("mismatch", []).append(f"round {r} tensor {i}")
                m0, m1 = list(aggs[0].model_weights), list(aggs[1].model_weights)
                if not all(np.array_equal(np.asarray(a), np.asarray(b)) for a, b in zip(m0, m1)):
                    res.setdefault("mismatch", []).append(f"round {r} model_weights")
            # every launch on its part's non-null stream; every part's buffers on its device
            handles = {ds.handle: ds for ds in sharded.group.streams}
            bad = 0
            for fn, st, cur in calls:
                if (fn.startswith("fa_rccl_") and fn not in ("fa_rccl_init", "fa_rccl_destroy")) or fn in ("fa_reduce_parts", "fa_yogi_step_parts"):
                    bad += int(list(st) != sharded.group.stream_handles())  # a per-part stream table
                elif fn in ("fa_host_gather", "fa_rccl_init", "fa_rccl_destroy", "fa_host_register",
                            "fa_host_unregister", "fa_h2d_pieces"):
                    continue
                elif cur is None or not st or st != cur.handle or (st not in handles and cur is not single.dstream):
                    bad += 1
            res["native_calls"] = len(calls)
            res["calls_off_their_stream"] = bad
            res["buffers_on_their_device"] = all(p._f[p._cur].device == p.device == ds.device and
                                                 (p.staging is None or p.staging.x.device == p.device)
                                                 for p, ds in zip(sharded.parts, sharded.group.streams))
            res["seconds"] = round(time.perf_counter() - t0, 3)
            ok = not res.get("mismatch") and bad == 0 and res["buffers_on_their_device"]
            res["ok"] = ok
            report["ok"] = report["ok"] and ok
            report["policies"][policy] = res
            sharded.group.close()
    finally:
        _native.call = kx.call = real
    return report


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--devices", required=True, help="comma-separated GPU ordinals, e.g. 0,1,2,3")
    a = p.parse_args(argv)
    devices = [int(d) for d in a.devices.split(",") if d.strip()]
    try:
        rep = run(devices)
    except Exception as e:  # reported, not raised: the caller (bench.py) records the failure
        rep = {"devices": devices, "ok": False, "error": f"{type(e).__name__}: {e}"}
    print(json.dumps(rep), flush=True)
    return 0 if rep.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
