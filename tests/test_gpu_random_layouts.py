"""Randomised differential test of the whole device path against the oracle (the CPU restatement pinned by
the reference's fixtures, oracle/cpu_reference.py): random state_dict layouts (0-d, empty, odd-sized and
int64 entries, dict or list uploads), random K, random staging capacities (chunk folding), every server
policy, two rounds each (ping-pong buffers, FedYoGi state, FedBuff staleness).  FedAvg / FedBuff are
bit-exact; FedYoGi within 1e-6 and q-FedAvg within 1e-5 (the tolerances of test_gpu_parity.py)."""
import argparse

import numpy as np
import pytest
import torch

from tests.golden_io import DEFAULT_ARGS, StateDictModule, assert_state_close, assert_state_equal

pytestmark = pytest.mark.gpu

POLICIES = ["fedavg", "fedbuff", "fed-yogi", "q-fedavg"]
SHAPES = [(), (0,), (1,), (3,), (5, 7), (64,), (33, 17), (4, 3, 3, 3), (1021,), (2, 2049), (8, 1, 5, 5)]


def _layout(rng):
    T = int(rng.integers(1, 9))
    names, tensors = [], []
    for i in range(T):
        shape = SHAPES[int(rng.integers(0, len(SHAPES)))]
        if rng.random() < 0.15:  # BatchNorm num_batches_tracked-like counters
            t = torch.tensor(int(rng.integers(0, 50)), dtype=torch.int64) if rng.random() < 0.7 else \
                torch.from_numpy(rng.integers(0, 50, size=shape).astype(np.int64))
        else:
            t = torch.from_numpy(np.asarray(rng.standard_normal(shape) * 0.05, dtype=np.float32))
        names.append(f"m{i}.w" if i % 2 else f"layer{i}.b")
        tensors.append(t)
    return names, tensors


def _uploads(rng, names, tensors, K, as_list_every):
    out = []
    for k in range(K):
        vals = []
        for t in tensors:
            a = t.numpy()
            if a.dtype == np.int64:  # ndarrays, 0-d ones included (param.data.cpu().numpy(), torch_client.py:76-78)
                vals.append(np.asarray(a + rng.integers(0, 7, size=a.shape), dtype=np.int64))
            else:
                vals.append(np.asarray(a + rng.standard_normal(a.shape) * 0.01, dtype=np.float32))
        up = vals if as_list_every and k % as_list_every == 0 else dict(zip(names, vals))
        out.append({"client_id": 101 + k, "update_weight": up, "moving_loss": float(rng.uniform(0.5, 2.0))})
    return out


@pytest.mark.parametrize("seed", range(96))
def test_random_layout_round_matches_oracle(gpu_device, seed):
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import OracleAggregator, OracleModel, OracleModelAdapter, OracleServerOptimizer

    rng = np.random.default_rng(1000 + seed)
    policy = POLICIES[seed % len(POLICIES)]
    names, tensors = _layout(rng)
    a = dict(DEFAULT_ARGS)
    a["gradient_policy"] = policy if policy in ("fed-yogi", "q-fedavg") else None
    a["learning_rate"] = float(rng.choice([0.05, 0.01, 0.1]))
    a["qfed_q"] = float(rng.choice([0.0, 1.0, 2.0]))
    args, oargs = argparse.Namespace(**a), argparse.Namespace(**a)
    cap = [None, 1, 2, 3][int(rng.integers(0, 4))]
    mode = a["gradient_policy"]
    adapter = TorchModelAdapter(StateDictModule(names, tensors),
                                optimizer=TorchServerOptimizer(mode, args, "cuda:0"), device="cuda:0",
                                staging_capacity=cap)
    oracle = OracleAggregator(OracleModelAdapter(OracleModel(names, tensors), OracleServerOptimizer(mode, oargs)),
                              oargs, asynchronous=policy == "fedbuff")
    agg = DeviceAsyncAggregator(adapter, args) if policy == "fedbuff" else DeviceAggregator(adapter, args)
    for r in range(2):
        K = int(rng.integers(1, 25))
        ups = _uploads(rng, names, tensors, K, as_list_every=int(rng.integers(0, 3)))
        if policy == "fedbuff":
            for o in (agg, oracle):
                o.round = 3 + r
            for res in ups:
                v = 3 + r - int(rng.integers(0, 6))
                agg.client_task_model_version[res["client_id"]] = v
                oracle.client_task_model_version[res["client_id"]] = v
        agg.start_round(K)
        oracle.start_round(K)
        for res in ups:
            oracle.on_result({**res, "update_weight": res["update_weight"]})  # its own result dict
            agg.on_result(res)
        got = adapter.get_weights()
        want = [t.numpy() for t in oracle.model_wrapper.get_weights()]
        ctx = f"seed {seed} {policy} r{r} K={K} cap={cap}"
        if policy in ("fedavg", "fedbuff"):
            assert_state_equal(got, want, ctx)
            assert_state_equal(list(agg.model_weights), [np.asarray(w) for w in oracle.model_weights], ctx + " mean")
        elif policy == "fed-yogi":  # the reference's torch.sqrt is MKL's, 1 ulp low on ~0.7 % of inputs
            assert_state_close(got, want, 1e-6, ctx)
        else:
            assert_state_close(got, want, 1e-5, ctx, int_slack=1)


@pytest.mark.parametrize("seed", range(32))
def test_random_layout_sharded_matches_oracle(gpu_device, seed):
    """The same random rounds through a ShardedModelAdapter of 2-4 parts on the one card (copy transport):
    the parts' slices fall anywhere, across tensors and through 0-d / empty entries."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from oracle.cpu_reference import OracleAggregator, OracleModel, OracleModelAdapter, OracleServerOptimizer

    rng = np.random.default_rng(5000 + seed)
    policy = POLICIES[seed % len(POLICIES)]
    names, tensors = _layout(rng)
    a = dict(DEFAULT_ARGS)
    a["gradient_policy"] = policy if policy in ("fed-yogi", "q-fedavg") else None
    a["qfed_q"] = float(rng.choice([0.0, 1.0, 2.0]))
    args, oargs = argparse.Namespace(**a), argparse.Namespace(**a)
    n = int(rng.integers(2, 5))
    cap = [None, 1, 3][int(rng.integers(0, 3))]
    mode = a["gradient_policy"]
    adapter = ShardedModelAdapter(StateDictModule(names, tensors), optimizer=TorchServerOptimizer(mode, args, "cuda:0"),
                                  devices=[0] * n, transport="copy", staging_capacity=cap)
    oracle = OracleAggregator(OracleModelAdapter(OracleModel(names, tensors), OracleServerOptimizer(mode, oargs)),
                              oargs, asynchronous=policy == "fedbuff")
    agg = DeviceAsyncAggregator(adapter, args) if policy == "fedbuff" else DeviceAggregator(adapter, args)
    for r in range(2):
        K = int(rng.integers(1, 17))
        ups = _uploads(rng, names, tensors, K, as_list_every=int(rng.integers(0, 3)))
        if policy == "fedbuff":
            for o in (agg, oracle):
                o.round = 3 + r
            for res in ups:
                v = 3 + r - int(rng.integers(0, 6))
                agg.client_task_model_version[res["client_id"]] = v
                oracle.client_task_model_version[res["client_id"]] = v
        agg.start_round(K)
        oracle.start_round(K)
        for res in ups:
            oracle.on_result({**res, "update_weight": res["update_weight"]})
            agg.on_result(res)
        got = adapter.get_weights()
        want = [t.numpy() for t in oracle.model_wrapper.get_weights()]
        ctx = f"seed {seed} {policy} parts={n} r{r} K={K} cap={cap}"
        if policy in ("fedavg", "fedbuff"):
            assert_state_equal(got, want, ctx)
            assert_state_equal(list(agg.model_weights), [np.asarray(w) for w in oracle.model_weights], ctx + " mean")
        elif policy == "fed-yogi":
            assert_state_close(got, want, 1e-6, ctx)
        else:
            assert_state_close(got, want, 1e-5, ctx, int_slack=1)
