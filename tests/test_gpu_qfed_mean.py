"""q-FedAvg rounds keep the reference's Aggregator.model_weights at any K (aggregator.py:497-507: the FedAvg
mean is computed on the same inputs even in q-FedAvg mode), and the retained results let go of their
uploads once they are staged (aggregator.py:466-467 retains them only for optimizers.py:73-98)."""
import argparse

import numpy as np
import pytest
import torch

from tests.golden_io import StateDictModule, assert_state_close

pytestmark = pytest.mark.gpu


def _model(seed=0):
    names = ["conv.weight", "bn.num_batches_tracked", "fc.weight", "fc.bias"]
    g = torch.Generator().manual_seed(seed)
    tensors = [torch.randn(16, 3, 5, 5, generator=g) * 0.05, torch.tensor(7, dtype=torch.int64),
               torch.randn(10, 1021, generator=g) * 0.05, torch.randn(10, generator=g) * 0.05]
    return names, tensors


def _uploads(names, tensors, K, seed=1):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(K):
        up = {}
        for n, t in zip(names, tensors):
            if t.dtype == torch.int64:
                up[n] = np.array(int(t) + int(rng.integers(0, 50)), dtype=np.int64)
            else:
                up[n] = t.numpy() + rng.normal(0, 0.01, size=tuple(t.shape)).astype(np.float32)
        out.append({"client_id": k, "update_weight": up, "moving_loss": float(rng.uniform(0.5, 2.0))})
    return out


@pytest.mark.parametrize("keep_mean", [True, "always"])
@pytest.mark.parametrize("sharded", [False, True])
def test_qfedavg_k2500_capacity333_model_weights(gpu_device, keep_mean, sharded):
    """K = 2500 through chunks of 333 (8 chunks): model_weights is the oracle's FedAvg mean bit for bit,
    the new model is the reference's q-FedAvg step within 1e-5, and client_training_results hold no arrays."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, StagedUpload
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import (OracleAggregator, OracleModel, OracleModelAdapter, OracleServerOptimizer,
                                      fedavg_close, fedavg_step)

    K = 2500
    names, tensors = _model()
    args = argparse.Namespace(gradient_policy="q-fedavg", learning_rate=0.05, qfed_q=1.0)
    opt = TorchServerOptimizer("q-fedavg", args, "cuda:0")
    model = StateDictModule(names, tensors)
    if sharded:
        adapter = ShardedModelAdapter(model, optimizer=opt, devices=[0, 0], transport="copy", staging_capacity=333)
    else:
        adapter = TorchModelAdapter(model, optimizer=opt, device="cuda:0", staging_capacity=333)

    class A(DeviceAggregator):
        device_keep_mean = keep_mean

    agg = A(adapter, args)
    oracle = OracleAggregator(OracleModelAdapter(OracleModel(names, tensors), OracleServerOptimizer("q-fedavg", args)),
                              args)
    results = _uploads(names, tensors, K)
    acc = None
    for k, res in enumerate(results):
        acc = fedavg_step(acc, [np.array(v) for v in res["update_weight"].values()], k == 0)
    want_mean = fedavg_close(acc, K)
    agg.start_round(K)
    oracle.start_round(K)
    for res in results:
        oracle.on_result({**res, "update_weight": dict(res["update_weight"])})
        agg.on_result(res)
    got_mean = list(agg.model_weights)
    for g, w in zip(got_mean, want_mean):
        assert np.asarray(g).dtype == np.asarray(w).dtype
        np.testing.assert_array_equal(np.asarray(g), np.asarray(w))
    assert_state_close(adapter.get_weights(), [t.numpy() for t in oracle.model_wrapper.get_weights()], 1e-5,
                       "q-fedavg k2500", int_slack=1)
    assert len(agg.client_training_results) == K
    assert all(type(r["update_weight"]) is StagedUpload for r in agg.client_training_results)
    if sharded:
        adapter.group.close()


def test_single_chunk_mean_survives_staging_reuse_with_always(gpu_device):
    """keep_mean="always": the q-FedAvg mean is fused into the round, so model_weights of round r is still
    readable after round r+1 has started (and overwritten the staged uploads)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import fedavg_close, fedavg_step

    names, tensors = _model(3)
    args = argparse.Namespace(gradient_policy="q-fedavg", learning_rate=0.05, qfed_q=1.0)
    adapter = TorchModelAdapter(StateDictModule(names, tensors), optimizer=TorchServerOptimizer("q-fedavg", args, None),
                                device="cuda:0")

    class A(DeviceAggregator):
        device_keep_mean = "always"

    agg = A(adapter, args)
    res = _uploads(names, tensors, 12, seed=4)
    acc = None
    for k, r in enumerate(res[:6]):
        acc = fedavg_step(acc, [np.array(v) for v in r["update_weight"].values()], k == 0)
    want = fedavg_close(acc, 6)
    agg.start_round(6)
    for r in res[:6]:
        agg.on_result(r)
    mw = agg.model_weights
    agg.start_round(6)
    for r in res[6:9]:  # the next round has started: its uploads overwrite the staging slots
        agg.on_result(r)
    torch.cuda.synchronize()
    # the lazy view is bound to the finished round's model version, which is still current
    for g, w in zip(list(mw), want):
        np.testing.assert_array_equal(np.asarray(g), np.asarray(w))
