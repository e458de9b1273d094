"""Generate golden input/output vectors from the REAL FedScale reference.

Run ONLY in the build container (it needs /root/reference, which never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

What it does
------------
It imports the reference's own hot-path code from /root/reference and drives it exactly the way the
reference's event loop does for one or more rounds:

* ``Aggregator.update_weight_aggregation``        fedscale/cloud/aggregation/aggregator.py:489-511
* ``AsyncAggregator.update_weight_aggregation``   fedscale/cloud/aggregation/async_aggregator.py:115-137
* ``TorchModelAdapter.set_weights/get_weights``   fedscale/cloud/internal/torch_model_adapter.py:23-47
* ``TorchServerOptimizer.update_round_gradient``  fedscale/cloud/aggregation/optimizers.py:31-108
* ``YoGi.update``                                  fedscale/utils/optimizer/yogi.py:15-36

The per-arrival driver below restates the three lines of ``client_completion_handler`` that touch the
reduction state (aggregator.py:466-467 q-FedAvg retention, :484 ``model_in_update += 1``, :485 the hook
call) and the round reset of ``round_completion_handler`` (aggregator.py:609, :620-623); the state
contract is the reference test's ``MockAggregator`` (fedscale/tests/cloud/aggregation/test_aggregator.py:11-17).

Importing ``aggregator.py`` pulls in off-path modules that are absent from this image (wandb,
tensorboard, torchvision, tensorflow, overrides, and the model-zoo / TF-adapter modules that import
them). They are replaced by empty ``sys.modules`` placeholders, exactly as SURVEY.md §8c records; none
of them is reached by the functions listed above. Nothing is written under /root/reference
(``PYTHONDONTWRITEBYTECODE`` is forced).

Outputs (data only — inputs and the reference's outputs):
    tests/golden/<scenario>.npz   arrays (client inputs stored as float16-exact values, outputs fp32/int64)
    tests/golden/<scenario>.json  metadata (tensor names/shapes/dtypes, K, policy, hyper-parameters)
"""
from __future__ import annotations

import argparse
import copy
import json
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


# ----------------------------------------------------------------------------------------------
# placeholders for absent, off-path imports
# ----------------------------------------------------------------------------------------------
def _install_placeholders():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Anything:  # attribute sink for e.g. torchvision.transforms.Compose
        def __getattr__(self, _):
            return _Anything()

        def __call__(self, *a, **k):
            return _Anything()

    mod("wandb")
    tb = mod("torch.utils.tensorboard", SummaryWriter=_Anything)
    torch.utils.tensorboard = tb
    tv = mod("torchvision")
    tv.models = mod("torchvision.models")
    tv.transforms = mod("torchvision.transforms")
    tv.datasets = mod("torchvision.datasets")
    mod("tensorflow")
    mod("overrides", overrides=lambda f: f)
    mod("fedscale.utils.models.torch_model_provider", get_cv_model=None)
    mod("fedscale.utils.models.tensorflow_model_provider", get_tensorflow_model=None)
    mod("fedscale.cloud.internal.tensorflow_model_adapter", TensorflowModelAdapter=object)


def _import_reference():
    sys.argv = [sys.argv[0]]  # config_parser.py:291 parses argv at import time
    sys.path.insert(0, REF)
    _install_placeholders()
    import fedscale.cloud.config_parser as parser
    from fedscale.cloud.aggregation.aggregator import Aggregator
    from fedscale.cloud.aggregation.async_aggregator import AsyncAggregator
    from fedscale.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale.cloud.internal.torch_model_adapter import TorchModelAdapter

    return parser, Aggregator, AsyncAggregator, TorchServerOptimizer, TorchModelAdapter


# ----------------------------------------------------------------------------------------------
# models (state_dict layouts); defined here, the tests only ever see names/shapes/dtypes + values
# ----------------------------------------------------------------------------------------------
class MixedNet(nn.Module):
    """fp32 params + BN buffers + int64 num_batches_tracked + a 0-d and an empty fp32 buffer."""

    def __init__(self):
        super().__init__()
        self.register_buffer("scale0d", torch.tensor(0.75))
        self.register_buffer("empty", torch.zeros(0))
        self.conv = nn.Conv2d(2, 3, 3)
        self.bn = nn.BatchNorm2d(3)
        self.fc = nn.Linear(12, 5)
        self.bn2 = nn.BatchNorm1d(5)


class FemnistCNN(nn.Module):
    """MnistCNN layout (fedscale/utils/models/simple/models.py:11-29) with a 62-way fc2 (FEMNIST): P=24,492."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 62)


class WideNet(nn.Module):
    """A few odd-sized fp32 tensors (P not a multiple of 4/64) for ordering tests at larger K."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(37, 23)
        self.b = nn.Linear(23, 1)
        self.register_buffer("c", torch.zeros(5, 7, 3))


def _f16_exact(rng, shape, scale, loc=None):
    x = rng.normal(0.0, scale, size=shape)
    if loc is not None:
        x = x + loc
    return x.astype(np.float16).astype(np.float32)


def _init_model(cls, seed):
    torch.manual_seed(seed)
    m = cls()
    rng = np.random.default_rng(seed)
    sd = m.state_dict()
    new = {}
    for k, v in sd.items():
        if v.dtype == torch.int64:
            new[k] = torch.tensor(int(rng.integers(0, 50)), dtype=torch.int64).reshape(v.shape)
        else:
            new[k] = torch.from_numpy(_f16_exact(rng, tuple(v.shape), 0.05))
    m.load_state_dict(new)
    return m


def _client_updates(model, K, seed, as_dict_every=2):
    """Full-weight uploads (torch_client.py:76-78,90): dict name->ndarray or list, base + noise."""
    rng = np.random.default_rng(seed)
    sd = model.state_dict()
    ups = []
    for k in range(K):
        w = {}
        for name, t in sd.items():
            base = t.numpy()
            if t.dtype == torch.int64:
                w[name] = np.array(base + int(rng.integers(0, 9)), dtype=np.int64).reshape(base.shape)
            else:
                w[name] = _f16_exact(rng, base.shape, 0.01, loc=base)
        ups.append(w if (k % as_dict_every == 0) else list(w.values()))
    return ups


def _meta_of(model):
    sd = model.state_dict()
    return {
        "names": list(sd.keys()),
        "shapes": [list(v.shape) for v in sd.values()],
        "dtypes": [str(v.dtype).replace("torch.", "") for v in sd.values()],
    }


def _save(name, meta, arrays):
    np.savez(os.path.join(OUT, name + ".npz"), **arrays)
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    sz = os.path.getsize(os.path.join(OUT, name + ".npz"))
    print(f"  {name}: {sz/1024:.1f} KiB")


def _compact(v):
    """fp32 inputs are stored as float16 when that round-trips exactly (halves the fixture size)."""
    if v.dtype == np.float32 and np.array_equal(v.astype(np.float16).astype(np.float32), v):
        return v.astype(np.float16)
    return v


def _store_inputs(arrays, ups, names):
    for k, u in enumerate(ups):
        vals = list(u.values()) if isinstance(u, dict) else u
        for i, v in enumerate(vals):
            v = np.asarray(v)
            arrays[f"client/{k}/{i}"] = _compact(v)


def _store_state(arrays, prefix, tensors):
    for i, t in enumerate(tensors):
        arrays[f"{prefix}/{i}"] = (t.detach().cpu().numpy() if torch.is_tensor(t) else np.asarray(t)).copy()


# ----------------------------------------------------------------------------------------------
def main():
    parser, Aggregator, AsyncAggregator, TorchServerOptimizer, TorchModelAdapter = _import_reference()

    class MockAggregator(Aggregator):  # test_aggregator.py:11-17 state contract
        def __init__(self, model_wrapper, args):
            self.model_weights = []
            self.model_in_update = 0
            self.tasks_round = 0
            self.model_wrapper = model_wrapper
            self.client_training_results = []
            self.args = args

    class MockAsyncAggregator(AsyncAggregator):
        def __init__(self, model_wrapper, args):
            MockAggregator.__init__(self, model_wrapper, args)
            self.round = 0
            self.client_task_model_version = {}
            self.aggregation_denominator = 0

    def make_args(policy, lr=0.05, q=1.0):
        a = argparse.Namespace(**vars(parser.args))
        a.gradient_policy = policy
        a.learning_rate = lr
        a.qfed_q = q
        return a

    def run_round(agg, results_list):
        agg.model_in_update = 0  # aggregator.py:620
        agg.client_training_results = []  # aggregator.py:622
        agg.tasks_round = len(results_list)  # aggregator.py:609
        for res in results_list:
            if agg.args.gradient_policy in ["q-fedavg"]:  # aggregator.py:466-467
                agg.client_training_results.append(res)
            agg.model_in_update += 1  # aggregator.py:484
            agg.update_weight_aggregation(res)  # aggregator.py:485

    def results_of(ups, losses=None, ids=None):
        return [
            {
                "client_id": (ids[k] if ids is not None else k + 1),
                "update_weight": u,
                "moving_loss": (float(losses[k]) if losses is not None else 1.0),
                "utility": 1.0,
                "trained_size": 20,
                "success": True,
                "wall_duration": 0.0,
            }
            for k, u in enumerate(ups)
        ]

    print("generating golden vectors from", REF)

    # 1. the reference test's KAT, with a real assert: 2w, 2w, 5w -> 3w (test_aggregator.py:43-54)
    torch.manual_seed(0)
    model = torch.nn.Linear(3, 2)
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(torch.from_numpy(_f16_exact(np.random.default_rng(1), tuple(p.shape), 0.5)))
    adapter = TorchModelAdapter(model)
    agg = MockAggregator(adapter, make_args(None))
    w = copy.deepcopy(adapter.get_weights())
    ups = [[x.numpy() * f for x in w] for f in (2, 2, 5)]
    meta = _meta_of(model)
    arrays = {}
    _store_state(arrays, "init", w)
    _store_inputs(arrays, ups, meta["names"])
    run_round(agg, results_of(ups))
    got = adapter.get_weights()
    for a, b in zip(got, w):
        assert np.array_equal(a.numpy(), b.numpy() * 3), "reference KAT 2,2,5 -> 3 failed"
    _store_state(arrays, "out/0", got)
    meta.update(policy="fedavg", rounds=[3], optimizer=None)
    _save("kat_linear_225", meta, arrays)

    # 2. FedAvg, mixed layout, K in {1,3,7}; optimizer present with mode None (aggregator.py:203-208)
    for K in (1, 3, 7):
        model = _init_model(MixedNet, 10 + K)
        adapter = TorchModelAdapter(model, optimizer=TorchServerOptimizer(None, make_args(None), None))
        agg = MockAggregator(adapter, make_args(None))
        meta = _meta_of(model)
        arrays = {}
        _store_state(arrays, "init", adapter.get_weights())
        ups = _client_updates(model, K, 100 + K)
        _store_inputs(arrays, ups, meta["names"])
        run_round(agg, results_of(ups))
        _store_state(arrays, "out/0", adapter.get_weights())
        meta.update(policy="fedavg", rounds=[K], dict_every=2, optimizer="none")
        _save(f"fedavg_mixed_k{K}", meta, arrays)

    # 3. FedAvg, C1 layout (FEMNIST small CNN, P=24,492), K=10
    model = _init_model(FemnistCNN, 21)
    adapter = TorchModelAdapter(model, optimizer=TorchServerOptimizer(None, make_args(None), None))
    agg = MockAggregator(adapter, make_args(None))
    meta = _meta_of(model)
    arrays = {}
    _store_state(arrays, "init", adapter.get_weights())
    ups = _client_updates(model, 10, 210)
    _store_inputs(arrays, ups, meta["names"])
    run_round(agg, results_of(ups))
    _store_state(arrays, "out/0", adapter.get_weights())
    meta.update(policy="fedavg", rounds=[10], dict_every=2, optimizer="none")
    _save("fedavg_femnist_cnn_k10", meta, arrays)

    # 4. FedAvg, larger K (ordering sensitivity), odd sizes
    model = _init_model(WideNet, 31)
    adapter = TorchModelAdapter(model)
    agg = MockAggregator(adapter, make_args(None))
    meta = _meta_of(model)
    arrays = {}
    _store_state(arrays, "init", adapter.get_weights())
    ups = _client_updates(model, 64, 310, as_dict_every=3)
    _store_inputs(arrays, ups, meta["names"])
    run_round(agg, results_of(ups))
    _store_state(arrays, "out/0", adapter.get_weights())
    meta.update(policy="fedavg", rounds=[64], dict_every=3, optimizer=None)
    _save("fedavg_wide_k64", meta, arrays)

    # 5. FedBuff (async_aggregator.py:115-137): staleness s_k = k mod 6 at round 10
    model = _init_model(MixedNet, 41)
    adapter = TorchModelAdapter(model)
    agg = MockAsyncAggregator(adapter, make_args(None))
    agg.round = 10
    K = 8
    ids = list(range(101, 101 + K))
    stale = [k % 6 for k in range(K)]
    for cid, s in zip(ids, stale):
        agg.client_task_model_version[cid] = agg.round - s
    meta = _meta_of(model)
    arrays = {}
    _store_state(arrays, "init", adapter.get_weights())
    ups = _client_updates(model, K, 410)
    _store_inputs(arrays, ups, meta["names"])
    run_round(agg, results_of(ups, ids=ids))
    assert agg.aggregation_denominator == 0
    _store_state(arrays, "out/0", adapter.get_weights())
    meta.update(policy="fedbuff", rounds=[K], dict_every=2, optimizer=None, round=10, staleness=stale)
    _save("fedbuff_k8", meta, arrays)

    # 6. FedYoGi, 3 rounds with m/v carry-over (optimizers.py:43-63, yogi.py:15-36)
    for cls, tag, Ks in ((MixedNet, "mixed", (4, 3, 5)), (WideNet, "wide", (6, 6, 6))):
        model = _init_model(cls, 51)
        args = make_args("fed-yogi")
        opt = TorchServerOptimizer("fed-yogi", args, None)
        adapter = TorchModelAdapter(model, optimizer=opt)
        agg = MockAggregator(adapter, args)
        meta = _meta_of(model)
        arrays = {}
        _store_state(arrays, "init", adapter.get_weights())
        k0 = 0
        for r, K in enumerate(Ks):
            ups = _client_updates(model, K, 510 + r)
            for k, u in enumerate(ups):
                vals = list(u.values()) if isinstance(u, dict) else u
                for i, v in enumerate(vals):
                    v = np.asarray(v)
                    arrays[f"client/{k0 + k}/{i}"] = _compact(v)
            k0 += K
            run_round(agg, results_of(ups))
            _store_state(arrays, f"out/{r}", adapter.get_weights())
            _store_state(arrays, f"yogi_m/{r}", opt.gradient_controller.m_t)
            _store_state(arrays, f"yogi_v/{r}", opt.gradient_controller.v_t)
        meta.update(policy="fed-yogi", rounds=list(Ks), dict_every=2, optimizer="fed-yogi",
                    yogi=dict(eta=args.yogi_eta, tau=args.yogi_tau, beta=args.yogi_beta, beta2=args.yogi_beta2))
        _save(f"fedyogi_{tag}_3rounds", meta, arrays)

    # 7. q-FedAvg, q in {0,1,2}; and an lr-decay pair of rounds (optimizers.py:65-104)
    for q, lrs, tag in ((0.0, [0.05], "q0"), (1.0, [0.05], "q1"), (2.0, [0.05], "q2"),
                        (1.0, [0.05, 0.049], "q1_lrdecay")):
        model = _init_model(MixedNet, 61)
        args = make_args("q-fedavg", lr=lrs[0], q=q)
        opt = TorchServerOptimizer("q-fedavg", args, None)
        adapter = TorchModelAdapter(model, optimizer=opt)
        agg = MockAggregator(adapter, args)
        meta = _meta_of(model)
        arrays = {}
        _store_state(arrays, "init", adapter.get_weights())
        k0 = 0
        all_losses = []
        Ks = []
        for r, lr in enumerate(lrs):
            args.learning_rate = lr  # update_default_task_config, aggregator.py:552-558
            K = 5
            rng = np.random.default_rng(610 + r)
            losses = [float(x) for x in rng.uniform(0.5, 2.0, size=K)]
            ups = _client_updates(model, K, 620 + r)
            for k, u in enumerate(ups):
                vals = list(u.values()) if isinstance(u, dict) else u
                for i, v in enumerate(vals):
                    v = np.asarray(v)
                    arrays[f"client/{k0 + k}/{i}"] = _compact(v)
            k0 += K
            all_losses += losses
            Ks.append(K)
            run_round(agg, results_of(ups, losses=losses))
            _store_state(arrays, f"out/{r}", adapter.get_weights())
        meta.update(policy="q-fedavg", rounds=Ks, dict_every=2, optimizer="q-fedavg", q=q, lrs=lrs,
                    losses=all_losses)
        _save(f"qfedavg_{tag}", meta, arrays)

    # 8. Auxo per-cohort FedAvg (examples/auxo/aggregator.py:451-472): two cohorts, interleaved arrivals.
    #    Auxo's own modules need three more off-path placeholders: nltk (clustering), and its `config`
    #    module (which would yaml.load a file shipped in the reference; it is never read on this path).
    import types as _t

    nl = _t.ModuleType("nltk")
    nlc = _t.ModuleType("nltk.cluster")
    nlc.KMeansClusterer, nlc.euclidean_distance = object, None
    nl.cluster = nlc
    sys.modules.update({"nltk": nl, "nltk.cluster": nlc})
    cfg = _t.ModuleType("config")
    cfg.auxo_config = {}
    sys.modules["config"] = cfg
    sys.path.insert(0, os.path.join(REF, "examples", "auxo"))
    from aggregator import AuxoAggregator  # examples/auxo/aggregator.py

    class MockAuxo(AuxoAggregator):
        def __init__(self, wrappers, K):
            self.model_weights = [[] for _ in wrappers]
            self.model_in_update = [0 for _ in wrappers]
            self.tasks_round = list(K)
            self.model_wrapper = wrappers
            self.client_training_results = [[] for _ in wrappers]

    models = [_init_model(MixedNet, 71), _init_model(MixedNet, 72)]
    wrappers = [TorchModelAdapter(m) for m in models]
    Ks = [4, 3]
    order = [0, 1, 0, 0, 1, 1, 0]
    agg = MockAuxo(wrappers, Ks)
    meta = _meta_of(models[0])
    arrays = {}
    for c, w in enumerate(wrappers):
        _store_state(arrays, f"init_c{c}", w.get_weights())
    ups = _client_updates(models[0], len(order), 710)
    _store_inputs(arrays, ups, meta["names"])
    for k, c in enumerate(order):
        agg.model_in_update[c] += 1  # examples/auxo/aggregator.py:307
        agg.update_weight_aggregation({"client_id": k + 1, "update_weight": ups[k], "moving_loss": 1.0}, c)
    for c, w in enumerate(wrappers):
        _store_state(arrays, f"out_c{c}", w.get_weights())
    meta.update(policy="auxo-cohorts", rounds=[len(order)], cohorts=order, cohort_K=Ks, dict_every=2, optimizer=None)
    _save("auxo_cohorts_fedavg", meta, arrays)

    # 9. HeteroFL sub-model combination (examples/heterofl/customized_aggregator.py:78-119): clients at
    #    model rates 1 / 0.5 / 0.25 / 0.125 upload prefix slices of every tensor; the global model takes the
    #    per-element mean over the clients that cover it.  The example's `config` module would open its
    #    YAML with a non-safe loader: a placeholder reads the same config.yml with yaml.safe_load (and
    #    shrinks resnet_hidden_size so the fixture stays small); its outdated logger import gets a placeholder.
    import yaml

    hdir = os.path.join(REF, "examples", "heterofl")
    hcfg = _t.ModuleType("config")
    with open(os.path.join(hdir, "config.yml")) as f:
        hcfg.cfg = yaml.safe_load(f)
    hcfg.cfg["resnet_hidden_size"] = [4, 8, 16, 32]
    sys.modules["config"] = hcfg
    sys.modules["fedscale.cloud.logger.aggregation_logging"] = _t.ModuleType("fedscale.cloud.logger.aggregation_logging")
    sys.path.insert(0, hdir)
    for m in ("aggregator", "client_manager", "resource_manager"):
        sys.modules.pop(m, None)  # auxo's same-named modules
    import customized_fllibs
    import resnet_heterofl
    from customized_aggregator import Customized_Aggregator

    class MockHetero(Customized_Aggregator):
        def __init__(self, model, results):
            self.model = model
            self.param_idx = {}
            self.client_training_results = results

    torch.manual_seed(81)
    gmodel = resnet_heterofl.resnet18(model_rate=1, track=False)
    with torch.no_grad():
        g = torch.Generator().manual_seed(82)
        for t in gmodel.state_dict().values():
            t.copy_((torch.randn(t.shape, generator=g) * 0.05).half().float())
    rates = [1, 0.5, 0.25, 0.125, 1, 0.5, 0.0625]
    rng = np.random.default_rng(83)
    results = []
    for r in rates:
        local = customized_fllibs.split_model(gmodel, r)
        for k in local:
            local[k] = torch.from_numpy(_f16_exact(rng, tuple(local[k].shape), 0.01, loc=local[k].numpy()))
        results.append({"model_rate": r, "local_parameters": local})
    meta = _meta_of(gmodel)
    arrays = {}
    _store_state(arrays, "init", list(gmodel.state_dict().values()))
    for m, res in enumerate(results):
        for i, v in enumerate(res["local_parameters"].values()):
            arrays[f"client/{m}/{i}"] = _compact(v.numpy())
    MockHetero(gmodel, results).combine_models()
    _store_state(arrays, "out/0", list(gmodel.state_dict().values()))
    meta.update(policy="heterofl", rounds=[len(rates)], rates=rates, optimizer=None)
    _save("heterofl_resnet18_small", meta, arrays)

    print("done")


if __name__ == "__main__":
    main()
