"""Round-3 golden vectors from the REAL FedScale reference (build container only; needs /root/reference).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden_r3.py

1. Full-precision fixtures.  gen_golden.py stores float16-exact inputs (half the bytes), and a sum of K <= 64
   such values near 0.05 is mostly exact in fp32, so those fixtures rarely distinguish one summation order
   from another.  These use unrounded fp32 inputs, so the reference's own outputs pin the arrival-order
   rounding of aggregator.py:500-507 (FedAvg) and async_aggregator.py:129-135 (FedBuff):
       fedavg_wide_k64_fp32, fedavg_wide_k200_fp32   (WideNet, P = 1,003)
       fedbuff_mixed_k64_fp32                        (MixedNet with int64 buffers, staleness k mod 6)
   Each meta records ``order_sensitive_elements``: how many output elements come out different when the
   same inputs are summed in reverse order (proof that the fixture pins the order).

2. Config 1's job configuration.  BASELINE config 1 is "FEMNIST small-CNN FedAvg, 10 clients/round ... via
   benchmark/configs".  The reference's launcher turns ``benchmark/configs/femnist/conf.yml``'s ``job_conf``
   list into one dict and then into ``--key value`` flags (docker/driver.py:81-95, 114-119), which the
   aggregator parses with config_parser.py (:291 ``parse_known_args``).  This does the same in a child
   process (config_parser parses sys.argv at import), with ``num_participants`` overridden to 10 as SURVEY
   §8d specifies, and writes the parsed flags the aggregation path reads to ``c1_femnist_job_conf.json``.

Outputs are data only (inputs, the reference's outputs, parsed flag values); no reference text is kept.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gen_golden as G  # noqa: E402  (the reference import with its placeholders, models, helpers)

CONF = os.path.join(G.REF, "benchmark", "configs", "femnist", "conf.yml")
#: the flags of config_parser.py that the aggregation hot path and config 1's round read
C1_FLAGS = ("job_name", "data_set", "model", "num_participants", "gradient_policy", "learning_rate", "local_steps",
            "batch_size", "use_cuda", "cuda_device", "rounds", "eval_interval", "yogi_eta", "yogi_tau", "yogi_beta",
            "yogi_beta2", "qfed_q", "engine", "experiment_mode")


def _fp32_updates(model, K, seed, as_dict_every=2, scale=0.01):
    """Full-weight uploads with UNROUNDED fp32 values (base + noise)."""
    rng = np.random.default_rng(seed)
    ups = []
    for k in range(K):
        w = {}
        for name, t in model.state_dict().items():
            base = t.numpy()
            if t.dtype == torch.int64:
                w[name] = np.array(base + int(rng.integers(0, 9)), dtype=np.int64).reshape(base.shape)
            else:
                w[name] = (base + rng.normal(0.0, scale, size=base.shape)).astype(np.float32)
        ups.append(w if (k % as_dict_every == 0) else list(w.values()))
    return ups


def _fp32_model(cls, seed):
    torch.manual_seed(seed)
    m = cls()
    rng = np.random.default_rng(seed)
    new = {}
    for k, v in m.state_dict().items():
        if v.dtype == torch.int64:
            new[k] = torch.tensor(int(rng.integers(0, 50)), dtype=torch.int64).reshape(v.shape)
        else:
            new[k] = torch.from_numpy(rng.normal(0.0, 0.05, size=tuple(v.shape)).astype(np.float32))
    m.load_state_dict(new)
    return m


def _order_sensitivity(ups, weights=None):
    """Elements whose fp32 arrival-order chain differs from the reverse-order chain."""
    vals = [list(u.values()) if isinstance(u, dict) else u for u in ups]
    n = 0
    for i in range(len(vals[0])):
        col = [np.asarray(v[i]) for v in vals]
        if col[0].dtype != np.float32:
            continue
        w = weights if weights is not None else [None] * len(col)
        fwd = rev = None
        for x, s in zip(col, w):
            t = x if s is None else x * s
            fwd = t if fwd is None else fwd + t
        for x, s in zip(col[::-1], w[::-1]):
            t = x if s is None else x * s
            rev = t if rev is None else rev + t
        n += int(np.count_nonzero(fwd != rev))
    return n


def gen_fp32_fixtures():
    parser, Aggregator, AsyncAggregator, TorchServerOptimizer, TorchModelAdapter = G._import_reference()

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

    import argparse

    def make_args():
        a = argparse.Namespace(**vars(parser.args))
        a.gradient_policy = None
        return a

    def run_round(agg, ups, ids=None):
        agg.model_in_update = 0  # aggregator.py:620
        agg.client_training_results = []  # aggregator.py:622
        agg.tasks_round = len(ups)  # aggregator.py:609
        for k, u in enumerate(ups):
            agg.model_in_update += 1  # aggregator.py:484
            agg.update_weight_aggregation({"client_id": ids[k] if ids else k + 1, "update_weight": u,
                                           "moving_loss": 1.0})  # aggregator.py:485

    def store_inputs(arrays, ups):
        # raw fp32 (no float16 compaction), one [K, *shape] stack per tensor (keeps K = 200 under 1 MB)
        vals = [list(u.values()) if isinstance(u, dict) else u for u in ups]
        for i in range(len(vals[0])):
            arrays[f"clients/{i}"] = np.stack([np.asarray(v[i]) for v in vals])

    for K, seed in ((64, 3100), (200, 3200)):
        model = _fp32_model(G.WideNet, seed)
        adapter = TorchModelAdapter(model)
        agg = MockAggregator(adapter, make_args())
        meta = G._meta_of(model)
        arrays = {}
        G._store_state(arrays, "init", adapter.get_weights())
        ups = _fp32_updates(model, K, seed + 1, as_dict_every=3)
        store_inputs(arrays, ups)
        run_round(agg, ups)
        G._store_state(arrays, "out/0", adapter.get_weights())
        meta.update(policy="fedavg", rounds=[K], dict_every=3, optimizer=None, inputs="fp32 (unrounded)",
                    order_sensitive_elements=_order_sensitivity(ups))
        G._save(f"fedavg_wide_k{K}_fp32", meta, arrays)

    model = _fp32_model(G.MixedNet, 3300)
    adapter = TorchModelAdapter(model)
    agg = MockAsyncAggregator(adapter, make_args())
    agg.round = 10
    K = 64
    ids = list(range(101, 101 + K))
    stale = [k % 6 for k in range(K)]
    for cid, s in zip(ids, stale):
        agg.client_task_model_version[cid] = agg.round - s
    meta = G._meta_of(model)
    arrays = {}
    G._store_state(arrays, "init", adapter.get_weights())
    ups = _fp32_updates(model, K, 3301)
    store_inputs(arrays, ups)
    run_round(agg, ups, ids=ids)
    G._store_state(arrays, "out/0", adapter.get_weights())
    w32 = [np.float32(1 / (1 + s) ** 0.5) for s in stale]
    meta.update(policy="fedbuff", rounds=[K], dict_every=2, optimizer=None, round=10, staleness=stale,
                inputs="fp32 (unrounded)", order_sensitive_elements=_order_sensitivity(ups, w32))
    G._save("fedbuff_mixed_k64_fp32", meta, arrays)


_CHILD = r"""
import json, sys
sys.dont_write_bytecode = True
sys.path.insert(0, %(ref)r)
sys.argv = ["aggregator"] + %(argv)r
import fedscale.cloud.config_parser as p
print(json.dumps({k: getattr(p.args, k) for k in %(flags)r}))
"""


def gen_c1_job_conf():
    import yaml

    with open(CONF) as f:
        yaml_conf = yaml.safe_load(f)
    job_conf = {}
    for conf in yaml_conf["job_conf"]:  # docker/driver.py:81-82
        job_conf.update(conf)
    job_conf["num_participants"] = 10  # config 1 runs 10 clients per round
    argv = []
    for name, val in job_conf.items():  # docker/driver.py:92-93 (--name value)
        argv += [f"--{name}", str(val)]
    code = _CHILD % {"ref": G.REF, "argv": argv, "flags": list(C1_FLAGS)}
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1"))
    parsed = json.loads(out.stdout.strip().splitlines()[-1])
    doc = {"source": "benchmark/configs/femnist/conf.yml job_conf, converted as docker/driver.py:81-95 and parsed "
                     "by fedscale/cloud/config_parser.py; num_participants overridden 50 -> 10 (SURVEY §8d)",
           "job_conf_num_participants": 50, "args": parsed}
    with open(os.path.join(HERE, "c1_femnist_job_conf.json"), "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print("  c1_femnist_job_conf:", parsed)


if __name__ == "__main__":
    gen_c1_job_conf()
    gen_fp32_fixtures()
    print("done")
