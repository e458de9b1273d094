"""Loader for the golden fixtures in tests/golden/ (data produced by tests/golden/gen_golden.py)."""
from __future__ import annotations

import argparse
import glob
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# config_parser.py defaults for the flags the path reads (config_parser.py:79-103,123)
DEFAULT_ARGS = dict(gradient_policy=None, learning_rate=0.05, min_learning_rate=5e-5, decay_factor=0.98,
                    decay_round=10, yogi_eta=3e-3, yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99,
                    qfed_q=1.0, max_staleness=5)


def scenario_names(kind="single"):
    """kind 'single': one global model per scenario; 'cohorts': Auxo multi-cohort scenarios; 'heterofl';
    'client': FedProx / local-DP client-side fixtures."""
    names = sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "*.json"))
                   if os.path.exists(p[:-5] + ".npz"))  # (c1_femnist_job_conf.json is a config, not a scenario)
    if kind == "client":  # client-side handler fixtures (gen_golden_client.py)
        return [n for n in names if n.startswith("client_")]
    names = [n for n in names if not n.startswith("client_")]
    coh = [n for n in names if n.startswith("auxo_")]
    het = [n for n in names if n.startswith("heterofl_")]
    if kind == "cohorts":
        return coh
    if kind == "heterofl":
        return het
    return [n for n in names if n not in coh and n not in het]


class Scenario:
    def __init__(self, name):
        self.name = name
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle defaults to False
        self.arrays = {k: z[k] for k in z.files}
        self.names = self.meta["names"]
        self.T = len(self.names)

    def _tensors(self, prefix):
        return [self.arrays[f"{prefix}/{i}"] for i in range(self.T)]

    def init_state(self, cohort=None):
        pre = "init" if cohort is None else f"init_c{cohort}"
        return [torch.from_numpy(np.array(a)) for a in self._tensors(pre)]

    def hetero_locals(self):
        """[per client: {name: local prefix-box array}] of a heterofl fixture."""
        out = []
        for m in range(len(self.meta["rates"])):
            vals = [a.astype(np.float32) if a.dtype == np.float16 else a for a in self._tensors(f"client/{m}")]
            out.append(dict(zip(self.names, vals)))
        return out

    def expected_cohort(self, c):
        return self._tensors(f"out_c{c}")

    def expected(self, r):
        return self._tensors(f"out/{r}")

    def yogi_state(self, r):
        return self._tensors(f"yogi_m/{r}"), self._tensors(f"yogi_v/{r}")

    def _client_tensors(self, k):
        if f"client/{k}/0" in self.arrays:
            return self._tensors(f"client/{k}")
        return [self.arrays[f"clients/{i}"][k] for i in range(self.T)]  # stacked [K, ...] per tensor

    def client(self, k):
        vals = []
        for a in self._client_tensors(k):
            vals.append(a.astype(np.float32) if a.dtype == np.float16 else a)
        every = self.meta.get("dict_every")
        if every and k % every == 0:
            return dict(zip(self.names, vals))
        return vals

    def rounds(self):
        """yield (round_index, [client k global indices])"""
        k0 = 0
        for r, K in enumerate(self.meta["rounds"]):
            yield r, list(range(k0, k0 + K))
            k0 += K

    def args(self):
        a = dict(DEFAULT_ARGS)
        a["gradient_policy"] = self.meta.get("optimizer") if self.meta.get("optimizer") not in ("none",) else None
        if self.meta["policy"] == "q-fedavg":
            a["qfed_q"] = self.meta["q"]
            a["learning_rate"] = self.meta["lrs"][0]
        return argparse.Namespace(**a)

    def results(self, ks, r=0):
        losses = self.meta.get("losses")
        out = []
        for k in ks:
            out.append({"client_id": k + 1 if self.meta["policy"] != "fedbuff" else 101 + k,
                        "update_weight": self.client(k),
                        "moving_loss": float(losses[k]) if losses else 1.0,
                        "utility": 1.0, "trained_size": 20, "success": True, "wall_duration": 0.0})
        return out


def assert_state_equal(got, want, ctx=""):
    assert len(got) == len(want), ctx
    for i, (g, w) in enumerate(zip(got, want)):
        g = g.detach().cpu().numpy() if torch.is_tensor(g) else np.asarray(g)
        w = np.asarray(w)
        assert g.dtype == w.dtype, f"{ctx} tensor {i}: dtype {g.dtype} != {w.dtype}"
        assert g.shape == w.shape, f"{ctx} tensor {i}: shape {g.shape} != {w.shape}"
        if not np.array_equal(g, w):
            bad = np.argwhere(g != w)
            raise AssertionError(f"{ctx} tensor {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}: "
                                 f"got {g[tuple(bad[0])] if g.ndim else g} want {w[tuple(bad[0])] if w.ndim else w}")


class StateDictModule(torch.nn.Module):
    """Minimal nn.Module exposing a fixed, ordered state_dict (names may contain dots)."""

    def __init__(self, names, tensors):
        super().__init__()
        from collections import OrderedDict

        self._sd = OrderedDict((n, t.detach().clone()) for n, t in zip(names, tensors))

    def state_dict(self, *a, **k):
        return self._sd

    def load_state_dict(self, new, strict=True):
        for n, dst in self._sd.items():
            dst.copy_(new[n])


def assert_state_close(got, want, rtol, ctx="", int_slack=0):
    """Per-tensor: |got - want| <= rtol * max(|want|, rms(want)) elementwise; ints within int_slack."""
    for i, (g, w) in enumerate(zip(got, want)):
        g = g.detach().cpu().numpy() if torch.is_tensor(g) else np.asarray(g)
        w = np.asarray(w)
        assert g.dtype == w.dtype and g.shape == w.shape, f"{ctx} tensor {i}: {g.dtype}{g.shape} vs {w.dtype}{w.shape}"
        if w.size == 0:
            continue
        if np.issubdtype(w.dtype, np.integer):
            if int_slack:  # the bound of 1 holds while |v| * rtol < 1 (tests/test_numerics_notes.py)
                assert np.max(np.abs(w.astype(np.float64))) * max(rtol, 1e-5) < 1, f"{ctx} tensor {i}: int slack"
            assert np.max(np.abs(g.astype(np.int64) - w.astype(np.int64))) <= int_slack, f"{ctx} tensor {i}"
            continue
        wd = w.astype(np.float64)
        scale = np.maximum(np.abs(wd), np.sqrt(np.mean(wd * wd)))
        err = np.abs(g.astype(np.float64) - wd)
        bad = err > rtol * scale
        assert not bad.any(), f"{ctx} tensor {i}: {bad.sum()} elements beyond rtol={rtol}, max rel {np.max(err / np.maximum(scale, 1e-30)):.3g}"


class ClientScenario:
    """A client-side fixture (tests/golden/gen_golden_client.py): FedProx steps or one local-DP upload."""

    def __init__(self, name):
        self.name = name
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            self.meta = json.load(f)
        z = np.load(os.path.join(GOLDEN, name + ".npz"))
        self.arrays = {k: z[k] for k in z.files}

    def list(self, prefix, n):
        return [self.arrays[f"{prefix}/{i}"] for i in range(n)]


def c1_job_args():
    """Config 1's aggregator flags: benchmark/configs/femnist/conf.yml's job_conf as the reference launcher
    converts it (docker/driver.py:81-95) and config_parser.py parses it, num_participants overridden to 10
    (tests/golden/gen_golden_r3.py wrote them from the real reference)."""
    with open(os.path.join(GOLDEN, "c1_femnist_job_conf.json")) as f:
        doc = json.load(f)
    a = dict(DEFAULT_ARGS)
    a.update(doc["args"])
    return argparse.Namespace(**a), doc
