"""bench.py's host side without a GPU: the config table is BASELINE.json's, the defaults keep the driver's
contract (N = 1, a K/W that finishes in minutes), and the CPU legs (the oracle on this host) produce the
fields the JSON line reports, for every policy."""
import json
import os
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_configs_are_baselines():
    cfgs = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"]
    assert len(cfgs) == 5
    want = {  # configs[1..4]: K x P (policy) as BASELINE.json names them; configs[0] is the C1 host round
        "c2": (100, 1_000_000, "fedavg"), "c3": (1000, 11_191_242, "fedavg"),
        "c4": (1000, 25_000_000, "fedyogi"), "c5": (10_000, 100_000_000, "qfedavg")}
    for name, (K, P, pol) in want.items():
        c = bench.CONFIGS[name]
        assert (c["clients"], c["params"], c["policy"]) == (K, P, pol), name
    assert "100 clients" in cfgs[1] and "1M" in cfgs[1]
    assert "FedYoGi" in cfgs[3] and "25M" in cfgs[3] and "q-FedAvg" in cfgs[4] and "100M" in cfgs[4]
    h = bench.CONFIGS["headline"]
    assert (h["clients"], h["params"], h["policy"]) == (1000, 25_000_000, "fedavg")  # the north star's target


def test_default_arguments(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0 and a.steps * 15e-3 < 60
    assert a.cfg == bench.CONFIGS["headline"] and a.scaling == "strong" and a.dist_backend == "nccl"
    monkeypatch.setattr(sys, "argv", ["bench.py", "--config", "c5", "--params", "1000"])
    a = bench.parse()
    assert a.cfg["policy"] == "qfedavg" and a.cfg["params"] == 1000 and a.cfg["clients"] == 10_000


@pytest.mark.parametrize("policy", ["fedavg", "fedyogi", "qfedavg"])
def test_cpu_leg_fields(policy):
    leg = bench.cpu_leg(policy, K=40, P=20_000, budget_s=0.2, seed=1, pool_n=4)
    assert leg["kind"] == "port" and leg["policy"] == policy and leg["pool_buffers"] == 4
    assert 0 < leg["accumulate_clients_timed"] <= 40 and leg["accumulate_ms_per_client"] > 0
    assert leg["finalize_ms"] > 0 and leg["round_s"] > 0
    assert leg["client_updates_per_s"] == pytest.approx(40 / leg["round_s"])
    assert leg["cores"] >= 1
    if policy == "qfedavg":
        assert leg["finalize_ms_per_retained_client"] > 0


def test_cpu_baseline_c1_times_arithmetic_and_reference_loop():
    r = bench.cpu_baseline_c1(seed=0, rounds=3)
    assert r["kind"] == "port" and r["cores"] == 1
    assert 0 < r["round_ms"] < r["handler_round_ms"]  # the whole loop costs more than its arithmetic
