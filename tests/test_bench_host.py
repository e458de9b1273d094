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
    assert a.gpus == 1 and a.steps > 0 and a.steps * 15e-3 < 60
    assert a.warmup == -1 and bench.WARMUP_S <= 2.0  # auto: >= 3 rounds and ~1 s of them, a bounded prefix
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


def test_pmc_traffic_belongs_to_its_run(tmp_path):
    """roofline.traffic is looked up by (workload, resident clients, launches per round, build id): any mismatch
    gives None (a stale entry must never be attached to a changed kernel or shape)."""
    import json

    f = tmp_path / "pmc.json"
    key = "fedavg_k1000_p25000000_per_gpu|C1000|L4|0123456789abcdef"
    f.write_text(json.dumps({"entries": {key: {"hbm_bytes_per_launch": 25.0e9}},
                             "history_pre_r05": {"fedavg_k1000_p25000000": {"hbm_bytes_per_launch": 1.0}}}))
    w = "fedavg_k1000_p25000000_per_gpu"
    assert bench.pmc_traffic(w, 1000, 4, "0123456789abcdef", str(f)) == 25.0e9
    assert bench.pmc_traffic(w, 1000, 4, "fedcba9876543210", str(f)) is None  # another library
    assert bench.pmc_traffic(w, 2048, 4, "0123456789abcdef", str(f)) is None  # another chunking
    assert bench.pmc_traffic(w, 1000, 2, "0123456789abcdef", str(f)) is None  # another launch plan
    assert bench.pmc_traffic("fedavg_k1000_p25000000", 1000, 4, "0123456789abcdef", str(f)) is None
    assert bench.pmc_traffic(w, 1000, 4, "0123456789abcdef", str(tmp_path / "missing.json")) is None


def test_committed_profiles_carry_their_own_traffic():
    """Every committed *_under_rocprof.json either has traffic null, or names the PMC CSVs it came from and its
    traffic is within 0.1 % of what those CSVs give (tools/pmc_parse.py's correction), or (a plain bench line run
    under the profiler) carries exactly the keyed pmc_traffic.json entry of its own workload, resident clients,
    launches per round and build id."""
    import glob
    import json

    sys.path.insert(0, os.path.join(bench.ROOT, "tools"))
    import pmc_parse

    n = 0
    for p in glob.glob(os.path.join(bench.ROOT, "profiles", "*under_rocprof*.json")):
        line = json.loads([ln for ln in open(p).read().splitlines() if ln.startswith("{")][-1])
        r = line["roofline"]
        if r.get("traffic") is None:
            continue
        if "traffic_source" not in r:
            assert r["traffic"] == bench.pmc_traffic(line["config"]["workload"], r["resident_clients"],
                                                     r["launches_per_step"], line["build_id"]), p
            continue
        src = r["traffic_source"]
        hbm = pmc_parse.traffic_per_launch(os.path.join(bench.ROOT, src["fetch"]), os.path.join(bench.ROOT, src["write"]),
                                           src["kernel"], int(r["launches_per_step"]))[0]
        assert abs(hbm / r["traffic"] - 1) < 1e-3, p
        n += 1
    assert n >= 6


def test_promote_inproc_value():
    """N > 1: value = the in-process drop-in's round; the SPMD figure stays as value_spmd; a failed in-process run
    leaves the SPMD value and says why."""
    res = {"value": 500000.0, "ms_per_step": 2.0, "scaling_vs_one_gpu": 7.0, "config": {"parallelism": "x"},
           "roofline": {"achieved": 7000.0, "frac": 0.875}, "hbm_gbps": 7000.0, "kernel_ms": 1.8}
    inproc = {"ok": True, "policies": {"fedavg": {"ok": True, "inproc_round_ms": 2.5, "speedup_vs_one_gpu": 5.6,
                                                  "devices": [0, 1, 2, 3, 4, 5, 6, 7], "transport": "rccl",
                                                  "rounds": 20, "part_kernel_ms": [1.8] * 7 + [2.0],
                                                  "part_alg_bytes": [12.5e9] * 8, "part_launches": [1] * 8}}}
    bench.promote_inproc(res, inproc, 1000, 20)
    assert res["value"] == 1000 / 2.5e-3 and res["ms_per_step"] == 2.5
    assert res["value_spmd"] == 500000.0 and res["ms_per_step_spmd"] == 2.0
    assert res["scaling_vs_one_gpu"] == 5.6 and res["scaling_vs_one_gpu_spmd"] == 7.0
    assert "ONE aggregator process" in res["config"]["parallelism"]
    assert res["roofline"]["achieved"] == 12.5e9 / 2.0e-3 / 1e9 and res["roofline_spmd"]["achieved"] == 7000.0
    assert res["kernel_ms"] == 2.0 and res["roofline"]["traffic"] is None
    res2 = {"value": 1.0, "ms_per_step": 2.0, "config": {"parallelism": "x"}}
    bench.promote_inproc(res2, {"ok": False, "policies": {"fedavg": {"ok": False, "error": "boom"}}}, 1000, 20)
    assert res2["value"] == 1.0 and "boom" in res2["value_source"] and "value_spmd" not in res2
    # parts sharing one card (a gloo rehearsal) are plumbing: the SPMD value stays
    res3 = {"value": 1.0, "ms_per_step": 2.0, "config": {"parallelism": "x"}}
    shared = {"ok": True, "inproc_round_ms": 2.5, "devices": [0, 0], "distinct_gpus": False, "transport": "copy"}
    bench.promote_inproc(res3, shared, 1000, 20)
    assert res3["value"] == 1.0 and "plumbing" in res3["value_source"] and "value_spmd" not in res3


def _line(n_gpus, with_cpu=True, with_pcie=True):
    res = {"metric": bench.CONFIGS and "m", "value": 1.0, "unit": "client-updates/s", "n_gpus": n_gpus, "steps": 5,
           "warmup": 2, "ms_per_step": 1.0, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "f32", "data": "synthetic", "config": {"workload": "w"},
           "roofline": {"bound": "hbm", "achieved": 1.0, "peak": 8000.0, "unit": "GB/s", "frac": 1 / 8000, "traffic": None},
           "cpu_baseline": ({"value": 80.0, "unit": "client-updates/s", "cores": 1, "kind": "port", "sample": "s"}
                            if with_cpu else None)}
    if with_pcie:
        res["pcie_inclusive"] = {"ok": True, "round_ms": 100.0, "client_updates_per_s": 640.0,
                                 "host_to_device_GBps": 64.0, "phases_ms": {}, "prediction": bench.pcie_prediction(n_gpus),
                                 "parts": [{"device": i, "params": 1, "host_numa_node": 0, "h2d_GBps_over_ingress": 8.0}
                                           for i in range(n_gpus)]}
    return res


@pytest.mark.parametrize("n", [2, 8])
def test_n_gt_1_line_must_carry_cpu_baseline_and_pcie_inclusive(n):
    """an N > 1 line without the CPU baseline or the PCIe-inclusive N-link round is incomplete (the
    north star wants both beside the 1/2/4/8-GPU figures)."""
    assert bench.check_line(_line(n)) == []
    assert "cpu_baseline (null)" in bench.check_line(_line(n, with_cpu=False))
    assert "pcie_inclusive" in bench.check_line(_line(n, with_pcie=False))
    bad = _line(n)
    bad["pcie_inclusive"]["parts"] = bad["pcie_inclusive"]["parts"][:-1]
    del bad["pcie_inclusive"]["parts"][0]["host_numa_node"]
    miss = bench.check_line(bad)
    assert any("parts (" in m for m in miss) and "pcie_inclusive.parts[0].host_numa_node" in miss
    failed = _line(n)
    failed["pcie_inclusive"] = {"ok": False, "error": "boom"}
    assert any("boom" in m for m in bench.check_line(failed))


def test_n1_line_schema():
    assert bench.check_line(_line(1, with_pcie=False)) == []
    off = _line(1, with_cpu=False, with_pcie=False)
    assert bench.check_line(off) == ["cpu_baseline (null)"]
    off["cpu_legs_off"] = True
    assert bench.check_line(off) == []
    broken = _line(1)
    del broken["roofline"]["traffic"]
    assert bench.check_line(broken) == ["roofline.traffic"]


def test_pcie_prediction_scales_with_links():
    p1, p8 = bench.pcie_prediction(1), bench.pcie_prediction(8)
    assert p8["host_to_device_GBps"] == 8 * p1["host_to_device_GBps"] == 8 * bench.PCIE_LINK_GBPS


def test_committed_rehearsal_lines_are_complete():
    """The N > 1 rehearsal lines committed this round (bench.py --gpus 2 / 8 under gloo on one card) carry every
    north-star quantity (labelled as plumbing)."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06_bench_gloo_rehearsal_*.json")))
    for p in paths:
        line = json.loads([ln for ln in open(p).read().splitlines() if ln.startswith("{")][-1])
        assert line["n_gpus"] > 1 and bench.check_line(line) == [], (p, bench.check_line(line))
        assert line["schema"]["complete"] and "plumbing" in json.dumps(line["pcie_inclusive"])
        if "plumbing_only" in line:  # (lines from round 6's last bench.py carry the machine-readable flag)
            assert "plumbing" in line["plumbing_only"] and "spmd" in line["value_source"]
