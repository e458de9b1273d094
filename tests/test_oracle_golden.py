"""The CPU oracle (oracle/cpu_reference.py) is bit-exact against every golden fixture that the real
reference produced (tests/golden/gen_golden.py). CPU only."""
import pytest

from oracle.cpu_reference import (OracleAggregator, OracleModel, OracleModelAdapter,
                                  OracleServerOptimizer)
from tests.golden_io import Scenario, assert_state_equal, scenario_names


@pytest.mark.parametrize("name", scenario_names())
def test_oracle_matches_reference_fixture(name):
    sc = Scenario(name)
    args = sc.args()
    model = OracleModel(sc.names, sc.init_state())
    policy = sc.meta["policy"]
    opt = None
    if sc.meta.get("optimizer") is not None:
        opt = OracleServerOptimizer(args.gradient_policy, args, None)
    adapter = OracleModelAdapter(model, optimizer=opt)
    agg = OracleAggregator(adapter, args, asynchronous=(policy == "fedbuff"))
    if policy == "fedbuff":
        agg.round = sc.meta["round"]
        for k, s in enumerate(sc.meta["staleness"]):
            agg.client_task_model_version[101 + k] = agg.round - s
    for r, ks in sc.rounds():
        if policy == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        assert_state_equal(adapter.get_weights(), sc.expected(r), f"{name} round {r}")
        if policy == "fed-yogi":
            m, v = sc.yogi_state(r)
            assert_state_equal(opt.gradient_controller.m_t, m, f"{name} m round {r}")
            assert_state_equal(opt.gradient_controller.v_t, v, f"{name} v round {r}")


@pytest.mark.parametrize("name", scenario_names("cohorts"))
def test_oracle_matches_auxo_cohort_fixture(name):
    from oracle.cpu_reference import OracleCohortAggregator

    sc = Scenario(name)
    wrappers = [OracleModelAdapter(OracleModel(sc.names, sc.init_state(c))) for c in range(len(sc.meta["cohort_K"]))]
    agg = OracleCohortAggregator(wrappers, sc.meta["cohort_K"])
    for k, c in enumerate(sc.meta["cohorts"]):
        agg.on_result({"client_id": k + 1, "update_weight": sc.client(k), "moving_loss": 1.0}, c)
    for c, w in enumerate(wrappers):
        assert_state_equal(w.get_weights(), sc.expected_cohort(c), f"{name} cohort {c}")


@pytest.mark.parametrize("name", scenario_names("heterofl"))
def test_oracle_matches_heterofl_fixture(name):
    from collections import OrderedDict

    from oracle.cpu_reference import heterofl_combine

    sc = Scenario(name)
    sd = OrderedDict(zip(sc.names, sc.init_state()))
    heterofl_combine(sd, sc.hetero_locals())
    assert_state_equal(list(sd.values()), sc.expected(0), name)


# ---- client-side handlers: oracle vs the real reference's outputs ----------------
from collections import OrderedDict  # noqa: E402

import numpy as np  # noqa: E402

from tests.golden_io import ClientScenario  # noqa: E402


@pytest.mark.parametrize("name", [n for n in scenario_names("client") if "_prox_" in n])
def test_oracle_fedprox_matches_reference(name):
    from oracle.cpu_reference import fedprox_update

    sc = ClientScenario(name)
    T = len(sc.meta["shapes"])
    glob = sc.list("global", T)
    for s in range(sc.meta["steps"]):
        got = fedprox_update(sc.list(f"in/{s}", T), glob, sc.meta["lr"], sc.meta["mu"])
        for g, w in zip(got, sc.list(f"out/{s}", T)):
            assert g.dtype == w.dtype and np.array_equal(g, w)


@pytest.mark.parametrize("name", [n for n in scenario_names("client") if "_dp_" in n])
def test_oracle_local_dp_matches_reference(name):
    from oracle.cpu_reference import dp_privatize

    sc = ClientScenario(name)
    m = sc.meta
    names, T = m["names"], len(m["names"])
    state = OrderedDict(zip(names, sc.list("in", T)))
    last = sc.list("last", sum(m["is_param"]))
    noise = dict(zip(names, sc.list("noise", T))) if m["noise_factor"] else None
    rec, up, total = dp_privatize(state, m["is_param"], last, m["clip"], m["noise_factor"], noise,
                                  norm_type=m["norm_type"])
    assert np.float32(total) == np.float32(m["total_norm"])
    for j, n in enumerate(names):
        for got, want in ((rec[n], sc.arrays[f"recovered/{j}"]), (up[n], sc.arrays[f"upload/{j}"])):
            assert got.dtype == want.dtype and got.shape == want.shape, n
            assert np.array_equal(got, want), n
