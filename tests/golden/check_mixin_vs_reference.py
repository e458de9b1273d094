"""Check the device mixins against the REAL reference aggregator classes (build container only; needs
/root/reference, with the off-path placeholders gen_golden.py installs).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/check_mixin_vs_reference.py

Run by tests/test_mixin_vs_reference.py in a child process (the placeholders never enter the test process).
For ``class A(DeviceAggregatorMixin, Aggregator)`` (fedscale/cloud/aggregation/aggregator.py) it checks that
* every method the mixin overrides exists on the reference class with the same parameter list (names,
  kinds, defaults), so the reference event loop's calls bind to the mixin unchanged;
* ``_reference_impl(name)`` is True for each of them: the next method in the MRO is the reference's own, so
  the mixin takes its device path (and a plugin that overrides one keeps its own);
* ``super()`` from the mixin reaches ``Aggregator.init_model`` (aggregator.py:198-211) and the MRO places
  the mixin first;
* tests/event_loop.py's restatement of the reference loop has the same parameter lists as the reference for
  every method it restates, and its class name makes ``_reference_impl`` behave as with the real class.
For ``class B(DeviceAsyncAggregatorMixin, AsyncAggregator)`` (async_aggregator.py) it checks that FedBuff's own
``create_client_task`` (:40) is recognised as a plugin override (``_reference_impl`` False), and the same
parameter-list checks; for Auxo (examples/auxo/aggregator.py:451-472) the cohort mixin's signatures.
Prints one JSON report; exit status 1 on any mismatch.
"""
from __future__ import annotations

import inspect
import json
import os
import sys

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)

import gen_golden as G  # noqa: E402

#: methods the aggregator mixin overrides (fedscale_amd/cloud/aggregation/aggregator.py)
MIXIN_OVERRIDES = ("init_model", "deserialize_response", "serialize_response", "create_client_task",
                   "get_test_config", "add_event_handler", "CLIENT_PING", "update_weight_aggregation",
                   "_is_first_result_in_round", "_is_last_result_in_round")
#: methods tests/event_loop.py restates from the reference (its control methods round_completion_handler /
#: event_monitor take test-harness arguments by design and are not compared)
EVENT_LOOP_RESTATED = ("get_client_conf", "create_client_task", "get_test_config", "serialize_response",
                       "deserialize_response", "add_event_handler", "CLIENT_PING", "CLIENT_EXECUTE_COMPLETION",
                       "client_completion_handler")


def params(fn):
    return [(p.name, p.kind.name, None if p.default is inspect.Parameter.empty else repr(p.default))
            for p in inspect.signature(fn).parameters.values()]


def compare(errors, what, mine, ref, allow_extra_defaults=False):
    a, b = params(mine), params(ref)
    if allow_extra_defaults:  # a default where the reference has none is a superset, not a mismatch
        a = [(n, k, d if rb[2] is not None else None) for (n, k, d), rb in zip(a, b)] if len(a) == len(b) else a
    if a != b:
        errors.append(f"{what}: {a} != reference {b}")


def main():
    _, Aggregator, AsyncAggregator, _, _ = G._import_reference()
    from fedscale_amd.cloud.aggregation import aggregator as M
    from tests import event_loop as EL

    errors, checked = [], []

    class A(M.DeviceAggregatorMixin, Aggregator):
        pass

    a = A.__new__(A)  # no reference __init__ (it opens gRPC and reads the job's data)
    assert A.__mro__[1] is M.DeviceAggregatorMixin and Aggregator in A.__mro__
    for name in MIXIN_OVERRIDES:
        ref = getattr(Aggregator, name, None)
        if ref is None:
            errors.append(f"Aggregator has no {name}")
            continue
        compare(errors, f"DeviceAggregatorMixin.{name}", getattr(M.DeviceAggregatorMixin, name), ref)
        if not a._reference_impl(name):
            errors.append(f"_reference_impl({name!r}) is False over the real Aggregator")
        checked.append(name)
    sup = super(M.DeviceAggregatorMixin, a).init_model
    if getattr(sup, "__qualname__", "") != "Aggregator.init_model":
        errors.append(f"super().init_model is {sup.__qualname__}, not Aggregator.init_model")

    for name in EVENT_LOOP_RESTATED:
        compare(errors, f"tests/event_loop.Aggregator.{name}", getattr(EL.Aggregator, name), getattr(Aggregator, name))

    class E(M.DeviceAggregatorMixin, EL.Aggregator):
        pass

    e = E.__new__(E)
    for name in MIXIN_OVERRIDES:
        if hasattr(EL.Aggregator, name) and not e._reference_impl(name):
            errors.append(f"_reference_impl({name!r}) is False over tests/event_loop.Aggregator")

    class B(M.DeviceAsyncAggregatorMixin, AsyncAggregator):
        pass

    b = B.__new__(B)
    if b._reference_impl("create_client_task"):
        errors.append("FedBuff's create_client_task (async_aggregator.py:40) was not seen as a plugin override")
    for name in ("deserialize_response", "serialize_response", "get_test_config", "CLIENT_PING"):
        if not b._reference_impl(name):
            errors.append(f"_reference_impl({name!r}) is False over AsyncAggregator")
    compare(errors, "DeviceAsyncAggregatorMixin.update_weight_aggregation",
            M.DeviceAsyncAggregatorMixin.update_weight_aggregation, AsyncAggregator.update_weight_aggregation)

    # Auxo per-cohort FedAvg (gen_golden.py installs the same placeholders for its off-path modules)
    import types as _t

    nl = _t.ModuleType("nltk")
    nlc = _t.ModuleType("nltk.cluster")
    nlc.KMeansClusterer, nlc.euclidean_distance = object, None
    nl.cluster = nlc
    cfg = _t.ModuleType("config")
    cfg.auxo_config = {}
    sys.modules.update({"nltk": nl, "nltk.cluster": nlc, "config": cfg})
    sys.path.insert(0, os.path.join(G.REF, "examples", "auxo"))
    from aggregator import AuxoAggregator  # examples/auxo/aggregator.py

    for name in ("update_weight_aggregation", "_is_first_result_in_round", "_is_last_result_in_round"):
        compare(errors, f"DeviceCohortAggregatorMixin.{name}", getattr(M.DeviceCohortAggregatorMixin, name),
                getattr(AuxoAggregator, name), allow_extra_defaults=True)

    report = {"ok": not errors, "overrides_checked": checked, "event_loop_checked": list(EVENT_LOOP_RESTATED),
              "errors": errors}
    print(json.dumps(report))
    return 0 if not errors else 1


if __name__ == "__main__":
    sys.exit(main())
