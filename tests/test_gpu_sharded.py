"""Multi-GPU behind the reference's single-process aggregator (``ShardedModelAdapter``).

The box these run on has one MI355X, so the model is sharded over ``[cuda:0, cuda:0]`` (two parts on one
card, device-to-device transport) and over ``[cuda:0]`` with the RCCL transport (a one-GPU communicator:
the collectives run through RCCL).  The per-element chains are the single-GPU ones, so FedAvg / FedBuff
are bit-exact against the reference's fixtures; FedYoGi and q-FedAvg keep the single-GPU tolerances
(see test_gpu_parity.py)."""
import pickle
import threading
import time

import numpy as np
import pytest
import torch

from tests.golden_io import Scenario, StateDictModule, assert_state_close, assert_state_equal, scenario_names

pytestmark = pytest.mark.gpu

QFED_RTOL = 1e-5
YOGI_RTOL = 1e-6
SHARDINGS = {"two_parts_one_gpu": ([0, 0], "copy"), "rccl_one_gpu": ([0], "rccl")}


def _sharded(sc, devices, transport, capacity=None):
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter

    args = sc.args()
    model = StateDictModule(sc.names, sc.init_state())
    opt = TorchServerOptimizer(args.gradient_policy, args, "cuda:0") if sc.meta.get("optimizer") is not None else None
    return args, opt, ShardedModelAdapter(model, optimizer=opt, devices=devices, staging_capacity=capacity,
                                          transport=transport)


def _yogi_state(adapter):
    """The sharded YoGi m/v reassembled into the reference's per-tensor lists (yogi.py:11-19)."""
    L = adapter.layout
    m = torch.zeros(L.ld)
    v = torch.zeros(L.ld)
    for p in adapter.parts:
        y = p.optimizer.gradient_controller
        m[p.layout.p0:p.layout.p1] = y.m[:p.layout.P].cpu()
        v[p.layout.p0:p.layout.p1] = y.v[:p.layout.P].cpu()
    y0 = adapter.parts[0].optimizer.gradient_controller
    return L.unpack(m, y0.ms.cpu()), L.unpack(v, y0.vs.cpu())


def _check(sc, r, got, adapter, ctx):
    pol = sc.meta["policy"]
    if pol == "q-fedavg":
        assert_state_close(got, sc.expected(r), QFED_RTOL, ctx, int_slack=1)
    elif pol == "fed-yogi":
        assert_state_close(got, sc.expected(r), YOGI_RTOL, ctx)
        m, v = _yogi_state(adapter)
        (assert_state_equal if r == 0 else lambda g, w, c: assert_state_close(g, w, YOGI_RTOL, c))(m, sc.yogi_state(r)[0], ctx + " m")
        (assert_state_equal if r == 0 else lambda g, w, c: assert_state_close(g, w, YOGI_RTOL, c))(v, sc.yogi_state(r)[1], ctx + " v")
    else:
        assert_state_equal(got, sc.expected(r), ctx)


@pytest.mark.parametrize("capacity", [None, 2])
@pytest.mark.parametrize("sharding", list(SHARDINGS))
@pytest.mark.parametrize("name", scenario_names())
def test_sharded_adapter_matches_reference_fixture(gpu_device, name, sharding, capacity):
    """Every fixture through DeviceAggregator over a ShardedModelAdapter."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator

    sc = Scenario(name)
    devices, transport = SHARDINGS[sharding]
    args, opt, adapter = _sharded(sc, devices, transport, capacity)
    assert adapter.group.transport == transport
    if sc.meta["policy"] == "fedbuff":
        agg = DeviceAsyncAggregator(adapter, args)
        agg.round = sc.meta["round"]
        for k, s in enumerate(sc.meta["staleness"]):
            agg.client_task_model_version[101 + k] = agg.round - s
    else:
        agg = DeviceAggregator(adapter, args)
    for r, ks in sc.rounds():
        if sc.meta["policy"] == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        _check(sc, r, adapter.get_weights(), adapter, f"{name} {sharding} r{r} cap={capacity}")
    adapter.group.close()


@pytest.mark.parametrize("name", ["fedavg_wide_k64", "fedyogi_wide_3rounds", "qfedavg_q1_lrdecay"])
def test_sharded_equals_single_gpu(gpu_device, name):
    """Two parts vs one GPU on the same inputs: FedAvg and fused FedYoGi bit-identical (same chains), the
    FedAvg mean (model_weights) bit-identical, q-FedAvg within the fp64 norm re-association."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    sc = Scenario(name)
    args, _, sharded = _sharded(sc, [0, 0], "copy")
    opt1 = TorchServerOptimizer(args.gradient_policy, args, "cuda:0") if sc.meta.get("optimizer") is not None else None
    single = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()), optimizer=opt1, device="cuda:0")
    aggs = [DeviceAggregator(sharded, args), DeviceAggregator(single, args)]
    for r, ks in sc.rounds():
        if sc.meta["policy"] == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        for agg in aggs:
            agg.start_round(len(ks))
            for res in sc.results(ks, r):
                agg.on_result(res)
        a, b = sharded.get_weights(), single.get_weights()
        if sc.meta["policy"] == "q-fedavg":
            assert_state_close(a, [t.numpy() for t in b], 1e-6, f"{name} r{r}", int_slack=1)
        else:
            assert_state_equal(a, [t.numpy() for t in b], f"{name} r{r}")
        assert_state_equal(list(aggs[0].model_weights), list(aggs[1].model_weights), f"{name} mean r{r}")


#: entry points that enqueue GPU work (their last argument is the stream, or the per-device stream table)
LAUNCHES = {"fa_reduce", "fa_reduce_mirror", "fa_reduce_yogi", "fa_yogi_step", "fa_qfed_accumulate", "fa_qfed_hs", "fa_qfed_finalize",
            "fa_sum_rows_f64", "fa_side_accumulate", "fa_side_close", "fa_side_yogi", "fa_side_qfed_accumulate",
            "fa_side_qfed_finalize", "fa_fill_synthetic", "fa_prefix_box_combine", "fa_rccl_all_gather",
            "fa_rccl_all_reduce", "fa_rccl_gather", "fa_rccl_broadcast", "fa_reduce_parts", "fa_yogi_step_parts"}
#: ... of them, those that take a per-part stream table (one stream per position of the adapter's group)
TABLE_LAUNCHES = {"fa_rccl_all_gather", "fa_rccl_all_reduce", "fa_rccl_gather", "fa_rccl_broadcast", "fa_reduce_parts",
                  "fa_yogi_step_parts"}


def _spy_native(monkeypatch):
    """Record (entry point, stream argument, innermost DeviceStream) of every native call."""
    from fedscale_amd import _native
    from fedscale_amd import kernels as kx
    from fedscale_amd.state import DeviceStream

    calls, real = [], _native.call

    def spy(fn, *args):
        calls.append((fn, args[-1] if args else None, DeviceStream.current()))
        return real(fn, *args)

    monkeypatch.setattr(_native, "call", spy)
    monkeypatch.setattr(kx, "call", spy)
    return calls


def _check_part_streams(calls, adapter, ctx):
    streams = {ds.handle: ds for ds in adapter.group.streams} if hasattr(adapter, "group") else {
        adapter.dstream.handle: adapter.dstream}
    launches = [c for c in calls if c[0] in LAUNCHES]
    assert launches, ctx
    for fn, st, cur in launches:
        if fn in TABLE_LAUNCHES:
            hs = list(st)
            assert hs == adapter.group.stream_handles() and all(hs), f"{ctx}: {fn} stream table {hs}"
            continue
        assert st, f"{ctx}: {fn} launched on the null stream"
        assert cur is not None, f"{ctx}: {fn} issued outside any part's DeviceStream"
        assert st == cur.handle, f"{ctx}: {fn} on stream {st:#x}, its part's stream is {cur.handle:#x}"
        assert st in streams and streams[st] is cur, f"{ctx}: {fn} on a stream no part of this adapter owns"
    return launches


@pytest.mark.parametrize("sharding", list(SHARDINGS))
@pytest.mark.parametrize("name", ["fedavg_wide_k64", "fedbuff_k8", "fedyogi_wide_3rounds", "qfedavg_q1_lrdecay"])
def test_every_native_call_runs_on_its_parts_stream(gpu_device, monkeypatch, name, sharding):
    """Every kernel launch and collective of a sharded round carries the non-null stream of the part whose
    buffers it touches (its own GPU's stream; the null stream would resolve against whatever device the
    calling thread has current), with chunk folds (capacity 2), every server step and egress; the results
    stay bit-exact / within tolerance of the reference fixtures."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator

    sc = Scenario(name)
    devices, transport = SHARDINGS[sharding]
    args, opt, adapter = _sharded(sc, devices, transport, capacity=2)
    calls = _spy_native(monkeypatch)
    if sc.meta["policy"] == "fedbuff":
        agg = DeviceAsyncAggregator(adapter, args)
        agg.round = sc.meta["round"]
        for k, s in enumerate(sc.meta["staleness"]):
            agg.client_task_model_version[101 + k] = agg.round - s
    else:
        agg = DeviceAggregator(adapter, args)
    for r, ks in sc.rounds():
        if sc.meta["policy"] == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        _check(sc, r, adapter.get_weights(), adapter, f"{name} {sharding} r{r}")
        list(agg.model_weights)  # the FedAvg mean's D2H runs on the parts' streams too
    launches = _check_part_streams(calls, adapter, f"{name} {sharding}")
    used = {c[1] for c in launches if c[0] not in TABLE_LAUNCHES}
    used |= {h for c in launches if c[0] in ("fa_reduce_parts", "fa_yogi_step_parts") for h in c[1]}
    assert used == set(adapter.group.stream_handles()), "every part launched on its own stream"
    if sc.meta["policy"] == "q-fedavg":
        assert any(c[0] in ("fa_rccl_all_gather", "fa_sum_rows_f64") for c in launches)
    adapter.group.close()


def test_single_adapter_runs_on_its_own_stream(gpu_device, monkeypatch):
    """The single-GPU adapter too: every launch on its DeviceStream (never the null stream), and the caller's
    stream is ordered after each call (a device buffer read right after a round on the default stream sees
    the round's result)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    sc = Scenario("fedyogi_wide_3rounds")
    args = sc.args()
    single = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()),
                               optimizer=TorchServerOptimizer(args.gradient_policy, args, "cuda:0"), device="cuda:0",
                               staging_capacity=3)
    calls = _spy_native(monkeypatch)
    agg = DeviceAggregator(single, args)
    for r, ks in sc.rounds():
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        cur = single._f[single._cur][:single.layout.P].cpu()  # default stream, no explicit sync
        got = single.get_weights()  # synchronises with the round's event
        flat = torch.cat([w.reshape(-1) for w, e in zip(got, single.layout.entries) if e.kind == "f"])
        assert torch.equal(cur, flat), f"round {r}: the caller's stream was not ordered after the round"
        assert_state_close(got, sc.expected(r), YOGI_RTOL, f"round {r}")
    launches = [c for c in calls if c[0] in LAUNCHES]
    assert launches and all(c[1] == single.dstream.handle and c[2] is single.dstream for c in launches)


def _executor_payload(res):
    return pickle.dumps(res)


@pytest.mark.parametrize("name", ["fedavg_femnist_cnn_k10", "fedyogi_mixed_3rounds", "qfedavg_q1_lrdecay",
                                  "fedavg_wide_k64"])
def test_reference_event_loop_drives_the_sharded_model(gpu_device, name):
    """The mixin over the reference's event-loop shape (tests/event_loop.py): 4 executor threads upload
    through CLIENT_EXECUTE_COMPLETION (servicer side, aggregator.py:919-963) and keep pinging
    (CLIENT_PING, :870-917: create_client_task, get_test_config, UPDATE_MODEL); the main thread reduces
    in queue order (event_monitor, :965-1007).  The model is sharded 2 ways.  The result equals the oracle
    run in the realised arrival order; every payload an executor received unpickles to exactly one model
    version; nothing deadlocks (every wait has a deadline)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin
    from oracle.cpu_reference import (OracleAggregator, OracleModel, OracleModelAdapter,
                                      OracleServerOptimizer)
    from tests import event_loop as EL

    sc = Scenario(name)
    args, opt, adapter = _sharded(sc, [0, 0], "copy")
    rounds = [len(ks) for _, ks in sc.rounds()]
    pol = sc.meta["policy"]
    if pol == "q-fedavg":
        args.learning_rate = sc.meta["lrs"][0]

    class A(DeviceAggregatorMixin, EL.Aggregator):
        pass

    agg = A(adapter, args, rounds)
    executors = [1, 2, 3, 4]
    versions = [adapter.get_weights()]  # version 0, then one per round (round_done)
    payloads = []
    errors = []
    stop = threading.Event()
    results = {k: res for r, ks in sc.rounds() for k, res in zip(ks, sc.results(ks, r))}
    order = sorted(results)
    lock = threading.Lock()
    upload_next = [0]

    def executor(e):
        try:
            i = 0
            while not stop.is_set():
                with lock:  # executors upload the clients of the CURRENT round only (as in FedScale)
                    k = None
                    if upload_next[0] < len(order):
                        cand = order[upload_next[0]]
                        r_of = next(r for r, ks in sc.rounds() if cand in ks)
                        if r_of == agg.round:
                            k = cand
                            upload_next[0] += 1
                if k is not None:
                    req = EL.request(e, client_id=k, event=EL.UPLOAD_MODEL, data=_executor_payload(results[k]))
                    ev, meta, data = agg.CLIENT_EXECUTE_COMPLETION(req, None)
                else:
                    if i % 3 == 0:
                        agg.individual_client_events[e].append(EL.CLIENT_TRAIN if i % 2 else EL.MODEL_TEST)
                    ev, meta, data = agg.CLIENT_PING(EL.request(e, client_id=k or 0), None)
                if ev in (EL.UPDATE_MODEL, EL.CLIENT_TRAIN, EL.MODEL_TEST):
                    payloads.append(data)
                i += 1
                time.sleep(0.0002)
        except Exception as ex:  # surfaced by the main thread
            errors.append(ex)

    def on_round(r):
        if pol == "q-fedavg" and r + 1 < len(sc.meta["lrs"]):
            args.learning_rate = sc.meta["lrs"][r + 1]

    threads = [threading.Thread(target=executor, args=(e,), daemon=True) for e in executors]
    for t in threads:
        t.start()
    try:
        agg.event_monitor(executors, deadline_s=60, on_round=on_round)
        for e in executors:
            agg.individual_client_events[e].append(EL.UPDATE_MODEL)
        time.sleep(0.05)
    finally:
        stop.set()
        for t in threads:
            t.join(timeout=30)
    assert not any(t.is_alive() for t in threads), "an executor thread is stuck"
    assert not errors, errors
    versions += agg.round_done

    # the oracle, fed in the order the main loop reduced
    oargs = sc.args()
    if pol == "q-fedavg":
        oargs.learning_rate = sc.meta["lrs"][0]
    oracle = OracleAggregator(OracleModelAdapter(OracleModel(sc.names, sc.init_state()),
                                                 OracleServerOptimizer(oargs.gradient_policy, oargs)), oargs)
    idx = {res["client_id"]: k for k, res in results.items()}
    done = 0
    for r, K in enumerate(rounds):
        if pol == "q-fedavg":
            oargs.learning_rate = sc.meta["lrs"][r]
        oracle.start_round(K)
        for cid in agg.processed[done:done + K]:
            oracle.on_result(results[idx[cid]])
        done += K
        want = oracle.model_wrapper.get_weights()
        got = versions[r + 1]
        if pol == "q-fedavg":
            assert_state_close(got, [t.numpy() for t in want], QFED_RTOL, f"{name} r{r}", int_slack=1)
        elif pol == "fed-yogi":
            assert_state_close(got, [t.numpy() for t in want], YOGI_RTOL, f"{name} r{r}")
            oracle.model_wrapper.model.load_state_dict(dict(zip(sc.names, got)))  # same trajectory
        else:
            assert_state_equal(got, [t.numpy() for t in want], f"{name} r{r}")

    # every egress payload is exactly one model version
    assert payloads, "no egress happened while the rounds ran"
    for data in payloads:
        w = pickle.loads(data)
        assert isinstance(w, list)
        assert any(all(torch.equal(a, b) for a, b in zip(w, v)) for v in versions), "a payload mixes versions"
    adapter.group.close()


def test_egress_is_consistent_under_concurrent_rounds(gpu_device):
    """8 threads call create_client_task / get_test_config / serialize_response of
    get_weights() (the servicer's paths, aggregator.py:788-816, 902-909) while the main thread completes
    20 rounds; every payload must unpickle to exactly one committed model version (single GPU and sharded)."""
    from fedscale_amd import synth
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from tests import event_loop as EL

    names, shapes = ["w", "b", "n"], [(1024, 1031), (77,), ()]
    dtypes = [torch.float32, torch.float32, torch.int64]
    for make in (lambda m: TorchModelAdapter(m, device="cuda:0"),
                 lambda m: ShardedModelAdapter(m, devices=[0, 0], transport="copy")):
        adapter = make(synth.LayoutModule(names, shapes, dtypes))

        class A(DeviceAggregator):
            resource_manager = EL._Resources()

            def get_client_conf(self, cid):
                return {}

        agg = A(adapter)
        rng = np.random.default_rng(0)
        versions = {0: adapter.get_weights()}
        payloads = []
        stop = threading.Event()
        errors = []

        def servicer(i):
            try:
                while not stop.is_set():
                    j = len(payloads) % 3
                    if j == 0:
                        _, w = agg.create_client_task(i)
                    elif j == 1:
                        _, w = agg.get_test_config(i)
                    else:
                        w = adapter.get_weights()
                    payloads.append(agg.serialize_response(w))
            except Exception as ex:
                errors.append(ex)

        threads = [threading.Thread(target=servicer, args=(i,), daemon=True) for i in range(8)]
        for t in threads:
            t.start()
        try:
            for r in range(20):
                agg.start_round(3)
                for k in range(3):
                    up = {"w": rng.standard_normal(shapes[0], dtype=np.float32),
                          "b": rng.standard_normal(shapes[1], dtype=np.float32), "n": np.array(r * 3 + k)}
                    agg.on_result({"client_id": k, "update_weight": up, "moving_loss": 1.0})
                versions[r + 1] = adapter.get_weights()
        finally:
            stop.set()
            for t in threads:
                t.join(timeout=30)
        assert not any(t.is_alive() for t in threads) and not errors, errors
        assert len(payloads) > 20
        for data in payloads:
            w = pickle.loads(data)
            assert sum(all(torch.equal(a, b) for a, b in zip(w, v)) for v in versions.values()) >= 1
        if hasattr(adapter, "group"):
            adapter.group.close()


def test_rccl_collectives_one_gpu(gpu_device):
    """fa_rccl_* with a one-GPU communicator: all-gather, all-reduce, gather and broadcast run through
    RCCL (ncclCommInitAll + grouped calls) and give the identities a world of one implies; the fixed-order
    f64 row sum combines per-shard partials."""
    from fedscale_amd import kernels as kx
    from fedscale_amd.state import DeviceGroup

    g = DeviceGroup([0], transport="rccl")
    x = torch.randn(1000, dtype=torch.float64, device="cuda:0")
    out = torch.empty(1000, dtype=torch.float64, device="cuda:0")
    g.all_gather([x], [out])
    assert torch.equal(out, x)
    y = torch.randn(333, device="cuda:0")
    root = torch.empty(333, device="cuda:0")
    g.gather([y], root)
    assert torch.equal(root, y)
    b = [y.clone()]
    g.broadcast(b)
    assert torch.equal(b[0], y)
    s = x.clone()
    g.sum_f64([s])
    assert torch.equal(s, x)
    rows = torch.randn(5, 77, dtype=torch.float64, device="cuda:0")
    o = torch.empty(77, dtype=torch.float64, device="cuda:0")
    kx.sum_rows_f64(rows, o)
    want = rows[0].clone()
    for i in range(1, 5):
        want = want + rows[i]
    assert torch.equal(o, want)
    info = g.rccl_info()  # what RCCL itself reports (fa_rccl_comm_info)
    assert info == {"transport": "rccl", "count": 1, "ranks": [0], "devices": [0], "devices_requested": [0]}
    g.close()
    assert DeviceGroup([0, 0], transport="copy").rccl_info()["count"] is None


def test_rccl_communicator_left_open_at_exit(gpu_device):
    """A ShardedModelAdapter that is never closed (the aggregator process simply exits): its RCCL
    communicator is destroyed by the exit hook while the HIP runtime is still up, and the process exits 0."""
    import os
    import subprocess
    import sys

    code = (
        "import torch\n"
        "from fedscale_amd.state import DeviceGroup\n"
        "g = DeviceGroup([0], transport='rccl')\n"
        "x = torch.ones(64, dtype=torch.float64, device='cuda:0')\n"
        "g.sum_f64([x])\n"
        "torch.cuda.synchronize()\n"
        "assert float(x.sum()) == 64.0\n"
        "print('ok', flush=True)\n"
    )
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])


def test_nccl_process_group_collectives_world1(gpu_device):
    """The torch.distributed (RCCL) branch of ShardGroup with device tensors, at world size 1 on the box:
    all_gather_into_tensor and all_reduce run through the nccl backend (the N-GPU SPMD bench uses them)."""
    import os

    import torch.distributed as dist

    from fedscale_amd.state import ShardGroup

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        g = ShardGroup(0, 1)
        x = torch.arange(4096, dtype=torch.float32, device="cuda:0")
        assert torch.equal(g.collective_all_gather(x), x)
        s = torch.ones(100, dtype=torch.float64, device="cuda:0")
        g.collective_all_reduce(s)
        assert torch.equal(s, torch.ones_like(s))
        assert dist.get_backend() == "nccl"
        from fedscale_amd.state import spmd_rccl_probe

        probe = spmd_rccl_probe(0)  # our own RCCL communicator over the process group's ranks
        assert probe["count"] == 1 and probe["counts_agree"]
        assert probe["rank_of_process"] == [0] and probe["device_of_rank"] == [0]
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("at_once", [True, False], ids=["parts_at_once", "per_part"])
def test_egress_never_mixes_part_versions(gpu_device, at_once):
    """A servicer thread asking for the model while the main thread is between two parts' commits gets
    the previous version whole (aggregator.py:177-178: 20 servicer threads read the model while the main
    loop applies rounds): part 0 already holds the new model, part 1 the old one, the version is still
    the old one, and egress must read the buffers of that version only."""
    import threading

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    g = torch.Generator().manual_seed(5)
    names = ["a.weight", "b.weight", "n"]
    tensors = [torch.randn(300, 70, generator=g), torch.randn(4097, generator=g), torch.tensor(3)]
    rng = np.random.default_rng(6)

    def uploads(n):
        return [{"client_id": k, "moving_loss": 1.0,
                 "update_weight": {"a.weight": rng.standard_normal((300, 70)).astype(np.float32),
                                   "b.weight": rng.standard_normal(4097).astype(np.float32),
                                   "n": np.array(int(rng.integers(0, 9)), dtype=np.int64)}} for k in range(n)]

    rounds = [uploads(5), uploads(6)]
    single = TorchModelAdapter(StateDictModule(names, tensors), device="cuda:0")
    sharded = ShardedModelAdapter(StateDictModule(names, tensors), devices=[0, 0], transport="copy")
    want = []
    agg1 = DeviceAggregator(single)
    for ups in rounds:
        agg1.start_round(len(ups))
        for res in ups:
            agg1.on_result(res)
        want.append([t.numpy().copy() for t in single.get_weights()])

    sharded.FINISH_PARTS_AT_ONCE = at_once
    started, done, seen = threading.Event(), threading.Event(), {}
    orig = sharded.parts[1]._commit_scratch

    def slow_commit(*a, **k):  # part 0 has committed round 2; part 1 has not
        started.set()
        assert done.wait(60), "servicer thread did not finish"
        return orig(*a, **k)

    def servicer():
        assert started.wait(60)
        try:
            seen["weights"] = [t.numpy().copy() for t in sharded.get_weights()]
        finally:
            done.set()

    agg = DeviceAggregator(sharded)
    agg.start_round(len(rounds[0]))
    for res in rounds[0]:  # round 1, never read back before the race
        agg.on_result(res)
    sharded.parts[1]._commit_scratch = slow_commit
    th = threading.Thread(target=servicer)
    th.start()
    agg.start_round(len(rounds[1]))
    for res in rounds[1]:
        agg.on_result(res)
    th.join(60)
    assert not th.is_alive()
    assert_state_equal(seen["weights"], want[0], "egress during the commit window")
    assert_state_equal(sharded.get_weights(), want[1], "after the round")


@pytest.mark.parametrize("devices", ["0", "0,0"])
def test_selfcheck_module(gpu_device, devices):
    """fedscale_amd.selfcheck (what bench.py --gpus N runs over the node's N GPUs) on the one-GPU box: a
    one-GPU RCCL communicator and two parts on one card; every server step bit-identical to one GPU (q-FedAvg
    within 1e-6), every launch on its part's stream."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "fedscale_amd.selfcheck", "--devices", devices], cwd=root,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    rep = json.loads(lines[-1])
    assert r.returncode == 0 and rep["ok"], rep
    assert set(rep["policies"]) == {"fedavg", "fedbuff", "fed-yogi", "q-fedavg"}
    assert all(v["calls_off_their_stream"] == 0 and v["native_calls"] > 0 for v in rep["policies"].values())


@pytest.mark.parametrize("parts", [1, 2, 3])
def test_adopt_resident_round_is_the_reference_mean(gpu_device, parts):
    """The bench hook of the in-process N-GPU round (DeviceRound.adopt_resident, fedscale_amd/inproc_bench.py):
    uploads written into every part's staging on its device, taken as the round's K arrivals, give the same
    model as the sequential fp32 mean (aggregator.py:497-507) of the same synthetic rows, bit for bit; and
    ShardedModelAdapter.close() releases the group and leaves the adapter usable."""
    from fedscale_amd import synth
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter

    K, P, seed = 9, 70_001, 31
    model = synth.LayoutModule(["a", "b"], [(50_000,), (20_001,)], [torch.float32] * 2)
    ad = ShardedModelAdapter(model, devices=[0] * parts, transport="copy", staging_capacity=K)
    with ad:
        for rep in range(2):
            rnd = ad.begin_round(K, "fedavg", capacity=K)
            for i, (p, r) in enumerate(zip(ad.parts, rnd.rounds)):
                with p.dstream:
                    x = r.staging.x
                    # part i's slice of client k = columns [p0, p1) of the whole-model row
                    full = torch.empty(K, -(-P // 64) * 64, device="cuda")
                    synth.fill(full, K, P, seed=seed + rep)
                    x[:, :p.layout.P].copy_(full[:, p.layout.p0:p.layout.p1])
            rnd.adopt_resident(K)
            with pytest.raises(ValueError):
                rnd.adopt_resident(1)  # the round already has its K arrivals
            ad.apply_round(rnd, float(np.float32(K)), float(K))
            got = np.concatenate([w.numpy().reshape(-1) for w in ad.get_weights()])
            acc = None
            for row in synth.host_columns(seed + rep, range(K), np.arange(P)):
                acc = row.copy() if acc is None else acc + row
            np.testing.assert_array_equal(got, np.divide(acc, np.float32(K)))
    ad.close()  # idempotent


def test_inproc_bench_module_rehearsal(gpu_device):
    """fedscale_amd.inproc_bench (what bench.py --gpus N runs on rank 0) on the one-GPU box: two parts on one card
    and the one-GPU adapter beside them, small sizes; the report carries the fields bench.py records."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "fedscale_amd.inproc_bench", "--devices", "0,0", "--clients", "16",
                        "--params", "1000000", "--rounds", "3", "--policies", "fedavg,fed-yogi"], cwd=root,
                       capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    both = json.loads(lines[-1])
    assert r.returncode == 0 and both["ok"], both
    for pol in ("fedavg", "fed-yogi"):
        rep = both["policies"][pol]
        assert rep["transport"] == "copy" and rep["distinct_gpus"] is False
        assert len(rep["part_kernel_ms"]) == 2 and all(t > 0 for t in rep["part_kernel_ms"])
        for k in ("inproc_round_ms", "egress_ms", "inproc_round_ms_incl_egress", "speedup_vs_one_gpu"):
            assert rep[k] > 0, (pol, k)
        assert rep["one_gpu"]["round_ms"] > 0


def test_batched_yogi_finish_matches_per_part(gpu_device):
    """Config 4's in-process finish: fa_reduce_parts + fa_yogi_step_parts (one native call per pass over every
    part) gives the same bits as each part's own two-pass finish, over three rounds (the YoGi state carries)."""
    from fedscale_amd import synth
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from fedscale_amd.inproc_bench import _model, _optimizer

    K, P = 24, 300_000
    outs = []
    for batched in (True, False):
        ad = ShardedModelAdapter(_model(P, 5), optimizer=_optimizer("fed-yogi", 0), devices=[0, 0, 0],
                                 staging_capacity=K)
        ad.FINISH_PARTS_AT_ONCE = batched
        got = []
        for rr in range(3):
            rnd = ad.begin_round(K, "fedavg", capacity=K)
            for i, (p, r) in enumerate(zip(ad.parts, rnd.rounds)):
                with p.dstream:
                    synth.fill(r.staging.x, K, p.layout.P, seed=100 * rr + i)
            rnd.adopt_resident(K)
            ad.apply_round(rnd, float(np.float32(K)), float(K))
            got.append([w.clone() for w in ad.get_weights()])
        outs.append(got)
        ad.close()
    for rr, (a, b) in enumerate(zip(*outs)):
        for i, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), f"round {rr} tensor {i}"


@pytest.mark.parametrize("parts", [2, 3])
def test_registered_payload_ingress_is_bit_exact(gpu_device, parts):
    """Round-4 N-GPU ingress: uploads decoded zero-copy from the executor's pickled payload (the mixin's
    deserialize_response, aggregator.py:704) are registered in place and every part's copy engine reads its slice
    of the large arrays straight out of the payload (RegisteredUpload, fa_h2d_pieces); small entries and int64
    entries come from the pinned row.  Mixed with plain dict uploads (the gather path) in the same round, over
    chunk folds: the model is the oracle's FedAvg mean bit for bit, and every registration is released."""
    from fedscale_amd import ingress
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from oracle.cpu_reference import fedavg_close, fedavg_step

    names = ["big0", "bn.running_mean", "bn.num_batches_tracked", "big1", "small", "big2"]
    shapes = [(700, 1000), (64,), (), (300_001,), (5,), (1, 1_200_000)]
    dtypes = [torch.float32, torch.float32, torch.int64, torch.float32, torch.float32, torch.float32]
    init = [torch.zeros(s, dtype=d) for s, d in zip(shapes, dtypes)]
    sharded = ShardedModelAdapter(StateDictModule(names, init), devices=[0] * parts, transport="copy",
                                  staging_capacity=4)
    agg = DeviceAggregator(sharded)
    rng = np.random.default_rng(parts)
    K = 11
    for r in range(2):
        agg.start_round(K)
        acc = None
        for k in range(K):
            up = {}
            for n, s, d in zip(names, shapes, dtypes):
                up[n] = (np.array(int(rng.integers(0, 50)), dtype=np.int64).reshape(s) if d == torch.int64 else
                         rng.standard_normal(s, dtype=np.float32))
            acc = fedavg_step(acc, up, k == 0)
            if k % 3 != 2:  # the deployed path: a pickled payload, decoded as views of its bytes
                res = ingress.loads(pickle.dumps({"client_id": k, "update_weight": up, "moving_loss": 1.0}))
                assert not res["update_weight"]["big0"].flags.owndata
            else:
                res = {"client_id": k, "update_weight": up, "moving_loss": 1.0}
            agg.on_result(res)
        want = fedavg_close(acc, K)  # the reference's model_weights (int64 entries as float64 means)
        assert_state_equal(list(agg.model_weights), want, f"round {r} mean")
        # ... loaded into the model (load_state_dict's copy_: float64 -> int64 truncates)
        loaded = [torch.as_tensor(np.asarray(w)).to(d).numpy() for w, d in zip(want, dtypes)]
        assert_state_equal(sharded.get_weights(), loaded, f"round {r} model")
    # every payload upload registered, except any whose pages a neighbour's registration already covered
    assert sharded.registered_uploads + sharded.registration_fallbacks == 2 * sum(1 for k in range(K) if k % 3 != 2)
    assert sharded.registered_uploads >= sharded.registration_fallbacks
    sharded.close()
    assert not sharded._regs


@pytest.mark.parametrize("kind", ["bytearray", "writable_memoryview", "readonly_bytes_view"])
def test_mutable_payload_buffers_are_copied_before_add_returns(gpu_device, kind):
    """the copy engine reads a registered payload AFTER on_result returns, so only an immutable root
    (bytes, or a read-only memoryview of bytes) may be registered.  Uploads whose arrays view a bytearray or a
    writable memoryview take the pinned-row gather (copied before add returns): overwriting the caller's buffer
    right after on_result must not change the mean."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.sharded_model_adapter import ShardedModelAdapter
    from oracle.cpu_reference import fedavg_close, fedavg_step

    names, shapes = ["big0", "big1"], [(600_000,), (700_000,)]
    init = [torch.zeros(s_) for s_ in shapes]
    sharded = ShardedModelAdapter(StateDictModule(names, init), devices=[0, 0], transport="copy",
                                  staging_capacity=8)
    agg = DeviceAggregator(sharded)
    rng = np.random.default_rng(11)
    K = 6
    agg.start_round(K)
    acc = None
    for k in range(K):
        vals = [rng.standard_normal(s_[0], dtype=np.float32) for s_ in shapes]
        acc = fedavg_step(acc, {n: v.copy() for n, v in zip(names, vals)}, k == 0)
        raw = b"".join(v.tobytes() for v in vals)
        root = {"bytearray": lambda: bytearray(raw), "writable_memoryview": lambda: memoryview(bytearray(raw)),
                "readonly_bytes_view": lambda: memoryview(bytes(raw))}[kind]()
        a0 = np.frombuffer(root, dtype=np.float32, count=shapes[0][0])
        a1 = np.frombuffer(root, dtype=np.float32, count=shapes[1][0], offset=4 * shapes[0][0])
        agg.on_result({"client_id": k, "update_weight": {"big0": a0, "big1": a1}, "moving_loss": 1.0})
        if kind != "readonly_bytes_view":  # the caller reuses its receive buffer at once
            mv = memoryview(root).cast("B")
            mv[:] = b"\xff" * len(mv)  # NaN bit patterns everywhere
    want = fedavg_close(acc, K)
    assert_state_equal(sharded.get_weights(), [np.asarray(w) for w in want], kind)
    if kind == "readonly_bytes_view":
        assert sharded.registered_uploads + sharded.registration_fallbacks == K
    else:
        assert sharded.registered_uploads == 0
    sharded.close()
