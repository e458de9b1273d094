"""Edge cases of the device path against the (fixture-pinned) CPU oracle: models with no fp32 entries,
a single scalar, many clients folded through a small staging buffer, FedBuff and FedYoGi with chunking."""
import argparse

import numpy as np
import pytest
import torch

from oracle.cpu_reference import (OracleAggregator, OracleModel, OracleModelAdapter, OracleServerOptimizer)
from tests.golden_io import StateDictModule, assert_state_close, assert_state_equal

pytestmark = pytest.mark.gpu


def _args(policy=None):
    return argparse.Namespace(gradient_policy=policy, yogi_eta=3e-3, yogi_tau=1e-8, yogi_beta=0.9, yogi_beta2=0.99,
                              learning_rate=0.05, qfed_q=1.0)


def _run(names, init, K, rounds, policy=None, asynchronous=False, capacity=None, seed=0):
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    args = _args(policy)
    dev = TorchModelAdapter(StateDictModule(names, init), device="cuda:0", staging_capacity=capacity,
                            optimizer=TorchServerOptimizer(policy, args, "cuda:0") if policy else None)
    ref = OracleModelAdapter(OracleModel(names, init), OracleServerOptimizer(policy, args) if policy else None)
    if asynchronous:
        agg, oagg = DeviceAsyncAggregator(dev, args), OracleAggregator(ref, args, asynchronous=True)
        for a in (agg, oagg):
            a.round = 7
            a.client_task_model_version = {k: 7 - (k % 5) for k in range(K)}
    else:
        agg, oagg = DeviceAggregator(dev, args), OracleAggregator(ref, args)
    rng = np.random.default_rng(seed)
    for r in range(rounds):
        agg.start_round(K)
        oagg.start_round(K)
        for k in range(K):
            upd = []
            for t in init:
                if t.dtype == torch.int64:
                    upd.append(np.array(int(rng.integers(0, 1000)), dtype=np.int64).reshape(tuple(t.shape)))
                else:
                    upd.append((t.numpy() + rng.normal(0, 0.01, size=tuple(t.shape))).astype(np.float32))
            res = {"client_id": k, "update_weight": upd, "moving_loss": float(rng.uniform(0.5, 2))}
            oagg.on_result(dict(res))  # its own dict: the device path releases the staged upload in res
            agg.on_result(res)
        yield r, dev.get_weights(), ref.get_weights()


def test_int_only_model(gpu_device):
    names = ["a.num_batches_tracked", "b.num_batches_tracked"]
    init = [torch.tensor(3), torch.tensor(9)]
    for r, got, want in _run(names, init, K=5, rounds=2):
        assert_state_equal(got, [w.numpy() for w in want], f"int-only r{r}")


def test_single_scalar_model(gpu_device):
    for r, got, want in _run(["s"], [torch.tensor(0.25)], K=3, rounds=2):
        assert_state_equal(got, [w.numpy() for w in want], f"scalar r{r}")


@pytest.mark.parametrize("asynchronous", [False, True])
def test_many_clients_small_staging(gpu_device, asynchronous):
    names = ["w", "b", "n"]
    init = [torch.randn(130, 77) * 0.05, torch.randn(77) * 0.05, torch.tensor(4)]
    for r, got, want in _run(names, init, K=2500, rounds=1, asynchronous=asynchronous, capacity=333):
        assert_state_equal(got, [w.numpy() for w in want], f"K=2500 cap=333 async={asynchronous}")


def test_fedyogi_chunked_three_rounds(gpu_device):
    names = ["w", "n", "b"]
    init = [torch.randn(300, 41) * 0.05, torch.tensor(2), torch.randn(41) * 0.05]
    for r, got, want in _run(names, init, K=37, rounds=3, policy="fed-yogi", capacity=8):
        assert_state_close(got, [w.numpy() for w in want], 1e-6, f"yogi r{r}")


def test_qfedavg_more_clients_than_a_chunk(gpu_device):
    names = ["w", "n"]
    init = [torch.randn(2000) * 0.05, torch.tensor(11)]
    for r, got, want in _run(names, init, K=1300, rounds=1, policy="q-fedavg", capacity=2000):
        assert_state_close(got, [w.numpy() for w in want], 1e-5, "qfed K=1300", int_slack=1)


@pytest.mark.parametrize("K,P", [(3, (1 << 28) + 1000), (5, 140_000_003)])
def test_qfed_accumulate_wide_rows_and_column_windows(gpu_device, K, P):
    """Rows longer than the one-descriptor-per-group limit (4 rows x 4 B x ld > 2 GiB) take the
    per-row-descriptor path, and P > 2^28 is cut into column windows; a ragged K exercises rows past K.
    delta is bit-exact against torch fp32 on the same device (IEEE division, same per-element order);
    the squared norms to 1e-9 (fp32 4-square partials summed in fp64, as the kernel documents)."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=11)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=11 + 90000, scale_noise=0.0)
    last = last[0]
    alpha = torch.rand(K, device="cuda") + 0.5
    lr = 0.05
    delta = torch.empty(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    kx.qfed_accumulate(x, K, P, last=last, alpha=alpha, lr=lr, delta=delta, sqnorm=sq,
                       workspace=kx.qfed_workspace(K, "cuda"), accumulate=False)
    want = None
    want_sq = []
    lr32 = torch.tensor(lr, dtype=torch.float32, device="cuda")
    for k in range(K):
        g = (last[:P] - x[k, :P]) / lr32
        t = alpha[k] * g
        want = t if want is None else want + t
        want_sq.append(float((g * g).double().sum()))
        del g, t
    assert torch.equal(delta[:P], want)
    np.testing.assert_allclose(sq.cpu().numpy(), np.array(want_sq), rtol=1e-9)


@pytest.mark.parametrize("chain", [False, True], ids=["plain", "chain"])
@pytest.mark.parametrize("K,P", [(37, 9_000_001), (5, 4_194_305), (3, 35_000_000)])
def test_qfed_deferred_gathers_same_bits(gpu_device, K, P, chain):
    """One call over several column windows gathers every window's partial norms once, at the end (the workspace
    of fa_qfed_workspace_bytes(K, ld, P) holds them all); the same windows as separate one-window calls gather
    after each.  Both add the same fp64 terms in the same order: norms, delta and chain are bit-identical, over
    a first and a FA_ACCUMULATE call.  (3 x 35 M: more windows than a one-window workspace holds, so the
    wrapper's workspace of fa_qfed_workspace_bytes(K) alone would gather per window: both sizes are run.)"""
    from fedscale_amd import _native
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd._native import FA_ACCUMULATE
    from fedscale_amd.bucket import round_up
    from fedscale_amd.state import raw_stream

    ld = round_up(P, 64)
    n = kx.qfed_launches(ld, P, chain)
    win = kx.qfed_window(chain)  # fedagg.hip qfed_window: one round of full-width tiles
    assert win % 4 == 0 and n == -(-P // win) and n > 1
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=21)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=21 + 90000, scale_noise=0.0)
    last = last[0]
    alpha = torch.rand(K, device="cuda") + 0.5
    st = raw_stream(0)

    def state():
        return (torch.zeros(ld, device="cuda"), torch.zeros(ld, device="cuda") if chain else None,
                torch.zeros(K, dtype=torch.float64, device="cuda"))

    runs = {}
    for name, ws in (("one_call_deferred", kx.qfed_workspace(K, "cuda", ld, P)),
                     ("one_call_small_ws", kx.qfed_workspace(K, "cuda"))):
        delta, ch, sq = state()
        for acc in (False, True):
            kx.qfed_accumulate(x, K, P, last=last, alpha=alpha, lr=0.05, delta=delta, sqnorm=sq, workspace=ws,
                               accumulate=acc, chain=ch)
        runs[name] = (delta, ch, sq)
    # the per-window reference: one call per window (a single window always gathers right after it)
    ws = kx.qfed_workspace(K, "cuda")
    delta, ch, sq = state()
    for acc in (False, True):
        for w0 in range(0, P, win):
            pw = min(win, P - w0)
            _native.call("fa_qfed_accumulate", x.data_ptr() + 4 * w0, ld, K, pw, last.data_ptr() + 4 * w0,
                         alpha.data_ptr(), 0.05, delta.data_ptr() + 4 * w0,
                         ch.data_ptr() + 4 * w0 if chain else None, sq.data_ptr(), ws.data_ptr(), ws.numel() * 8,
                         FA_ACCUMULATE if acc else 0, st)
    torch.cuda.synchronize()
    for name, (d1, c1, s1) in runs.items():
        assert torch.equal(s1, sq), f"{name}: squared norms differ from the per-window gathers"
        assert torch.equal(d1, delta), name
        if chain:
            assert torch.equal(c1, ch), name


@pytest.mark.parametrize("name", ["fedavg_wide_k64", "fedbuff_k8", "qfedavg_q1"])
def test_async_ingress_staging_matches_reference(gpu_device, name):
    """ClientStaging(async_ingress=True): the gather + H2D of each update runs on a background thread in
    arrival order; the chunked folds drain it first.  Results stay those of the reference fixture."""
    from fedscale_amd.bucket import ClientStaging
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from tests.golden_io import Scenario, StateDictModule, assert_state_close, assert_state_equal

    sc = Scenario(name)
    args = sc.args()
    opt = TorchServerOptimizer(args.gradient_policy, args, "cuda:0") if sc.meta.get("optimizer") else None
    adapter = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()), optimizer=opt, device="cuda:0",
                                staging_capacity=5)
    adapter.staging = ClientStaging(adapter.layout, adapter.device, 5, async_ingress=True)
    policy = sc.meta["policy"]
    if policy == "fedbuff":
        agg = DeviceAsyncAggregator(adapter, args)
        agg.round = sc.meta["round"]
        for k, s in enumerate(sc.meta["staleness"]):
            agg.client_task_model_version[101 + k] = agg.round - s
    else:
        agg = DeviceAggregator(adapter, args)
    for r, ks in sc.rounds():
        if policy == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        got = adapter.get_weights()
        if policy == "q-fedavg":
            assert_state_close(got, sc.expected(r), 1e-5, f"{name} r{r}", int_slack=1)
        else:
            assert_state_equal(got, sc.expected(r), f"{name} r{r}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fedavg_femnist_cnn_k10", "fedavg_wide_k64", "fedyogi_wide_3rounds"])
def test_zero_copy_payload_ingress_matches_reference(gpu_device, name, monkeypatch):
    """Executor payloads (pickle.dumps of the result, torch_client.py:76-91) through the mixin's
    deserialize_response (fedscale_amd/ingress.py: arrays as read-only views of the payload; every other
    one decoded on arrival by add_event_handler on a servicer thread) into the device round: results stay those of the reference fixture, and the fast path really ran."""
    import pickle
    import threading

    from fedscale_amd import ingress
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from tests.golden_io import Scenario, StateDictModule, assert_state_close, assert_state_equal

    monkeypatch.setattr(ingress, "MIN_BYTES", 256)  # strip every array that pickles as BINBYTES (>= 256 B)
    monkeypatch.setattr(ingress, "MIN_PAYLOAD", 0)  # the fixtures' payloads are small
    sc = Scenario(name)
    args = sc.args()
    opt = TorchServerOptimizer(args.gradient_policy, args, "cuda:0") if sc.meta.get("optimizer") else None
    adapter = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()), optimizer=opt, device="cuda:0")
    agg = DeviceAggregator(adapter, args)
    agg.device_decode_on_arrival = True
    policy = sc.meta["policy"]
    for r, ks in sc.rounds():
        if policy == "q-fedavg":
            args.learning_rate = sc.meta["lrs"][r]
        agg.start_round(len(ks))
        for i, res in enumerate(sc.results(ks, r)):
            if i % 2:  # decoded on arrival by a servicer thread (add_event_handler), popped by the main loop
                th = threading.Thread(target=agg.add_event_handler, args=(i, "upload_model", None, pickle.dumps(res)))
                th.start()
                th.join()
                got_res = agg.deserialize_response(agg.server_events_queue.popleft()[3])
            else:
                got_res = agg.deserialize_response(pickle.dumps(res))
            uw = got_res["update_weight"]
            views = [v for v in (uw.values() if isinstance(uw, dict) else uw)
                     if isinstance(v, np.ndarray) and v.nbytes >= 256]
            assert views and all(not v.flags.writeable for v in views)
            agg.on_result(got_res)
        got = adapter.get_weights()
        if policy == "fed-yogi":  # the sqrt of the reference's torch CPU path: within 1e-5 (north_star)
            assert_state_close(got, sc.expected(r), 1e-5, f"{name} r{r}")
        else:
            assert_state_equal(got, sc.expected(r), f"{name} r{r}")


def test_get_weights_of_a_large_model_clones_in_parallel(gpu_device):
    """get_weights() of a model above CLONE_PARALLEL_MIN_BYTES clones the host snapshot with the native
    multi-threaded copy: the same values as the reference's per-entry clone (torch_model_adapter.py:41-47), each
    entry its own tensor, and writing to one returned tensor changes neither the snapshot nor the next call."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import fedavg_close, fedavg_step
    from tests.golden_io import StateDictModule

    names = ["w0", "w1", "tiny"]
    init = [torch.zeros(3_000_000), torch.zeros(2000, 1001), torch.zeros(3)]
    ad = TorchModelAdapter(StateDictModule(names, init), device="cuda:0")
    assert ad.layout.P_full * 4 >= ad.CLONE_PARALLEL_MIN_BYTES
    agg = DeviceAggregator(ad)
    rng = np.random.default_rng(4)
    acc = None
    agg.start_round(3)
    for k in range(3):
        up = [rng.standard_normal(tuple(t.shape)).astype(np.float32) for t in init]
        acc = fedavg_step(acc, up, k == 0)
        agg.on_result({"client_id": k, "update_weight": up, "moving_loss": 1.0})
    want = fedavg_close(acc, 3)
    got = ad.get_weights()
    assert_state_equal(got, want, "parallel clone")
    assert len({t.data_ptr() for t in got}) == len(got)
    got[0].fill_(7.0)
    assert_state_equal(ad.get_weights(), want, "a second call after the caller wrote into the first list")


def test_qfed_round_without_capacity_is_sized_by_free_hbm(gpu_device, monkeypatch):
    """A q-FedAvg DeviceRound given no capacity (TorchServerOptimizer's reference-typed list path) stages at most
    what default_capacity admits, not fa_qfed_max_chunk() clients: 2048 rows of a 100 M-parameter model would not
    fit the card."""
    from fedscale_amd import round as rd
    from fedscale_amd.bucket import BucketLayout

    seen = []

    def small(layout, K, device, *a, **k):
        seen.append(K)
        return 4

    monkeypatch.setattr(rd, "default_capacity", small)
    lay = BucketLayout(["w"], [(1000,)], [torch.float32])
    last = dict(last_f32=torch.zeros(lay.ld, dtype=torch.float32, device="cuda:0"),
                last_i64=torch.zeros(max(1, lay.ldq), dtype=torch.int64, device="cuda:0"))
    rnd = rd.DeviceRound(lay, "cuda:0", 11, "qfedavg", **last)
    assert seen and rnd.staging.capacity == 4 and rnd.cap == 4
    rnd2 = rd.DeviceRound(lay, "cuda:0", 11, "qfedavg", capacity=6, **last)  # an explicit capacity is kept
    assert rnd2.staging.capacity == 6 and rnd2.cap == 6
