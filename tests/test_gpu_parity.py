"""GPU parity: the HIP path (through the C ABI) against the golden fixtures of the real reference and
the CPU oracle.

* FedAvg / FedBuff (and the int64 side table): bit-exact — the kernels reproduce the reference's fp32
  op order (sequential arrival-order sum, true division, no FMA).
* FedYoGi: m and v bit-exact whenever they depend on the inputs only; the new model within
  YOGI_RTOL = 1e-6.  Reason: the reference's ``torch.sqrt`` on the CPU is not IEEE-correctly rounded
  (this torch build dispatches it to MKL VML; 0.7 % of fp32 inputs come out 1 ulp low, see
  tests/test_numerics_notes.py), while the GPU kernel uses the correctly rounded sqrt.
* q-FedAvg: within QFED_RTOL = 1e-5 (the north-star tolerance) because torch's CPU sum order for
  ||g||^2 is implementation-defined; the delta chain and the hs recurrence are checked bit-exact
  separately (test_qfed_kernels_delta_bit_exact_and_hs)."""
import numpy as np
import pytest
import torch

from oracle.cpu_reference import OracleYoGi, fedavg_flat, fedbuff_flat
from tests.golden_io import (Scenario, StateDictModule, assert_state_close, assert_state_equal,
                             scenario_names)

pytestmark = pytest.mark.gpu

QFED_RTOL = 1e-5
YOGI_RTOL = 1e-6


def _device_run(sc, capacity=None):
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator, DeviceAsyncAggregator
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    args = sc.args()
    model = StateDictModule(sc.names, sc.init_state())
    opt = TorchServerOptimizer(args.gradient_policy, args, "cuda:0") if sc.meta.get("optimizer") is not None else None
    adapter = TorchModelAdapter(model, optimizer=opt, device="cuda:0", staging_capacity=capacity)
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
        yield r, adapter, opt, agg


@pytest.mark.parametrize("bulk", ["zerocopy", "bulk", "perupdate"])
@pytest.mark.parametrize("capacity", [None, 2])
@pytest.mark.parametrize("name", scenario_names())
def test_device_path_matches_reference_fixture(gpu_device, name, capacity, bulk, monkeypatch):
    """Every fixture through the device path: small single-chunk rounds read the pinned mirror and write the
    egress snapshot from the kernel (zerocopy, the default for small models), the small-model bulk staging
    with one H2D per drain and a D2H for egress (bulk), and the per-update H2D ring of large models."""
    from fedscale_amd.bucket import ClientStaging
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    monkeypatch.setattr(ClientStaging, "BULK_MAX_BYTES", ClientStaging.BULK_MAX_BYTES if bulk != "perupdate" else -1)
    if bulk != "zerocopy":
        monkeypatch.setattr(ClientStaging, "ZERO_COPY_MAX_BYTES", -1)
        monkeypatch.setattr(TorchModelAdapter, "EGRESS_MIRROR_MAX_BYTES", -1)
    sc = Scenario(name)
    for r, adapter, opt, agg in _device_run(sc, capacity):
        got = adapter.get_weights()
        if sc.meta["policy"] == "q-fedavg":
            assert_state_close(got, sc.expected(r), QFED_RTOL, f"{name} r{r}", int_slack=1)
        elif sc.meta["policy"] == "fed-yogi":
            assert_state_close(got, sc.expected(r), YOGI_RTOL, f"{name} r{r}")
            m, v = sc.yogi_state(r)
            if r == 0:  # before any sqrt-dependent value feeds back
                assert_state_equal(opt.gradient_controller.m_t, m, f"{name} m r{r}")
                assert_state_equal(opt.gradient_controller.v_t, v, f"{name} v r{r}")
            else:
                assert_state_close(opt.gradient_controller.m_t, m, YOGI_RTOL, f"{name} m r{r}")
                assert_state_close(opt.gradient_controller.v_t, v, YOGI_RTOL, f"{name} v r{r}")
        else:
            assert_state_equal(got, sc.expected(r), f"{name} r{r} cap={capacity}")


def test_model_weights_is_the_fedavg_mean(gpu_device):
    """Aggregator.model_weights after the last result = the mean (aggregator.py:505-507), lazily fetched."""
    sc = Scenario("fedavg_mixed_k7")
    from oracle.cpu_reference import fedavg_close, fedavg_step

    acc = None
    for k in range(7):
        acc = fedavg_step(acc, sc.client(k), k == 0)
    want = fedavg_close(acc, 7)
    for _, adapter, _, agg in _device_run(sc):
        got = list(agg.model_weights)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(np.asarray(g), np.asarray(w))
            assert np.asarray(g).dtype == np.asarray(w).dtype


def test_model_weights_after_qfedavg_round(gpu_device):
    """The reference keeps the FedAvg mean in model_weights even in q-FedAvg mode (aggregator.py:505-507)."""
    sc = Scenario("qfedavg_q1")
    from oracle.cpu_reference import fedavg_close, fedavg_step

    acc = None
    for k in range(5):
        acc = fedavg_step(acc, sc.client(k), k == 0)
    want = fedavg_close(acc, 5)
    for _, adapter, _, agg in _device_run(sc):
        got = list(agg.model_weights)
        for g, w in zip(got, want):
            np.testing.assert_array_equal(np.asarray(g), np.asarray(w))


def test_get_model_syncs_module(gpu_device):
    sc = Scenario("fedavg_femnist_cnn_k10")
    for r, adapter, _, _ in _device_run(sc):
        m = adapter.get_model()
        assert_state_equal(list(m.state_dict().values()), sc.expected(r), "get_model")


def test_reference_typed_optimizer_api(gpu_device):
    """TorchServerOptimizer.update_round_gradient with the reference's list/nn.Module types."""
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from oracle.cpu_reference import OracleModel, OracleServerOptimizer

    sc = Scenario("fedyogi_mixed_3rounds")
    args = sc.args()
    ours = TorchServerOptimizer("fed-yogi", args, None)
    theirs = OracleServerOptimizer("fed-yogi", args, None)
    m_ours = StateDictModule(sc.names, sc.init_state())
    m_theirs = OracleModel(sc.names, sc.init_state())
    rng = np.random.default_rng(5)
    for r in range(3):
        last = [t.clone() for t in m_theirs.state_dict().values()]
        cur = []
        for t in last:
            if t.dtype == torch.int64:
                cur.append(t.to(torch.float64) + float(rng.integers(0, 4)) / 3)
            else:
                cur.append(t + torch.from_numpy(rng.normal(0, 0.01, size=tuple(t.shape)).astype(np.float32)))
        ours.update_round_gradient([t.clone() for t in last], [c.clone() for c in cur], m_ours)
        theirs.update_round_gradient(last, cur, m_theirs)
        assert_state_close(list(m_ours.state_dict().values()), list(m_theirs.state_dict().values()), YOGI_RTOL,
                           f"round {r}")
        # keep both on the same trajectory (the reference's sqrt is not IEEE: see module docstring)
        m_ours.load_state_dict(dict(m_theirs.state_dict()))


def test_yogi_update_api_matches_oracle(gpu_device):
    """YoGi.update(list) -> list of steps, 3 calls with state carry-over, fp32 and fp64 gradients."""
    from fedscale_amd.utils.optimizer.yogi import YoGi

    ours, theirs = YoGi(3e-3, 1e-8, 0.9, 0.99), OracleYoGi(3e-3, 1e-8, 0.9, 0.99)
    rng = np.random.default_rng(0)
    shapes = [(17, 5), (3,), (), (64,), (1,)]
    for it in range(3):
        grads = [torch.from_numpy(rng.normal(0, 0.02, size=s).astype(np.float32)) for s in shapes]
        grads.append(torch.tensor(float(it) + 0.5, dtype=torch.float64))
        got = ours.update([g.cuda() for g in grads])
        want = theirs.update(grads)
        assert_state_close([g.cpu() for g in got], [w.numpy() for w in want], YOGI_RTOL, f"step {it}")
        assert_state_equal([t.cpu() for t in ours.m_t], [t.numpy() for t in theirs.m_t], f"m {it}")
        assert_state_equal([t.cpu() for t in ours.v_t], [t.numpy() for t in theirs.v_t], f"v {it}")


# ---------------------------------------------------------------------------------------------
# kernel level, random inputs, edge shapes
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("K", [1, 2, 3, 7, 8, 9, 17, 64])
@pytest.mark.parametrize("P", [1, 3, 4, 5, 63, 64, 65, 1000, 4099, 70001, 8_400_017])
def test_reduce_kernel_bit_exact(gpu_device, K, P):
    from fedscale_amd import kernels as kx
    from fedscale_amd.bucket import round_up

    rng = np.random.default_rng(K * 100003 + P)
    ld = round_up(P, 64)
    xh = np.zeros((K, ld), dtype=np.float32)
    xh[:, :P] = rng.normal(0.1, 1.0, size=(K, P)).astype(np.float32)
    x = torch.from_numpy(xh).cuda()
    out = torch.full((ld,), 7.0, device="cuda")
    kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
    np.testing.assert_array_equal(out[:P].cpu().numpy(), fedavg_flat(xh[:, :P]))
    # weighted (FedBuff) and chunked continuation
    s = [1 / (1 + (k % 6)) ** 0.5 for k in range(K)]
    a = torch.tensor(np.asarray(s, dtype=np.float32), device="cuda")
    acc = torch.zeros(ld, device="cuda")
    h = K // 2
    if h:
        kx.reduce(x[:h], h, P, acc, a=a[:h])
        kx.reduce(x[h:], K - h, P, acc, a=a[h:], acc_in=acc, denom=float(np.float32(sum(s))), finalize=True)
    else:
        kx.reduce(x, K, P, acc, a=a, denom=float(np.float32(sum(s))), finalize=True)
    np.testing.assert_array_equal(acc[:P].cpu().numpy(), fedbuff_flat(xh[:, :P], s))
    # untouched tail: out[P:] beyond the float4 columns is not written
    if ld > (P + 3) // 4 * 4:
        assert float(out[ld - 1]) == 7.0


def test_reduce_kernel_special_values(gpu_device):
    from fedscale_amd import kernels as kx

    K, P = 5, 256
    xh = np.random.default_rng(1).normal(size=(K, P)).astype(np.float32)
    xh[0, 0] = np.inf
    xh[1, 1] = np.nan
    xh[:, 2] = [3e38, 3e38, -3e38, 0, 0]       # overflow then back: inf - inf
    xh[:, 3] = [1e-45, 1e-45, 0, 0, 0]         # denormals
    xh[:, 4] = [-0.0] * K
    x = torch.from_numpy(xh).cuda()
    out = torch.empty(P, device="cuda")
    kx.reduce(x, K, P, out, denom=5.0, finalize=True)
    with np.errstate(all="ignore"):
        want = fedavg_flat(xh)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    assert np.signbit(got[4]) == np.signbit(want[4])


def test_qfed_kernels_delta_bit_exact_and_hs(gpu_device):
    from fedscale_amd import kernels as kx

    rng = np.random.default_rng(3)
    K, P, ld = 37, 100003, 100032
    L = rng.normal(0, 0.05, size=ld).astype(np.float32)
    L[P:] = 0
    xh = (L[None, :] + rng.normal(0, 0.01, size=(K, ld))).astype(np.float32)
    xh[:, P:] = 0
    losses = rng.uniform(0.5, 2.0, size=K)
    lr, q = 0.05, 1.0
    alpha = np.array([np.float32(np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    x = torch.from_numpy(xh).cuda()
    Ld = torch.from_numpy(L).cuda()
    delta = torch.zeros(ld, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    ws = kx.qfed_workspace(K, "cuda")
    h = 20
    kx.qfed_accumulate(x[:h], h, P, last=Ld, alpha=torch.from_numpy(alpha[:h]).cuda(), lr=lr, delta=delta,
                       sqnorm=sq[:h], workspace=ws, accumulate=False)
    kx.qfed_accumulate(x[h:], K - h, P, last=Ld, alpha=torch.from_numpy(alpha[h:]).cuda(), lr=lr, delta=delta,
                       sqnorm=sq[h:], workspace=ws, accumulate=True)
    # host emulation of optimizers.py:82-93 in fp32
    d = None
    sq_ref = np.zeros(K)
    for k in range(K):
        g = (L[:P] - xh[k, :P]) / np.float32(lr)
        t = alpha[k] * g
        d = t if d is None else d + t
        sq_ref[k] = np.sum((g * g).astype(np.float64))
    np.testing.assert_array_equal(delta[:P].cpu().numpy(), d)
    np.testing.assert_allclose(sq.cpu().numpy(), sq_ref, rtol=1e-9)  # fp32 4-square partials, fp64 sums
    # hs recurrence (fp32, arrival order) is bit-exact given the same sqnorm
    c1 = np.array([np.float32(q * np.float_power(l + 1e-10, q - 1)) for l in losses], dtype=np.float32)
    c2 = np.array([np.float32((1.0 / lr) * np.float_power(l + 1e-10, q)) for l in losses], dtype=np.float32)
    hs = torch.zeros(2, device="cuda")
    kx.qfed_hs(sq, torch.from_numpy(c1).cuda(), torch.from_numpy(c2).cuda(), K, hs)
    s32 = sq.cpu().numpy().astype(np.float32)
    hh = np.float32(0)
    for k in range(K):
        hh = np.float32(hh + np.float32(c1[k] * s32[k] + c2[k]))
    assert hs[0].item() == float(hh)
    assert hs[1].item() == float(np.float32(hh + np.float32(1e-10)))


def test_synthetic_generator_matches_host_twin(gpu_device):
    from fedscale_amd import synth

    K, P, ld = 5, 10007, 10048
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=1234, k0=17)
    cols = np.array([0, 1, 2, 3, 4095, 4096, 10006])
    want = synth.host_columns(1234, range(17, 17 + K), cols)
    np.testing.assert_array_equal(x[:, cols].cpu().numpy(), want)
    assert float(x[:, P:].abs().sum()) == 0.0


def test_errors_are_loud(gpu_device):
    from fedscale_amd import kernels as kx
    from fedscale_amd._native import FedAggError, call

    x = torch.zeros(2, 64, device="cuda")
    out = torch.zeros(64, device="cuda")
    with pytest.raises(TypeError):
        kx.reduce(x.double(), 2, 64, out)
    with pytest.raises(ValueError):
        kx.reduce(x.cpu(), 2, 64, out)
    with pytest.raises(FedAggError):  # the C ABI itself rejects a misaligned pointer
        call("fa_reduce", x.data_ptr() + 4, 64, 2, 60, None, None, out.data_ptr(), 1.0, 2, None)


def test_pickled_adapter_size_matches_reference(gpu_device):
    """aggregator.py:422-424 sizes simulated transfers from pickle.dumps(model_wrapper)."""
    import pickle

    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter
    from oracle.cpu_reference import OracleModelAdapter, OracleServerOptimizer

    sc = Scenario("fedyogi_wide_3rounds")
    args = sc.args()
    net = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.BatchNorm1d(200))
    ours = TorchModelAdapter(net, optimizer=TorchServerOptimizer("fed-yogi", args, None))
    ref = OracleModelAdapter(net, OracleServerOptimizer("fed-yogi", args))
    a, b = len(pickle.dumps(ours)), len(pickle.dumps(ref))
    assert abs(a - b) < 0.02 * b, (a, b)
    back = pickle.loads(pickle.dumps(ours))
    assert_state_equal(back.get_weights(), ours.get_weights(), "unpickled adapter")


@pytest.mark.parametrize("last_zero", [0.0, -0.0])
@pytest.mark.parametrize("lr", [0.05, 0.049, 0.1, 1 / 3, 7e-5, 123.456, 1e-20, 3e25])
def test_qfed_division_is_correctly_rounded(gpu_device, lr, last_zero):
    """g = (L - W) / lr inside k_qfed_accum (constant-divisor division with one FMA correction) equals
    IEEE fp32 division for values over the whole exponent range, zeros of both signs, denormals, inf and
    NaN.  With L = -0, L - W = a exactly, -0 included (L = +0 turns a = -0 into +0)."""
    from fedscale_amd import kernels as kx

    rng = np.random.default_rng(int(lr * 1e6) % 1000)
    n = 1 << 22
    mant = rng.uniform(1.0, 2.0, size=n)
    expo = rng.integers(-149, 128, size=n)
    a = (mant * np.exp2(expo.astype(np.float64))).astype(np.float32)
    a[rng.random(n) < 0.5] *= -1
    a[:16] = [0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.1754944e-38, 3.4028235e38, -3.4028235e38,
              7.8886091e-31, 7.8886e-31, 1e30, 1.0000001e30, 1.0, -1.0]
    ld = n
    x = torch.from_numpy(-a).cuda().view(1, ld)  # last = +-0 -> L - W = a exactly (but for a = -0)
    last = torch.full((ld,), last_zero, device="cuda")
    delta = torch.empty(ld, device="cuda")
    sq = torch.zeros(1, dtype=torch.float64, device="cuda")
    with np.errstate(all="ignore"):
        want = (np.float32(last_zero) - (-a)) / np.float32(lr)  # the kernel's (L - W)
    assert np.signbit(want[1]) == np.signbit(np.float32(last_zero))
    kx.qfed_accumulate(x, 1, n, last=last, alpha=torch.ones(1, device="cuda"), lr=lr, delta=delta, sqnorm=sq,
                       workspace=kx.qfed_workspace(1, "cuda"), accumulate=False)
    got = delta.cpu().numpy()
    same = (got == want) | (np.isnan(got) & np.isnan(want))
    assert same.all(), f"{(~same).sum()} mismatches, e.g. a={a[~same][:3]} got={got[~same][:3]} want={want[~same][:3]}"
    assert (np.signbit(got) == np.signbit(want))[~np.isnan(want)].all()


@pytest.mark.parametrize("lr", [0.05, 3e-6, 7.5e5])
def test_qfed_inf_and_overflow_in_otherwise_fast_waves(gpu_device, lr):
    """Waves whose values are all in the fast-division range except a lone +-inf / NaN, or whose squares
    overflow fp32: the per-client finiteness check (QF_INFCHK 2) must send them to the IEEE division.
    Two clients, so the fallback of one client does not leak into the other's delta or norm."""
    from fedscale_amd import kernels as kx

    rng = np.random.default_rng(11)
    n = 1 << 20
    K = 2
    a = (rng.uniform(1.0, 2.0, size=(K, n)) * np.exp2(rng.integers(-40, 40, size=(K, n)).astype(np.float64)))
    a = a.astype(np.float32)
    a[rng.random((K, n)) < 0.5] *= -1
    for pos in rng.choice(n, size=24, replace=False):  # lone specials in different waves
        a[0, pos] = rng.choice([np.inf, -np.inf, np.nan])
    big = rng.choice(n, size=24, replace=False)  # |g| beyond 2^64: g*g overflows, the value stays finite
    a[1, big] = np.float32(2.0 ** 79) * np.float32(1.5)
    x = torch.from_numpy(-a).cuda()
    last = torch.zeros(n, device="cuda")
    delta = torch.empty(n, device="cuda")
    sq = torch.zeros(K, dtype=torch.float64, device="cuda")
    alpha = torch.tensor([1.0, 0.5], device="cuda")
    with np.errstate(all="ignore"):
        g = (np.float32(0) - (-a)) / np.float32(lr)
        want = g[0] * np.float32(1.0)
        want = want + g[1] * np.float32(0.5)
    kx.qfed_accumulate(x, K, n, last=last, alpha=alpha, lr=lr, delta=delta, sqnorm=sq,
                       workspace=kx.qfed_workspace(K, "cuda"), accumulate=False)
    got = delta.cpu().numpy()
    same = (got == want) | (np.isnan(got) & np.isnan(want))
    assert same.all(), f"{(~same).sum()} mismatches, e.g. got={got[~same][:3]} want={want[~same][:3]}"
    s = sq.cpu().numpy()
    assert np.isnan(s[0]) or np.isinf(s[0])
    with np.errstate(all="ignore"):
        ref1 = np.sum(np.square(g[1]).astype(np.float64))
    assert np.isinf(s[1]) == np.isinf(ref1)
    if not np.isinf(ref1):
        assert abs(s[1] - ref1) <= 1e-9 * ref1


@pytest.mark.parametrize("capacity", [None, 2])
@pytest.mark.parametrize("name", scenario_names("cohorts"))
def test_auxo_cohorts_match_reference_fixture(gpu_device, name, capacity):
    """Two cohorts with interleaved arrivals, each reduced on its own device adapter (bit-exact)."""
    from fedscale_amd.cloud.aggregation.aggregator import DeviceCohortAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    sc = Scenario(name)
    n = len(sc.meta["cohort_K"])
    wrappers = [TorchModelAdapter(StateDictModule(sc.names, sc.init_state(c)), device="cuda:0",
                                  staging_capacity=capacity) for c in range(n)]
    agg = DeviceCohortAggregator(wrappers, sc.meta["cohort_K"])
    for k, c in enumerate(sc.meta["cohorts"]):
        agg.on_result({"client_id": k + 1, "update_weight": sc.client(k), "moving_loss": 1.0}, c)
    for c, w in enumerate(wrappers):
        assert_state_equal(w.get_weights(), sc.expected_cohort(c), f"{name} cohort {c}")


@pytest.mark.parametrize("name", scenario_names("heterofl"))
def test_heterofl_combine_matches_reference_fixture(gpu_device, name):
    """HeteroFL sub-model combination (examples/heterofl/customized_aggregator.py:78-119), bit-exact."""
    from collections import OrderedDict

    from fedscale_amd.cloud.aggregation.heterofl import DeviceHeteroFLMixin

    sc = Scenario(name)

    class Agg(DeviceHeteroFLMixin):
        pass

    agg = Agg()
    agg.model = StateDictModule(sc.names, sc.init_state())
    agg.client_training_results = [{"model_rate": r, "local_parameters": loc}
                                   for r, loc in zip(sc.meta["rates"], sc.hetero_locals())]
    agg.combine_models()
    assert_state_equal(list(agg.model.state_dict().values()), sc.expected(0), name)


def test_egress_bytes_cached_per_model_version(gpu_device):
    """serialize_response of get_weights(): pickled once per model version, identical to pickle.dumps of
    the reference's plain list, unpickles without fedscale_amd types."""
    import pickle

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import TorchModelAdapter

    sc = Scenario("fedavg_mixed_k3")
    adapter = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()), device="cuda:0")
    agg = DeviceAggregator(adapter, sc.args())
    b0 = agg.serialize_response(adapter.get_weights())
    assert agg.serialize_response(adapter.get_weights()) is b0  # cached
    for r, ks in sc.rounds():
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
    w = adapter.get_weights()
    b1 = agg.serialize_response(w)
    assert b1 is not b0 and agg.serialize_response(adapter.get_weights()) is b1
    got = pickle.loads(b1)
    assert type(got) is list and all(type(t) is torch.Tensor for t in got)
    assert_state_equal(got, sc.expected(0), "egress")
    assert all(torch.equal(a, b) for a, b in zip(got, w))
    assert pickle.loads(agg.serialize_response({"x": 1})) == {"x": 1}  # other responses: plain pickle


def test_egress_handles_from_create_client_task(gpu_device):
    """create_client_task / get_test_config (aggregator.py:788-816) through the mixin hand the servicer an
    EgressHandle: serialised it is the cached bytes of its own model version (also after the model moved
    on), used as a list it is get_weights() of that version; a plugin's own create_client_task wins."""
    import pickle
    import types

    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregator
    from fedscale_amd.cloud.internal.torch_model_adapter import EgressHandle, TorchModelAdapter

    sc = Scenario("fedyogi_wide_3rounds")
    args = sc.args()
    from fedscale_amd.cloud.aggregation.optimizers import TorchServerOptimizer

    adapter = TorchModelAdapter(StateDictModule(sc.names, sc.init_state()),
                                optimizer=TorchServerOptimizer(args.gradient_policy, args, "cuda:0"), device="cuda:0")

    class Aggregator:  # stands for the reference class: the mixin replaces only its own methods
        def create_client_task(self, executor_id):
            raise AssertionError("the mixin should not call the reference create_client_task")

        def get_test_config(self, client_id):
            raise AssertionError("the mixin should not call the reference get_test_config")

        def get_client_conf(self, client_id):
            return {"learning_rate": 0.05}

        def CLIENT_PING(self, request, context):  # the UPDATE_MODEL branch, aggregator.py:902-907
            self.individual_client_events[request.executor_id].popleft()
            return self.serialize_response(self.model_wrapper.get_weights())

    class Agg(DeviceAggregator, Aggregator):
        pass

    agg = Agg(adapter, args)
    agg.resource_manager = types.SimpleNamespace(get_next_task=lambda e: 100 + e)
    agg.individual_client_events = {0: __import__("collections").deque(["update_model"] * 2)}
    ping = types.SimpleNamespace(executor_id=0, client_id=0)
    conf, h0 = agg.create_client_task(3)
    assert conf == {"client_id": 103, "task_config": {"learning_rate": 0.05}}
    assert isinstance(h0, EgressHandle)
    b0 = agg.serialize_response(h0)
    assert b0 is h0.egress_payload and b0 is agg.serialize_response(agg.get_test_config(5)[1])
    w0 = adapter.get_weights()
    assert_state_equal(pickle.loads(b0), w0, "handle bytes r-init")
    assert agg.CLIENT_PING(ping, None) is b0  # UPDATE_MODEL: the cached bytes, no clone
    for r, ks in sc.rounds():
        agg.start_round(len(ks))
        for res in sc.results(ks, r):
            agg.on_result(res)
        h = agg.create_client_task(0)[1]
        assert_state_equal(list(h), adapter.get_weights(), f"handle as list r{r}")
        assert len(h) == len(w0) and torch.equal(h[0], adapter.get_weights()[0])
    assert agg.CLIENT_PING(ping, None) is agg.serialize_response(agg.create_client_task(0)[1])
    # the first handle still serialises (and reads) as the version it was made from
    assert agg.serialize_response(h0) is b0
    assert_state_equal(list(h0), w0, "old handle")
    assert pickle.loads(pickle.dumps(h0)).__class__ is list  # pickles as the plain list
    assert_state_equal(pickle.loads(pickle.dumps(h0)), w0, "old handle pickled")
    # opt-out: the reference's fresh clone
    agg.device_egress_handles = False
    assert type(agg.create_client_task(1)[1]) is not EgressHandle


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_heterofl_random_prefix_boxes_bit_exact(gpu_device, seed):
    """Random global shapes (row lengths off the 4-grid, conv kernels, 1-D and 0-d-free vectors, rows in
    both kernel modes) and random per-client prefix boxes, more clients than one load batch, against the
    oracle restatement of combine_models — bit-exact."""
    from collections import OrderedDict

    from fedscale_amd.cloud.aggregation.heterofl import combine_prefix_boxes
    from oracle.cpu_reference import heterofl_combine

    rng = np.random.default_rng(seed)
    shapes = [(37, 29, 3, 3), (64, 300), (5, 1023), (130,), (7, 2, 5), (258, 257), (3, 1025, 1), (11, 255)]
    glob = OrderedDict((f"t{i}", torch.from_numpy(rng.normal(0, 1, size=s).astype(np.float32)))
                       for i, s in enumerate(shapes))
    K = 19
    locs = []
    for m in range(K):
        loc = OrderedDict()
        for n, v in glob.items():
            s = tuple(v.shape)
            o = int(rng.integers(0, s[0] + 1)) if m % 4 else s[0]
            box = (o,) + ((int(rng.integers(1, s[1] + 1)),) if len(s) > 1 else ()) + s[2:]
            loc[n] = rng.normal(0, 1, size=box).astype(np.float32)
        locs.append(loc)
    want = OrderedDict((n, v.clone()) for n, v in glob.items())
    heterofl_combine(want, locs)
    got = OrderedDict((n, v.clone()) for n, v in glob.items())
    combine_prefix_boxes(got, locs, device=gpu_device)
    for n in glob:
        assert torch.equal(got[n], want[n]), n


class _ReferenceHeteroFLHandler:
    """The reduction lines of examples/heterofl/customized_aggregator.py:55-71 (append the result, count
    it, combine at the K-th) — the base a DeviceHeteroFLMixin sits on in a real deployment."""

    def client_completion_handler(self, results):
        self.client_training_results.append(results)
        self.model_in_update += 1
        if self.model_in_update == self.tasks_round:
            self.combine_models()


@pytest.mark.parametrize("name", scenario_names("heterofl"))
def test_heterofl_staged_on_arrival_matches_reference_fixture(gpu_device, name):
    """Uploads staged on the device as they arrive (PrefixBoxStaging), combined at the K-th result."""
    from fedscale_amd.cloud.aggregation.heterofl import DeviceHeteroFLMixin

    sc = Scenario(name)

    class Agg(DeviceHeteroFLMixin, _ReferenceHeteroFLHandler):
        pass

    agg = Agg()
    agg.model = StateDictModule(sc.names, sc.init_state())
    for rnd in range(2):  # two rounds: the staging is rebuilt at each round's first result
        if rnd == 1:
            agg.model = StateDictModule(sc.names, sc.init_state())
        agg.client_training_results, agg.model_in_update = [], 0
        agg.tasks_round = len(sc.meta["rates"])
        for r, loc in zip(sc.meta["rates"], sc.hetero_locals()):
            agg.client_completion_handler({"model_rate": r, "local_parameters": loc})
        assert agg._hetero_staging is None  # consumed by combine_models
        assert_state_equal(list(agg.model.state_dict().values()), sc.expected(0), f"{name} round {rnd}")


def test_heterofl_staging_random_boxes_bit_exact(gpu_device):
    from collections import OrderedDict

    from fedscale_amd.cloud.aggregation.heterofl import PrefixBoxStaging
    from oracle.cpu_reference import heterofl_combine

    rng = np.random.default_rng(11)
    shapes = [(37, 29, 3, 3), (64, 300), (130,), (258, 257), (11, 255)]
    glob = OrderedDict((f"t{i}", torch.from_numpy(rng.normal(0, 1, size=s).astype(np.float32)))
                       for i, s in enumerate(shapes))
    locs = []
    for m in range(13):
        loc = OrderedDict()
        for n, v in glob.items():
            s = tuple(v.shape)
            o = int(rng.integers(0, s[0] + 1)) if m % 3 else s[0]
            box = (o,) + ((int(rng.integers(1, s[1] + 1)),) if len(s) > 1 else ()) + s[2:]
            loc[n] = rng.normal(0, 1, size=box).astype(np.float32)
        locs.append(loc)
    want = OrderedDict((n, v.clone()) for n, v in glob.items())
    heterofl_combine(want, locs)
    st = PrefixBoxStaging([tuple(v.shape) for v in glob.values()], len(locs), gpu_device)
    for loc in locs:
        st.add(list(glob.keys()), loc)
    got = OrderedDict((n, v.clone()) for n, v in glob.items())
    st.combine(got)
    for n in glob:
        assert torch.equal(got[n], want[n]), n


def test_heterofl_int64_entries_follow_the_reference_cast(gpu_device):
    """int64 state_dict entries (num_batches_tracked): the reference adds them into an fp32 tmp_v and
    stores tmp_v / count truncated back to int64 (customized_aggregator.py:114-118)."""
    from collections import OrderedDict

    from fedscale_amd.cloud.aggregation.heterofl import combine_prefix_boxes
    from oracle.cpu_reference import heterofl_combine

    rng = np.random.default_rng(5)
    glob = OrderedDict([("conv.weight", torch.from_numpy(rng.normal(size=(16, 8, 3, 3)).astype(np.float32))),
                        ("bn.num_batches_tracked", torch.tensor(7, dtype=torch.int64)),
                        ("fc.weight", torch.from_numpy(rng.normal(size=(10, 300)).astype(np.float32))),
                        ("steps", torch.tensor([3, 9, 11], dtype=torch.int64))])
    locs = []
    for m in range(5):
        locs.append(OrderedDict([("conv.weight", rng.normal(size=(16 - 2 * m, 8 - m, 3, 3)).astype(np.float32)),
                                 ("bn.num_batches_tracked", np.array(10 + 3 * m, dtype=np.int64)),
                                 ("fc.weight", rng.normal(size=(10, 300 - 40 * m)).astype(np.float32)),
                                 ("steps", np.array([1 + m, 2 * m, 5], dtype=np.int64)[:3 - (m % 2)])]))
    want = OrderedDict((n, v.clone()) for n, v in glob.items())
    heterofl_combine(want, locs)
    got = OrderedDict((n, v.clone()) for n, v in glob.items())
    combine_prefix_boxes(got, locs, device=gpu_device)
    for n in glob:
        assert got[n].dtype == want[n].dtype and torch.equal(got[n], want[n]), n


@pytest.mark.parametrize("K,P", [(1, 5), (3, 1000), (7, 70001), (64, 1_000_003), (13, 4_194_307)])
def test_qfed_fused_chain_kernel(gpu_device, K, P):
    """fa_qfed_accumulate with the fused FedAvg chain (LDS-DMA prefetch kernel on QF_CHAIN_V = 8-float4 tiles):
    delta equals the plain launch's bit for bit, the chain equals fa_reduce's FedAvg sum of the same rows bit for
    bit, and a chunked launch pair continues both chains exactly (FA_ACCUMULATE).  The per-client squared norms
    are summed over tiles of another width (the plain kernel's are 16 float4 wide) from fp32 partials of 8 squares
    instead of 4 (QF_CHAIN_PART, round 4), i.e. in another order: chain and plain launches are NOT bit-reproducible
    against each other on the norms (include/fedagg.h).  Their sums agree to ~1e-10 relative, so their fp32
    roundings (what hs consumes, optimizers.py:97's torch.sum of fp32) agree to within one ulp."""
    from fedscale_amd import kernels as kx
    from fedscale_amd import synth
    from fedscale_amd.bucket import round_up

    ld = round_up(P, 64)
    x = torch.empty(K, ld, device="cuda")
    synth.fill(x, K, P, seed=K + P)
    last = torch.empty(1, ld, device="cuda")
    synth.fill(last, 1, P, seed=K + P + 90000, scale_noise=0.0)
    last = last[0]
    alpha = torch.rand(K, device="cuda") + 0.5
    ws = kx.qfed_workspace(K, "cuda")
    outs = {}
    for use_chain in (False, True):
        delta = torch.full((ld,), float("nan"), device="cuda")
        chain = torch.full((ld,), float("nan"), device="cuda") if use_chain else None
        sq = torch.zeros(K, dtype=torch.float64, device="cuda")
        h = max(1, K // 2)
        kx.qfed_accumulate(x[:h], h, P, last=last, alpha=alpha[:h], lr=0.05, delta=delta, sqnorm=sq[:h],
                           workspace=ws, accumulate=False, chain=chain)
        if K > h:
            kx.qfed_accumulate(x[h:], K - h, P, last=last, alpha=alpha[h:], lr=0.05, delta=delta, sqnorm=sq[h:],
                               workspace=ws, accumulate=True, chain=chain)
        outs[use_chain] = (delta[:P].clone(), sq.clone(), None if chain is None else chain[:P].clone())
    assert torch.equal(outs[True][0], outs[False][0])
    n1, n0 = outs[True][1], outs[False][1]
    f1, f0 = n1.float(), n0.float()
    assert bool((f1 == f0).logical_or(torch.nextafter(f0, f1) == f1).all())  # within one fp32 ulp
    assert float(((n1 - n0).abs() / n0.abs().clamp_min(1e-300)).max()) < 1e-9
    want = torch.empty(ld, device="cuda")
    kx.reduce(x, K, P, want)
    assert torch.equal(outs[True][2], want[:P])
