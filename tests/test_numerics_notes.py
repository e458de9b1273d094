"""Documents (and guards) the numerics facts the parity tolerances rest on (CPU only)."""
import numpy as np
import torch


def test_torch_cpu_sqrt_vs_ieee():
    """torch.sqrt on the CPU may differ from the IEEE correctly-rounded sqrt by at most 1 ulp (this
    build: MKL VML, ~0.7 % of inputs 1 ulp low).  The reference's FedYoGi (yogi.py:29) inherits it; the
    GPU path uses IEEE sqrt, hence YOGI_RTOL in tests/test_gpu_parity.py."""
    x = np.random.default_rng(0).uniform(1e-9, 1e-5, size=1_000_000).astype(np.float32)
    ieee = np.sqrt(x).view(np.int32).astype(np.int64)
    th = torch.sqrt(torch.from_numpy(x)).numpy().view(np.int32).astype(np.int64)
    assert np.max(np.abs(ieee - th)) <= 1
    assert np.mean(ieee != th) < 0.02


def test_torch_cpu_elementwise_ops_are_ieee():
    """Division by a Python scalar, reciprocal, add/mul: IEEE (the kernels rely on this)."""
    rng = np.random.default_rng(1)
    x = rng.normal(size=1_000_000).astype(np.float32)
    y = rng.normal(size=1_000_000).astype(np.float32)
    t, u = torch.from_numpy(x), torch.from_numpy(y)
    np.testing.assert_array_equal((t / 0.05).numpy(), x / np.float32(0.05))
    np.testing.assert_array_equal(t.reciprocal().numpy(), np.float32(1) / x)
    np.testing.assert_array_equal((0.9 * t + (1.0 - 0.9) * u).numpy(), np.float32(0.9) * x + np.float32(0.1) * y)
    np.testing.assert_array_equal((t ** 2).numpy(), x * x)


def test_qfedavg_int64_entries_move_by_at_most_one():
    """Why q-FedAvg's int64 state_dict entries are compared with a slack of 1 (int_slack=1), and why 1 is the
    bound.  The new value of an int64 entry is a truncation of an fp32 expression (optimizers.py:101-104, then
    load_state_dict's float32 -> int64 copy): n = trunc(fp32(L) - fp32(d / h)), with d the entry's delta and
    h = hs + 1e-10.  h carries the norm sum, which the reference forms with torch's CPU reduction order and
    the device in fp64, so h, and with it d / h, may differ by a relative rtol <= 1e-5.  For one
    value v = L - d/h with |v| * rtol < 1, a relative change <= rtol moves v by less than 1, and trunc of two
    reals less than 1 apart differs by at most 1 (it is 0 unless an integer lies between them).  The fixtures
    satisfy |v| * 1e-5 < 1 (int64 counters < 100), which assert_state_close's precondition checks."""
    rng = np.random.default_rng(7)
    rtol = 1e-5
    L = rng.integers(-60000, 60000, size=200_000).astype(np.float32)
    q = (rng.standard_normal(200_000) * 50).astype(np.float32)  # d / h
    v = L - q
    assert np.all(np.abs(v).astype(np.float64) * rtol < 1)
    e = rng.uniform(-rtol, rtol, size=200_000)
    q2 = (q.astype(np.float64) * (1 + e)).astype(np.float32)
    n1 = np.trunc(L - q).astype(np.int64)
    n2 = np.trunc(L - q2).astype(np.int64)
    assert np.max(np.abs(n1 - n2)) <= 1
    assert np.any(n1 != n2)  # the slack is needed: near-integer values do move
