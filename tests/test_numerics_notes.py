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
