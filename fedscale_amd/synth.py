"""Deterministic synthetic client updates (full-weight uploads = base + small noise).

Device side: ``fill(x, K, P, seed, k0)`` launches ``fa_fill_synthetic``.  Host side: ``host_columns``
recomputes any (client, column) value bit-exactly with numpy, so a full-size device result can be
checked column-sampled against a CPU sequential sum without materialising K x P on the host.

value(k, p) = fp32(tri(seed, p) * scale_base) + fp32(tri(seed + 1 + k, p) * scale_noise)
tri(s, p)   = (u1 + u2 - 2^24) * 2^-24 with u1, u2 the top 24 bits of two chained 32-bit mixes of
              (s, p): exact in fp32, triangular on (-1, 1).
"""
from __future__ import annotations

import numpy as np

from . import kernels as kx

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def _tri(stream: int, p: np.ndarray) -> np.ndarray:
    p = np.asarray(p, dtype=np.int64).astype(np.uint64)
    lo = p & M32
    hi = p >> np.uint64(32)
    s = _mix32(np.array([stream & 0xFFFFFFFF], dtype=np.uint64))
    h = _mix32(_mix32((lo + s) & M32) ^ hi)
    u1 = (h >> np.uint64(8)).astype(np.int64)
    u2 = (_mix32(h) >> np.uint64(8)).astype(np.int64)
    return (u1 + u2 - (1 << 24)).astype(np.float32) * np.float32(5.9604644775390625e-08)


def host_columns(seed: int, clients, cols, scale_base: float = 0.05, scale_noise: float = 0.01) -> np.ndarray:
    """[len(clients), len(cols)] fp32 values identical to what fa_fill_synthetic writes."""
    cols = np.asarray(cols, dtype=np.int64)
    b = _tri(seed, cols) * np.float32(scale_base)
    out = np.empty((len(clients), len(cols)), dtype=np.float32)
    for i, k in enumerate(clients):
        n = _tri((seed + 1 + int(k)) & 0xFFFFFFFF, cols) * np.float32(scale_noise)
        out[i] = b + n
    return out


def fill(x, K: int, P: int, *, seed: int, k0: int = 0, scale_base: float = 0.05, scale_noise: float = 0.01):
    """Device: x[0:K, :P] <- clients k0 .. k0+K-1 (columns [P, ld) zeroed)."""
    done = 0
    while done < K:  # the kernel takes <= 65535 clients per launch (grid.y)
        n = min(65535, K - done)
        kx.fill_synthetic(x[done:done + n], n, P, seed=seed, k0=k0 + done, scale_base=scale_base,
                          scale_noise=scale_noise)
        done += n
    return x


# ------------------------------------------------------------------------------------------------
# state_dict layouts of the BASELINE configs (synthetic workloads: shapes only, no weights)
# ------------------------------------------------------------------------------------------------
def resnet18_layout(num_classes: int = 10):
    """torchvision ResNet-18 state_dict (config 3, CIFAR-10 head): 102 fp32 tensors with
    P = 11,191,242 (11,181,642 parameters + 9,600 BN running stats) and 20 int64 num_batches_tracked."""
    import torch

    ent = []

    def bn(p, c):
        for n in ("weight", "bias", "running_mean", "running_var"):
            ent.append((f"{p}.{n}", (c,), torch.float32))
        ent.append((f"{p}.num_batches_tracked", (), torch.int64))

    ent.append(("conv1.weight", (64, 3, 7, 7), torch.float32))
    bn("bn1", 64)
    inp = 64
    for li, (planes, stride) in enumerate([(64, 1), (128, 2), (256, 2), (512, 2)], 1):
        for b in range(2):
            p = f"layer{li}.{b}"
            s = stride if b == 0 else 1
            ent.append((f"{p}.conv1.weight", (planes, inp, 3, 3), torch.float32))
            bn(f"{p}.bn1", planes)
            ent.append((f"{p}.conv2.weight", (planes, planes, 3, 3), torch.float32))
            bn(f"{p}.bn2", planes)
            if b == 0 and (s != 1 or inp != planes):
                ent.append((f"{p}.downsample.0.weight", (planes, inp, 1, 1), torch.float32))
                bn(f"{p}.downsample.1", planes)
            inp = planes
    ent.append(("fc.weight", (num_classes, 512), torch.float32))
    ent.append(("fc.bias", (num_classes,), torch.float32))
    return [e[0] for e in ent], [e[1] for e in ent], [e[2] for e in ent]


def femnist_cnn_layout():
    """MnistCNN (fedscale/utils/models/simple/models.py:11-29) with a 62-way fc2: P = 24,492 (config 1)."""
    import torch

    ent = [("conv1.weight", (10, 1, 5, 5)), ("conv1.bias", (10,)), ("conv2.weight", (20, 10, 5, 5)),
           ("conv2.bias", (20,)), ("fc1.weight", (50, 320)), ("fc1.bias", (50,)), ("fc2.weight", (62, 50)),
           ("fc2.bias", (62,))]
    return [e[0] for e in ent], [e[1] for e in ent], [torch.float32] * len(ent)


class LayoutModule:
    """A stand-in model object exposing state_dict()/load_state_dict() for a given layout (CPU tensors)."""

    def __init__(self, names, shapes, dtypes, seed: int = 0):
        import torch
        from collections import OrderedDict

        g = torch.Generator().manual_seed(seed)
        self._sd = OrderedDict()
        for n, s, d in zip(names, shapes, dtypes):
            self._sd[n] = (torch.randn(s, generator=g) * 0.05).to(d) if d.is_floating_point else torch.zeros(s, dtype=d)

    def state_dict(self, *a, **k):
        return self._sd

    def load_state_dict(self, new, strict=True):
        for n, dst in self._sd.items():
            dst.copy_(new[n])
