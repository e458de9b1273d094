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
