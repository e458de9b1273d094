"""CPU-only checks: the C ABI library loads and exports every symbol of include/*.h, the host-side
layout / packing / sharding logic, the host twin of the synthetic generator, and that the product
package never reaches into oracle/."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    names = set()
    for h in ("fedagg.h", "fedclient.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    from fedscale_amd import _native

    lib = ctypes.CDLL(_native.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 22
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/*.h but not exported"
    assert sorted(_native.SIGNATURES) == names, "ctypes binding out of sync with include/*.h"
    _native.load()  # types every entry point, checks the ABI version (no GPU call)
    assert _native.load().fa_abi_version() == _native.ABI_VERSION


def test_error_path_without_gpu():
    from fedscale_amd._native import FedAggError, call

    with pytest.raises(FedAggError, match="ld"):
        call("fa_reduce", None, 6, 1, 8, None, None, None, 1.0, 2, None)  # validation precedes any HIP call


def test_sgd_prox_step_argument_errors_without_gpu():
    """fa_sgd_prox_step validates before any HIP call: momentum without buffers, nesterov with dampening,
    misaligned pointers (fake device addresses are never dereferenced)."""
    import ctypes

    from fedscale_amd._native import FedAggError, call

    arr = lambda *v: (ctypes.c_uint64 * len(v))(*v)
    n = (ctypes.c_int64 * 1)(8)
    with pytest.raises(FedAggError, match="momentum buffer"):
        call("fa_sgd_prox_step", arr(256), arr(512), None, None, n, 1, 0.1, 0.9, 0.0, 0.0, 0, 1, 0.0, 1, None)
    with pytest.raises(FedAggError, match="nesterov"):
        call("fa_sgd_prox_step", arr(256), arr(512), arr(768), None, n, 1, 0.1, 0.9, 0.1, 0.0, 1, 1, 0.0, 1, None)
    with pytest.raises(FedAggError, match="aligned"):
        call("fa_sgd_prox_step", arr(256), arr(512), arr(770), None, n, 1, 0.1, 0.9, 0.0, 0.0, 0, 1, 0.0, 1, None)
    with pytest.raises(FedAggError, match="NULL reference"):
        call("fa_sgd_prox_step", arr(256), arr(0), None, None, n, 1, 0.1, 0.0, 0.0, 0.0, 0, 1, 0.0, 1, None)


def test_kernels_reject_host_tensors():
    from fedscale_amd import kernels as kx

    x = torch.zeros(2, 64)
    with pytest.raises(ValueError, match="device tensor"):
        kx.reduce(x, 2, 64, torch.zeros(64))


def test_layout_and_sharding():
    from fedscale_amd.bucket import BucketLayout

    names = ["a", "n", "b", "c"]
    shapes = [(3, 5), (), (1000,), (7,)]
    dtypes = [torch.float32, torch.int64, torch.float32, torch.float32]
    full = BucketLayout(names, shapes, dtypes)
    assert full.P_full == 15 + 1000 + 7 and full.Q == 1 and full.P == full.P_full
    assert full.ld % 64 == 0 and full.ld >= full.P
    for world in (2, 3, 4, 8):
        shards = [BucketLayout(names, shapes, dtypes, r, world) for r in range(world)]
        assert all(s.ld == shards[0].ld and s.ld % 64 == 0 for s in shards)
        assert sum(s.P for s in shards) == full.P_full
        assert shards[0].p0 == 0 and all(shards[i].p1 == shards[i + 1].p0 or shards[i + 1].P == 0
                                         for i in range(world - 1))
    with pytest.raises(NotImplementedError):
        BucketLayout(["h"], [(2,)], [torch.float16])


def test_pack_host_roundtrip_and_shards():
    from fedscale_amd.bucket import BucketLayout

    rng = np.random.default_rng(0)
    names = ["w", "cnt", "b", "s0", "e"]
    vals = [rng.normal(size=(33, 7)).astype(np.float32), np.array(12, dtype=np.int64),
            rng.normal(size=(129,)).astype(np.float32), np.float32(0.25), np.zeros(0, np.float32)]
    shapes = [np.shape(v) for v in vals]
    dtypes = [torch.float32, torch.int64, torch.float32, torch.float32, torch.float32]
    world = 3
    parts = []
    for r in range(world):
        lay = BucketLayout(names, shapes, dtypes, r, world)
        f = np.zeros(lay.ld, np.float32)
        i = np.zeros(lay.ldq, np.int64)
        lay.pack_host(lay.values_of(dict(zip(names, vals))), f, i)
        parts.append(f)
        assert i[0] == 12
    flat = torch.from_numpy(np.concatenate(parts))
    out = BucketLayout(names, shapes, dtypes).unpack(flat, torch.tensor([12]))
    for o, v in zip(out, vals):
        np.testing.assert_array_equal(o.numpy(), np.asarray(v))
    lay = BucketLayout(names, shapes, dtypes)
    with pytest.raises(TypeError):
        lay.pack_host([v.astype(np.float64) if i == 0 else v for i, v in enumerate(vals)],
                      np.zeros(lay.ld, np.float32), np.zeros(1, np.int64))
    with pytest.raises(ValueError):
        lay.pack_host(vals[:-1], np.zeros(lay.ld, np.float32), np.zeros(1, np.int64))


def test_synth_host_twin_properties():
    from fedscale_amd import synth

    v = synth.host_columns(7, [0, 1, 2], np.arange(10000))
    assert v.dtype == np.float32 and v.shape == (3, 10000)
    assert np.all(np.abs(v) < 0.0601)
    assert abs(float(v.mean())) < 2e-3
    np.testing.assert_array_equal(v, synth.host_columns(7, [0, 1, 2], np.arange(10000)))
    assert not np.array_equal(v[0], v[1])


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "fedscale_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f"{f} imports oracle"


@pytest.mark.parametrize("workers", [1, 4, 8])
def test_native_host_gather(workers):
    """fa_host_gather (host-only native code, no GPU): pieces land at their offsets, pool path included."""
    from fedscale_amd.bucket import BucketLayout

    rng = np.random.default_rng(workers)
    shapes = [(1024, 1025), (3,), (700, 999), (), (5, 7, 11), (2048, 513)]  # > 4 MB in total
    names = [f"t{i}" for i in range(len(shapes))]
    vals = [rng.normal(size=s).astype(np.float32) for s in shapes]
    lay = BucketLayout(names, shapes, [torch.float32] * len(shapes))
    f = np.full(lay.ld, -1, np.float32)
    lay.pack_host(vals, f, np.zeros(1, np.int64), workers=workers)
    np.testing.assert_array_equal(f[:lay.P], np.concatenate([v.reshape(-1) for v in vals]))
    assert np.all(f[lay.P:] == -1)


@pytest.mark.parametrize("workers", [1, 3, 16])
def test_native_host_gather_streaming_copy_odd_offsets(workers):
    """The streaming-store copy of large pieces (>= 64 KiB): byte-exact at destination and source offsets
    off every alignment, with tails shorter than a cache line, and nothing written outside the pieces."""
    from fedscale_amd import _native

    rng = np.random.default_rng(10 + workers)
    sizes = [65536, 65537 + 13, 3, 1 << 20, 200_001, 64 * 1024 + 63, 5_000_000]
    src_buf = rng.integers(0, 256, size=sum(sizes) + 64 * len(sizes), dtype=np.uint8)
    srcs, offs, pos, s_at = [], [], 7, 1
    for n in sizes:
        srcs.append(src_buf.ctypes.data + s_at)
        offs.append(pos)
        s_at += n + 5
        pos += n + 3  # gaps of 3 bytes stay untouched
    dst = np.full(pos + 64, 0xAB, dtype=np.uint8)
    ps = np.asarray(srcs, dtype=np.uint64)
    po = np.asarray(offs, dtype=np.int64)
    pn = np.asarray(sizes, dtype=np.int64)
    _native.call("fa_host_gather", dst.ctypes.data, ps.ctypes.data, po.ctypes.data, pn.ctypes.data, len(sizes), workers)
    want = np.full_like(dst, 0xAB)
    s_at = 1
    for o, n in zip(offs, sizes):
        want[o:o + n] = src_buf[s_at:s_at + n]
        s_at += n + 5
    np.testing.assert_array_equal(dst, want)


def test_qfed_workspace_sizes():
    """fa_qfed_workspace_bytes (host-only): the one-window size for (K, 0, 0); for a call's (ld, P) room for every
    column window's partial norms of either launch form (chain windows are 2,097,152 columns, plain 4,194,304),
    so fa_qfed_accumulate gathers once per call; fa_qfed_accumulate refuses a workspace below the one-window size."""
    from fedscale_amd._native import FA_ACCUMULATE, FedAggError, call, load

    lib = load()
    for K in (1, 37, 462, 1024):
        one = lib.fa_qfed_workspace_bytes(K, 0, 0)
        assert one >= (256 + 16) * K * 8
        for P in (1_000_000, 25_000_000, 100_000_000):
            ld = -(-P // 64) * 64
            nwin = -(-P // 2_097_152)
            b = lib.fa_qfed_workspace_bytes(K, ld, P)
            assert b >= one and b >= nwin * (256 + 16) * K * 8, (K, P, b)
    with pytest.raises(FedAggError, match="workspace"):
        call("fa_qfed_accumulate", 16, 64, 4, 64, 16, 16, 0.05, 16, None, 16, 16, 8, FA_ACCUMULATE, None)
