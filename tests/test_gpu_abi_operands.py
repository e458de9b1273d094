"""Every launching entry point of the C ABI checks every operand before it queues anything (fa_device.h,
DevScope::operand / table): a pageable host buffer handed in any operand position returns FA_E_ARG, names
the operand, and leaves every output untouched; pinned host memory is accepted only where include/fedagg.h
allows it (the zero-copy round's x / mirror / xi).  Called straight through ctypes (no Python wrapper
validation in between).  The wrong-device half of the check is covered on the CPU against a mock runtime
(tests/test_abi_operands.py): the box has one GPU."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

K, LD, P, Q = 4, 64, 60, 3
FIN, ACC = 2, 1


def _u64(ptrs):
    return np.asarray(ptrs, dtype=np.uint64)


_STREAMS = []


def _stream():
    """A non-null stream (the per-part tables, fa_reduce_parts / fa_yogi_step_parts, refuse the null stream),
    created blocking (hipStreamCreate's default flags), so it is ordered after the tensors torch fills on the null
    stream; the tests synchronize the whole device."""
    if not _STREAMS:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        _STREAMS.append(s.value)
    return _STREAMS[0]


class Case:
    """An entry point, its operands (device tensors, or lists of them for pointer tables), the operands a
    launch writes, and how the ABI arguments are formed from a {name: pointer or [pointers]} map."""

    def __init__(self, name, ops, outs, args, host_ok=()):
        self.name, self.ops, self.outs, self.args, self.host_ok = name, ops, outs, args, set(host_ok)


def _cases(dev, st):
    def f(n, v=7.0, dt=torch.float32):
        return torch.full((n,), v, dtype=dt, device=dev)

    x = f(K * LD, 0.5)
    hp = [ctypes.c_float(3e-3), ctypes.c_float(1e-8), ctypes.c_float(0.9), ctypes.c_float(0.1), ctypes.c_float(0.01)]
    from fedscale_amd import _native as N

    lib = N.load()
    ws_q = lib.fa_qfed_workspace_bytes(K, LD, P)
    numel = np.asarray([40, 24], dtype=np.int64)
    ws_dp = lib.fa_dp_workspace_bytes(numel.ctypes.data, 2)
    tab = lambda v: [f(40, v), f(24, v)]  # noqa: E731 (a two-tensor model)
    tab64 = lambda v, dt: [f(40, v, dt), f(24, v, dt)]  # noqa: E731
    keep = []  # host arrays whose addresses are in flight

    def t(ps):
        a = _u64(ps)
        keep.append(a)
        return a.ctypes.data

    def host(dt, vals):  # a host array of per-tensor scalars (read by the host, never by a kernel)
        a = np.asarray(vals, dtype=dt)
        keep.append(a)
        return a.ctypes.data

    box_desc = torch.tensor([[0, 1, 4, 4]] * K, dtype=torch.int64, device=dev).reshape(-1)
    cases = [
        Case("fa_reduce", dict(x=x, a=f(K, 1.0), acc_in=f(LD, 0.0), out=f(LD)), ["out"],
             lambda p: (p["x"], LD, K, P, p["a"], p["acc_in"], p["out"], ctypes.c_float(4.0), FIN | ACC, st),
             host_ok=["x"]),
        Case("fa_reduce_mirror", dict(x=x, a=f(K, 1.0), acc_in=f(LD, 0.0), out=f(LD), mirror=f(LD)), ["out", "mirror"],
             lambda p: (p["x"], LD, K, P, p["a"], p["acc_in"], p["out"], p["mirror"], ctypes.c_float(4.0), FIN | ACC,
                        st), host_ok=["x", "mirror"]),
        Case("fa_reduce_yogi", dict(x=x, a=f(K, 1.0), acc_in=f(LD, 0.0), last=f(LD), m=f(LD), v=f(LD), out=f(LD),
                                    mean_out=f(LD)), ["m", "v", "out", "mean_out"],
             lambda p: (p["x"], LD, K, P, p["a"], p["acc_in"], ctypes.c_float(4.0), p["last"], p["m"], p["v"], p["out"],
                        p["mean_out"], *hp, FIN | ACC, st)),
        Case("fa_yogi_step", dict(cur=f(LD), last=f(LD), m=f(LD), v=f(LD), out=f(LD)), ["m", "v", "out"],
             lambda p: (p["cur"], p["last"], p["m"], p["v"], p["out"], P, *hp, 0, st)),
        Case("fa_qfed_accumulate", dict(x=x, last=f(LD), alpha=f(K, 1.0), delta=f(LD), chain=f(LD),
                                        sqnorm=f(K, 0.0, torch.float64), workspace=f(ws_q // 8 + 1, 0.0, torch.float64)),
             ["delta", "chain", "sqnorm"],
             lambda p: (p["x"], LD, K, P, p["last"], p["alpha"], ctypes.c_float(0.05), p["delta"], p["chain"],
                        p["sqnorm"], p["workspace"], ws_q, ACC, st)),
        Case("fa_qfed_hs", dict(sqnorm=f(K, 1.0, torch.float64), c1=f(K, 1.0), c2=f(K, 1.0), hs_out=f(2)), ["hs_out"],
             lambda p: (p["sqnorm"], p["c1"], p["c2"], K, p["hs_out"], st)),
        Case("fa_qfed_finalize", dict(last=f(LD), delta=f(LD), hs_dev=f(2, 2.0), out=f(LD)), ["out"],
             lambda p: (p["last"], p["delta"], p["hs_dev"], p["out"], P, st)),
        Case("fa_sum_rows_f64", dict(x=f(2 * K, 1.0, torch.float64), out=f(K, 0.0, torch.float64)), ["out"],
             lambda p: (p["x"], K, 2, K, p["out"], st)),
        Case("fa_side_accumulate", dict(xi=f(K * Q, 3, torch.int64), w=f(K, 1.0, torch.float64),
                                        acc_d=f(Q, 9.0, torch.float64)), ["acc_d"],
             lambda p: (p["xi"], Q, K, Q, 1, p["w"], None, p["acc_d"], 0, st), host_ok=["xi"]),
        Case("fa_side_close", dict(acc_i=f(Q, 8, torch.int64), cur=f(Q, 0.0, torch.float64),
                                   model=f(Q, 5, torch.int64)), ["cur", "model"],
             lambda p: (p["acc_i"], None, Q, 0, ctypes.c_double(4.0), p["cur"], p["model"], st)),
        Case("fa_side_yogi", dict(cur=f(Q, 1.0, torch.float64), last=f(Q, 1, torch.int64), m=f(Q, 0.0, torch.float64),
                                  v=f(Q, 0.0, torch.float64), step=f(Q, 0.0, torch.float64), model=f(Q, 5, torch.int64)),
             ["m", "v", "step", "model"],
             lambda p: (p["cur"], p["last"], p["m"], p["v"], p["step"], p["model"], Q, *[ctypes.c_double(h.value)
                                                                                         for h in hp], 0, st)),
        Case("fa_side_qfed_accumulate", dict(xi=f(K * Q, 3, torch.int64), last=f(Q, 1, torch.int64),
                                             alpha=f(K, 1.0), delta_s=f(Q), sqnorm=f(K, 0.0, torch.float64)),
             ["delta_s", "sqnorm"],
             lambda p: (p["xi"], Q, K, Q, p["last"], p["alpha"], ctypes.c_float(0.05), p["delta_s"], p["sqnorm"], 0,
                        st)),
        Case("fa_side_qfed_finalize", dict(last=f(Q, 1, torch.int64), delta_s=f(Q), hs_dev=f(2, 2.0),
                                           model=f(Q, 5, torch.int64)), ["model"],
             lambda p: (p["last"], p["delta_s"], p["hs_dev"], p["model"], Q, st)),
        Case("fa_fill_synthetic", dict(x=f(K * LD)), ["x"],
             lambda p: (p["x"], LD, K, P, 1, 0, ctypes.c_float(0.05), ctypes.c_float(0.01), st)),
        Case("fa_prefix_box_combine",
             dict(xs=f(K * 16, 1.0), desc=box_desc + 0, tensors=torch.tensor([0, 1, 4, 1], dtype=torch.int64,
                                                                               device=dev),
                  chunk_tensor=torch.tensor([0, -1], dtype=torch.int32, device=dev),
                  chunk_first=torch.tensor([0], dtype=torch.int64, device=dev), **{"global": f(4)}), ["global"],
             lambda p: (p["xs"], p["desc"], K, p["tensors"], 1, p["chunk_tensor"], p["chunk_first"], 1, p["global"],
                        st)),
        Case("fa_dp_normals", dict(out=f(64)), ["out"], lambda p: (p["out"], 64, 5, 0, st)),
        # the in-process N-GPU finish: two parts (on the one card), tables of per-part operands
        Case("fa_reduce_parts", {"x": [f(K * LD, 0.5), f(K * LD, 0.25)], "acc_in": [f(LD, 0.0), f(LD, 0.0)],
                                 "out": [f(LD), f(LD)]}, ["out"],
             lambda p: (2, t(p["x"]), host(np.int64, [LD, LD]), host(np.int32, [K, K]), host(np.int64, [P, P]),
                        t(p["acc_in"]), t(p["out"]), ctypes.c_float(4.0), host(np.int32, [FIN | ACC] * 2),
                        t([st, st]))),
        Case("fa_yogi_step_parts", {k: [f(LD), f(LD)] for k in ("cur", "last", "m", "v", "out")}, ["m", "v", "out"],
             lambda p: (2, t(p["cur"]), t(p["last"]), t(p["m"]), t(p["v"]), t(p["out"]), host(np.int64, [P, P]), *hp,
                        0, t([st, st]))),
        # client-side pointer tables (include/fedclient.h)
        Case("fa_prox_update", {"param": tab(1.0), "global": tab(2.0)}, ["param"],
             lambda p: (t(p["param"]), t(p["global"]), numel.ctypes.data, 2, ctypes.c_float(0.1), st)),
        Case("fa_sgd_prox_step", {"param": tab(1.0), "grad": tab(0.5), "momentum_buf": tab(0.0), "global": tab(2.0)}, ["param", "momentum_buf"],
             lambda p: (t(p["param"]), t(p["grad"]), t(p["momentum_buf"]), t(p["global"]), numel.ctypes.data, 2,
                        ctypes.c_float(0.1), ctypes.c_float(0.9), ctypes.c_double(0.0), ctypes.c_float(5e-4), 0, 0,
                        ctypes.c_float(0.01), 1, st)),
        Case("fa_sgd_prox_step_groups", {"param": tab(1.0), "grad": tab(0.5), "momentum_buf": tab(0.0), "global": tab(2.0)},
             ["param", "momentum_buf"],
             lambda p: (t(p["param"]), t(p["grad"]), t(p["momentum_buf"]), t(p["global"]), numel.ctypes.data, 2,
                        host(np.float32, [0.1, 0.2]), host(np.float32, [0.9, 0.9]), host(np.float64, [0.0, 0.0]),
                        host(np.float32, [5e-4, 0.0]), host(np.int32, [0, 0]), ctypes.c_float(0.01), 1, st)),
        Case("fa_dp_clip_coef", dict(param=tab(1.0), last=tab(0.5), workspace=f(ws_dp // 8 + 1, 0.0, torch.float64),
                                     coef_out=f(3)), ["coef_out"],
             lambda p: (t(p["param"]), t(p["last"]), numel.ctypes.data, 2, ctypes.c_float(1.0), 0, p["workspace"],
                        p["coef_out"], st)),
        Case("fa_dp_apply", dict(param=tab(1.0), last=tab(0.5), upload=tab(0.0), coef=f(3, 0.5)), ["param", "upload"],
             lambda p: (t(p["param"]), t(p["last"]), t(p["upload"]), numel.ctypes.data, t([0, 40]), 2, p["coef"],
                        ctypes.c_float(0.1), 3, 1, st)),
        Case("fa_dp_noise_i64", dict(x=tab64(3, torch.int64), out=tab64(0.0, torch.float64)), ["out"],
             lambda p: (t(p["x"]), t(p["out"]), numel.ctypes.data, t([0, 40]), 2, ctypes.c_float(0.1), 3, st)),
    ]
    return cases, keep


def _ptrs(ops, bad_name=None, bad_ptr=None, bad_index=0):
    p = {}
    for n, v in ops.items():
        if isinstance(v, list):
            p[n] = [x.data_ptr() for x in v]
            if n == bad_name:
                p[n][bad_index] = bad_ptr
        else:
            p[n] = bad_ptr if n == bad_name else v.data_ptr()
    return p


def _snapshot(case):
    out = {}
    for n in case.outs:
        v = case.ops[n]
        out[n] = [x.clone() for x in v] if isinstance(v, list) else v.clone()
    return out


def _unchanged(case, snap):
    torch.cuda.synchronize()
    for n, want in snap.items():
        got = case.ops[n]
        if isinstance(got, list):
            assert all(torch.equal(a, b) for a, b in zip(got, want)), f"{case.name}: {n} was written"
        else:
            assert torch.equal(got, want), f"{case.name}: {n} was written"


def test_pageable_operand_in_every_position_is_rejected_before_any_launch(gpu_device):
    from fedscale_amd import _native as N

    lib = N.load()
    st = _stream()
    pageable = np.zeros(1 << 20, dtype=np.float64)  # plain malloc'd host memory: pageable
    bad = pageable.ctypes.data
    cases, keep = _cases(gpu_device, st)
    exported = {n for n in N.SIGNATURES}
    checked = set()
    for case in cases:
        assert case.name in exported
        fn = getattr(lib, case.name)
        for name, v in case.ops.items():
            snap = _snapshot(case)
            rc = fn(*case.args(_ptrs(case.ops, name, bad, bad_index=1 if isinstance(v, list) else 0)))
            msg = lib.fa_last_error_string().decode()
            assert rc == -1, (case.name, name, rc, msg)  # FA_E_ARG
            assert "pageable" in msg and "nothing was launched" in msg, (case.name, name, msg)
            assert (f"{name}[1]" if isinstance(v, list) else name) in msg, (case.name, name, msg)
            _unchanged(case, snap)
            checked.add((case.name, name))
        # the same call with every operand valid goes through (the case's arguments are right)
        rc = fn(*case.args(_ptrs(case.ops)))
        assert rc == 0, (case.name, lib.fa_last_error_string().decode())
    torch.cuda.synchronize()
    del keep
    # every launching entry point of the ABI is covered (queries, host-only and RCCL calls are not launches)
    host_or_query = {"fa_abi_version", "fa_build_id", "fa_build_defs", "fa_last_error_string", "fa_pointer_kind",
                     "fa_reduce_launches", "fa_qfed_launches", "fa_qfed_max_chunk", "fa_qfed_workspace_bytes", "fa_host_gather",
                     "fa_pickle_strip", "fa_dp_workspace_bytes", "fa_host_register", "fa_host_unregister",
                     "fa_h2d_pieces", "fa_unranged_operands", "fa_set_strict_operands"}  # (fa_h2d_pieces: below)
    rccl = {n for n in exported if n.startswith("fa_rccl_")}
    assert exported - host_or_query - rccl == {c.name for c in cases}


def test_pinned_host_operand_only_where_the_header_allows_it(gpu_device):
    from fedscale_amd import _native as N

    lib = N.load()
    st = _stream()
    pinned = torch.zeros(1 << 17, dtype=torch.float64).pin_memory()
    cases, keep = _cases(gpu_device, st)
    for case in cases:
        fn = getattr(lib, case.name)
        for name, v in case.ops.items():
            if isinstance(v, list):
                continue
            snap = _snapshot(case)
            pinned.zero_()
            rc = fn(*case.args(_ptrs(case.ops, name, pinned.data_ptr())))
            msg = lib.fa_last_error_string().decode()
            if name in case.host_ok:  # the zero-copy operands: pinned memory is read / written over PCIe
                assert rc == 0, (case.name, name, msg)
                torch.cuda.synchronize()
            else:
                assert rc == -1 and "pinned host memory" in msg, (case.name, name, rc, msg)
                _unchanged(case, snap)
    del keep


def test_operand_extent_beyond_its_allocation_is_rejected(gpu_device):
    """A buffer too short for the call (here: P columns over an allocation of P/2) is refused, not overrun.  The
    short operand is its own hipMalloc (torch's caching allocator would hand out a slice of a larger segment)."""
    from fedscale_amd import _native as N

    lib = N.load()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    st = _stream()
    big = 1 << 22
    cur = torch.ones(big, device=gpu_device)
    m, v, out = (torch.zeros(big, device=gpu_device) for _ in range(3))
    short = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(short), big // 2 * 4) == 0
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    assert hip.hipMemset(short, 0, big // 2 * 4) == 0
    try:
        rc = lib.fa_yogi_step(cur.data_ptr(), short.value, m.data_ptr(), v.data_ptr(), out.data_ptr(), big,
                              3e-3, 1e-8, 0.9, 0.1, 0.01, 0, st)
        msg = lib.fa_last_error_string().decode()
        assert rc == -1 and "last" in msg and "past the end of its allocation" in msg, msg
        rc = lib.fa_yogi_step(cur.data_ptr(), short.value, m.data_ptr(), v.data_ptr(), out.data_ptr(), big // 2,
                              3e-3, 1e-8, 0.9, 0.1, 0.01, 0, st)  # the same operand, within its allocation
        assert rc == 0, lib.fa_last_error_string().decode()
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(out[big // 2:])) == 0 and int(torch.count_nonzero(out[:big // 2])) > 0
    finally:
        torch.cuda.synchronize()
        hip.hipFree(short)


def test_rccl_buffers_are_checked(gpu_device):
    from fedscale_amd import _native as N

    lib = N.load()
    if not lib.fa_rccl_available():
        pytest.skip("RCCL not loadable")
    comm = ctypes.c_void_p()
    devs = np.zeros(1, dtype=np.int32)
    N.call("fa_rccl_init", 1, devs.ctypes.data, ctypes.byref(comm))
    try:
        st = _stream()
        send = torch.ones(64, device=gpu_device)
        recv = torch.zeros(64, device=gpu_device)
        pageable = np.zeros(64, dtype=np.float32)
        sts = _u64([st])
        for s_ptr, r_ptr, name in ((pageable.ctypes.data, recv.data_ptr(), "send[0]"),
                                   (send.data_ptr(), pageable.ctypes.data, "recv[0]")):
            st_tab, rt_tab = _u64([s_ptr]), _u64([r_ptr])  # held: the library reads the tables during the call
            rc = lib.fa_rccl_all_reduce(comm, st_tab.ctypes.data, rt_tab.ctypes.data, 64, N.FA_DT_F32,
                                        sts.ctypes.data)
            msg = lib.fa_last_error_string().decode()
            assert rc == -1 and name in msg and "pageable" in msg, msg
        torch.cuda.synchronize()
        assert int(torch.count_nonzero(recv)) == 0
        st_tab, rt_tab = _u64([send.data_ptr()]), _u64([recv.data_ptr()])
        N.call("fa_rccl_all_reduce", comm, st_tab.ctypes.data, rt_tab.ctypes.data, 64, N.FA_DT_F32, sts.ctypes.data)
        torch.cuda.synchronize()
        assert torch.equal(recv, send)
    finally:
        N.call("fa_rccl_destroy", comm)


def test_h2d_pieces_checks_every_piece(gpu_device):
    """fa_h2d_pieces (round-4 N-GPU ingress): a source must be registered (fa_host_register, checked against the
    library's own list of registrations, extent included) or pinned host memory, a destination device memory of its
    stream's device holding the piece; a bad piece anywhere refuses the whole call before any copy is enqueued."""
    from fedscale_amd import _native as N

    lib = N.load()
    st = _stream()
    host = np.arange(1 << 18, dtype=np.float32)  # pageable until registered
    pinned = torch.arange(1 << 10, dtype=torch.float32).pin_memory()
    dst = torch.zeros(1 << 18, device=gpu_device)
    streams = _u64([st])

    def call(pieces):
        d = _u64([p[0] for p in pieces])
        s = _u64([p[1] for p in pieces])
        nb = np.asarray([p[2] for p in pieces], dtype=np.int64)
        si = np.zeros(len(pieces), dtype=np.int32)
        rc = lib.fa_h2d_pieces(d.ctypes.data, s.ctypes.data, nb.ctypes.data, si.ctypes.data, len(pieces),
                               streams.ctypes.data, 1)
        return rc, lib.fa_last_error_string().decode()

    half = host.nbytes // 2
    good = (dst.data_ptr(), pinned.data_ptr(), pinned.numel() * 4)
    rc, msg = call([good, (dst.data_ptr() + 4096, host.ctypes.data, half)])
    assert rc == -1 and "src" in msg and "not registered" in msg, msg
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(dst)) == 0  # the good piece before it was not copied either
    N.call("fa_host_register", host.ctypes.data, host.nbytes)
    try:
        rc, msg = call([good, (dst.data_ptr() + 4096, host.ctypes.data + half, half + 4)])
        assert rc == -1 and "src" in msg, msg  # 4 bytes past the registration
        rc, msg = call([(host.ctypes.data, pinned.data_ptr(), 64)])
        assert rc == -1 and "dst" in msg, msg
        rc, msg = call([good, (dst.data_ptr() + pinned.numel() * 4, host.ctypes.data + 4096, half)])
        assert rc == 0, msg
        torch.cuda.synchronize()
        want = np.concatenate([pinned.numpy(), host[1024:1024 + half // 4]])
        np.testing.assert_array_equal(dst[:want.size].cpu().numpy(), want)
    finally:
        N.call("fa_host_unregister", host.ctypes.data)
    rc, msg = call([(dst.data_ptr(), host.ctypes.data, 64)])  # released: no longer a valid source
    assert rc == -1, msg


_EXPANDABLE_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from fedscale_amd import kernels as kx
from oracle.cpu_reference import fedavg_flat
K, P, ld = 7, 50_000, 50_048
rng = np.random.default_rng(3)
h = rng.standard_normal((K, ld), dtype=np.float32)
x = torch.from_numpy(h).to("cuda:0")          # expandable (VMM) segments: HIP may report no address range
out = torch.empty(ld, device="cuda:0")
kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
got = out[:P].cpu().numpy()
want = fedavg_flat(h[:, :P])[:P]
assert np.array_equal(got, want), "mean differs"
from fedscale_amd import _native
st = _native.operand_stats()
if st["unranged"] > 0:  # HIP gave no range for the segment: counted, and refused under strict checks (ABI 5)
    _native.load().fa_set_strict_operands(1)
    try:
        kx.reduce(x, K, P, out, denom=float(np.float32(K)), finalize=True)
        raise SystemExit("strict operand checks accepted a rangeless operand")
    except _native.FedAggError as e:
        assert "strict operand checks" in str(e), e
    _native.load().fa_set_strict_operands(0)
print("OK", st["unranged"], torch.cuda.memory_stats().get("num_alloc_retries", 0))
"""


def test_expandable_segments_allocator_is_accepted(gpu_device):
    """operands in torch's expandable (VMM) segments pass DevScope::operand — the type and device checks
    hold; the extent check is skipped only where HIP reports no range — and the mean stays bit-exact."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTORCH_HIP_ALLOC_CONF="expandable_segments:True",
               PYTORCH_CUDA_ALLOC_CONF="expandable_segments:True")
    r = subprocess.run([sys.executable, "-c", _EXPANDABLE_CHILD, root], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-2000:]


def test_host_registered_pinned_x_is_accepted(gpu_device):
    """a client chunk in host memory registered with hipHostRegister (fa_host_register: what
    torch's host-register pinned mode and the registered ingress do) is accepted where the header allows host
    memory (fa_reduce's x, the zero-copy round), and the kernel reads it correctly."""
    import numpy as np

    from fedscale_amd import _native
    from oracle.cpu_reference import fedavg_flat

    K, P, ld = 5, 40_000, 40_000
    page = 4096
    raw = np.zeros(K * ld * 4 + 2 * page, dtype=np.uint8)
    off = (-raw.ctypes.data) % page
    h = raw[off:off + K * ld * 4].view(np.float32).reshape(K, ld)
    h[:] = np.random.default_rng(5).standard_normal((K, ld), dtype=np.float32)
    _native.call("fa_host_register", h.ctypes.data, h.nbytes)
    try:
        out = torch.empty(ld, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        _native.call("fa_reduce", h.ctypes.data, ld, K, P, None, None, out.data_ptr(), float(np.float32(K)),
                     _native.FA_FINALIZE, st)
        torch.cuda.synchronize()
        assert np.array_equal(out[:P].cpu().numpy(), fedavg_flat(h[:, :P])[:P])
        # one row more than the registration holds: refused before anything is queued
        st = torch.cuda.current_stream().cuda_stream
        with pytest.raises(_native.FedAggError, match="past the end of its registration|past the end of its allocation"):
            _native.call("fa_reduce", h.ctypes.data, ld, K + 1, P, None, None, out.data_ptr(),
                         float(np.float32(K)), _native.FA_FINALIZE, st)
    finally:
        _native.call("fa_host_unregister", h.ctypes.data)


def test_host_memory_registered_outside_the_library_is_refused(gpu_device):
    """pinned host memory HIP reports no range for and that no fa_host_register call covers has no known
    extent, so it is refused (FA_E_ARG) rather than handed to a kernel that might read past it."""
    import ctypes

    import numpy as np

    from fedscale_amd import _native

    K, P, ld = 3, 8192, 8192
    page = 4096
    raw = np.zeros(K * ld * 4 + 2 * page, dtype=np.uint8)
    off = (-raw.ctypes.data) % page
    h = raw[off:off + K * ld * 4].view(np.float32).reshape(K, ld)
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipHostRegister(ctypes.c_void_p(h.ctypes.data), ctypes.c_size_t(h.nbytes), 0) == 0
    try:
        out = torch.empty(ld, device="cuda:0")
        st = torch.cuda.current_stream().cuda_stream
        lib = _native.load()
        rc = lib.fa_reduce(h.ctypes.data, ld, K, P, None, None, out.data_ptr(), float(np.float32(K)),
                           _native.FA_FINALIZE, st)
        msg = lib.fa_last_error_string().decode()
        if rc == 0:  # this HIP reports a range for registered memory: the extent was checked against it
            torch.cuda.synchronize()
            assert "unknown extent" not in msg
        else:
            assert rc == -1 and "unknown extent" in msg, msg
    finally:
        hip.hipHostUnregister(ctypes.c_void_p(h.ctypes.data))
