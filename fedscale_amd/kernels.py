"""Typed torch-tensor wrappers over the C ABI (include/fedagg.h).

Each wrapper validates device / dtype / contiguity / size on the host (stricter than the reference,
identical on valid input) and launches on the current HIP stream of the tensor's device.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native as N
from ._native import FA_ACCUMULATE, FA_FINALIZE, FA_YOGI_INIT, call, ptr
from .state import raw_stream


def _dev(t: torch.Tensor, dtype, name: str, min_numel: int = 0, align: int = 16):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cuda":
        raise ValueError(f"{name}: must be a device tensor (got {t.device}); the HIP path has no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.numel() < min_numel:
        raise ValueError(f"{name}: has {t.numel()} elements, needs >= {min_numel}")
    if t.data_ptr() % align:
        raise ValueError(f"{name}: device pointer must be {align}-byte aligned")


def _cols(P: int) -> int:
    return (P + 3) // 4 * 4


def _stream(t: torch.Tensor):
    """The current stream of the tensor's device on this thread (an adapter's DeviceStream inside its calls)."""
    return raw_stream(t.device.index)


def _pinned(t: torch.Tensor, dtype, name: str, min_numel: int = 0):
    """A page-locked host tensor a kernel may read or write over PCIe (fa_reduce_mirror's host operands)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor, got {type(t).__name__}")
    if t.device.type != "cpu" or not t.is_pinned():
        raise ValueError(f"{name}: a host operand must be pinned (page-locked) memory")
    if t.dtype != dtype or not t.is_contiguous() or t.numel() < min_numel or t.data_ptr() % 16:
        raise ValueError(f"{name}: needs a contiguous, 16-byte aligned {dtype} buffer of >= {min_numel} elements")


def _check_x(x: torch.Tensor, K: int, P: int, host_ok: bool = False):
    if host_ok and isinstance(x, torch.Tensor) and x.device.type == "cpu":
        _pinned(x, torch.float32, "x")
    else:
        _dev(x, torch.float32, "x")
    if x.dim() != 2:
        raise ValueError("x: expected a [K, ld] client-major buffer")
    if K > x.shape[0]:
        raise ValueError(f"x: K={K} > rows {x.shape[0]}")
    ld = x.shape[1]
    if ld < P or ld % 4:
        raise ValueError(f"x: ld={ld} must be >= P={P} and a multiple of 4")
    return ld


def reduce(x: torch.Tensor, K: int, P: int, out: torch.Tensor, *, a: Optional[torch.Tensor] = None,
           acc_in: Optional[torch.Tensor] = None, denom: float = 1.0, finalize: bool = False,
           host_ok: bool = False) -> torch.Tensor:
    """In-order weighted column reduction of x[:K, :P] (fa_reduce); ``host_ok``: x may be a pinned host
    tensor, read by the kernel over PCIe."""
    ld = _check_x(x, K, P, host_ok) if K > 0 else (x.shape[1] if x is not None else _cols(P))
    _dev(out, torch.float32, "out", _cols(P))
    if a is not None:
        _dev(a, torch.float32, "a", K, align=4)
    if acc_in is not None:
        _dev(acc_in, torch.float32, "acc_in", _cols(P))
    flags = (FA_ACCUMULATE if acc_in is not None else 0) | (FA_FINALIZE if finalize else 0)
    call("fa_reduce", ptr(x) if K > 0 else None, ld, K, P, ptr(a), ptr(acc_in), ptr(out), float(denom), flags,
         _stream(out))
    return out


def reduce_parts(xs, Ks, Ps, outs, acc_ins, streams, *, denom: float, finalize: bool):
    """fa_reduce over every part of a model sharded over this process's GPUs, in one native call (unweighted):
    part i reduces xs[i][:Ks[i], :Ps[i]] (continuing acc_ins[i] when not None) into outs[i] on streams[i] (a
    hipStream_t of that part's GPU).  The library checks every part's stream and operands before launching."""
    import numpy as np

    n = len(xs)
    for name, seq in (("x", xs), ("out", outs)):
        for t in seq:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device.type != "cuda":
                raise ValueError(f"reduce_parts: {name} must be contiguous float32 device tensors")
    ptrs = lambda ts: np.asarray([0 if t is None else t.data_ptr() for t in ts], dtype=np.uint64)  # noqa: E731
    x_t, o_t, a_t = ptrs(xs), ptrs(outs), ptrs(acc_ins)
    ld = np.asarray([t.shape[-1] for t in xs], dtype=np.int64)
    K = np.asarray(Ks, dtype=np.int32)
    P = np.asarray(Ps, dtype=np.int64)
    fl = np.asarray([(FA_ACCUMULATE if a is not None else 0) | (FA_FINALIZE if finalize else 0) for a in acc_ins],
                    dtype=np.int32)
    import ctypes

    st = (ctypes.c_void_p * n)(*streams)  # a per-part stream table (as the fa_rccl_* calls take it)
    call("fa_reduce_parts", n, x_t.ctypes.data, ld.ctypes.data, K.ctypes.data, P.ctypes.data, a_t.ctypes.data,
         o_t.ctypes.data, float(denom), fl.ctypes.data, st)


def yogi_step_parts(curs, lasts, ms, vs, outs, Ps, streams, *, eta, tau, beta, omb, omb2, init):
    """fa_yogi_step over every part of a sharded model in one native call (part i on streams[i])."""
    import ctypes

    import numpy as np

    n = len(curs)
    for i in range(n):
        for nm, ts in (("cur", curs), ("last", lasts), ("m", ms), ("v", vs), ("out", outs)):
            _dev(ts[i], torch.float32, f"{nm}[{i}]", _cols(Ps[i]))
    tab = lambda ts: np.asarray([t.data_ptr() for t in ts], dtype=np.uint64)  # noqa: E731
    c_t, l_t, m_t, v_t, o_t = tab(curs), tab(lasts), tab(ms), tab(vs), tab(outs)
    P = np.asarray(Ps, dtype=np.int64)
    st = (ctypes.c_void_p * n)(*streams)
    call("fa_yogi_step_parts", n, c_t.ctypes.data, l_t.ctypes.data, m_t.ctypes.data, v_t.ctypes.data, o_t.ctypes.data,
         P.ctypes.data, float(eta), float(tau), float(beta), float(omb), float(omb2), FA_YOGI_INIT if init else 0, st)


def reduce_mirror(x: torch.Tensor, K: int, P: int, out: torch.Tensor, mirror: torch.Tensor, *,
                  a: Optional[torch.Tensor] = None, acc_in: Optional[torch.Tensor] = None,
                  denom: float = 1.0) -> torch.Tensor:
    """The finalizing reduce (fa_reduce_mirror) with the mean written to ``out`` and to ``mirror``; ``x`` and
    ``mirror`` may be pinned host tensors (the kernel reads / writes them over PCIe)."""
    ld = _check_x(x, K, P, host_ok=True) if K > 0 else _cols(P)
    _dev(out, torch.float32, "out", _cols(P))
    if mirror.device.type == "cpu":
        _pinned(mirror, torch.float32, "mirror", _cols(P))
    else:
        _dev(mirror, torch.float32, "mirror", _cols(P))
    if a is not None:
        _dev(a, torch.float32, "a", K, align=4)
    if acc_in is not None:
        _dev(acc_in, torch.float32, "acc_in", _cols(P))
    flags = (FA_ACCUMULATE if acc_in is not None else 0) | FA_FINALIZE
    call("fa_reduce_mirror", ptr(x) if K > 0 else None, ld, K, P, ptr(a), ptr(acc_in), ptr(out), ptr(mirror),
         float(denom), flags, _stream(out))
    return out


def reduce_yogi(x, K, P, *, last, m, v, out, denom, eta, tau, beta, omb, omb2, init, a=None, acc_in=None,
                mean_out=None):
    ld = _check_x(x, K, P) if K > 0 else x.shape[1]
    for n, t in (("last", last), ("m", m), ("v", v), ("out", out)):
        _dev(t, torch.float32, n, _cols(P))
    if a is not None:
        _dev(a, torch.float32, "a", K, align=4)
    if acc_in is not None:
        _dev(acc_in, torch.float32, "acc_in", _cols(P))
    if mean_out is not None:
        _dev(mean_out, torch.float32, "mean_out", _cols(P))
    flags = (FA_ACCUMULATE if acc_in is not None else 0) | FA_FINALIZE | (FA_YOGI_INIT if init else 0)
    call("fa_reduce_yogi", ptr(x) if K > 0 else None, ld, K, P, ptr(a), ptr(acc_in), float(denom), ptr(last),
         ptr(m), ptr(v), ptr(out), ptr(mean_out), float(eta), float(tau), float(beta), float(omb), float(omb2), flags,
         _stream(out))
    return out


def yogi_step(cur, last, m, v, out, P, *, eta, tau, beta, omb, omb2, init):
    for n, t in (("cur", cur), ("last", last), ("m", m), ("v", v), ("out", out)):
        _dev(t, torch.float32, n, _cols(P))
    call("fa_yogi_step", ptr(cur), ptr(last), ptr(m), ptr(v), ptr(out), P, float(eta), float(tau), float(beta),
         float(omb), float(omb2), FA_YOGI_INIT if init else 0, _stream(out))
    return out


def qfed_max_chunk() -> int:
    return N.load().fa_qfed_max_chunk()


def qfed_launches(ld: int, P: int, chain: bool = False) -> int:
    """k_qfed_accum launches one fa_qfed_accumulate call makes for rows of ld floats, with or without the fused
    FedAvg chain (fa_qfed_launches)."""
    return int(N.load().fa_qfed_launches(int(ld), int(P), 1 if chain else 0))


def qfed_window(chain: bool = False) -> int:
    """Columns of one k_qfed_accum column window (one round of full-width tiles; the chain launches' tiles have their
    own width): the largest P one launch covers, found from fa_qfed_launches."""
    lo, hi = 1, 1 << 28  # launches(lo) == 1 < launches(hi)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if qfed_launches((mid + 63) // 64 * 64, mid, chain) == 1:
            lo = mid
        else:
            hi = mid
    return lo


def reduce_launches(K: int, P: int, weighted: bool = False) -> int:
    """Kernel launches one fa_reduce call makes at (K, P) on the current device (fa_reduce_launches)."""
    return int(N.load().fa_reduce_launches(int(K), int(P), 1 if weighted else 0))


def qfed_workspace(K: int, device, ld: int = 0, P: int = 0) -> torch.Tensor:
    """Workspace of fa_qfed_accumulate for chunks of <= K clients; with the rows' (ld, P) it holds every column
    window's partial norms, so each call gathers them once instead of after every window (same bits)."""
    nbytes = N.load().fa_qfed_workspace_bytes(K, int(ld), int(P))
    return torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)


def qfed_accumulate(x, K, P, *, last, alpha, lr, delta, sqnorm, workspace, accumulate, chain=None):
    """q-FedAvg phase 1 over one chunk (fa_qfed_accumulate); ``chain`` (optional) carries the plain FedAvg
    sum of the same updates (the reference's model_weights before the division)."""
    ld = _check_x(x, K, P)
    _dev(last, torch.float32, "last", _cols(P))
    _dev(delta, torch.float32, "delta", _cols(P))
    if chain is not None:
        _dev(chain, torch.float32, "chain", _cols(P))
    _dev(alpha, torch.float32, "alpha", K, align=4)
    _dev(sqnorm, torch.float64, "sqnorm", K, align=8)
    _dev(workspace, torch.float64, "workspace")
    if workspace.numel() * 8 < N.load().fa_qfed_workspace_bytes(K, 0, 0):
        raise ValueError("workspace too small")
    call("fa_qfed_accumulate", ptr(x), ld, K, P, ptr(last), ptr(alpha), float(lr), ptr(delta), ptr(chain),
         ptr(sqnorm), ptr(workspace), workspace.numel() * 8, FA_ACCUMULATE if accumulate else 0, _stream(delta))


def qfed_hs(sqnorm, c1, c2, K, hs_out):
    _dev(sqnorm, torch.float64, "sqnorm", K, align=8)
    _dev(c1, torch.float32, "c1", K, align=4)
    _dev(c2, torch.float32, "c2", K, align=4)
    _dev(hs_out, torch.float32, "hs_out", 2)
    call("fa_qfed_hs", ptr(sqnorm), ptr(c1), ptr(c2), K, ptr(hs_out), _stream(hs_out))


def qfed_finalize(last, delta, hs, out, P):
    for n, t in (("last", last), ("delta", delta), ("out", out)):
        _dev(t, torch.float32, n, _cols(P))
    _dev(hs, torch.float32, "hs", 2)
    call("fa_qfed_finalize", ptr(last), ptr(delta), ptr(hs), ptr(out), P, _stream(out))


def sum_rows_f64(x: torch.Tensor, out: torch.Tensor):
    """out[k] = fixed-order sum over the rows of x[n, K] (fa_sum_rows_f64); out may alias x[0]."""
    _dev(x, torch.float64, "x", align=8)
    if x.dim() != 2:
        raise ValueError("x: expected [n, K]")
    n, K = x.shape
    _dev(out, torch.float64, "out", K, align=8)
    if out.device != x.device:
        raise ValueError("out and x must be on the same device")
    call("fa_sum_rows_f64", ptr(x), K, n, K, ptr(out), _stream(out))
    return out


# ---- side table (int64 entries) ---------------------------------------------------------------
def side_accumulate(xi, K, Q, mode, *, w=None, acc_i=None, acc_d=None, accumulate=False):
    """``xi`` may be a pinned host tensor (the staging mirror): the kernel then reads it over PCIe."""
    if Q == 0 or K == 0:
        return
    if xi.device.type == "cpu":
        _pinned(xi, torch.int64, "xi")
    else:
        _dev(xi, torch.int64, "xi", align=8)
    ldq = xi.shape[1]
    if mode == 0:
        _dev(acc_i, torch.int64, "acc_i", Q, align=8)
    else:
        _dev(acc_d, torch.float64, "acc_d", Q, align=8)
        _dev(w, torch.float64, "w", K, align=8)
    call("fa_side_accumulate", ptr(xi), ldq, K, Q, mode, ptr(w), ptr(acc_i), ptr(acc_d),
         FA_ACCUMULATE if accumulate else 0, _stream(acc_i if mode == 0 else acc_d))


def side_close(Q, mode, denom, *, acc_i=None, acc_d=None, cur=None, model=None):
    if Q == 0:
        return
    ref = acc_i if mode == 0 else acc_d
    call("fa_side_close", ptr(acc_i), ptr(acc_d), Q, mode, float(denom), ptr(cur), ptr(model), _stream(ref))


def side_yogi(cur, last, m, v, Q, *, step=None, model=None, eta, tau, beta, omb, omb2, init):
    if Q == 0:
        return
    call("fa_side_yogi", ptr(cur), ptr(last), ptr(m), ptr(v), ptr(step), ptr(model), Q, float(eta), float(tau), float(beta),
         float(omb), float(omb2), FA_YOGI_INIT if init else 0, _stream(cur))


def side_qfed_accumulate(xi, K, Q, *, last, alpha, lr, delta_s, sqnorm, accumulate):
    if Q == 0 or K == 0:
        return
    _dev(xi, torch.int64, "xi", align=8)
    call("fa_side_qfed_accumulate", ptr(xi), xi.shape[1], K, Q, ptr(last), ptr(alpha), float(lr), ptr(delta_s),
         ptr(sqnorm), FA_ACCUMULATE if accumulate else 0, _stream(xi))


def side_qfed_finalize(last, delta_s, hs, model, Q):
    if Q == 0:
        return
    call("fa_side_qfed_finalize", ptr(last), ptr(delta_s), ptr(hs), ptr(model), Q, _stream(model))


def fill_synthetic(x: torch.Tensor, K: int, P: int, *, seed: int, k0: int = 0, scale_base: float = 0.05,
                   scale_noise: float = 0.01):
    _dev(x, torch.float32, "x")
    ld = x.shape[1]
    if K > x.shape[0] or ld < P:
        raise ValueError("fill_synthetic: x too small")
    call("fa_fill_synthetic", ptr(x), ld, K, P, seed & 0xFFFFFFFF, k0, float(scale_base), float(scale_noise),
         _stream(x))
    return x


# ---- client-side handlers (include/fedclient.h): multi-tensor launches over HOST pointer tables -----
# The reference calls FedProx after EVERY local step (torch_client.py:238-240), so the per-call host cost
# matters as much as the kernel: a validated pointer table is cached per tensor-list signature (device
# pointers + sizes), and a repeat call is one ctypes call into the library.
class _Plan:
    """Validated host tables (device pointers, element counts) for fixed tensor lists."""

    def __init__(self, lists, numel):
        import numpy as np

        self.arrays = [None if lst is None else
                       np.asarray([0 if t is None else t.data_ptr() for t in lst], dtype=np.uint64) for lst in lists]
        self.numel = np.asarray(numel, dtype=np.int64)
        self.T = len(numel)

    def ptr(self, i):
        a = self.arrays[i]
        return None if a is None else a.ctypes.data


_PLANS: "dict" = {}
_PLANS_MAX = 32


def _sig(*lists):
    out = []
    for lst in lists:
        if lst is None:
            out.append(None)
        else:
            out.append(tuple(0 if t is None else t.data_ptr() for t in lst))
            out.append(tuple(0 if t is None else t.numel() for t in lst))
            out.append(tuple(None if t is None else (t.dtype, t.device, t.is_contiguous()) for t in lst))
    return tuple(out)


def _cached_plan(kind, lists, build):
    key = (kind,) + _sig(*lists)
    plan = _PLANS.get(key)
    if plan is None:
        plan = build()
        if len(_PLANS) >= _PLANS_MAX:
            _PLANS.pop(next(iter(_PLANS)))
        _PLANS[key] = plan
    return plan


def _fp32_list(ts, name, device=None, allow_none=False, dtype=torch.float32, align=4):
    dev = device
    for i, t in enumerate(ts):
        if t is None and allow_none:
            continue
        _dev(t, dtype, f"{name}[{i}]", align=align)
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"{name}[{i}]: on {t.device}, expected {dev}")
    return dev


def prox_update(params, global_model, c: float):
    """param[t] += c * (param[t] - global[t]) for every tensor, one multi-tensor launch (fa_prox_update)."""
    params = params if isinstance(params, list) else list(params)
    global_model = global_model if isinstance(global_model, list) else list(global_model)
    if not params:
        return

    def build():
        if len(params) != len(global_model):
            raise ValueError(f"{len(params)} parameters but {len(global_model)} global tensors")
        dev = _fp32_list(params, "param")
        _fp32_list(global_model, "global_model", dev)
        for i, (p, g) in enumerate(zip(params, global_model)):
            if p.shape != g.shape:
                raise ValueError(f"param[{i}] shape {tuple(p.shape)} != global_model[{i}] shape {tuple(g.shape)}")
        return _Plan([params, global_model], [p.numel() for p in params])

    plan = _cached_plan("prox", (params, global_model), build)
    call("fa_prox_update", plan.ptr(0), plan.ptr(1), plan.numel.ctypes.data, plan.T, float(c),
         _stream(params[0]))


def sgd_prox_step(params, grads, bufs, global_model, lr: float, momentum: float, dampening: float,
                  weight_decay: float, nesterov: bool, first: bool, c: float, fma: bool = True):
    """torch.optim.SGD step + FedProx step over every tensor in one multi-tensor launch (fa_sgd_prox_step).
    ``bufs`` None when momentum == 0; ``global_model`` None: no proximal step."""
    params, grads = list(params), list(grads)
    if not params:
        return
    bufs = list(bufs) if bufs is not None else None
    global_model = list(global_model) if global_model is not None else None
    if momentum != 0 and bufs is None:
        raise ValueError("momentum != 0 needs momentum buffers")

    def build():
        dev = _fp32_list(params, "param")
        for name, lst in (("grad", grads), ("momentum_buffer", bufs), ("global_model", global_model)):
            if lst is None:
                continue
            if len(lst) != len(params):
                raise ValueError(f"{len(params)} parameters but {len(lst)} {name} tensors")
            _fp32_list(lst, name, dev)
            for i, (p, t) in enumerate(zip(params, lst)):
                if p.shape != t.shape:
                    raise ValueError(f"{name}[{i}] shape {tuple(t.shape)} != param[{i}] shape {tuple(p.shape)}")
        return _Plan([params, grads, bufs if bufs is not None else [None] * len(params),
                      global_model if global_model is not None else [None] * len(params)],
                     [p.numel() for p in params])

    plan = _cached_plan("sgdprox", (params, grads, bufs, global_model), build)
    call("fa_sgd_prox_step", plan.ptr(0), plan.ptr(1), plan.ptr(2) if bufs is not None else None,
         plan.ptr(3) if global_model is not None else None, plan.numel.ctypes.data, plan.T, float(lr),
         float(momentum), float(dampening), float(weight_decay), int(bool(nesterov)), int(bool(first)), float(c),
         int(bool(fma)), _stream(params[0]))


def sgd_prox_step_groups(params, grads, bufs, global_model, lr, momentum, dampening, weight_decay, flags,
                         c: float, fma: bool = True):
    """torch.optim.SGD step (per-tensor group scalars) + FedProx over every tensor in one multi-tensor
    launch (fa_sgd_prox_step_groups).  ``bufs[i]`` None where the tensor's momentum is 0; ``global_model``
    None: no proximal step; scalars are sequences of len(params); flags: FA_SGD_NESTEROV | FA_SGD_FIRST."""
    import numpy as np

    params, grads = list(params), list(grads)
    T = len(params)
    if not T:
        return
    bufs = list(bufs) if bufs is not None else [None] * T
    global_model = list(global_model) if global_model is not None else None

    def build():
        dev = _fp32_list(params, "param")
        for name, lst, none_ok in (("grad", grads, False), ("momentum_buffer", bufs, True),
                                   ("global_model", global_model, False)):
            if lst is None:
                continue
            if len(lst) != T:
                raise ValueError(f"{T} parameters but {len(lst)} {name} tensors")
            _fp32_list(lst, name, dev, allow_none=none_ok)
            for i, (p, t) in enumerate(zip(params, lst)):
                if t is not None and p.shape != t.shape:
                    raise ValueError(f"{name}[{i}] shape {tuple(t.shape)} != param[{i}] shape {tuple(p.shape)}")
        return _Plan([params, grads, bufs, global_model if global_model is not None else [None] * T],
                     [p.numel() for p in params])

    plan = _cached_plan("sgdgroups", (params, grads, bufs, global_model), build)
    lr_a = np.asarray(lr, dtype=np.float32)
    mom_a = np.asarray(momentum, dtype=np.float32)
    damp_a = np.asarray(dampening, dtype=np.float64)
    wd_a = np.asarray(weight_decay, dtype=np.float32)
    fl_a = np.asarray(flags, dtype=np.int32)
    for a in (lr_a, mom_a, damp_a, wd_a, fl_a):
        if a.shape != (T,):
            raise ValueError(f"per-tensor scalars: expected {T} values, got shape {a.shape}")
    call("fa_sgd_prox_step_groups", plan.ptr(0), plan.ptr(1), plan.ptr(2),
         plan.ptr(3) if global_model is not None else None, plan.numel.ctypes.data, T, lr_a.ctypes.data,
         mom_a.ctypes.data, damp_a.ctypes.data, wd_a.ctypes.data, fl_a.ctypes.data, float(c), int(bool(fma)),
         _stream(params[0]))


def sgd_prox_step_groups_raw(pptr, gptr, bptr, globptr, numel, T: int, lr, momentum, dampening, weight_decay,
                             flags, c: float, fma: bool, stream):
    """fa_sgd_prox_step_groups on tables the caller has already validated (uint64 pointer arrays, int64
    element counts, per-tensor scalar arrays of the ABI's types): the per-step launch of a plan that
    ClientOptimizer.step_and_update checked when it built it (cloud/execution/optimizers.py)."""
    call("fa_sgd_prox_step_groups", pptr.ctypes.data, gptr.ctypes.data, bptr.ctypes.data,
         globptr.ctypes.data if globptr is not None else None, numel.ctypes.data, T, lr.ctypes.data,
         momentum.ctypes.data, dampening.ctypes.data, weight_decay.ctypes.data, flags.ctypes.data, float(c),
         int(bool(fma)), stream)


def dp_clip_coef(params, last, max_norm: float, norm_inf: bool, coef_out: torch.Tensor):
    """coef_out[0:3] <- (total norm of param - last, clip coefficient, apply flag) (fa_dp_clip_coef)."""
    params = list(params)
    last = list(last) if last is not None else [None] * len(params)

    def build():
        dev = _fp32_list(params, "param", coef_out.device)
        _fp32_list(last, "last", dev, allow_none=True)
        for i, (p, l) in enumerate(zip(params, last)):
            if l is not None and l.numel() != p.numel():
                raise ValueError(f"last[{i}] has {l.numel()} elements, param has {p.numel()}")
        plan = _Plan([params, last], [p.numel() for p in params])
        plan.ws_bytes = N.load().fa_dp_workspace_bytes(plan.numel.ctypes.data, plan.T)
        return plan

    plan = _cached_plan("dpnorm", (params, last), build)
    _dev(coef_out, torch.float32, "coef_out", 3, align=4)
    ws = torch.empty((plan.ws_bytes + 7) // 8, dtype=torch.float64, device=coef_out.device)
    call("fa_dp_clip_coef", plan.ptr(0), plan.ptr(1), plan.numel.ctypes.data, plan.T, float(max_norm),
         1 if norm_inf else 0, ptr(ws), ptr(coef_out), _stream(coef_out))


def dp_apply(params, last, upload, noise_offset, coef: torch.Tensor, sigma: float, seed: int,
             write_param: bool = True, scale_only: bool = False):
    """Recover (+ clip) and noise every tensor in one multi-tensor launch (fa_dp_apply)."""
    import numpy as np

    params = list(params)
    T = len(params)
    last = list(last) if last is not None else [None] * T
    upload = None if scale_only else list(upload)

    def build():
        dev = _fp32_list(params, "param", coef.device)
        _fp32_list(last, "last", dev, allow_none=True)
        for i, (p, l) in enumerate(zip(params, last)):
            if l is not None and l.numel() != p.numel():
                raise ValueError(f"last[{i}] has {l.numel()} elements, param has {p.numel()}")
        if upload is not None:
            _fp32_list(upload, "upload", dev)
            for i, (p, u) in enumerate(zip(params, upload)):
                if u.numel() != p.numel():
                    raise ValueError(f"upload[{i}] has {u.numel()} elements, param has {p.numel()}")
        plan = _Plan([params, last, upload], [p.numel() for p in params])
        plan.offs = np.asarray(noise_offset if noise_offset is not None else [0] * T, dtype=np.int64)
        return plan

    plan = _cached_plan(("dpapply", None if noise_offset is None else tuple(noise_offset)),
                        (params, last, upload), build)
    _dev(coef, torch.float32, "coef", 3, align=4)
    flags = (N.FA_DP_WRITE_PARAM if write_param else 0) | (N.FA_DP_SCALE_ONLY if scale_only else 0)
    call("fa_dp_apply", plan.ptr(0), plan.ptr(1), plan.ptr(2), plan.numel.ctypes.data, plan.offs.ctypes.data, T,
         ptr(coef), float(sigma), int(seed) & 0xFFFFFFFFFFFFFFFF, flags, _stream(coef))


def dp_noise_i64(xs, outs, noise_offset, sigma: float, seed: int):
    """outs[t] <- float64(xs[t]) + noise, all int64 entries in one launch (fa_dp_noise_i64)."""
    import numpy as np

    xs, outs = list(xs), list(outs)
    if not xs:
        return

    def build():
        dev = _fp32_list(xs, "x", dtype=torch.int64, align=8)
        _fp32_list(outs, "out", dev, dtype=torch.float64, align=8)
        for i, (x, o) in enumerate(zip(xs, outs)):
            if o.numel() != x.numel():
                raise ValueError(f"out[{i}] has {o.numel()} elements, x has {x.numel()}")
        plan = _Plan([xs, outs], [x.numel() for x in xs])
        plan.offs = np.asarray(noise_offset, dtype=np.int64)
        return plan

    plan = _cached_plan(("dpi64", tuple(noise_offset)), (xs, outs), build)
    call("fa_dp_noise_i64", plan.ptr(0), plan.ptr(1), plan.numel.ctypes.data, plan.offs.ctypes.data, plan.T,
         float(sigma), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream(xs[0]))


def dp_normals(out: torch.Tensor, seed: int, noise_offset: int = 0):
    _dev(out, torch.float32, "out", align=4)
    call("fa_dp_normals", ptr(out), out.numel(), int(seed) & 0xFFFFFFFFFFFFFFFF, int(noise_offset), _stream(out))
    return out
