"""ctypes binding of libfedagg.so — the C ABI declared in include/fedagg.h and include/fedclient.h.

This is the only way the package reaches the GPU.  There is no fallback: if the shared library is
missing or a call fails, a ``FedAggError`` is raised.  Build it with ``python __graft_entry__.py``
(or ``make -C fedscale_amd/csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FEDAGG_LIB", os.path.join(_HERE, "libfedagg.so"))
ABI_VERSION = 5  # fedagg.hip FA_ABI_VERSION

FA_ACCUMULATE = 1
FA_FINALIZE = 2
FA_YOGI_INIT = 4
FA_DP_WRITE_PARAM = 1
FA_DP_SCALE_ONLY = 2
FA_DT_F32, FA_DT_F64, FA_DT_I64 = 0, 1, 2
FA_SGD_NESTEROV, FA_SGD_FIRST = 1, 2


class FedAggError(RuntimeError):
    pass


_c_void_p, _i32, _i64, _f32, _f64, _u32 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float,
                                             ctypes.c_double, ctypes.c_uint32)

# name -> (restype, argtypes);  must list every symbol of include/fedagg.h and include/fedclient.h
SIGNATURES = {
    "fa_abi_version": (_i32, []),
    "fa_build_id": (ctypes.c_char_p, []),
    "fa_build_defs": (ctypes.c_char_p, []),
    "fa_last_error_string": (ctypes.c_char_p, []),
    "fa_pointer_kind": (_i32, [_c_void_p]),
    "fa_unranged_operands": (_i64, []),
    "fa_set_strict_operands": (_i32, [_i32]),
    "fa_reduce": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _c_void_p, _f32, _i32, _c_void_p]),
    "fa_reduce_mirror": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32, _i32,
                                _c_void_p]),
    "fa_reduce_launches": (_i64, [_i32, _i64, _i32]),
    "fa_reduce_parts": (_i32, [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32, _c_void_p,
                               _c_void_p]),
    "fa_qfed_launches": (_i64, [_i64, _i64, _i32]),
    "fa_reduce_yogi": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _f32, _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _f32, _f32, _f32, _f32, _f32, _i32, _c_void_p]),
    "fa_yogi_step": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _f32, _f32, _f32, _f32,
                            _f32, _i32, _c_void_p]),
    "fa_yogi_step_parts": (_i32, [_i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32, _f32,
                                  _f32, _f32, _f32, _i32, _c_void_p]),
    "fa_qfed_max_chunk": (_i32, []),
    "fa_qfed_workspace_bytes": (_i64, [_i32, _i64, _i64]),
    "fa_qfed_accumulate": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p, _f32, _c_void_p, _c_void_p,
                                  _c_void_p, _c_void_p, _i64, _i32, _c_void_p]),
    "fa_qfed_hs": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p]),
    "fa_qfed_finalize": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p]),
    "fa_side_accumulate": (_i32, [_c_void_p, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _i32,
                                  _c_void_p]),
    "fa_side_close": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _f64, _c_void_p, _c_void_p, _c_void_p]),
    "fa_side_yogi": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _f64, _f64,
                            _f64, _f64, _f64, _i32, _c_void_p]),
    "fa_side_qfed_accumulate": (_i32, [_c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _f32, _c_void_p,
                                       _c_void_p, _i32, _c_void_p]),
    "fa_side_qfed_finalize": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p]),
    "fa_fill_synthetic": (_i32, [_c_void_p, _i64, _i32, _i64, _u32, _i32, _f32, _f32, _c_void_p]),
    "fa_host_gather": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32]),
    "fa_host_register": (_i32, [_c_void_p, _i64]),
    "fa_host_unregister": (_i32, [_c_void_p]),
    "fa_h2d_pieces": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32]),
    "fa_pickle_strip": (_i64, [_c_void_p, _i64, _i64, _c_void_p, _i64, _c_void_p, _i32, _c_void_p]),
    "fa_prefix_box_combine": (_i32, [_c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p, _c_void_p, _i32,
                                     _c_void_p, _c_void_p]),
    "fa_sum_rows_f64": (_i32, [_c_void_p, _i64, _i32, _i64, _c_void_p, _c_void_p]),
    # shard group (RCCL over the GPUs of this process; tables are host arrays of device pointers / streams)
    "fa_rccl_available": (_i32, []),
    "fa_rccl_init": (_i32, [_i32, _c_void_p, ctypes.POINTER(_c_void_p)]),
    "fa_rccl_destroy": (_i32, [_c_void_p]),
    "fa_rccl_all_gather": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _i32, _c_void_p]),
    "fa_rccl_all_reduce": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _i32, _c_void_p]),
    "fa_rccl_gather": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i64, _i32, _i32, _c_void_p]),
    "fa_rccl_broadcast": (_i32, [_c_void_p, _c_void_p, _i64, _i32, _i32, _c_void_p]),
    "fa_rccl_comm_info": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p]),
    "fa_rccl_unique_id": (_i32, [_c_void_p]),
    "fa_rccl_init_rank": (_i32, [_i32, _c_void_p, _i32, _i32, ctypes.POINTER(_c_void_p)]),
    # include/fedclient.h (client-side handlers; pointer tables are host arrays)
    "fa_prox_update": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i32, _f32, _c_void_p]),
    "fa_sgd_prox_step": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _f32, _f32, _f64,
                                _f32, _i32, _i32, _f32, _i32, _c_void_p]),
    "fa_sgd_prox_step_groups": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p,
                                       _c_void_p, _c_void_p, _c_void_p, _c_void_p, _f32, _i32, _c_void_p]),
    "fa_dp_workspace_bytes": (_i64, [_c_void_p, _i32]),
    "fa_dp_clip_coef": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i32, _f32, _i32, _c_void_p, _c_void_p,
                               _c_void_p]),
    "fa_dp_apply": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _f32,
                           ctypes.c_uint64, _i32, _c_void_p]),
    "fa_dp_noise_i64": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _f32, ctypes.c_uint64,
                               _c_void_p]),
    "fa_dp_normals": (_i32, [_c_void_p, _i64, ctypes.c_uint64, _i64, _c_void_p]),
}

_lib = None
_info = None
_lock = threading.Lock()


def check_build(lib, path: str, tree: str = None) -> dict:
    """The library's build id against the one the sources of ``tree`` (default: this checkout) produce with the
    library's own extra definitions (fedscale_amd/buildinfo.py); FedAggError on a mismatch — a library built
    from other sources (a stale or foreign binary) is never used."""
    from . import buildinfo

    bid = lib.fa_build_id().decode(errors="replace")
    defs = lib.fa_build_defs().decode(errors="replace")
    tree = tree or buildinfo.ROOT
    try:
        want = buildinfo.source_id(defs, root=tree)
    except OSError as e:
        raise FedAggError(f"{path}: cannot verify its build id {bid}: the library's sources are not readable "
                          f"under {tree} ({e})")
    if bid != want:
        raise FedAggError(f"{path}: build id {bid} (defs {defs!r}), but the sources under {tree} build {want}: the "
                          f"library is stale or was built from other sources (run `python __graft_entry__.py`)")
    return {"path": os.path.abspath(path), "build_id": bid, "defs": defs, "verified_against": tree}


def load(path: str = None, tree: str = None):
    """Load (once) and type the shared library.  Raises FedAggError when it is absent, has another ABI version,
    or was not built from the sources in the tree (``check_build``)."""
    global _lib, _info
    with _lock:
        if _lib is not None and path is None and tree is None:
            return _lib
        path = path or LIB_PATH
        if not os.path.exists(path):
            raise FedAggError(f"{path} not found: the HIP extension is not built "
                              f"(run `python __graft_entry__.py` to build it; there is no CPU fallback)")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                raise FedAggError(f"{path}: no symbol {name} (an older build; run `python __graft_entry__.py`)")
            fn.restype = res
            fn.argtypes = args
        v = lib.fa_abi_version()
        if v != ABI_VERSION:
            raise FedAggError(f"{path}: ABI version {v}, expected {ABI_VERSION}")
        info = check_build(lib, path, tree)
        if os.environ.get("FEDAGG_STRICT_OPERANDS", "") not in ("", "0"):
            lib.fa_set_strict_operands(1)  # refuse device operands whose extent HIP cannot report (fa_device.h)
        if tree is None:
            _lib, _info = lib, info
        return lib


def build_info() -> dict:
    """{path, build_id, defs, verified_against} of the loaded library (loads it)."""
    load()
    return dict(_info)


def operand_stats() -> dict:
    """{unranged, strict}: device operands accepted so far without an extent check (HIP reports no range for VMM /
    expandable segments; fa_unranged_operands) and whether such operands are refused instead
    (fa_set_strict_operands, env FEDAGG_STRICT_OPERANDS=1)."""
    lib = load()
    prev = lib.fa_set_strict_operands(0)
    lib.fa_set_strict_operands(prev)
    return {"unranged": int(lib.fa_unranged_operands()), "strict": bool(prev)}


def call(name: str, *args):
    """Call an fa_* entry point; raise on a non-zero return code."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.fa_last_error_string().decode(errors="replace")
        raise FedAggError(f"{name} failed ({rc}): {msg}")
    return rc


def ptr(t) -> int:
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
