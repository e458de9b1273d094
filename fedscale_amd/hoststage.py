"""Loader of the host staging extension (fedscale_amd/csrc/hoststage.c, built by ``__graft_entry__.build()``).

Like the HIP library, the module must carry the build id of the source in this tree (fedscale_amd/buildinfo.py);
a missing or stale module raises (no silent Python fallback).
"""
from __future__ import annotations

_mod = None


def load():
    global _mod
    if _mod is None:
        from . import buildinfo

        try:
            from . import _hoststage as m
        except ImportError as e:
            raise ImportError(f"{buildinfo.host_module_path()}: the host staging extension is not built "
                              f"(run `python __graft_entry__.py`): {e}") from None
        want = "FA_BUILD_ID=" + buildinfo.host_source_id()
        if m.build_id() != want:
            raise ImportError(f"{m.__file__}: build id {m.build_id()}, the tree's source builds {want} "
                              f"(stale; run `python __graft_entry__.py`)")
        _mod = m
    return _mod


def stage(values: list, dsts: list) -> int:
    """Copy values[i] into dsts[i] (validated: plain C-contiguous ndarray of the destination's shape and dtype);
    -1 when every entry was copied, else the index of the first entry left to the caller (nothing after it was
    written)."""
    return load().stage(values, dsts)
