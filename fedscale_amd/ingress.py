"""Zero-copy unpickling of an executor's result payload (the aggregator's ``deserialize_response``).

The reference aggregator turns every UPLOAD_MODEL payload back into a dict with ``pickle.loads``
(aggregator.py:695-704, called at :994).  The executor made that payload with ``pickle.dumps`` of the
training result (torch_client.py:76-91, protocol 4): each ``update_weight`` array is a numpy
``_reconstruct`` + BUILD whose state carries the array's raw bytes as one BINBYTES/BINBYTES8 string, so
``pickle.loads`` copies every byte of the update once, single-threaded, before the aggregator has even
looked at it (≈45 MB per ResNet-18 update; DESIGN.md §5 measures it as the ingress bound).

``loads`` produces the same object tree without that copy:

1. ``fa_pickle_strip`` (csrc/ingress_host.cpp) walks the opcode stream and replaces each byte string of
   at least ``min_bytes`` with a 12-byte tag ``b"FAPB" + index`` while recording where the raw bytes lie;
2. the few-KiB stripped stream is unpickled with ``_Unpickler``, whose ``find_class`` hands numpy's
   ``_reconstruct`` a placeholder that records the BUILD state instead of copying it;
3. placeholders whose data is a tag become ``np.frombuffer`` views of the payload (read-only, kept
   alive by the payload ``bytes``), the others are rebuilt exactly as numpy would.

The result is element-for-element the object ``pickle.loads`` returns (tests/test_ingress.py), except
that large arrays are read-only views.  Anything the fast path does not recognise — another protocol,
out-of-band buffers, a tag that is not consumed by an array, an array nested inside an object the
post-pass cannot rebuild — falls back to ``pickle.loads`` of the original payload.
"""
from __future__ import annotations

import ctypes
import io
import math
import pickle

import numpy as np

from . import _native

#: byte strings shorter than this stay inline (small tensors, strings, scalars): below a few KiB numpy's
#: own rebuild (C) is cheaper than a view built in Python (measured on a ResNet-18 payload)
MIN_BYTES = 4096

#: payloads smaller than this go straight to pickle.loads: below about a MiB its single copy costs less
#: than the strip + placeholder pass (measured: 98 KB FEMNIST update 25 us vs 92 us; 45 MB ResNet-18
#: update 39 ms vs 1 ms on this container's host)
MIN_PAYLOAD = 1 << 20

_TAG = b"FAPB"
_RECONSTRUCT = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}


class _ArrayStub:
    """Stands in for ``numpy._core.multiarray._reconstruct(cls, shape, dtype)``; BUILD hands it the state."""

    __slots__ = ("reconstruct", "args", "state")

    def __init__(self, reconstruct, args):
        self.reconstruct = reconstruct
        self.args = args
        self.state = None

    def __setstate__(self, state):
        self.state = state


class _Unpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _RECONSTRUCT:
            real = super().find_class(module, name)
            return lambda *args: _ArrayStub(real, args)
        return super().find_class(module, name)


_LEAVES = frozenset((str, int, float, bool, bytes, type(None), complex))


class _Fallback(Exception):
    pass


class _Materializer:
    def __init__(self, payload, regions):
        self.payload = payload
        self.regions = regions
        self.used = 0
        self.done = {}  # id(stub) -> array: a memoised array (pickled once, referenced twice) stays one object

    def array(self, stub: _ArrayStub):
        a = self.done.get(id(stub))
        if a is None:
            a = self.done[id(stub)] = self._build(stub)
        return a

    def _build(self, stub: _ArrayStub):
        if stub.state is None:
            raise _Fallback("array without BUILD state")
        st = stub.state
        if not (isinstance(st, tuple) and len(st) == 5):
            raise _Fallback("unexpected ndarray state")
        version, shape, dtype, fortran, data = st
        if isinstance(data, (bytes, bytearray)) and len(data) == 12 and data[:4] == _TAG:
            cls = stub.args[0] if stub.args else np.ndarray
            if cls is not np.ndarray or dtype.hasobject:
                raise _Fallback("tagged data on a non-plain array")
            idx = int.from_bytes(data[4:], "little")
            if idx >= len(self.regions):
                raise _Fallback("tag index out of range")
            off, n = self.regions[idx]
            count = math.prod(shape)
            if count * dtype.itemsize != n:
                raise _Fallback("tagged byte count does not match the array")
            self.used += 1
            a = np.frombuffer(self.payload, dtype=dtype, count=count, offset=off)
            return a.reshape(shape, order="F") if fortran else a.reshape(shape)
        a = stub.reconstruct(*stub.args)  # exactly what pickle.loads does for an inline array
        a.__setstate__(st)
        return a

    def walk(self, obj, depth=0):
        if depth > 64:
            raise _Fallback("nesting too deep")
        t = type(obj)
        if t is _ArrayStub:
            return self.array(obj)
        if t is dict:  # (the upload's name -> array dict: leaves handled inline, no call per array)
            for k, v in obj.items():
                if type(k) is _ArrayStub:
                    raise _Fallback("array used as a key")
                tv = type(v)
                if tv is _ArrayStub:
                    obj[k] = self.array(v)
                elif tv not in _LEAVES:
                    nv = self.walk(v, depth + 1)
                    if nv is not v:
                        obj[k] = nv
            return obj
        if t is list:
            for i, v in enumerate(obj):
                tv = type(v)
                if tv is _ArrayStub:
                    obj[i] = self.array(v)
                elif tv not in _LEAVES:
                    nv = self.walk(v, depth + 1)
                    if nv is not v:
                        obj[i] = nv
            return obj
        if t is tuple:
            items = [self.walk(v, depth + 1) for v in obj]
            if any(a is not b for a, b in zip(items, obj)):
                return tuple(items)
            return obj
        if t in _LEAVES:
            return obj
        if isinstance(obj, (np.generic, np.ndarray)):
            return obj
        # any other object could hold a stub where the post-pass cannot see it
        raise _Fallback(f"cannot walk {t.__name__}")


def _strip_call(lib, payload, min_bytes, out, out_cap, regions, max_regions, nreg):
    n = lib.fa_pickle_strip(payload, len(payload), min_bytes, out, out_cap, regions, max_regions,
                            ctypes.byref(nreg))
    if n < 0:
        msg = lib.fa_last_error_string().decode(errors="replace")
        raise _native.FedAggError(f"fa_pickle_strip failed ({n}): {msg}")
    return int(n)


def strip(payload: bytes, min_bytes: int = MIN_BYTES):
    """(stripped stream, [(offset, length), ...]) of ``payload`` via fa_pickle_strip (raises FedAggError).

    ``payload`` is passed by pointer (ctypes hands the ``bytes`` buffer over without copying)."""
    lib = _native.load()
    nreg = ctypes.c_int32(0)
    out_cap, max_regions = 1 << 16, 512
    out = ctypes.create_string_buffer(out_cap)
    regions = (ctypes.c_int64 * (2 * max_regions))()
    n = _strip_call(lib, payload, min_bytes, out, out_cap, regions, max_regions, nreg)
    if n > out_cap or nreg.value > max_regions:  # second pass with exact sizes
        out_cap, max_regions = max(n, 1), max(nreg.value, 1)
        out = ctypes.create_string_buffer(out_cap)
        regions = (ctypes.c_int64 * (2 * max_regions))()
        n = _strip_call(lib, payload, min_bytes, out, out_cap, regions, max_regions, nreg)
    r = nreg.value
    return ctypes.string_at(out, n), [(regions[2 * i], regions[2 * i + 1]) for i in range(r)]


def loads(payload, min_bytes: int | None = None, min_payload: int | None = None):
    """``pickle.loads(payload)`` without copying the large byte strings (module docstring)."""
    min_bytes = MIN_BYTES if min_bytes is None else int(min_bytes)
    min_payload = MIN_PAYLOAD if min_payload is None else int(min_payload)
    if (type(payload) is not bytes or len(payload) < max(2 * min_bytes, min_payload)
            or payload[:2] != b"\x80\x04"):
        return pickle.loads(payload)
    try:
        stream, regions = strip(payload, min_bytes)
    except Exception:
        return pickle.loads(payload)
    if not regions:
        return pickle.loads(payload)
    try:
        obj = _Unpickler(io.BytesIO(stream)).load()
        m = _Materializer(payload, regions)
        obj = m.walk(obj)
        if m.used != len(regions):
            raise _Fallback("not every stripped byte string became an array")
        return obj
    except Exception:
        return pickle.loads(payload)
