"""Flat device layout of a state_dict ("bucket") and the client-update staging area.

HBM layout:
  * fp32 entries of the state_dict, concatenated in state_dict order -> one flat vector of P elements.
    A rank owns the contiguous slice [p0, p1) of it: the boundaries are r*P/N rounded to the nearest
    multiple of 64, so every slice starts 256-byte aligned and holds P/N floats within 64 (shard_bounds).
    Every rank's row stride ``ld`` is the same (the largest slice rounded up to 64 floats) and the padding is
    kept at zero, so the reassembly is a plain all-gather of ld floats per rank followed by unshard().
  * non-fp32 entries (int64 BatchNorm ``num_batches_tracked`` ...) -> the "side table" of Q int64
    elements, replicated on every rank (it is a few hundred bytes).
  * a round's client updates live client-major: x[slot, :] (fp32, [capacity, ld]) and xi[slot, :]
    (int64, [capacity, Q]).  Positional mapping to state_dict keys follows
    torch_model_adapter.py:31-34 (weights[i] <-> i-th key).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import hoststage

ALIGN = 64  # floats: 256-byte rows, and the shard granule


class _NullCtx:
    __slots__ = ()

    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL_CTX = _NullCtx()


def default_pack_workers() -> int:
    """Host threads for the ingress gather (FEDAGG_PACK_WORKERS overrides; the GPU box gives a GPU 16)."""
    env = os.environ.get("FEDAGG_PACK_WORKERS")
    if env:
        return max(1, int(env))
    return max(1, min(8, (os.cpu_count() or 2) // 2))


def round_up(n: int, m: int) -> int:
    return (n + m - 1) // m * m


def shard_bounds(P: int, world: int) -> List[int]:
    """[b_0 = 0, b_1, ..., b_world = P]: b_r = r*P/world rounded to the nearest multiple of ALIGN (ties down), so
    every slice [b_r, b_r+1) starts 64-float aligned and |slice - P/world| <= 64 (each boundary is within 32 of
    its ideal).  Rounds 1-4 cut equal slices of round_up(ceil(P/world), 64), which left the last one up to
    64*(world-1) floats short (256 at 100 M over 8)."""
    if world < 1:
        raise ValueError("world >= 1")
    b = [0]
    for r in range(1, world):
        b.append(min(P, max(b[-1], ((2 * r * P + ALIGN * world - 1) // (2 * ALIGN * world)) * ALIGN)))
    b.append(P)
    return b


def shard_ld(P: int, world: int) -> int:
    """The row stride every rank of a P-float model over ``world`` uses: the largest slice, rounded up to 64."""
    b = shard_bounds(P, world)
    return max(ALIGN, round_up(max(b[r + 1] - b[r] for r in range(world)), ALIGN))


@dataclass
class Entry:
    index: int
    name: str
    shape: Tuple[int, ...]
    dtype: torch.dtype
    offset: int  # into the fp32 vector (kind 'f') or the side table (kind 'i')
    numel: int
    kind: str  # 'f' fp32 bucket | 'i' int64 side table


_SUPPORTED = {torch.float32: "f", torch.int64: "i"}
_F32, _I64 = np.dtype(np.float32), np.dtype(np.int64)


class BucketLayout:
    def __init__(self, names: Sequence[str], shapes: Sequence[Sequence[int]], dtypes: Sequence[torch.dtype],
                 rank: int = 0, world: int = 1):
        if world < 1 or not (0 <= rank < world):
            raise ValueError(f"bad shard ({rank}, {world})")
        self.entries: List[Entry] = []
        pf = pi = 0
        for i, (n, s, d) in enumerate(zip(names, shapes, dtypes)):
            if d not in _SUPPORTED:
                raise NotImplementedError(
                    f"state_dict entry {n!r} has dtype {d}; the device path supports float32 parameters/buffers "
                    f"and int64 buffers (FedScale models)")
            numel = int(np.prod(s)) if len(s) else 1
            kind = _SUPPORTED[d]
            e = Entry(i, n, tuple(int(v) for v in s), d, pf if kind == "f" else pi, numel, kind)
            if kind == "f":
                pf += numel
            else:
                pi += numel
            self.entries.append(e)
        self.names = list(names)
        self.T = len(self.entries)
        self.P_full = pf
        self.Q = pi
        self.rank, self.world = rank, world
        self.bounds = shard_bounds(pf, world)  # balanced, 64-aligned slice boundaries
        self.p0, self.p1 = self.bounds[rank], self.bounds[rank + 1]
        self.P = self.p1 - self.p0
        self.ld = shard_ld(pf, world)  # row stride of every rank (multiple of 64, >= every P)
        self.ldq = max(1, self.Q)
        self.f_entries = [e for e in self.entries if e.kind == "f"]
        self.i_entries = [e for e in self.entries if e.kind == "i"]
        # static half of host_gather_plan: per entry (index, name, shape, kind, source byte offset of this
        # rank's slice or -1 when the entry has none); destination offsets and sizes of the copied pieces
        self._gather_entries = []
        offs, sizes = [], []
        for e in self.entries:
            src = -1
            if e.kind == "f":
                lo, hi = max(e.offset, self.p0), min(e.offset + e.numel, self.p1)
                if lo < hi:
                    src = 4 * (lo - e.offset)
                    offs.append(4 * (lo - self.p0))
                    sizes.append(4 * (hi - lo))
            self._gather_entries.append((e.index, e.name, e.shape, e.kind, src, e.offset))
        self._gather_offs = np.asarray(offs, dtype=np.int64)
        self._gather_sizes = np.asarray(sizes, dtype=np.int64)

    def unshard(self, gathered):
        """The P_full-float model from an all-gather of every rank's ld-float row (rank r's slice is the first
        P_r floats of row r): a view when the slices fill their rows, else one compaction copy (torch or numpy)."""
        if self.world == 1:
            return gathered[:self.P_full]
        ld, b = self.ld, self.bounds
        if all(b[r + 1] - b[r] == ld for r in range(self.world - 1)):
            return gathered[:self.P_full]
        parts = [gathered[r * ld:r * ld + (b[r + 1] - b[r])] for r in range(self.world)]
        return torch.cat(parts) if isinstance(gathered, torch.Tensor) else np.concatenate(parts)

    @classmethod
    def from_state_dict(cls, sd, rank: int = 0, world: int = 1) -> "BucketLayout":
        return cls(list(sd.keys()), [tuple(v.shape) for v in sd.values()], [v.dtype for v in sd.values()],
                   rank, world)

    def same_structure(self, names, shapes) -> bool:
        return list(names) == self.names and [tuple(s) for s in shapes] == [e.shape for e in self.entries]

    # ---- host-side packing ----------------------------------------------------------------------
    def values_of(self, update) -> list:
        """dict name->array | list -> list in state_dict order (aggregator.py:494-496)."""
        if type(update) is dict:
            update = list(update.values())
        if len(update) != self.T:
            raise ValueError(f"update has {len(update)} tensors, the model has {self.T}")
        return update

    def pack_host(self, values: list, f_out: np.ndarray, i_out: np.ndarray, workers: int = 1):
        """Copy this rank's slice of the fp32 entries into f_out[:P] and the int entries into i_out[:Q].

        The fp32 byte ranges go to ``fa_host_gather`` (native, multi-threaded memcpy into the pinned row):
        a single memcpy stream is slower than the H2D copy engine."""
        self.run_host_gather(self.host_gather_plan(values), f_out, i_out, workers)

    def host_gather_plan(self, values: list):
        """Validate an update (shapes, dtypes) and list its byte ranges for ``run_host_gather``: the cheap,
        synchronous half of pack_host (the caller's errors surface here, at the add, as in the reference).
        The plan holds a reference to every source array until the copy has run."""
        values = self.values_of(values)
        ptrs, keep, side = [], [], []
        for idx, name, shape, kind, src, off in self._gather_entries:
            a = values[idx]
            if type(a) is not np.ndarray:
                if isinstance(a, torch.Tensor):
                    a = a.detach().cpu().numpy()
                a = np.asarray(a)
            if a.shape != shape:
                raise ValueError(f"{name}: shape {tuple(a.shape)} != model shape {shape}")
            if kind == "f":
                if a.dtype != _F32:
                    raise TypeError(f"{name}: dtype {a.dtype}, the model entry is float32")
                if src >= 0:
                    if not a.flags.c_contiguous:
                        a = np.ascontiguousarray(a)
                    keep.append(a)
                    ptrs.append(a.__array_interface__["data"][0] + src)
            else:
                if a.dtype != _I64:
                    raise TypeError(f"{name}: dtype {a.dtype}, the model entry is int64")
                side.append((off, a.reshape(-1)))
        return (np.array(ptrs, dtype=np.uint64), self._gather_offs, self._gather_sizes, keep, side)

    def run_host_gather(self, plan, f_out: np.ndarray, i_out: np.ndarray, workers: int = 1):
        """The copying half of pack_host (no Python-level validation left; releases the GIL in C)."""
        from . import _native

        ps, po, pn, keep, side = plan
        if not f_out.flags.c_contiguous or f_out.dtype != np.float32 or f_out.size < self.P:
            raise ValueError("pack_host: f_out must be a contiguous float32 array of >= P elements")
        for off, a in side:
            i_out[off:off + a.size] = a
        if len(ps):
            if len(ps) != len(po):
                raise ValueError("pack_host: plan and layout disagree")
            ptr = lambda a: a.__array_interface__["data"][0]  # noqa: E731 (cheaper than .ctypes.data)
            _native.call("fa_host_gather", ptr(f_out), ptr(ps), ptr(po), ptr(pn), len(ps), int(workers))
        del keep

    def pack_device(self, values: list, f_dst: torch.Tensor, i_dst: torch.Tensor):
        """Same as pack_host for a list of tensors already resident on this device (D2D copies)."""
        values = self.values_of(values)
        for e in self.entries:
            v = values[e.index]
            if not isinstance(v, torch.Tensor):
                v = torch.as_tensor(np.asarray(v))
            if tuple(v.shape) != e.shape:
                raise ValueError(f"{e.name}: shape {tuple(v.shape)} != model shape {e.shape}")
            if v.dtype != e.dtype:
                raise TypeError(f"{e.name}: dtype {v.dtype} != model dtype {e.dtype}")
            flat = v.reshape(-1)
            if e.kind == "f":
                lo, hi = max(e.offset, self.p0), min(e.offset + e.numel, self.p1)
                if lo < hi:
                    f_dst[lo - self.p0:hi - self.p0].copy_(flat[lo - e.offset:hi - e.offset], non_blocking=True)
            else:
                i_dst[e.offset:e.offset + e.numel].copy_(flat, non_blocking=True)

    def unpack(self, f_full: torch.Tensor, i_side: torch.Tensor) -> list:
        """Views of a FULL (gathered, length >= P_full) fp32 vector + side table as state_dict tensors."""
        out = []
        for e in self.entries:
            src = f_full if e.kind == "f" else i_side
            out.append(src[e.offset:e.offset + e.numel].view(e.shape))
        return out


class HostRow:
    """One arriving update gathered ONCE into pinned host rows covering the whole model: ``f`` the fp32
    bucket (length >= P_full), ``i`` the side table.  A model sharded over the devices of one process
    hands the same row to every part's ``ClientStaging.put``: each part copies its slice [p0, p1) to its own
    device, so an upload crosses PCIe once, split over the GPUs' links.  ``pending`` collects the events of
    those copies; the row is rewritten only after all of them (``wait``)."""

    __slots__ = ("f", "i", "f_np", "i_np", "pending")

    def __init__(self, ld: int, ldq: int):
        self.f = torch.zeros(ld, dtype=torch.float32).pin_memory()
        self.i = torch.zeros(ldq, dtype=torch.int64).pin_memory()
        self.f_np, self.i_np = self.f.numpy(), self.i.numpy()
        self.pending = []

    def wait(self):
        for ev in self.pending:
            ev.synchronize()
        self.pending = []


class RegisteredUpload:
    """One arriving update whose LARGE fp32 entries the GPUs' copy engines read straight out of the host memory
    that holds them — the executor's payload, registered in place (``fa_host_register``) — while the small
    entries and the side table are gathered into a pinned ``row`` (round 4, N-GPU ingress: one host-DRAM pass per
    large byte instead of three).  ``segs``: the whole-model segments (row offset, elements, large-entry index or
    -1 for "from the row"), fixed per layout; ``src``: the address of every large entry's first element.  Each
    part's ``ClientStaging.put`` copies the pieces of its slice and appends its event to ``events`` (and to the
    row's ``pending``); the registration is released once they have all completed."""

    __slots__ = ("row", "segs", "src", "events")

    def __init__(self, row: "HostRow", segs, src: np.ndarray):
        self.row, self.segs, self.src, self.events = row, segs, src, []


class PieceSegments:
    """Whole-model segments of a layout for ``RegisteredUpload``: fp32 entries of at least ``min_bytes`` are their
    own segment (read from the registered upload), runs of smaller entries one segment each (read from the pinned
    row).  ``large``: the fp32-entry positions (in ``layout.f_entries`` order) of the large entries."""

    def __init__(self, layout: "BucketLayout", min_bytes: int):
        if layout.world != 1:
            raise ValueError("PieceSegments: a whole-model layout (the coordinator's)")
        self.large = [j for j, e in enumerate(layout.f_entries) if e.numel and 4 * e.numel >= min_bytes]
        li = {j: n for n, j in enumerate(self.large)}
        segs = []
        for j, e in enumerate(layout.f_entries):
            if e.numel == 0:
                continue
            if j in li:
                segs.append((e.offset, e.numel, li[j]))
            elif segs and segs[-1][2] < 0 and segs[-1][0] + segs[-1][1] == e.offset:
                segs[-1] = (segs[-1][0], segs[-1][1] + e.numel, -1)
            else:
                segs.append((e.offset, e.numel, -1))
        self.segs = segs
        # positions in host_gather_plan's piece lists (one piece per NON-EMPTY fp32 entry of a whole-model layout)
        piece, k = {}, 0
        for j, e in enumerate(layout.f_entries):
            if e.numel:
                piece[j] = k
                k += 1
        self.large_pieces = [piece[j] for j in self.large]
        self.small_pieces = np.asarray([piece[j] for j in piece if j not in li], dtype=np.int64)

    def part_plan(self, p0: int, p1: int):
        """(dst byte offsets in the part's row, byte counts, large index or -1, source byte offsets) of the pieces
        of slice [p0, p1): relative to the large entry's first byte, or to the start of the pinned row."""
        dst, nb, kind, soff = [], [], [], []
        for off, n, k in self.segs:
            lo, hi = max(off, p0), min(off + n, p1)
            if lo >= hi:
                continue
            dst.append(4 * (lo - p0))
            nb.append(4 * (hi - lo))
            kind.append(k)
            soff.append(4 * (lo - off) if k >= 0 else 4 * lo)
        return (np.asarray(dst, dtype=np.uint64), np.asarray(nb, dtype=np.int64), np.asarray(kind, dtype=np.int64),
                np.asarray(soff, dtype=np.uint64))


class ClientStaging:
    """Device staging area for up to ``capacity`` client updates of one round (chunk).

    Host -> device ingress goes through a ring of pinned host buffers; each H2D copy is enqueued on the
    caller's current stream, so stream order guarantees a slot is not overwritten while a kernel still
    reads it.  With ``async_ingress`` the gather into the pinned row and the H2D enqueue run on one
    background thread, in arrival order: ``put`` validates the update and returns.  It is off by default:
    measured with the executor's pickled payloads, the background copy and the main thread's
    ``pickle.loads`` (aggregator.py:704) serialise on the GIL and halve the rate.
    ``drain()`` waits for every queued copy to be enqueued; DeviceRound calls it before any kernel reads
    the slots.  Small staging areas (``bulk``, <= BULK_MAX_BYTES) skip the per-update H2D: updates are
    gathered into a pinned mirror of the whole area and ``drain()`` moves the pending rows in one copy.
    """

    #: staging areas of at most this many bytes take the bulk path: every update is gathered into a
    #: pinned mirror of the whole area and one H2D per drain() moves all pending rows (small models pay
    #: the per-update copy-enqueue latency otherwise)
    BULK_MAX_BYTES = 64 << 20
    #: single-chunk rounds of at most this many staged bytes are read by the kernels straight out of the pinned
    #: mirror (no H2D): at config 1's 1 MB the copy is mostly latency (26.5 us of the 49.8 us device floor)
    ZERO_COPY_MAX_BYTES = 4 << 20

    def __init__(self, layout: BucketLayout, device, capacity: int, ring: int = 2,
                 pack_workers: Optional[int] = None, async_ingress: bool = False, bulk: Optional[bool] = None,
                 dstream=None):
        """``dstream``: the owning adapter's DeviceStream; the staging's buffers, H2D copies and events are
        issued on it (None: the caller's current stream)."""
        self.dstream = dstream
        if dstream is None:
            self._init(layout, device, capacity, ring, pack_workers, async_ingress, bulk)
        else:
            with dstream:
                self._init(layout, device, capacity, ring, pack_workers, async_ingress, bulk)

    def _on(self):
        """Context for GPU work: the dstream, unless it is already current (or there is none)."""
        ds = self.dstream
        if ds is None:
            return _NULL_CTX
        from .state import DeviceStream

        return _NULL_CTX if DeviceStream.current() is ds else ds

    def _init(self, layout, device, capacity, ring, pack_workers, async_ingress, bulk):
        self.layout = layout
        self.pack_workers = pack_workers or default_pack_workers()
        self.device = torch.device(device)
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.capacity = int(capacity)
        self.generation = 0  # bumped by every DeviceRound that takes the slots over
        self.side_scratch = None  # (int64, float64) side-table sums of FedAvg / FedBuff rounds, reused
        self.x = torch.zeros(self.capacity, layout.ld, dtype=torch.float32, device=self.device)
        self.xi = torch.zeros(self.capacity, layout.ldq, dtype=torch.int64, device=self.device)
        self._ring = []  # pinned rows for host updates, allocated on the first one (a part of a sharded
        self._ring_n = ring  # model is fed HostRows by its coordinator and never needs its own)
        self._next = 0
        self._row_evs = {}  # id(HostRow) -> event of this part's last H2D out of that row
        self.async_ingress = async_ingress
        self._pool = None
        nbytes = self.capacity * (layout.ld * 4 + layout.ldq * 8)
        self.bulk = (not async_ingress and nbytes <= self.BULK_MAX_BYTES) if bulk is None else bool(bulk)
        if self.bulk and async_ingress:
            raise ValueError("bulk staging and async_ingress are exclusive")
        self._views = None
        if self.bulk:
            self._hx = torch.zeros(self.capacity, layout.ld, dtype=torch.float32).pin_memory()
            self._hxi = torch.zeros(self.capacity, layout.ldq, dtype=torch.int64).pin_memory()
            self._hx_np, self._hxi_np = self._hx.numpy(), self._hxi.numpy()
            self._bulk_lo = self._bulk_hi = 0  # host rows [lo, hi) not yet copied to the device
            self._bulk_ev = torch.cuda.Event()
            self._bulk_busy = False  # an H2D out of the mirror may still be running
            # whole-model layouts: per slot, numpy views of every entry's place in the pinned mirror, so a
            # small update (config 1: 8 tensors, 98 KB) is validated and copied entry by entry in a few µs
            # instead of building a gather plan and crossing into the native gather
            self._views = [None] * self.capacity if layout.world == 1 else None  # built per slot on first use
            self._dsts = [None] * self.capacity  # the views alone (hoststage.stage's destinations)
            self._stage = hoststage.load().stage  # the native call itself (no Python wrapper per upload)
            self.head_acc = None  # DeviceRound._launch_head's running chain (one per staging, reused)
            self._head_key = None

    def _copy_in(self, slot, plan, r, stream, on_current: bool):
        """Gather into ring entry r's pinned rows, then enqueue their H2D on ``stream`` and record r's event
        (the caller has waited for that event's previous record, so re-recording it is safe)."""
        lay = self.layout
        hf, hi, ev = r[0], r[1], r[6]
        lay.run_host_gather(plan, r[4], r[5], workers=self.pack_workers)
        if on_current:  # the common case: no stream switch needed
            self.x[slot, :lay.P].copy_(hf[:lay.P], non_blocking=True)
            if lay.Q:
                self.xi[slot, :lay.Q].copy_(hi[:lay.Q], non_blocking=True)
        else:
            with torch.cuda.stream(stream):
                self.x[slot, :lay.P].copy_(hf[:lay.P], non_blocking=True)
                if lay.Q:
                    self.xi[slot, :lay.Q].copy_(hi[:lay.Q], non_blocking=True)
        ev.record(stream)
        return ev

    def put_small(self, slot: int, update: dict) -> bool:
        """A small whole-model upload (a dict, config 1) into its slot of the pinned mirror; False: not taken (the
        caller goes on with ``put``, which converts or raises as for any upload)."""
        values = list(update.values())
        return len(values) == self.layout.T and self._put_bulk_views(slot, values)

    def put(self, slot: int, update):
        if self._views is not None and type(update) is dict and self.put_small(slot, update):
            return  # a small whole-model upload (config 1): the common case
        if type(update) is HostRow:
            return self._put_row(slot, update)
        if type(update) is RegisteredUpload:
            return self._put_registered(slot, update)
        lay = self.layout
        values = lay.values_of(update)
        if self.bulk and self._views is not None and self._put_bulk_views(slot, values):
            return
        on_dev = [isinstance(v, torch.Tensor) and v.device == self.device for v in values]
        if all(on_dev):
            with self._on():
                if self.dstream is not None:
                    self.dstream.wait_caller()  # the caller's device tensors
                self.drain()  # keep the slots' arrival order with any queued host copies
                lay.pack_device(values, self.x[slot], self.xi[slot])
            return
        plan = lay.host_gather_plan(values)  # validation errors surface here, synchronously
        if self.bulk:
            self._put_bulk(slot, plan)
            return
        if not self._ring:
            for _ in range(self._ring_n):
                hf = torch.zeros(lay.ld, dtype=torch.float32).pin_memory()
                hi = torch.zeros(lay.ldq, dtype=torch.int64).pin_memory()
                # pinned rows, event of the last H2D, pending job, numpy views of the rows, the row's own event
                self._ring.append([hf, hi, None, None, hf.numpy(), hi.numpy(), torch.cuda.Event()])
        r = self._ring[self._next]
        if r[3] is not None:  # the job that last used this pinned row
            r[2] = r[3].result()
            r[3] = None
        if r[2] is not None:
            r[2].synchronize()  # the previous H2D out of this pinned row has completed
        stream = self.dstream.stream if self.dstream is not None else torch.cuda.current_stream(self._dev_index)
        if self.async_ingress:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor

                self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="fedagg-ingress")
            r[3] = self._pool.submit(self._copy_in, slot, plan, r, stream, False)
        else:
            with self._on():
                r[2] = self._copy_in(slot, plan, r, stream, True)
        self._next = (self._next + 1) % len(self._ring)

    def _put_row(self, slot: int, row: "HostRow"):
        """An update already gathered into a pinned row of the whole model (``HostRow``): copy this part's
        slice [p0, p1) and the side table to the device (one H2D on this device's stream and link)."""
        lay = self.layout
        if self.bulk:
            self._claim_bulk(slot)
            self._hx_np[slot, :lay.P] = row.f_np[lay.p0:lay.p1]
            if lay.Q:
                self._hxi_np[slot, :lay.Q] = row.i_np[:lay.Q]
            self._bulk_hi = slot + 1
            return
        with self._on():  # this part's device and stream: the copy crosses this GPU's own link
            self.x[slot, :lay.P].copy_(row.f[lay.p0:lay.p1], non_blocking=True)
            if lay.Q:
                self.xi[slot, :lay.Q].copy_(row.i[:lay.Q], non_blocking=True)
            ev = self._row_evs.get(id(row))
            if ev is None:
                ev = self._row_evs[id(row)] = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self._dev_index))
        row.pending.append(ev)

    def _put_registered(self, slot: int, up: "RegisteredUpload"):
        """This part's slice of an upload read partly from its registered host memory (``RegisteredUpload``):
        one native call enqueues every piece's H2D on this device's stream (``fa_h2d_pieces``)."""
        from . import _native

        lay = self.layout
        plan = getattr(self, "_reg_plan", None)
        if plan is None or plan[0] is not up.segs:
            plan = self._reg_plan = (up.segs, up.segs.part_plan(lay.p0, lay.p1))
        dst, nb, kind, soff = plan[1]
        rowbase = np.uint64(up.row.f.data_ptr())
        src = np.where(kind >= 0, up.src[np.maximum(kind, 0)] + soff, rowbase + soff).astype(np.uint64)
        if self.bulk:  # a small staging area keeps its pinned mirror: the pieces are host copies into it
            self._claim_bulk(slot)
            mirror = self._hx_np[slot]
            for d, n, s_ in zip(dst.tolist(), nb.tolist(), src.tolist()):
                ctypes_src = np.ctypeslib.as_array((ctypes.c_float * (n // 4)).from_address(s_))
                mirror[d // 4:(d + n) // 4] = ctypes_src
            if lay.Q:
                self._hxi_np[slot, :lay.Q] = up.row.i_np[:lay.Q]
            self._bulk_hi = slot + 1
            return
        with self._on():
            st = torch.cuda.current_stream(self._dev_index)
            if len(nb):
                dsts = (np.uint64(self.x[slot].data_ptr()) + dst).astype(np.uint64)
                sidx = np.zeros(len(nb), dtype=np.int32)
                streams = np.asarray([st.cuda_stream], dtype=np.uint64)
                _native.call("fa_h2d_pieces", dsts.ctypes.data, src.ctypes.data, nb.ctypes.data, sidx.ctypes.data,
                             len(nb), streams.ctypes.data, 1)
            if lay.Q:
                self.xi[slot, :lay.Q].copy_(up.row.i[:lay.Q], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        up.row.pending.append(ev)
        up.events.append(ev)

    def _put_bulk_views(self, slot: int, values) -> bool:
        """Small whole-model update of plain numpy arrays: validate (shape, dtype) and copy each entry into
        its pinned view — in one native call (fedscale_amd/csrc/hoststage.c), which stops at the first entry it
        does not take (not a plain C-contiguous array of the entry's shape and dtype) and leaves it and the rest
        to the loop below.  False when an entry is not a plain ndarray: the general path converts and reports it
        (and rewrites every entry of the slot)."""
        views = self._views[slot]
        if views is None:
            views = self._views[slot] = [
                (e.name, e.shape, _F32 if e.kind == "f" else _I64,
                 (self._hx_np[slot, e.offset:e.offset + e.numel] if e.kind == "f" else
                  self._hxi_np[slot, e.offset:e.offset + e.numel]).reshape(e.shape))
                for e in self.layout.entries]
            self._dsts[slot] = [v[3] for v in views]
        if type(values) is not list:
            values = list(values)
        if self._bulk_busy or self._bulk_hi != slot or slot == self._bulk_lo:
            self._claim_bulk(slot)  # (the steady state — the next contiguous slot, the mirror idle — needs none)
        # validated entry by entry as it is copied: an error leaves the slot uncommitted (_bulk_hi is not
        # advanced), so the next update written to it overwrites every entry
        i = self._stage(values, self._dsts[slot])
        if i < 0:
            self._bulk_hi = slot + 1
            return True
        for (name, shape, dt, dst), a in zip(views[i:], values[i:]):
            if type(a) is not np.ndarray:
                return False
            if a.shape != shape:
                raise ValueError(f"{name}: shape {tuple(a.shape)} != model shape {shape}")
            if a.dtype != dt:
                raise TypeError(f"{name}: dtype {a.dtype}, the model entry is {'float32' if dt == _F32 else 'int64'}")
            dst[...] = a
        self._bulk_hi = slot + 1
        return True

    def _claim_bulk(self, slot: int):
        if self._bulk_busy:  # the mirror's previous H2D must finish before its rows are rewritten
            self._bulk_ev.synchronize()
            self._bulk_busy = False
        if self._bulk_hi > self._bulk_lo and slot != self._bulk_hi:
            self.drain()  # keep pending rows contiguous
        if self._bulk_hi == self._bulk_lo:
            self._bulk_lo = self._bulk_hi = slot

    def _put_bulk(self, slot: int, plan):
        lay = self.layout
        self._claim_bulk(slot)
        lay.run_host_gather(plan, self._hx_np[slot], self._hxi_np[slot], workers=self.pack_workers)
        self._bulk_hi = slot + 1

    def _drain_bulk(self):
        lo, hi = self._bulk_lo, self._bulk_hi
        if hi > lo:
            with self._on():
                # whole rows: one contiguous block (the mirror's padding columns are zero, as on the device)
                self.x[lo:hi].copy_(self._hx[lo:hi], non_blocking=True)
                if self.layout.Q:
                    self.xi[lo:hi].copy_(self._hxi[lo:hi], non_blocking=True)
                self._bulk_ev.record(torch.cuda.current_stream(self._dev_index))
            self._bulk_busy = True
            self._bulk_lo = self._bulk_hi = 0

    def host_rows(self, n: int):
        """(x, xi) of the pinned mirror when slots [0, n) were all written since the last drain and are small
        enough for the round's kernels to read them over PCIe (``ZERO_COPY_MAX_BYTES``): the H2D copy and its
        latency are skipped (fa_reduce_mirror, tools/c1_zero_copy_probe.py).  None otherwise.  A caller that
        uses them calls ``release_host_rows()`` after its launches; the device slots [0, n) then stay stale."""
        if (not self.bulk or self.layout.world != 1 or n <= 0 or self._bulk_lo != 0 or self._bulk_hi != n
                or n * (self.layout.ld * 4 + self.layout.ldq * 8) > self.ZERO_COPY_MAX_BYTES):
            return None
        return self._hx, self._hxi

    def release_host_rows(self):
        """After the launches that read ``host_rows()``: the mirror's rows are rewritten only once the stream
        has passed them (the same event as an H2D out of the mirror).  The reads were issued on the dstream
        (or, without one, on the current stream of this device)."""
        self._bulk_ev.record(self.dstream.stream if self.dstream is not None
                             else torch.cuda.current_stream(self._dev_index))
        self._bulk_busy = True
        self._bulk_lo = self._bulk_hi = 0

    def drain(self):
        """Wait until every queued copy has been enqueued on its stream (re-raising a copy's error)."""
        if self.bulk:
            self._drain_bulk()
            return
        for r in self._ring:
            if r[3] is not None:
                r[2] = r[3].result()
                r[3] = None
