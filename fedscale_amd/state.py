"""Flat device snapshots of a model state and the multi-GPU (sharded) plumbing.

``FlatState`` is what the device path hands around instead of the reference's list-of-tensors:
``f32`` is this rank's slice of the fp32 bucket, ``side`` the replicated side table (int64 for a model
state, float64 for a FedAvg mean of int64 entries).

``DeviceGroup`` is the N GPUs that ONE process drives: the multi-GPU drop-in behind FedScale's single
aggregator process (``ShardedModelAdapter``; its cross-device steps are RCCL collectives issued from the
library, ``fa_rccl_*``).  ``ShardGroup`` is one process per GPU, torch.distributed over RCCL (the SPMD
benchmark and tests), with two ways to spread a round over the ranks:

* ``mode="params"`` (default): every rank owns a balanced, 64-aligned slice of the fp32 bucket
  (``bucket.shard_bounds``; every row ``ld`` wide) and reduces its slice of every client update.  The only collectives are the all-gather that reassembles the global model
  for egress and, for q-FedAvg, one exchange of the K per-client partial squared norms (all-gather +
  fixed-order sum, ``sum_partials``).  The per-element chain is the reference's, so the result is
  bit-exact.
* ``mode="clients"``: every rank holds the whole model and reduces a contiguous block of the round's
  arrivals (rank r takes arrival indices [r*K/N, (r+1)*K/N)).  The per-rank partial sums meet in one RCCL
  all-reduce (the "final RCCL reduce" of the north star) and the server step then runs replicated, so
  egress needs no gather.  Summing per-rank partials re-associates the fp32 chain: the result is within
  the north-star tolerance (1e-5 relative), not bit-exact; int64 side-table sums stay exact.
"""
from __future__ import annotations

import atexit
import threading
from dataclasses import dataclass
from typing import Optional

import torch

from .bucket import BucketLayout


# Thin wrappers over torch's per-thread device / current-stream state.  A stream is named by its key
# (stream_id, device_index, device_type); the raw torch._C calls skip torch.cuda.current_stream()'s Stream-object
# construction, which costs several µs per call on the per-round path (config 1 rounds take ~0.1 ms).
_C = torch._C
_FAST = all(hasattr(_C, n) for n in ("_cuda_getDevice", "_cuda_setDevice", "_cuda_getCurrentStream",
                                      "_cuda_setStream", "_cuda_getCurrentRawStream"))


def _get_device() -> int:
    return _C._cuda_getDevice() if _FAST else torch.cuda.current_device()


def _set_device(i: int):
    if _FAST:
        _C._cuda_setDevice(i)
    else:
        torch.cuda.set_device(i)


def _stream_key(s) -> tuple:
    return (s.stream_id, s.device_index, s.device_type)


def _get_stream(i: int) -> tuple:
    """Key of the current stream of device i (this thread)."""
    if _FAST:
        return tuple(_C._cuda_getCurrentStream(i))
    return _stream_key(torch.cuda.current_stream(i))


def _set_stream(key: tuple):
    if _FAST:
        _C._cuda_setStream(stream_id=key[0], device_index=key[1], device_type=key[2])
    else:
        torch.cuda.set_stream(_stream_obj(key))


_STREAM_OBJS: dict = {}


def _stream_obj(key: tuple):
    """A torch Stream object for a key (cached: callers' streams are few, usually the default one)."""
    s = _STREAM_OBJS.get(key)
    if s is None:
        s = _STREAM_OBJS[key] = torch.cuda.Stream(stream_id=key[0], device_index=key[1], device_type=key[2])
    return s


def raw_stream(index: int) -> int:
    """hipStream_t of the current stream of device ``index`` on this thread (what the C ABI takes)."""
    if _FAST:
        return _C._cuda_getCurrentRawStream(index)
    return torch.cuda.current_stream(index).cuda_stream


class DeviceStream:
    """A GPU and the HIP stream an adapter (or one part of a sharded adapter) issues ALL its work on.

    ``with ds:`` makes the GPU current and the stream current on it, for torch ops and for the library
    (``kernels._stream`` passes the current stream of the tensor's device), and restores both on exit.  So
    one host thread drives several GPUs and every launch, copy and event of a part lands on the part's own
    device, whatever device the caller had current (the null stream would resolve against the caller's
    current device).  Work the adapter does not own — device tensors handed in by the caller — is ordered
    by ``wait_caller()``: the stream waits for the stream that was current on this device at entry."""

    __slots__ = ("device", "index", "stream", "handle", "key", "_join_ev")
    _tls = threading.local()

    def __init__(self, device, stream: "Optional[torch.cuda.Stream]" = None):
        d = torch.device(device) if not isinstance(device, int) else torch.device("cuda", device)
        if d.type != "cuda":
            raise ValueError(f"device {d}: the aggregation path runs on the GPU only (no CPU fallback)")
        if d.index is None:
            d = torch.device("cuda", _get_device())
        self.device, self.index = d, d.index
        self.stream = stream if stream is not None else torch.cuda.Stream(device=d)
        self.handle = self.stream.cuda_stream  # never 0: a stream of this device, not the null stream
        self.key = _stream_key(self.stream)
        self._join_ev = None  # one event, re-recorded for every join (no event create/destroy per call)

    @classmethod
    def current(cls) -> "Optional[DeviceStream]":
        """The innermost DeviceStream entered on this thread (None outside any)."""
        st = getattr(cls._tls, "stack", None)
        return st[-1][0] if st else None

    def __enter__(self):
        st = getattr(self._tls, "stack", None)
        if st is None:
            st = self._tls.stack = []
        prev_dev = _get_device()
        if prev_dev != self.index:
            _set_device(self.index)
        prev = _get_stream(self.index)  # the caller's stream on this device
        _set_stream(self.key)
        st.append((self, prev_dev, prev))
        return self

    def __exit__(self, *exc):
        return self._exit(False)

    def _exit(self, join: bool, done=None):
        _, prev_dev, prev = self._tls.stack.pop()
        if join and prev != self.key:  # no host sync: the caller's stream is ordered after our work
            # ``done()``: an event the body has ALREADY recorded on this stream after all of its work (an adapter's
            # commit event), or None — then one is recorded here
            ev = done() if done is not None else None
            if ev is None:
                ev = self._join_ev
                if ev is None:
                    ev = self._join_ev = torch.cuda.Event()
                ev.record(self.stream)
            _stream_obj(prev).wait_event(ev)
        _set_stream(prev)
        if prev_dev != self.index:
            _set_device(prev_dev)
        return False

    def joined(self, done=None) -> "_Joined":
        """Like ``with ds:``, and on exit the caller's stream on this device waits for everything issued
        inside (an event, no host sync): an adapter's public calls keep the ordering a caller on its own
        stream expects (device buffers it reads afterwards are written), while the work itself runs on
        ``stream``.  ``done``: a callable returning an event the body recorded on ``stream`` after ALL of its
        work (or None), which the caller's stream then waits on instead of a fresh record."""
        return _Joined(self, done)

    def wait_caller(self):
        """Order this stream after the work the caller queued on this device before its outermost entry."""
        for ds, _, prev in getattr(self._tls, "stack", None) or ():
            if ds is self:
                if prev != self.key:
                    self.stream.wait_stream(_stream_obj(prev))
                return
        cur = _get_stream(self.index)
        if cur != self.key:
            self.stream.wait_stream(_stream_obj(cur))


class _Joined:
    __slots__ = ("ds", "done")

    def __init__(self, ds: DeviceStream, done=None):
        self.ds, self.done = ds, done

    def __enter__(self):
        return self.ds.__enter__()

    def __exit__(self, *exc):
        return self.ds._exit(True, None if exc[0] is not None else self.done)


@dataclass
class FlatState:
    layout: BucketLayout
    f32: torch.Tensor
    side: torch.Tensor


MODES = ("params", "clients")


class ShardGroup:
    """rank/world of the GPUs sharing a round; ``None`` group = the default process group."""

    def __init__(self, rank: int = 0, world: int = 1, group=None, mode: str = "params"):
        if mode not in MODES:
            raise ValueError(f"shard mode {mode!r} not in {MODES}")
        self.rank, self.world, self.group, self.mode = rank, world, group, mode

    @classmethod
    def from_env(cls, group=None, mode: str = "params") -> "ShardGroup":
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_rank(group), dist.get_world_size(group), group, mode)
        return cls(mode=mode)

    @property
    def shards_params(self) -> bool:
        """The fp32 bucket is split across ranks (egress needs the all-gather)."""
        return self.world > 1 and self.mode == "params"

    @property
    def shards_clients(self) -> bool:
        """Each rank reduces a block of the round's clients over the whole model."""
        return self.world > 1 and self.mode == "clients"

    def client_block(self, K: int, rank: Optional[int] = None):
        """[k0, k1): the arrival indices rank ``rank`` reduces in client mode (contiguous, balanced)."""
        r = self.rank if rank is None else rank
        return r * K // self.world, (r + 1) * K // self.world

    def owner(self, k: int, K: int) -> int:
        """The rank that reduces arrival index k of a K-client round (client mode)."""
        return ((k + 1) * self.world - 1) // K

    def _host_staged(self, t: torch.Tensor) -> bool:
        """gloo (CPU tests, several ranks sharing one GPU) moves device tensors through the host."""
        import torch.distributed as dist

        return t.device.type == "cuda" and dist.get_backend(self.group) == "gloo"

    def all_gather(self, shard: torch.Tensor) -> torch.Tensor:
        """Concatenate the equal-size shards of every rank (RCCL all-gather over xGMI).  In client mode the
        model is replicated, so the local copy already is the whole model."""
        if not self.shards_params:
            return shard
        return self.collective_all_gather(shard)

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks (RCCL all-reduce; the K per-client partial norms of q-FedAvg)."""
        if self.world == 1:
            return t
        return self.collective_all_reduce(t)

    def sum_partials(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks in a FIXED rank order (all-gather, then ((t_0 + t_1) + t_2) + ...): the
        per-client partial squared norms of q-FedAvg over the parameter shards.  Unlike an all-reduce,
        whose internal order depends on the ring, the bits do not depend on the transport."""
        if self.world == 1:
            return t
        allp = self.collective_all_gather(t.reshape(-1)).view(self.world, -1)
        if t.device.type == "cuda" and t.dtype == torch.float64:
            from . import kernels as kx

            kx.sum_rows_f64(allp, t.view(-1))
            return t
        acc = allp[0].clone()
        for r in range(1, self.world):
            acc += allp[r]
        t.copy_(acc.view_as(t))
        return t

    # raw collectives (no world-1 short cut): what the wrappers above issue, callable at any world size
    def collective_all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist

        if self._host_staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def collective_all_gather(self, shard: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        if self._host_staged(shard):
            return self.collective_all_gather(shard.cpu()).to(shard.device)
        out = torch.empty(world * shard.numel(), dtype=shard.dtype, device=shard.device)
        if shard.device.type == "cpu":
            parts = list(out.chunk(world))
            dist.all_gather(parts, shard.contiguous(), group=self.group)
            return torch.cat(parts)
        dist.all_gather_into_tensor(out, shard.contiguous(), group=self.group)
        return out


class PartOf(ShardGroup):
    """Part r of N of a model sharded over the devices of ONE process (``DeviceGroup``): the shard
    geometry of rank r of N, but no process-group collectives — the cross-part steps are issued by the
    coordinating ``ShardedModelAdapter`` for all parts at once."""

    def __init__(self, rank: int, world: int, devices: "DeviceGroup"):
        super().__init__(rank, world, None, "params")
        self.devices = devices

    def all_gather(self, shard):
        raise RuntimeError("in-process shard: the coordinating adapter reassembles the parts")

    def all_reduce_sum(self, t):
        raise RuntimeError("in-process shard: the coordinating adapter combines the parts")

    def sum_partials(self, t):
        raise RuntimeError("in-process shard: the coordinating adapter combines the parts")


def _close_live_groups():
    for g in list(_LIVE_GROUPS):
        try:
            g.close()
        except Exception:
            pass


#: groups with an open RCCL communicator, held STRONGLY until closed: a communicator is destroyed only by an
#: explicit close() or by the exit hook below (while the HIP runtime is still up) — never from a GC
#: finalizer, which may run on any thread, gRPC servicer threads included
_LIVE_GROUPS: "set" = set()
atexit.register(_close_live_groups)


def comm_info(comm, n_local: int) -> dict:
    """{count, ranks, devices} of an fa_rccl handle as RCCL reports them (fa_rccl_comm_info)."""
    import ctypes

    from . import _native

    cnt = ctypes.c_int32(-1)
    ranks = (ctypes.c_int32 * n_local)()
    devs = (ctypes.c_int32 * n_local)()
    _native.call("fa_rccl_comm_info", comm, ctypes.byref(cnt), ranks, devs)
    return {"count": cnt.value, "ranks": list(ranks), "devices": list(devs)}


def spmd_rccl_probe(device_index: int, group=None, timeout_s: float = 90.0) -> dict:
    """One process per GPU (torch.distributed initialised): open an RCCL communicator of our own over the ranks
    (fa_rccl_unique_id on rank 0, broadcast through the process group, fa_rccl_init_rank on every rank), ask RCCL
    for its rank count, rank and device, gather those to every rank and close it.  What a multi-GPU record shows
    as "RCCL saw N ranks".

    Collective-safe on every path: ncclCommInitRank blocks until all ranks have joined, so each rank
    runs its part in a child process (``fedscale_amd.rccl_probe``) under ``timeout_s``; a rank whose init fails or
    hangs is killed at the deadline, and every rank then reaches the same all_gather of (ok, result | error), so the
    ranks always leave together, with the failures named."""
    import ctypes
    import json
    import os
    import subprocess
    import sys

    import torch.distributed as dist

    from . import _native

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    # agree first on RCCL being loadable everywhere and on rank 0's id, and skip together otherwise
    avail = [None] * world
    dist.all_gather_object(avail, bool(_native.load().fa_rccl_available()), group=group)
    if not all(avail):
        return {"skipped": "RCCL could not be loaded on ranks %s" % [r for r, a in enumerate(avail) if not a]}
    idbuf = (ctypes.c_char * 128)()
    msg = [None]
    if rank == 0:
        try:
            _native.call("fa_rccl_unique_id", idbuf)
            msg = [bytes(idbuf)]
        except _native.FedAggError as e:
            msg = [str(e)]
    dist.broadcast_object_list(msg, src=0, group=group)
    if not isinstance(msg[0], bytes):
        return {"error": "fa_rccl_unique_id on rank 0: %s" % msg[0]}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "fedscale_amd.rccl_probe", "--nranks", str(world), "--rank", str(rank),
           "--device", str(device_index), "--id", msg[0].hex()]
    try:
        r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=timeout_s)
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        mine = json.loads(lines[-1]) if lines else {
            "ok": False, "error": "rc %s: %s" % (r.returncode, r.stderr[-300:])}
    except subprocess.TimeoutExpired:
        mine = {"ok": False, "error": f"no result within {timeout_s:g} s (ncclCommInitRank did not complete)"}
    every = [None] * world
    dist.all_gather_object(every, mine, group=group)  # every rank gets here, whatever its child did
    bad = {i: e.get("error") for i, e in enumerate(every) if not e.get("ok")}
    if bad:
        return {"error": "RCCL probe failed on ranks %s" % sorted(bad), "rank_errors": bad}
    return {"count": every[0]["count"], "counts_agree": all(e["count"] == every[0]["count"] for e in every),
            "rank_of_process": [e["user_rank"] for e in every], "device_of_rank": [e["cu_device"] for e in every],
            "source": "fa_rccl_init_rank + fa_rccl_comm_info (ncclCommCount / ncclCommUserRank / ncclCommCuDevice), "
                      "one child process per rank with a %g s deadline" % timeout_s}


class DeviceGroup:
    """The GPUs ONE aggregator process drives (FedScale's aggregator is a single process, aggregator.py:
    177-192, 919-963).  Cross-device steps are RCCL collectives over xGMI issued for every device at once
    from the calling thread (``fa_rccl_*``, one communicator for the group); when a device appears more
    than once (several shards on one card, as in tests) or RCCL is unavailable, the same steps run as
    device-to-device copies.  Either way the combination order is fixed (all-gather, then a fixed-order
    sum), so the result does not depend on the transport.

    Position i of the group owns ``streams[i]``, a ``DeviceStream`` of ``devices[i]``: the part of a
    ``ShardedModelAdapter`` at that position issues all its work on it, and the group's collectives run on
    it (RCCL gets one explicit stream per device, never the null stream).  A collective first orders each
    position's stream after the caller's current stream on that device and, at the end, the caller's
    current streams after the group's, so plain tensors handed in and read back need no extra sync.

    ``transport``: "rccl", "copy" or None (choose: RCCL whenever the devices are distinct)."""

    def __init__(self, devices, transport: Optional[str] = None):
        devs = [torch.device(d) if not isinstance(d, int) else torch.device("cuda", d) for d in devices]
        if not devs:
            raise ValueError("DeviceGroup needs at least one device")
        for d in devs:
            if d.type != "cuda" or d.index is None:
                raise ValueError(f"device {d}: a DeviceGroup holds indexed GPUs (cuda:N); no CPU fallback")
        self.devices = devs
        self.world = len(devs)
        distinct = len({d.index for d in devs}) == len(devs)
        if transport is None:
            from . import _native

            transport = "rccl" if distinct and _native.load().fa_rccl_available() else "copy"
        if transport not in ("rccl", "copy"):
            raise ValueError(f"transport {transport!r}")
        if transport == "rccl" and not distinct:
            raise ValueError("RCCL needs one shard per GPU (a device appears twice)")
        self.transport = transport
        self.streams = [DeviceStream(d) for d in devs]
        self._comm = None

    # ---- RCCL communicator ------------------------------------------------------------------------
    def _rccl(self):
        if self._comm is None:
            import ctypes

            from . import _native

            devs = (ctypes.c_int32 * self.world)(*[d.index for d in self.devices])
            h = ctypes.c_void_p()
            _native.call("fa_rccl_init", self.world, devs, ctypes.byref(h))
            self._comm = h
            _LIVE_GROUPS.add(self)  # destroyed by close() or at interpreter exit, never by GC
        return self._comm

    def rccl_info(self) -> dict:
        """What RCCL itself reports for the group's communicator (fa_rccl_comm_info: ncclCommCount, and per
        position ncclCommUserRank / ncclCommCuDevice); the copy transport has no communicator."""
        if self.transport != "rccl":
            return {"transport": self.transport, "count": None,
                    "note": "no RCCL communicator: a device hosts several parts (copy transport)"}
        return {"transport": "rccl", **comm_info(self._rccl(), self.world),
                "devices_requested": [d.index for d in self.devices]}

    def close(self):
        if self._comm is not None:
            from . import _native

            comm, self._comm = self._comm, None
            _LIVE_GROUPS.discard(self)
            _native.call("fa_rccl_destroy", comm)

    def stream_handles(self) -> list:
        """The hipStream_t of every position (what the fa_rccl_* stream tables hold)."""
        return [ds.handle for ds in self.streams]

    def _tables(self, *lists):
        import ctypes

        out = []
        for lst in lists:
            out.append((ctypes.c_void_p * self.world)(*[None if t is None else t.data_ptr() for t in lst]))
        streams = (ctypes.c_void_p * self.world)(*self.stream_handles())
        return out, streams

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        from . import _native

        return {torch.float32: _native.FA_DT_F32, torch.float64: _native.FA_DT_F64,
                torch.int64: _native.FA_DT_I64}[t.dtype]

    def _enter(self):
        """Every position's stream waits for the caller's current stream on its device."""
        for ds in self.streams:
            cur = torch.cuda.current_stream(ds.index)
            if cur != ds.stream:
                ds.stream.wait_stream(cur)

    def _leave(self):
        """The caller's current streams wait for the group's work."""
        for ds in self.streams:
            cur = torch.cuda.current_stream(ds.index)
            if cur != ds.stream:
                cur.wait_stream(ds.stream)

    def _barrier(self):
        """Every position's stream waits for what every position has queued so far (copy transport: a copy
        reads another position's buffer, so both sides must be ordered)."""
        evs = []
        for ds in self.streams:
            ev = torch.cuda.Event()
            ev.record(ds.stream)
            evs.append(ev)
        for ds in self.streams:
            for ev in evs:
                ds.stream.wait_event(ev)

    def _copy_each(self, fn):
        """Run fn(i) under position i's DeviceStream for every i, between two barriers."""
        self._barrier()
        for i, ds in enumerate(self.streams):
            with ds:
                fn(i)
        self._barrier()

    # ---- collectives over the parts ---------------------------------------------------------------
    def all_gather(self, parts, outs):
        """outs[i][r*n:(r+1)*n] = parts[r] for every part i (n = parts[r].numel(), equal for all r)."""
        n = parts[0].numel()
        self._enter()
        if self.transport == "rccl":
            from . import _native

            (send, recv), streams = self._tables(parts, outs)
            _native.call("fa_rccl_all_gather", self._rccl(), send, recv, n, self._dt(parts[0]), streams)
        else:
            def copy(i):
                for r, p in enumerate(parts):
                    outs[i][r * n:(r + 1) * n].copy_(p.reshape(-1), non_blocking=True)

            self._copy_each(copy)
        self._leave()
        return outs

    def gather(self, parts, out_root, root: int = 0):
        """out_root[r*n:(r+1)*n] = parts[r], on device ``root``."""
        n = parts[0].numel()
        self._enter()
        if self.transport == "rccl":
            import ctypes

            from . import _native

            (send,), streams = self._tables(parts)
            _native.call("fa_rccl_gather", self._rccl(), send, ctypes.c_void_p(out_root.data_ptr()), n,
                         self._dt(parts[0]), root, streams)
        else:
            def copy(i):
                if i == root:
                    for r, p in enumerate(parts):
                        out_root[r * n:(r + 1) * n].copy_(p.reshape(-1), non_blocking=True)

            self._copy_each(copy)
        self._leave()
        return out_root

    def broadcast(self, bufs, root: int = 0):
        """bufs[i] <- bufs[root] for every part i."""
        n = bufs[root].numel()
        self._enter()
        if self.transport == "rccl":
            from . import _native

            (b,), streams = self._tables(bufs)
            _native.call("fa_rccl_broadcast", self._rccl(), b, n, self._dt(bufs[root]), root, streams)
        else:
            def copy(i):
                if i != root:
                    bufs[i].copy_(bufs[root], non_blocking=True)

            self._copy_each(copy)
        self._leave()
        return bufs

    def sum_f64(self, parts, scratch=None):
        """parts[i] <- ((parts[0] + parts[1]) + ...) on every device: per-shard fp64 partials (q-FedAvg's
        per-client squared norms), combined by an all-gather and a fixed-order sum (fa_sum_rows_f64), each
        position's sum on its own stream."""
        from . import kernels as kx

        n = parts[0].numel()
        if scratch is None:
            scratch = []
            for ds in self.streams:
                with ds:  # allocated on the stream that uses it (the caching allocator reuses per stream)
                    scratch.append(torch.empty(self.world * n, dtype=torch.float64, device=ds.device))
        self.all_gather(parts, scratch)
        self._enter()
        for ds, p, o in zip(self.streams, parts, scratch):
            with ds:
                kx.sum_rows_f64(o.view(self.world, n), p)
        self._leave()
        return parts
