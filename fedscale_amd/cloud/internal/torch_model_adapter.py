"""Device-resident TorchModelAdapter — drop-in for fedscale/cloud/internal/torch_model_adapter.py:10-53.

The global model lives in HBM as a flat bucket (``fedscale_amd.bucket``), double-buffered: the round's
result is written into the spare buffer while the current one is the optimizer's ``last_model``
(torch_model_adapter.py:30 clones it; the ping-pong makes that clone free).  ``self.model`` (the
nn.Module the reference exposes through ``get_model``) is synchronised from HBM lazily, on egress
(``get_weights`` / ``get_model``), which is where the reference's pickling of the model happens anyway
(aggregator.py:788-804, 902-909).

Reference API (same names, argument meaning and error behaviour on valid input):
    TorchModelAdapter(model, optimizer=None)
    set_weights(weights, is_aggregator=True, client_training_results=None)
    get_weights() -> list of CPU tensors (cloned), in state_dict order
    get_model()   -> the nn.Module holding the current global weights
Device fast path used by ``DeviceAggregatorMixin``:
    begin_round(K, policy) -> DeviceRound;  apply_round(round, denom32, denom64, client_training_results)
"""
from __future__ import annotations

import itertools
import threading
from typing import List, Optional

import numpy as np
import torch

from ...bucket import BucketLayout, ClientStaging
from ... import hoststage
from ... import kernels as kx
from ..._native import FA_ACCUMULATE, FA_FINALIZE
from ...kernels import qfed_max_chunk as kx_qfed_max_chunk
from ...round import DeviceRound, default_capacity
from ...state import DeviceStream, FlatState, ShardGroup
from .model_adapter_base import ModelAdapterBase


_EGRESS_IDS = itertools.count(1)
#: per servicer thread: the adapter whose next get_weights() call hands out an EgressHandle
#: (set by the aggregator mixin around the reference CLIENT_PING's UPDATE_MODEL branch)
_HANDLE_ONCE = threading.local()


class EgressWeights(list):
    """The list get_weights() returns: a plain list of cloned CPU tensors plus an ``egress_key``.  It
    pickles as a plain list, so executors unpickle it without this package."""

    egress_key = None

    def __reduce_ex__(self, protocol):
        return (list, (list(self),))


class EgressHandle:
    """Stands for ``get_weights()`` where the caller only serialises it: what the mixin's
    ``create_client_task`` / ``get_test_config`` return in place of the weights (aggregator.py:788-804,
    806-816), which the servicer passes straight to ``serialize_response`` (:905-907).

    It holds the pickled bytes of its model version (``egress_bytes``, made once per version), so
    serialising it copies nothing and always yields the version current when it was made. Any other use
    (indexing, iteration, ``len``, pickling) unpickles those bytes once: the same list of CPU tensors
    ``get_weights()`` returns."""

    __slots__ = ("egress_key", "egress_payload", "_weights")

    def __init__(self, key, payload: bytes):
        self.egress_key = key
        self.egress_payload = payload
        self._weights = None

    def weights(self) -> list:
        if self._weights is None:
            import pickle

            self._weights = pickle.loads(self.egress_payload)
        return self._weights

    def __len__(self):
        return len(self.weights())

    def __getitem__(self, i):
        return self.weights()[i]

    def __iter__(self):
        return iter(self.weights())

    def __reduce_ex__(self, protocol):
        return (list, (list(self.weights()),))


class _HostBuf:
    """Pinned host buffers for one model version (fp32 bucket ``f``, side table ``s``) with their state_dict
    views, made once: buffers are pooled across versions, so egress clones from ready-made views."""

    __slots__ = ("f", "s", "views", "np_views", "np_list", "ev")

    def __init__(self, layout: BucketLayout):
        # round_up(P, 4) floats: fa_reduce_mirror writes whole float4 columns into ``f``
        self.f = torch.empty(max(4, (layout.P_full + 3) // 4 * 4), dtype=torch.float32, pin_memory=True)
        self.s = torch.empty(max(1, layout.Q), dtype=torch.int64)
        self.views = layout.unpack(self.f, self.s)
        self.np_views = [v.numpy() for v in self.views]
        self.np_list = list(self.np_views)  # (hoststage.stage takes a list)
        # recorded after the kernel that writes this buffer (fa_reduce_mirror); re-recorded only while the buffer
        # is out of the pool, i.e. while no reader can be waiting on it
        self.ev = torch.cuda.Event()


class _HostSnapshot:
    """One model version's host copy (a ``_HostBuf``) and its reader count.  ``pending``: the round's kernel
    writes the buffer itself (fa_reduce_mirror) and the first reader waits for that kernel (``buf.ev``)."""

    __slots__ = ("version", "buf", "readers", "pending")

    def __init__(self, version, buf: _HostBuf, pending: bool = False):
        self.version, self.buf, self.readers, self.pending = version, buf, 0, pending


def _resolve_device(device) -> torch.device:
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"device {d}: the aggregation path runs on the GPU only (no CPU fallback)")
    if d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class TorchModelAdapter(ModelAdapterBase):
    """``dstream``: the ``DeviceStream`` (GPU + HIP stream) every kernel, copy and event of this adapter is
    issued on — made for ``device`` when not given; a ``ShardedModelAdapter`` hands each part its own.  Each
    public call runs under ``dstream.joined()``: the adapter's GPU is current for the call (whatever the
    caller had current) and the caller's stream on that GPU is ordered after the call's work — except
    ``apply_round`` of a round that exposes no device state (``_round_exposes_device_state``), whose results every
    public reader waits for by itself."""

    def __init__(self, model: torch.nn.Module, optimizer=None, device=None, shards: Optional[ShardGroup] = None,
                 staging_capacity: Optional[int] = None, _load_from=None, dstream: Optional[DeviceStream] = None):
        self.model = model
        self.optimizer = optimizer
        self.device = _resolve_device(device)
        if dstream is not None and dstream.device != self.device:
            raise ValueError(f"dstream is on {dstream.device}, the adapter on {self.device}")
        self.dstream = dstream if dstream is not None else DeviceStream(self.device)
        self.shards = shards or ShardGroup()
        sd = model.state_dict()
        if self.shards.shards_params:
            self.layout = BucketLayout.from_state_dict(sd, self.shards.rank, self.shards.world)
        else:  # single GPU, or client mode: every rank holds the whole model
            self.layout = BucketLayout.from_state_dict(sd)
        L, dev = self.layout, self.device
        with self.dstream.joined():
            self.dstream.wait_caller()  # _load_from may hold the caller's device tensors
            self._f = [torch.zeros(L.ld, dtype=torch.float32, device=dev) for _ in range(2)]
            self._s = [torch.zeros(L.ldq, dtype=torch.int64, device=dev) for _ in range(2)]
            self._cur = 0
            # float64 side table + fp32 mean of the last round: the reference's Aggregator.model_weights
            self._mean_s = torch.zeros(L.ldq, dtype=torch.float64, device=dev)
            self._mean_f: Optional[torch.Tensor] = None
            self._mean_valid = False
            self.staging: Optional[ClientStaging] = None
            self.staging_capacity = staging_capacity
            cur_f = torch.zeros(L.ld, dtype=torch.float32, device=dev)
            cur_s = torch.zeros(L.ldq, dtype=torch.float64, device=dev)
            self._pack_values(list(_load_from) if _load_from is not None else list(sd.values()), cur_f, cur_s)
            self._f[0].copy_(cur_f)
            self._s[0].copy_(cur_s.to(torch.int64))
            self._ready = torch.cuda.Event()  # the kernels that wrote the current model buffers
            self._ready.record(self.dstream.stream)
            self._ready_stream = self.dstream.stream
        self._init_egress(_load_from is None)

    def _init_egress(self, module_in_sync: bool):
        """Egress state, shared with the servicer threads (aggregator.py:177-178: 20 of them call
        get_weights / serialize the model while the main thread applies rounds).  Host snapshots are
        immutable per model version; the lock guards (version, current snapshot, cached bytes)."""
        self._version = 0  # bumps on every device-side model update
        self._egress_lock = threading.Lock()
        self._pickle_lock = threading.Lock()  # one thread pickles a version; the others take its bytes
        self._snap: Optional[_HostSnapshot] = None
        self._snap_pool: list = []  # pinned buffers of retired snapshots no reader holds any more
        self._egress_cache = None
        self._egress_id = next(_EGRESS_IDS)
        self._module_version = 0 if module_in_sync else -1
        self._egress_ds: Optional[DeviceStream] = None  # D2H stream of egress (made on first use)

    # ---- internal buffers ---------------------------------------------------------------------
    def _snapshot(self) -> FlatState:
        return FlatState(self.layout, self._f[self._cur], self._s[self._cur])

    def _scratch_buffers(self):
        return self._f[1 - self._cur], self._s[1 - self._cur]

    def _commit_scratch(self, host: Optional[_HostBuf] = None):
        """Make the scratch buffers the model.  ``host``: a pinned buffer the round's kernel is writing the new
        model into (fa_reduce_mirror); it becomes the new version's egress snapshot, so egress needs no D2H."""
        self._ready_stream = self.dstream.stream  # every write to the model buffers is issued on it
        self._ready.record(self._ready_stream)
        self._commit_ev = self._ready
        with self._egress_lock:  # (buffer, version) flip atomically for the servicer threads
            self._cur = 1 - self._cur
            self._version += 1
            if host is not None:
                host.ev.record(self._ready_stream)  # this version's kernel: what its readers wait for
                old, self._snap = self._snap, _HostSnapshot(self._version, host, pending=True)
                if old is not None and old.readers == 0:
                    self._snap_pool.append(old.buf)

    #: FedAvg / FedBuff rounds of models of at most this many fp32 bytes (and no int64 entries) write the new
    #: model into its egress snapshot from the reduce's epilogue (fa_reduce_mirror): no D2H, no copy stream
    EGRESS_MIRROR_MAX_BYTES = 4 << 20

    def _mirror_target(self) -> Optional[_HostBuf]:
        """A free pinned snapshot buffer for fa_reduce_mirror, when this adapter's rounds qualify."""
        L = self.layout
        if L.world != 1 or L.Q or self.shards.world != 1 or L.P_full * 4 > self.EGRESS_MIRROR_MAX_BYTES:
            return None
        with self._egress_lock:
            if self._snap_pool:
                return self._snap_pool.pop()
        return _HostBuf(L)  # allocated with this adapter's GPU current (inside its DeviceStream)

    def _sqnorm_allreduce(self):
        return self.shards.sum_partials if self.shards.shards_params else None

    def _pack_values(self, values: list, f_dst: torch.Tensor, s_dst: torch.Tensor):
        """weights list -> device fp32 bucket slice + side table (converted to s_dst's dtype)."""
        L = self.layout
        values = L.values_of(values)
        for e in L.entries:
            v = values[e.index]
            t = v.detach() if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            if tuple(t.shape) != e.shape:
                raise ValueError(f"{e.name}: shape {tuple(t.shape)} != model shape {e.shape}")
            flat = t.reshape(-1)
            if e.kind == "f":
                lo, hi = max(e.offset, L.p0), min(e.offset + e.numel, L.p1)
                if lo < hi:
                    # np.asarray(w, dtype=float32) (torch_model_adapter.py:32)
                    f_dst[lo - L.p0:hi - L.p0].copy_(flat[lo - e.offset:hi - e.offset].to(torch.float32))
            else:
                s_dst[e.offset:e.offset + e.numel].copy_(flat.to(s_dst.dtype))

    # ---- reference API --------------------------------------------------------------------------
    def set_weights(self, weights, is_aggregator=True, client_training_results=None):
        """torch_model_adapter.py:23-39 on the device."""
        with self.dstream.joined():
            self.dstream.wait_caller()  # weights may be the caller's device tensors
            L = self.layout
            last = self._snapshot()
            cur_f = torch.zeros(L.ld, dtype=torch.float32, device=self.device)
            cur_s = torch.zeros(L.ldq, dtype=torch.float64, device=self.device)
            self._pack_values(list(weights), cur_f, cur_s)
            self._mean_f, self._mean_s, self._mean_valid = cur_f, cur_s, True
            opt = self.optimizer
            if opt is not None and is_aggregator and getattr(opt, "mode", None) in ("fed-yogi", "q-fedavg"):
                opt.update_round_gradient(last, FlatState(L, cur_f, cur_s), self, client_training_results)
                return
            nf, ns = self._scratch_buffers()
            nf.copy_(cur_f)
            ns.copy_(cur_s.to(torch.float32).to(torch.int64))  # float32 -> int64 load truncates (:31-35)
            self._commit_scratch()

    def _copy_to_host(self, f_cpu: torch.Tensor, s_cpu: torch.Tensor):
        """D2H of the current model into pinned f_cpu[:P_full] / s_cpu[:Q] (the caller holds the egress
        lock, so no round commits meanwhile; synchronous).  Parameter-sharded SPMD ranks all-gather
        first: every rank must then call egress from its main thread, in step (bench / tests)."""
        L = self.layout
        es = self._egress_ds
        if es is None:
            es = self._egress_ds = DeviceStream(self.device)
        with es:  # its own stream, ordered after the round's kernels by an event: one host wait, at the end
            es.stream.wait_event(self._ready)
            full = self.shards.all_gather(self._f[self._cur])
            full = L.unshard(full) if self.shards.shards_params else full[:L.P_full]
            if L.P_full == f_cpu.numel():  # (a _HostBuf holds exactly P_full floats, at least one)
                f_cpu.copy_(full, non_blocking=True)
            else:
                f_cpu[:L.P_full].copy_(full, non_blocking=True)
            if L.Q:
                s_cpu[:L.Q].copy_(self._s[self._cur][:L.Q], non_blocking=True)
            es.stream.synchronize()

    def _acquire_host(self) -> "_HostSnapshot":
        """The host snapshot of the current model version (one D2H per version), held by the caller until
        ``_release_host``: a later version goes to another pinned buffer, so readers of this one never see
        it change (aggregator.py:788-804, 902-909 read the model from up to 20 servicer threads)."""
        with self._egress_lock:
            snap = self._snap
            if snap is not None and snap.pending and snap.version == self._version:
                snap.readers += 1  # held: it cannot return to the pool while this thread waits
                wait = snap.buf.ev
            else:
                wait = None
        if wait is not None:
            # the kernel of THIS version wrote the snapshot (fa_reduce_mirror): wait for it alone, outside the
            # lock, so neither the next round's kernels nor the other egress readers hold this thread up
            wait.synchronize()
            with self._egress_lock:
                snap.pending = False
            return snap
        with self._egress_lock:
            snap = self._snap
            if snap is not None and snap.pending and snap.version == self._version:
                snap.buf.ev.synchronize()  # (another thread published a pending version meanwhile)
                snap.pending = False
            if snap is None or snap.version != self._version:
                buf = self._snap_pool.pop() if self._snap_pool else _HostBuf(self.layout)
                self._copy_to_host(buf.f, buf.s)
                old, snap = snap, _HostSnapshot(self._version, buf)
                self._snap = snap
                if old is not None and old.readers == 0:
                    self._snap_pool.append(old.buf)
            snap.readers += 1
            return snap

    def _release_host(self, snap: "_HostSnapshot"):
        with self._egress_lock:
            snap.readers -= 1
            if snap.readers == 0 and snap is not self._snap:
                self._snap_pool.append(snap.buf)

    #: models of at least this many bytes clone the snapshot with the native multi-threaded copy (fa_host_gather):
    #: one memcpy stream moves ~10 GB/s, so get_weights() of the headline's 100 MB model spent 10 of its 13 ms on
    #: the clones (bench.py headline_model_pcie_inclusive, phases_ms)
    CLONE_PARALLEL_MIN_BYTES = 16 << 20

    def _clone_weights(self, snap: "_HostSnapshot") -> list:
        # the reference's params.data.clone() per entry (torch_model_adapter.py:47): a fresh CPU tensor each,
        # copied through numpy (half the per-tensor cost of Tensor.clone on small models)
        views = snap.buf.np_views
        if self.layout.P_full * 4 < self.CLONE_PARALLEL_MIN_BYTES:
            return [torch.from_numpy(a.copy()) for a in views]
        from ... import _native
        from ...bucket import default_pack_workers

        outs = [np.empty(a.shape, dtype=a.dtype) for a in views]  # independent tensors, as clone() returns
        off = np.zeros(1, dtype=np.int64)
        workers = default_pack_workers()
        for a, o in zip(views, outs):  # one multi-threaded copy per entry (small ones stay one memcpy in C)
            if a.nbytes:
                sp = np.asarray([a.__array_interface__["data"][0]], dtype=np.uint64)
                nn = np.asarray([a.nbytes], dtype=np.int64)
                _native.call("fa_host_gather", o.__array_interface__["data"][0], sp.ctypes.data, off.ctypes.data,
                             nn.ctypes.data, 1, workers)
        return [torch.from_numpy(o) for o in outs]

    def get_weights(self) -> List[torch.Tensor]:
        """torch_model_adapter.py:41-47: cloned CPU tensors in state_dict order (gathers the shards).
        Inside ``handle_next_get_weights`` (this thread only) the one next call returns an EgressHandle.

        The list is tagged with (adapter, model version) so that the aggregator's serialize_response can
        hand out the pickled bytes of this version, made once per round (``egress_bytes``)."""
        if getattr(_HANDLE_ONCE, "adapter", None) is self:  # the caller only serialises this list
            _HANDLE_ONCE.adapter = None
            return self.egress_handle()
        pre = self._preallocate_clones()  # (small models) before the wait for the round's kernel, which hides it
        snap = self._acquire_host()
        try:
            if pre is not None and hoststage.stage(snap.buf.np_list, pre[0]) < 0:
                out = EgressWeights(pre[1])
            else:
                out = EgressWeights(self._clone_weights(snap))
            out.egress_key = (self._egress_id, snap.version)
        finally:
            self._release_host(snap)
        return out

    def _preallocate_clones(self):
        """(numpy arrays, the CPU tensors over them) for the clones of a small model (below CLONE_PARALLEL_MIN_BYTES):
        fresh, independent storage per call, as ``params.data.clone()`` gives (torch_model_adapter.py:47).  Made
        before get_weights() waits for a round's kernel, they cost nothing on the round's critical path; the copy
        after the wait is one native call (fedscale_amd/csrc/hoststage.c) over all of them."""
        L = self.layout
        if L.P_full * 4 >= self.CLONE_PARALLEL_MIN_BYTES:
            return None
        specs = self.__dict__.get("_clone_specs")
        if specs is None:
            specs = self._clone_specs = [(e.shape, np.float32 if e.kind == "f" else np.int64) for e in L.entries]
        arrs = [np.empty(shape, dtype) for shape, dtype in specs]
        return arrs, [torch.from_numpy(a) for a in arrs]

    def egress_bytes(self, key) -> Optional[bytes]:
        """``pickle.dumps`` of get_weights() for model version ``key`` — the bytes the reference's
        serialize_response makes per executor request (aggregator.py:788-804, 902-909) — made once per
        model version from the adapter's own host copy.  None when ``key`` is not the current version.
        Thread-safe: the bytes always belong to exactly the version of ``key``."""
        import pickle

        with self._egress_lock:
            if key != (self._egress_id, self._version):
                return None
            c = self._egress_cache
            if c is not None and c[0] == key:
                return c[1]
        with self._pickle_lock:  # one thread pickles; the others wait and take its bytes
            with self._egress_lock:
                c = self._egress_cache
                if c is not None and c[0] == key:
                    return c[1]
            snap = self._acquire_host()
            try:
                if (self._egress_id, snap.version) != key:
                    return None  # a round committed meanwhile: the caller's list is of an older version
                b = pickle.dumps(self._clone_weights(snap))
            finally:
                self._release_host(snap)
            with self._egress_lock:
                c = self._egress_cache
                if c is None or c[0][1] < key[1]:
                    self._egress_cache = (key, b)
            return b

    def egress_handle(self) -> EgressHandle:
        """``get_weights()`` for a caller that only serialises it: no clone (``EgressHandle``)."""
        while True:
            with self._egress_lock:
                key = (self._egress_id, self._version)
            b = self.egress_bytes(key)
            if b is not None:  # else a round committed between the two lines: take the new version
                return EgressHandle(key, b)

    def handle_next_get_weights(self):
        """Context: the next get_weights() on this thread returns ``egress_handle()`` (no clone). For a
        caller that only serialises the list, such as the servicer's UPDATE_MODEL branch
        (aggregator.py:902-907)."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            _HANDLE_ONCE.adapter = self
            try:
                yield
            finally:
                _HANDLE_ONCE.adapter = None

        return ctx()

    def get_model(self):
        if self._module_version != self._version:
            sd = self.model.state_dict()
            self.model.load_state_dict({n: t for n, t in zip(sd.keys(), self.get_weights())})
            self._module_version = self._version
        return self.model

    def __reduce__(self):
        """Pickle like the reference adapter (model + optimizer): the aggregator sizes simulated model
        transfers with ``sys.getsizeof(pickle.dumps(self.model_wrapper))`` (aggregator.py:422-424), so the
        device buffers must not inflate it.  Unpickling rebuilds the HBM state on the current device."""
        return (self.__class__, (self.get_model(), self.optimizer))

    # ---- device fast path -----------------------------------------------------------------------
    def begin_round(self, K: int, policy: str, capacity: Optional[int] = None, keep_mean=True) -> DeviceRound:
        """``keep_mean`` for q-FedAvg rounds: True fuses the FedAvg chain when the round spans several chunks
        (the staged updates are then gone by the end of the round), "always" in every round (the mean is then
        independent of the staging's later reuse), False never (model_weights of such rounds raises)."""
        cap = capacity or self.staging_capacity
        K_local = K
        if self.shards.shards_clients:  # this rank stages only its block of the arrivals
            k0, k1 = self.shards.client_block(K)
            K_local = max(1, k1 - k0)
        if cap:
            want = min(cap, K_local)
        elif self.staging is not None and self.staging.capacity >= K_local:
            want = K_local  # the round fits the staging already allocated (no free-memory query)
        else:
            want = min(default_capacity(self.layout, K_local, self.device), K_local)
        if policy == "qfedavg":  # phase-1 chunks hold at most fa_qfed_max_chunk() clients
            want = min(want, kx_qfed_max_chunk())
        if self.staging is None or self.staging.capacity < want:
            self.staging = None
            self.staging = ClientStaging(self.layout, self.device, want, dstream=self.dstream)
        snap = self._snapshot()
        chain = keep_mean == "always" or (bool(keep_mean) and want < K_local)
        return DeviceRound(self.layout, self.device, K, policy, capacity=want, staging=self.staging,
                           last_f32=snap.f32, last_i64=snap.side,
                           clients=self.shards if self.shards.shards_clients else None, mean_chain=chain,
                           dstream=self.dstream)

    def apply_round(self, rnd: DeviceRound, denom32: float, denom64: float, client_training_results=None,
                    keep_mean: bool = True):
        """Finish a round: reduce the last chunk with the server step fused, then swap buffers."""
        self._commit_ev = None
        if self._round_exposes_device_state():
            with self.dstream.joined(self._take_commit_event):
                self._apply_round(rnd, denom32, denom64, keep_mean)
        else:
            with self.dstream:
                self._apply_round(rnd, denom32, denom64, keep_mean)

    def _round_exposes_device_state(self) -> bool:
        """Whether a round leaves device buffers a caller can read through the public API — the FedYoGi optimizer's
        ``m_t`` / ``v_t`` (device views, yogi.py's reference attributes) — so the caller's stream must be ordered
        after the round (DeviceStream.joined).  Otherwise every public reader of the round's results is ordered
        by the adapter itself (get_weights / egress wait on the round's event, model_weights reads on the adapter's
        stream), and the join — a hipStreamWaitEvent on a kernel still running, 5 us against 0.5 us on an idle one
        (profiles/r06_launch_api_probe.log), ~6 % of config 1's round — is skipped."""
        opt = self.optimizer
        return opt is not None and getattr(opt, "mode", None) == "fed-yogi"

    def _take_commit_event(self):
        """The event ``_commit_scratch`` recorded for the round just applied (after all of its work on the
        dstream): the caller's stream waits on it instead of a second record (DeviceStream.joined)."""
        ev, self._commit_ev = getattr(self, "_commit_ev", None), None
        return ev

    def _apply_round(self, rnd: DeviceRound, denom32: float, denom64: float, keep_mean):
        L = self.layout
        out_f, out_s = self._scratch_buffers()
        opt = self.optimizer
        mode = getattr(opt, "mode", None) if opt is not None else None
        if rnd.policy == "qfedavg":
            if mode != "q-fedavg":
                raise RuntimeError("a q-FedAvg round needs the q-fedavg server optimizer")
            rnd.qfed_fold()
            allreduce = self._sqnorm_allreduce()
            if allreduce is not None and rnd.cg is None:
                allreduce(rnd.sqnorm)
            self._finish_qfed(rnd)
            return
        elif mode == "fed-yogi":
            # the FedAvg mean (aggregator.py:505-507) into its own buffer, then the YoGi step over it
            # (optimizers.py:43-63, yogi.py:15-36) as a second streaming pass: the same bits as the fused
            # epilogue (fa_reduce_yogi), 1 % faster at 1000 x 25 M — the fused epilogue's last/m/v traffic sits
            # at the end of every tile with one wave per SIMD to hide it (tools/yogi_ab.py,
            # profiles/r03_yogi_fused_vs_unfused.log)
            last = self._snapshot()
            y = opt.gradient_controller
            y.bind(L, self.device)
            if self._mean_f is None or self._mean_f is last.f32 or self._mean_f is out_f:
                self._mean_f = torch.zeros(L.ld, dtype=torch.float32, device=self.device)
            mean_f = self._mean_f
            rnd.finalize_mean(denom32, denom64, out=mean_f, cur_side=self._mean_s, model_side=None)
            kx.yogi_step(mean_f, last.f32, y.m, y.v, out_f, L.P, init=not y.initialized, **y.fp32_hparams())
            y.step_side(self._mean_s, last.side, model=out_s)
            y.initialized = True
            self._mean_valid = True
        elif mode == "q-fedavg":
            raise RuntimeError("q-fedavg optimizer but the round was not staged as q-FedAvg")
        else:
            host = self._mirror_target()
            if not self._finish_small(rnd, denom32, out_f, host):
                rnd.finalize_mean(denom32, denom64, out=out_f, cur_side=self._mean_s, model_side=out_s,
                                  mirror=None if host is None else host.f)
            self._mean_f = out_f  # FedAvg without a server step: the mean IS the new model
            self._mean_valid = True
            self._commit_scratch(host)
            return
        self._commit_scratch()

    #: the small-round finish (``_finish_small``); False takes DeviceRound.finalize_mean for every round
    SMALL_ROUND_FINISH = True

    def _finish_small(self, rnd: DeviceRound, denom32: float, out_f: torch.Tensor, host) -> bool:
        """FedAvg's finishing reduce for a small single-chunk round whose updates are all still in the staging's
        pinned mirror and whose model has no int64 entries (config 1, the FEMNIST CNN): the one fa_reduce_mirror
        launch DeviceRound.finalize_mean would make (x read over PCIe from the mirror, the mean written to the new
        model buffer and to its egress snapshot), issued straight through the C ABI.  The same launch on the same
        stream, so the same bits; the host cost of the general path's argument checks (which the ABI repeats on
        every operand, fa_device.h) is paid once per (rows, model buffer, snapshot) triple and cached.  False:
        the round does not qualify (the caller takes finalize_mean)."""
        L = self.layout
        if (not self.SMALL_ROUND_FINISH or host is None or L.Q or rnd.policy != "fedavg" or rnd.chunks_done
                or rnd.cg is not None):
            return False
        rnd._check_complete()
        st = rnd.staging
        n = rnd.slot
        zc = st.host_rows(n)
        if zc is None:
            return False
        x = zc[0]
        h = rnd.head  # rows [0, h) already reduced into rnd.head_acc (DeviceRound._launch_head)
        acc = rnd.head_acc if h else None
        key = (x.data_ptr(), n, h, out_f.data_ptr(), host.f.data_ptr(), acc.data_ptr() if h else 0)
        cache = self.__dict__.setdefault("_small_keys", set())
        if key not in cache:  # the wrapper's checks, once per operand set (kernels.reduce_mirror)
            kx._check_x(x, n, L.P, host_ok=True)
            kx._dev(out_f, torch.float32, "out", kx._cols(L.P))
            kx._pinned(host.f, torch.float32, "mirror", kx._cols(L.P))
            if h:
                kx._dev(acc, torch.float32, "acc_in", kx._cols(L.P))
            if len(cache) > 64:
                cache.clear()
            cache.add(key)
        flags = FA_FINALIZE | (FA_ACCUMULATE if h else 0)
        try:
            kx.call("fa_reduce_mirror", key[0] + h * x.shape[1] * 4, x.shape[1], n - h, L.P, None, key[5] or None,
                    key[3], key[4], denom32, flags, self.dstream.handle)
        finally:
            st.release_host_rows()  # the mirror's rows are rewritten only after the stream has passed the reads
        return True

    def _finish_qfed(self, rnd: DeviceRound):
        """hs + step of a folded q-FedAvg round (its norms already summed over the shards), then commit."""
        with self.dstream.joined():
            out_f, out_s = self._scratch_buffers()
            rnd.qfed_finish(out=out_f, model_side=out_s)
            self._mean_valid = False
            self._mean_round = rnd  # the mean can still be recomputed lazily from the staged updates
            self._commit_scratch()

    def round_mean_weights(self):
        """The reference's Aggregator.model_weights after the last result of a round (the FedAvg mean,
        aggregator.py:505-507): fp32 entries float32, int64 entries float64 — materialised lazily."""
        return LazyWeights(self)

    def _fetch_mean(self) -> list:
        with self.dstream.joined():  # the D2H copies run on the stream that computed the mean
            mean_f, mean_s = self._mean_device()
            L = self.layout
            full = self.shards.all_gather(mean_f[:L.ld])
            full = L.unshard(full) if self.shards.shards_params else full[:L.P_full]
            return self._mean_lists(full.to("cpu").numpy(), mean_s[:L.Q].to("cpu").numpy())

    def _mean_lists(self, f_cpu, s_cpu) -> list:
        out = []
        for e in self.layout.entries:
            src = f_cpu if e.kind == "f" else s_cpu
            out.append(np.array(src[e.offset:e.offset + e.numel].reshape(e.shape)))
        return out

    def _mean_device(self):
        """(fp32 mean slice, float64 side mean) of the last round on this device (written on ``dstream``)."""
        with self.dstream.joined():
            return self._mean_device_on_stream()

    def _mean_device_on_stream(self):
        rnd = getattr(self, "_mean_round", None)
        if not self._mean_valid and rnd is not None:
            L = self.layout
            mean_f = torch.zeros(L.ld, dtype=torch.float32, device=self.device)
            if rnd.mean_from_staging(mean_f, self._mean_s):
                self._mean_f, self._mean_valid = mean_f, True
            self._mean_round = None
        if not self._mean_valid or self._mean_f is None:
            raise RuntimeError("the FedAvg mean of this round is not available on the device: a q-FedAvg "
                               "round keeps it only while all K updates are still staged (one chunk), and "
                               "fed-yogi keeps it unless keep_mean=False")
        return self._mean_f, self._mean_s


class LazyWeights:
    """List-like stand-in for ``Aggregator.model_weights``: fetched from HBM on first access."""

    def __init__(self, adapter: TorchModelAdapter):
        self._adapter = adapter
        self._version = adapter._version
        self._cache = None

    def _get(self):
        if self._cache is None:
            if self._adapter._version != self._version:
                raise RuntimeError("model_weights of an earlier round: the device buffers were reused")
            self._cache = self._adapter._fetch_mean()
        return self._cache

    def __len__(self):
        return self._adapter.layout.T

    def __getitem__(self, i):
        return self._get()[i]

    def __iter__(self):
        return iter(self._get())

    def __deepcopy__(self, memo):
        import copy

        return copy.deepcopy(self._get(), memo)
