"""Model adapter sharded over the GPUs of ONE process — the multi-GPU drop-in behind FedScale's
single-process aggregator.

FedScale's aggregator is one process: every upload lands in it (``CLIENT_EXECUTE_COMPLETION``,
fedscale/cloud/aggregation/aggregator.py:919-963, queued at :958-959 and reduced on the main thread by
client_completion_handler :454-487), and egress is served from its 20 gRPC servicer threads
(:177-178; ``get_weights`` at :788-816, :902-903).  So the shards cannot be one process per GPU behind that
loop.  ``ShardedModelAdapter`` keeps the reference interface of ``TorchModelAdapter``
(torch_model_adapter.py:10-53) and drives N devices from the one process:

* the fp32 bucket is split into N equal 64-aligned slices, one part per device (``BucketLayout`` rank r of
  N); each part is a full ``TorchModelAdapter`` over its slice (ping-pong model buffers, staging, its own
  YoGi m/v, the replicated int64 side table);
* ingress: an upload is gathered ONCE into a pinned row of the whole model (``HostRow``) and each part
  copies its slice to its own device — one H2D per GPU, over the GPUs' own PCIe links;
* the per-part reductions run on each part's own stream of its own device (``DeviceStream``: the part's GPU is
  made current for every call, so a part's kernels can never land on another GPU or on the null stream),
  independently (FedAvg, FedBuff and fused FedYoGi need no cross-device step: every output element depends
  only on its own column);
* q-FedAvg's one exchange, the per-client squared norms summed over the shards (optimizers.py:96-97), is
  an RCCL all-gather over xGMI issued for all devices at once, followed by a fixed-order sum on every
  device (``DeviceGroup.sum_f64``), so the result does not depend on the transport;
* egress: per-part D2H straight into the pinned host snapshot (no collective; never a collective from a
  servicer thread), one snapshot per model version, immutable while any thread reads it.

The element chains are the single-GPU ones, so FedAvg / FedBuff results are bit-identical to one GPU and
to the reference; q-FedAvg only re-associates the fp64 norm sum (north-star tolerance).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from ...bucket import BucketLayout, HostRow, PieceSegments, RegisteredUpload, default_pack_workers
from ...round import default_capacity
from ...state import DeviceGroup, PartOf, ShardGroup
from .torch_model_adapter import TorchModelAdapter


class ShardedRound:
    """One round over the parts: the arrival is gathered once (``HostRow``) and staged by every part."""

    def __init__(self, adapter: "ShardedModelAdapter", rounds):
        self.adapter, self.rounds = adapter, rounds
        self.policy, self.K = rounds[0].policy, rounds[0].K
        self.cg = None

    @property
    def n(self) -> int:
        return self.rounds[0].n

    def add(self, update, **kw):
        row = self.adapter._stage_row(update)  # validates the update; nothing is staged if it raises
        for rnd in self.rounds:
            rnd.add(row, **kw)

    def adopt_resident(self, n: int):
        """Bench hook: ``n`` arrivals already written into every part's staging slots on its device
        (``DeviceRound.adopt_resident``)."""
        for rnd in self.rounds:
            rnd.adopt_resident(n)


class ShardedModelAdapter(TorchModelAdapter):
    """``TorchModelAdapter`` whose fp32 bucket is split over ``devices`` (GPU ordinals or torch devices;
    default: every visible GPU) of this process.  ``transport``: "rccl" (default when the devices are
    distinct), or "copy" (device-to-device copies; required when a device hosts several parts)."""

    #: pinned full-model rows an upload is gathered into before the per-device copies (the host packs
    #: update k+1 while update k is still crossing PCIe)
    INGRESS_ROWS = 2
    #: round 4: an upload whose large arrays all view ONE host buffer (the executor's payload decoded zero-copy by
    #: the mixin's deserialize_response, fedscale_amd/ingress.py) has that buffer registered in place, and every
    #: GPU's copy engine reads its slice of the large arrays straight out of it (``RegisteredUpload``): one
    #: host-DRAM pass per byte instead of three (profiles/r04_register_probe.log).  Entries below this size, and
    #: uploads that do not qualify, take the pinned-row gather.  -1 turns it off.
    REGISTER_MIN_ENTRY_BYTES = 1 << 20
    #: registrations kept while their copies may still run (older ones are waited for and released first)
    REGISTER_MAX_PENDING = 4

    def __init__(self, model: torch.nn.Module, optimizer=None, devices=None, staging_capacity: Optional[int] = None,
                 transport: Optional[str] = None):
        if devices is None:
            devices = list(range(torch.cuda.device_count()))
        self.group = devices if isinstance(devices, DeviceGroup) else DeviceGroup(devices, transport)
        N = self.group.world
        self.model = model
        self.optimizer = optimizer
        self.device = self.group.devices[0]
        self.dstream = self.group.streams[0]
        self.shards = ShardGroup()  # this process is one rank; its parts are in self.parts
        self.layout = BucketLayout.from_state_dict(model.state_dict())  # the whole model (host side)
        self.staging_capacity = staging_capacity
        self.parts = []
        for r, dev in enumerate(self.group.devices):
            opt = optimizer.for_shard(dev) if optimizer is not None else None
            self.parts.append(TorchModelAdapter(model, optimizer=opt, device=dev, shards=PartOf(r, N, self.group),
                                                staging_capacity=staging_capacity, dstream=self.group.streams[r]))
        self._rows = []
        self._next_row = 0
        self._regs = {}  # registered address -> [payload object, events of the copies out of it]
        self._reg_segs = None
        self.registered_uploads = 0  # uploads staged out of their registered payload (the rest: pinned-row gather)
        self.registration_fallbacks = 0  # qualifying uploads that took the gather (page shared / register refused)
        self.pack_workers = default_pack_workers()
        self._init_egress(True)
        self._egress_src = self._part_buffers()

    def __reduce__(self):
        return (self.__class__, (self.get_model(), self.optimizer, [d.index for d in self.group.devices], None,
                                 self.group.transport))

    def close(self):
        """Destroy the device group's RCCL communicator now (its HBM and proxy threads) rather than at interpreter
        exit, where ``state._LIVE_GROUPS`` would otherwise hold it, and release every registered upload (after its
        copies).  Idempotent; the adapter stays usable (the next collective re-creates the communicator).  Call it
        from the thread that drives the rounds."""
        self._release_registrations(block=True)
        self.group.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- ingress ----------------------------------------------------------------------------------
    def _stage_row(self, update):
        """Gather one upload into the next pinned full-model row (validated like the reference's list
        handling, aggregator.py:494-496; multi-threaded native gather) — or, when its large arrays view one
        registrable host buffer, only its small entries (``RegisteredUpload``)."""
        L = self.layout
        if not self._rows:
            self._rows = [HostRow(L.ld, L.ldq) for _ in range(self.INGRESS_ROWS)]
        row = self._rows[self._next_row]
        plan = L.host_gather_plan(L.values_of(update))
        reg = self._register(plan)
        row.wait()  # every part's H2D out of this row has completed
        if reg is not None:
            segs, src, addr = reg
            ps, po, pn, keep, side = plan
            small = segs.small_pieces
            L.run_host_gather((ps[small], po[small], pn[small], keep, side), row.f_np, row.i_np,
                              workers=self.pack_workers)
            out = RegisteredUpload(row, segs, src)
            self._regs[addr][1].append(out)
            self.registered_uploads += 1
        else:
            L.run_host_gather(plan, row.f_np, row.i_np, workers=self.pack_workers)
            out = row
        self._next_row = (self._next_row + 1) % len(self._rows)
        return out

    def _register(self, plan):
        """(segments, large-entry addresses, registered address) when the upload's large fp32 arrays all view one
        host buffer that is (or now gets) registered; None: take the pinned-row gather."""
        from ... import _native

        if self.REGISTER_MIN_ENTRY_BYTES < 0:
            return None
        if self._reg_segs is None:
            self._reg_segs = PieceSegments(self.layout, self.REGISTER_MIN_ENTRY_BYTES)
        segs = self._reg_segs
        if not segs.large:
            return None
        ps, po, pn, keep, side = plan
        root = None
        for j in segs.large_pieces:  # the arrays as handed in (host_gather_plan keeps them, contiguous)
            r = keep[j]
            while isinstance(r.base, np.ndarray):
                r = r.base
            r = r.base
            # Only an IMMUTABLE payload may be read after on_result returns (the copy engine reads the registered
            # buffer asynchronously): the gRPC payload's bytes, or a read-only view of bytes (np.frombuffer wraps
            # each such view in a memoryview of its own, so the bytes object is the identity).  A bytearray,
            # writable memoryview, mmap or numpy-owned buffer the caller could reuse takes the pinned-row gather,
            # which has copied everything before add returns, as the reference's copy at add time does.
            if type(r) is memoryview and r.readonly and type(r.obj) is bytes:
                r = r.obj
            if type(r) is not bytes or (root is not None and r is not root):
                return None
            root = r
        try:
            buf = np.frombuffer(root, dtype=np.uint8)
        except (TypeError, ValueError):
            return None
        lo, n = buf.ctypes.data, buf.nbytes
        page = 4096
        a0, a1 = lo // page * page, -(-(lo + n) // page) * page  # whole pages of the payload's own mapping
        self._release_registrations(block=False)
        if a0 in self._regs and a1 > self._regs[a0][2]:
            # the first page is registered, but by an earlier payload whose registration ends before this one does:
            # its tail pages are not registered, so this upload takes the gather
            self.registration_fallbacks += 1
            return None
        if a0 not in self._regs:
            # two payloads next to each other on the heap can share a boundary page, and a range already registered
            # cannot be registered again: this upload takes the gather, the next ones are tried afresh
            if any(b0 < a1 and a0 < b1 for b0, (_, _, b1) in self._regs.items()):
                self.registration_fallbacks += 1
                return None
            if len(self._regs) >= self.REGISTER_MAX_PENDING:
                self._release_registrations(block=True, keep=self.REGISTER_MAX_PENDING - 1)
            try:
                _native.call("fa_host_register", a0, a1 - a0)
            except _native.FedAggError:
                self.registration_fallbacks += 1  # e.g. memory the runtime will not pin: this upload only
                return None
            self._regs[a0] = [root, [], a1]
        return segs, np.asarray([ps[j] for j in segs.large_pieces], dtype=np.uint64), a0

    def _release_registrations(self, block: bool, keep: int = 0):
        """Unregister uploads whose copies have all completed (``block``: wait for the oldest ones, until at most
        ``keep`` remain)."""
        from ... import _native

        for addr in list(self._regs):
            ups = self._regs[addr][1]
            done = all(ev.query() for up in ups for ev in up.events)
            if not done and block and len(self._regs) > keep:
                for up in ups:
                    for ev in up.events:
                        ev.synchronize()
                done = True
            if done:
                del self._regs[addr]
                _native.call("fa_host_unregister", addr)

    # ---- rounds -----------------------------------------------------------------------------------
    def begin_round(self, K: int, policy: str, capacity: Optional[int] = None, keep_mean=True) -> ShardedRound:
        cap = capacity or self.staging_capacity
        if not cap and all(p.staging is not None and p.staging.capacity >= K for p in self.parts):
            cap = K  # the round fits the staging every part already holds (no free-memory query)
        if not cap:  # one capacity for all parts, so they fold their chunks in step; parts sharing a
            # device share its budget (half of the free HBM)
            per_dev = {}
            for p in self.parts:
                per_dev[p.device] = per_dev.get(p.device, 0) + 1
            cap = min(default_capacity(p.layout, K, p.device, budget_fraction=0.5 / per_dev[p.device])
                      for p in self.parts)
        return ShardedRound(self, [p.begin_round(K, policy, capacity=cap, keep_mean=keep_mean) for p in self.parts])

    def apply_round(self, rnd: ShardedRound, denom32: float, denom64: float, client_training_results=None,
                    keep_mean: bool = True):
        if rnd.policy == "qfedavg":
            self._apply_qfed(rnd)
        elif not self._finish_parts_at_once(rnd, denom32, denom64):
            for p, r in zip(self.parts, rnd.rounds):
                p.apply_round(r, denom32, denom64, None, keep_mean)
        self._commit()
        self._release_registrations(block=False)

    #: FedAvg rounds (without a server step, or with FedYoGi's) finish every part with ONE native call per pass
    #: (fa_reduce_parts, then fa_yogi_step_parts)
    FINISH_PARTS_AT_ONCE = True

    def _finish_parts_at_once(self, rnd: ShardedRound, denom32: float, denom64: float) -> bool:
        """FedAvg rounds of two or more parts: every part's finishing reduce goes out in one native call instead of
        one Python call chain per part — the same launches on the same streams, so the same bits; the per-part host
        cost was the in-process round's serial part.  Without a server step the mean IS the new model
        (aggregator.py:505-511); with FedYoGi (config 4, optimizers.py:43-63, yogi.py:15-36) the mean goes to its
        own buffer and one more call steps every part (``TorchModelAdapter._apply_round``'s two-pass finish).  The
        side table and the version commit follow per part.  False: take the per-part path (q-FedAvg, one part,
        FedBuff, a per-client round)."""
        from ... import kernels as kx

        opt = self.optimizer
        mode = getattr(opt, "mode", None) if opt is not None else None
        if (not self.FINISH_PARTS_AT_ONCE or rnd.policy != "fedavg" or len(self.parts) < 2
                or mode not in (None, "fed-yogi") or any(r.cg is not None for r in rnd.rounds)):
            return False
        yogi = mode == "fed-yogi"
        ys = [p.optimizer.gradient_controller for p in self.parts] if yogi else None
        if yogi and len({y.initialized for y in ys}) != 1:
            return False
        xs, Ks, Ps, means, accs, lasts, outs = [], [], [], [], [], [], []
        for i, (p, r) in enumerate(zip(self.parts, rnd.rounds)):
            r._check_complete()
            r.staging.drain()
            out_f, out_s = p._scratch_buffers()
            mean_f = out_f
            if yogi:
                last = p._snapshot()
                if ys[i].layout is None or p._mean_f is None or p._mean_f is last.f32 or p._mean_f is out_f:
                    with p.dstream:  # first round: the YoGi state and the mean buffer on the part's device
                        ys[i].bind(p.layout, p.device)
                        if p._mean_f is None or p._mean_f is last.f32 or p._mean_f is out_f:
                            p._mean_f = torch.zeros(p.layout.ld, dtype=torch.float32, device=p.device)
                mean_f = p._mean_f
                lasts.append(last)
            xs.append(r.staging.x)
            Ks.append(r.slot)
            Ps.append(p.layout.P)
            means.append(mean_f)
            outs.append((out_f, out_s))
            accs.append(None if r.chunks_done == 0 else r.acc)
        streams = [p.dstream.handle for p in self.parts]
        kx.reduce_parts(xs, Ks, Ps, means, accs, streams, denom=denom32, finalize=True)
        if yogi:
            y0 = ys[0]
            kx.yogi_step_parts(means, [last.f32 for last in lasts], [y.m for y in ys], [y.v for y in ys],
                               [o[0] for o in outs], Ps, streams, init=not y0.initialized, **y0.fp32_hparams())
        for i, (p, r) in enumerate(zip(self.parts, rnd.rounds)):
            out_f, out_s = outs[i]
            with p.dstream.joined():  # the caller's stream on this GPU is ordered after the part's work
                L = p.layout
                kx.side_accumulate(r.staging.xi, r.slot, L.Q, 0, acc_i=r.acc_i, acc_d=r.acc_d,
                                   accumulate=r.chunks_done > 0)
                kx.side_close(L.Q, 0, denom64, acc_i=r.acc_i, acc_d=r.acc_d, cur=p._mean_s,
                              model=None if yogi else out_s)
                if yogi:
                    ys[i].step_side(p._mean_s, lasts[i].side, model=out_s)
                    ys[i].initialized = True
                else:
                    p._mean_f = out_f
                p._mean_valid = True
                p._commit_scratch()
        return True

    def _apply_qfed(self, rnd: ShardedRound):
        mode = getattr(self.optimizer, "mode", None)
        if mode != "q-fedavg":
            raise RuntimeError("a q-FedAvg round needs the q-fedavg server optimizer")
        for r in rnd.rounds:
            r.qfed_fold()
        # optimizers.py:96-97: each client's squared norm is the sum over ALL parameters, i.e. over the shards
        self.group.sum_f64([r.sqnorm for r in rnd.rounds])
        for p, r in zip(self.parts, rnd.rounds):
            p._finish_qfed(r)

    def _part_buffers(self):
        return [(p._f[p._cur], p._s[p._cur]) for p in self.parts]

    def _commit(self):
        """The parts have committed their new buffers one by one; the model version and the buffers egress
        reads change together here, so a servicer thread never snapshots a mix of old and new parts."""
        with self._egress_lock:
            self._egress_src = self._part_buffers()
            self._version += 1

    # ---- reference API ----------------------------------------------------------------------------
    def set_weights(self, weights, is_aggregator=True, client_training_results=None):
        """torch_model_adapter.py:23-39 over the parts.  FedYoGi runs per part (no cross-shard step);
        q-FedAvg stages the retained results (aggregator.py:466-467) and runs the sharded round."""
        weights = list(weights)
        opt = self.optimizer
        if opt is not None and is_aggregator and getattr(opt, "mode", None) == "q-fedavg":
            rnd = self.begin_round(len(client_training_results), "qfedavg")
            a = opt.args
            from ..aggregation.aggregator import StagedUpload

            for res in client_training_results:
                if isinstance(res["update_weight"], StagedUpload):
                    raise RuntimeError("a retained q-FedAvg result's update_weight was released after it was "
                                       "staged in HBM (device_release_uploads); set_weights cannot re-stage it")
                rnd.add(res["update_weight"], loss=res["moving_loss"], learning_rate=a.learning_rate, q=a.qfed_q)
            self._apply_qfed(rnd)
            for p in self.parts:  # the reference's model_weights: the list it was handed
                with p.dstream.joined():
                    p.dstream.wait_caller()
                    p._mean_f = torch.zeros(p.layout.ld, dtype=torch.float32, device=p.device)
                    p._pack_values(weights, p._mean_f, p._mean_s)
                p._mean_valid, p._mean_round = True, None
        else:
            for p in self.parts:
                p.set_weights(weights, is_aggregator, client_training_results)
        self._commit()

    def _copy_to_host(self, f_cpu: torch.Tensor, s_cpu: torch.Tensor):
        """Per-part D2H into the pinned snapshot (each over its own device's link); no collective.  Reads
        the buffers of the committed version (``_egress_src``, swapped with ``_version`` under the egress
        lock the caller holds), not the parts' live pointers, which flip one part at a time."""
        for p in self.parts:
            p._ready.synchronize()  # every part's writes, whatever stream they ran on
        src = self._egress_src
        for p, (f_dev, _) in zip(self.parts, src):
            L = p.layout
            if L.P:
                f_cpu[L.p0:L.p1].copy_(f_dev[:L.P], non_blocking=True)
        s_cpu[:self.layout.Q].copy_(src[0][1][:self.layout.Q])
        for p in self.parts:
            torch.cuda.current_stream(p.device).synchronize()

    def _fetch_mean(self) -> list:
        L = self.layout
        f_cpu = np.empty(max(1, L.P_full), dtype=np.float32)
        s_cpu = None
        for p in self.parts:
            with p.dstream.joined():  # the D2H copies run on the stream that computed the part's mean
                mean_f, mean_s = p._mean_device()
                if p.layout.P:
                    f_cpu[p.layout.p0:p.layout.p1] = mean_f[:p.layout.P].cpu().numpy()
                if s_cpu is None:
                    s_cpu = mean_s[:L.Q].cpu().numpy()
        return self._mean_lists(f_cpu, s_cpu)

    # the server optimizer's YoGi state lives in the parts (one m/v slice per device)
    def shard_optimizers(self):
        return [p.optimizer for p in self.parts]

