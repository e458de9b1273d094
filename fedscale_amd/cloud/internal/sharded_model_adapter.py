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

from ...bucket import BucketLayout, HostRow, default_pack_workers
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
        self.pack_workers = default_pack_workers()
        self._init_egress(True)
        self._egress_src = self._part_buffers()

    def __reduce__(self):
        return (self.__class__, (self.get_model(), self.optimizer, [d.index for d in self.group.devices], None,
                                 self.group.transport))

    def close(self):
        """Destroy the device group's RCCL communicator now (its HBM and proxy threads) rather than at interpreter
        exit, where ``state._LIVE_GROUPS`` would otherwise hold it.  Idempotent; the adapter stays usable (the next
        collective re-creates the communicator).  Call it from the thread that drives the rounds."""
        self.group.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- ingress ----------------------------------------------------------------------------------
    def _stage_row(self, update) -> HostRow:
        """Gather one upload into the next pinned full-model row (validated like the reference's list
        handling, aggregator.py:494-496; multi-threaded native gather)."""
        L = self.layout
        if not self._rows:
            self._rows = [HostRow(L.ld, L.ldq) for _ in range(self.INGRESS_ROWS)]
        row = self._rows[self._next_row]
        plan = L.host_gather_plan(L.values_of(update))
        row.wait()  # every part's H2D out of this row has completed
        L.run_host_gather(plan, row.f_np, row.i_np, workers=self.pack_workers)
        self._next_row = (self._next_row + 1) % len(self._rows)
        return row

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
        else:
            for p, r in zip(self.parts, rnd.rounds):
                p.apply_round(r, denom32, denom64, None, keep_mean)
        self._commit()

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

