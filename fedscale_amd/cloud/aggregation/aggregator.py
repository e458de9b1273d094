"""Device aggregation hook — drop-in for ``Aggregator.update_weight_aggregation``.

Reference: fedscale/cloud/aggregation/aggregator.py:489-511 (sync FedAvg, + the q-FedAvg retention of
:466-467 and the server step reached through set_weights, :508-511) and
fedscale/cloud/aggregation/async_aggregator.py:115-137 (FedBuff).  The plugin API of the reference is
subclassing ``Aggregator`` and overriding ``update_weight_aggregation(self, results)``
(precedents: AsyncAggregator, MNN/TFLite aggregators, examples/auxo); so is this::

    from fedscale.cloud.aggregation.aggregator import Aggregator
    from fedscale_amd.cloud.aggregation.aggregator import DeviceAggregatorMixin

    class MI355XAggregator(DeviceAggregatorMixin, Aggregator):
        pass

State contract (the reference test's MockAggregator, fedscale/tests/cloud/aggregation/test_aggregator.py:11-17):
``model_weights, model_in_update, tasks_round, model_wrapper, client_training_results`` (+ ``args``,
and for FedBuff ``round, client_task_model_version, aggregation_denominator``).  ``model_in_update`` is
incremented by the caller before the call (aggregator.py:484); the first/last tests are ==1 / ==K
(:430-434).  ``model_wrapper`` must be a ``fedscale_amd`` TorchModelAdapter.
"""
from __future__ import annotations

import numpy as np

from ..internal.torch_model_adapter import TorchModelAdapter


class _Decoded:
    """An upload payload already decoded by the servicer thread (``add_event_handler``)."""

    __slots__ = ("value",)

    def __init__(self, value):
        self.value = value


class StagedUpload:
    """What a retained q-FedAvg result holds in place of ``update_weight`` once the upload is staged in HBM
    (``device_release_uploads``): the device round is the only consumer, so the host arrays are let go."""

    __slots__ = ("arrival",)

    def __init__(self, arrival: int):
        self.arrival = arrival

    def __repr__(self):
        return f"<update {self.arrival} of this round, staged in HBM>"


class DeviceAggregatorMixin:
    #: clients staged per chunk (None: as many as fit in half of the free HBM)
    device_round_capacity = None
    #: keep the FedAvg mean as ``model_weights`` (aggregator.py:505-507): fed-yogi rounds write it in the
    #: fused pass (P*4 bytes); q-FedAvg rounds that span several staging chunks fuse the FedAvg chain into
    #: their phase-1 kernel (measured 9 % of it), single-chunk ones recompute it from the staged updates
    #: when model_weights is read; "always" fuses the chain in every q-FedAvg round (the mean then survives
    #: the next round's reuse of the staging); False keeps no mean
    device_keep_mean = True
    #: drop the retained q-FedAvg results' ``update_weight`` (aggregator.py:466-467) once it is staged in
    #: HBM: the device round never reads it again, and with zero-copy ingress each retained array would
    #: pin its whole upload payload in host memory (45 GB for 1000 ResNet-18 uploads)
    device_release_uploads = True
    #: unpickle executor payloads without copying their arrays (fedscale_amd/ingress.py); the arrays of
    #: ``update_weight`` are then read-only views of the payload
    device_zero_copy_ingress = True
    #: create_client_task / get_test_config hand the servicer an EgressHandle (the cached pickled bytes of
    #: the model version) instead of a fresh clone of the model per request
    device_egress_handles = True
    #: the servicer thread that receives an upload (CLIENT_EXECUTE_COMPLETION, aggregator.py:958-959) runs
    #: its zero-copy decode, to overlap the main loop's gather + H2D of the previous update. Off: measured
    #: +4 % on one box and -10 % on another (GIL contention once the main loop is at the H2D bound)
    device_decode_on_arrival = False
    #: pickled bytes kept for past model versions' get_weights() lists (FedBuff's model_cache holds
    #: max_staleness + 1 of them, config_parser.py:123)
    device_egress_past_versions = 8
    #: GPU ordinals to shard the model over inside this process (None: FEDAGG_DEVICES, else one GPU)
    device_shards = None
    #: opt-in: bind the main thread (which stages every upload into pinned memory) to the CPUs of the GPU's NUMA
    #: node, so the staging lands next to the GPU's PCIe link (fedscale_amd/hostnuma.py; single-GPU adapters).  Off
    #: by default: the affinity is process-wide in effect (every thread the main thread starts later inherits it:
    #: torch's intra-op pool, gRPC work), for ~7 us on config 1's round (profiles/r03_numa_probe.log).  When on,
    #: torch's intra-op thread count is lowered to the node's CPUs and the binding is logged
    device_numa_bind = False

    _device_round = None

    # same predicates as aggregator.py:430-434 (defined here too so the mixin also works standalone)
    def _is_first_result_in_round(self):
        return self.model_in_update == 1

    def _is_last_result_in_round(self):
        return self.model_in_update == self.tasks_round

    def _aggregation_device(self):
        """The GPU of the reference's ``self.device`` (aggregator.py:47: ``args.cuda_device`` when
        ``use_cuda``, e.g. "cuda:3"; None = the current device).  The device path has no CPU fallback."""
        d = getattr(self, "device", None)
        if d is None:
            return None
        import torch

        d = torch.device(d) if not isinstance(d, int) else torch.device("cuda", d)
        if d.type != "cuda":
            raise ValueError(f"the aggregator device is {d} (use_cuda=False?): the device aggregation path runs on "
                             f"a GPU only; set use_cuda and cuda_device, or use the reference Aggregator")
        return d

    def init_model(self):
        """aggregator.py:198-211, re-wired onto the device adapter + device server optimizer, on the GPU the
        reference's ``--cuda_device`` selects (``self.device``, aggregator.py:47).  With ``device_shards``
        (or FEDAGG_DEVICES="0,1,...") naming more than one GPU, the model is sharded over them inside this
        one process (``ShardedModelAdapter``)."""
        from .optimizers import TorchServerOptimizer

        super().init_model()
        model = self.model_wrapper.get_model()
        devs = self.device_shards
        if devs is None:
            import os

            env = os.environ.get("FEDAGG_DEVICES")
            devs = [int(d) for d in env.split(",") if d.strip()] if env else None
        if devs is not None and len(devs) > 1:
            from ..internal.sharded_model_adapter import ShardedModelAdapter

            opt = TorchServerOptimizer(self.args.gradient_policy, self.args, devs[0])
            self.model_wrapper = ShardedModelAdapter(model, optimizer=opt, devices=devs)
        else:
            dev = devs[0] if devs else self._aggregation_device()
            opt = TorchServerOptimizer(self.args.gradient_policy, self.args, dev)
            self.model_wrapper = TorchModelAdapter(model, optimizer=opt, device=dev)
            if self.device_numa_bind:
                from ...hostnuma import bind_to_gpu

                bind_to_gpu(getattr(self.model_wrapper, "device", dev), match_torch_threads=True, log=True)

    def _wrapper(self) -> TorchModelAdapter:
        w = self.model_wrapper
        if not isinstance(w, TorchModelAdapter):
            raise TypeError(f"model_wrapper is {type(w).__name__}; the device path needs "
                            f"fedscale_amd.cloud.internal.torch_model_adapter.TorchModelAdapter")
        return w

    def _device_policy(self) -> str:
        opt = self._wrapper().optimizer
        return "qfedavg" if (opt is not None and getattr(opt, "mode", None) == "q-fedavg") else "fedavg"

    def deserialize_response(self, responses):
        """aggregator.py:695-704 (``pickle.loads``) without the copy of every array's bytes: the same
        object tree, large arrays as read-only views of ``responses`` (fedscale_amd/ingress.py)."""
        sup = getattr(super(), "deserialize_response", None)
        # only in place of the plain pickle.loads: a subclass that converts the payload (the TFLite / MNN
        # aggregators, aggregator_tflite.py:47-58) keeps its own path
        if type(responses) is _Decoded:  # decoded on arrival (add_event_handler)
            return responses.value
        if self.device_zero_copy_ingress and self._reference_impl("deserialize_response") and \
                type(responses) is bytes:
            from ...ingress import loads

            return loads(responses)
        if sup is not None:
            return sup(responses)
        import pickle

        return pickle.loads(responses)

    def add_event_handler(self, client_id, event, meta, data):
        """aggregator.py:830-840, called by the servicer thread (CLIENT_EXECUTE_COMPLETION :958-959). The
        reference queues the raw payload and the main loop unpickles it (:993-994). Here an upload is
        decoded (zero-copy, ``deserialize_response``) on this thread before it is queued, so the decode
        overlaps the main loop's native gather and H2D of the previous update, which release the GIL.
        A payload that fails to decode is queued as it came, so the main loop raises as before."""
        if (self.device_decode_on_arrival and event == "upload_model" and type(data) is bytes  # commons.UPLOAD_MODEL
                and self.device_zero_copy_ingress and self._reference_impl("deserialize_response")
                and self._reference_impl("add_event_handler")):
            try:
                data = _Decoded(self.deserialize_response(data))
            except Exception:
                pass
        sup = getattr(super(), "add_event_handler", None)
        if sup is not None:
            return sup(client_id, event, meta, data)
        import collections

        self.__dict__.setdefault("server_events_queue", collections.deque()).append((client_id, event, meta, data))

    def serialize_response(self, responses):
        """aggregator.py:706-715 (``pickle.dumps``), with the global model's bytes made once per model
        version: the reference pickles get_weights() again for every executor request
        (create_client_task :804, get_test_config :816, UPDATE_MODEL :903)."""
        payload = getattr(responses, "egress_payload", None)
        if type(payload) is bytes:  # an EgressHandle: the bytes of its own model version
            return payload
        key = getattr(responses, "egress_key", None)
        if key is not None:
            wrappers = self.model_wrapper if isinstance(self.model_wrapper, list) else [self.model_wrapper]
            for w in wrappers:
                b = w.egress_bytes(key) if isinstance(w, TorchModelAdapter) else None
                if b is not None:
                    return b
            # a past model version: FedBuff hands out the lists of its model_cache
            # (async_aggregator.py:54,71-73) again for every client task; each list object pickles once
            import pickle

            old = self.__dict__.setdefault("_egress_past", {})
            hit = old.get(id(responses))
            if hit is not None and hit[0] is responses:
                return hit[1]
            b = pickle.dumps(list(responses))
            if len(old) >= self.device_egress_past_versions:
                old.pop(next(iter(old)))
            old[id(responses)] = (responses, b)  # holds the list, so its id stays unique
            return b
        sup = getattr(super(), "serialize_response", None)
        if sup is not None:
            return sup(responses)
        import pickle

        return pickle.dumps(responses)

    def _reference_impl(self, name) -> bool:
        """True when the next ``name`` in the MRO is the reference Aggregator's own (a plugin that
        overrides it, e.g. Auxo's create_client_task, keeps its version)."""
        sup = getattr(super(), name, None)
        return sup is None or getattr(sup, "__qualname__", "").split(".")[-2:] == ["Aggregator", name]

    def _egress_weights(self):
        """``self.model_wrapper.get_weights()`` as the servicer uses it (serialised, :905-907): an
        EgressHandle on the cached bytes of this model version instead of a clone of the model."""
        w = self.model_wrapper
        if self.device_egress_handles and isinstance(w, TorchModelAdapter):
            return w.egress_handle()
        return w.get_weights()

    def create_client_task(self, executor_id):
        """aggregator.py:788-804 with the weights handed over as an EgressHandle (``_egress_weights``)."""
        if not self._reference_impl("create_client_task"):
            return super().create_client_task(executor_id)
        next_client_id = self.resource_manager.get_next_task(executor_id)
        train_config = None
        if next_client_id is not None:
            train_config = {"client_id": next_client_id, "task_config": self.get_client_conf(next_client_id)}
        return train_config, self._egress_weights()

    def get_test_config(self, client_id):
        """aggregator.py:806-816 with the weights handed over as an EgressHandle."""
        if not self._reference_impl("get_test_config"):
            return super().get_test_config(client_id)
        return {"client_id": client_id}, self._egress_weights()

    def CLIENT_PING(self, request, context):
        """aggregator.py:870-912, the reference servicer itself. Its UPDATE_MODEL branch (:902-903) calls
        ``model_wrapper.get_weights()`` only to serialise it (:905-907), so for that one call the adapter
        hands back an EgressHandle on the cached bytes instead of cloning the model."""
        sup = super().CLIENT_PING
        w = self.model_wrapper
        q = getattr(self, "individual_client_events", {}).get(request.executor_id)
        if (self.device_egress_handles and isinstance(w, TorchModelAdapter) and q
                and q[0] == "update_model" and self._reference_impl("CLIENT_PING")):  # commons.UPDATE_MODEL
            with w.handle_next_get_weights():
                return sup(request, context)
        return sup(request, context)

    def update_weight_aggregation(self, results):
        rnd = self._device_round
        if rnd is None or self._is_first_result_in_round():
            w = self._wrapper()
            rnd = self._device_round = w.begin_round(self.tasks_round, self._device_policy(),
                                                     capacity=self.device_round_capacity,
                                                     keep_mean=self.device_keep_mean)
        if rnd.policy == "qfedavg":
            a = self._wrapper().optimizer.args  # optimizers.py:69 reads the live args at step time
            rnd.add(results["update_weight"], loss=results["moving_loss"], learning_rate=a.learning_rate,
                    q=a.qfed_q)
            if self.device_release_uploads:
                results["update_weight"] = StagedUpload(rnd.n - 1)
        else:
            rnd.add(results["update_weight"])
        if self._is_last_result_in_round():
            w = self._wrapper()
            K = self.tasks_round
            # np.divide(w, K): fp32 entries divide by fp32(K), int64 sums by float64(K)
            w.apply_round(rnd, float(np.float32(K)), float(K),
                          client_training_results=self.client_training_results, keep_mean=self.device_keep_mean)
            self.model_weights = w.round_mean_weights()
            self._device_round = None


class DeviceAsyncAggregatorMixin(DeviceAggregatorMixin):
    """FedBuff (async_aggregator.py:115-137): staleness-weighted accumulate, divide by the weight sum."""

    def update_weight_aggregation(self, results):
        w = self._wrapper()
        # async_aggregator.py:125-126 — Python-float weight and denominator
        s = 1 / (1 + self.round - self.client_task_model_version[results["client_id"]]) ** 0.5
        self.aggregation_denominator += s
        if self._is_first_result_in_round() or self._device_round is None:
            self._device_round = w.begin_round(self.tasks_round, "fedbuff", capacity=self.device_round_capacity)
        self._device_round.add(results["update_weight"], weight=s)
        if self._is_last_result_in_round():
            den = self.aggregation_denominator
            # np.divide(fp32 array, Python float) divides by fp32(den) (NEP 50); float64 sides by den
            w.apply_round(self._device_round, float(np.float32(den)), float(den), client_training_results=None,
                          keep_mean=self.device_keep_mean)
            self.model_weights = w.round_mean_weights()
            self.aggregation_denominator = 0
            self._device_round = None


class DeviceCohortAggregatorMixin(DeviceAggregatorMixin):
    """Auxo per-cohort FedAvg (examples/auxo/aggregator.py:451-472), one device round per cohort.

    Every reduction field is a list indexed by ``cohort_id`` (``model_wrapper``, ``model_in_update``,
    ``tasks_round``, ``model_weights``); each cohort's ``model_wrapper`` is its own device-resident
    TorchModelAdapter, so cohorts reduce concurrently and independently.  As in the reference,
    set_weights runs without client_training_results (:472)."""

    def _is_first_result_in_round(self, cohort_id=0):
        return self.model_in_update[cohort_id] == 1

    def _is_last_result_in_round(self, cohort_id=0):
        return self.model_in_update[cohort_id] == self.tasks_round[cohort_id]

    def update_weight_aggregation(self, results, cohort_id=0):
        w = self.model_wrapper[cohort_id]
        if not isinstance(w, TorchModelAdapter):
            raise TypeError(f"model_wrapper[{cohort_id}] is {type(w).__name__}; the device path needs "
                            f"fedscale_amd's TorchModelAdapter")
        rounds = self.__dict__.setdefault("_device_rounds", {})
        if self._is_first_result_in_round(cohort_id) or cohort_id not in rounds:
            rounds[cohort_id] = w.begin_round(self.tasks_round[cohort_id], "fedavg",
                                              capacity=self.device_round_capacity)
        rounds[cohort_id].add(results["update_weight"])
        if self._is_last_result_in_round(cohort_id):
            K = self.tasks_round[cohort_id]
            w.apply_round(rounds.pop(cohort_id), float(np.float32(K)), float(K), client_training_results=None,
                          keep_mean=self.device_keep_mean)
            self.model_weights[cohort_id] = w.round_mean_weights()


class DeviceAggregator(DeviceAggregatorMixin):
    """Standalone holder of the hot-path state contract (for tools, tests and non-FedScale callers)."""

    def __init__(self, model_wrapper: TorchModelAdapter, args=None):
        self.model_weights = []
        self.model_in_update = 0
        self.tasks_round = 0
        self.model_wrapper = model_wrapper
        self.client_training_results = []
        self.args = args

    def start_round(self, tasks_round: int):
        """round_completion_handler's reset (aggregator.py:609, 620-623)."""
        self.tasks_round = tasks_round
        self.model_in_update = 0
        self.client_training_results = []

    def on_result(self, results):
        """client_completion_handler's reduction lines (aggregator.py:466-467, 482-487)."""
        if self.args is not None and getattr(self.args, "gradient_policy", None) in ["q-fedavg"]:
            self.client_training_results.append(results)
        self.model_in_update += 1
        self.update_weight_aggregation(results)


class DeviceAsyncAggregator(DeviceAsyncAggregatorMixin, DeviceAggregator):
    def __init__(self, model_wrapper: TorchModelAdapter, args=None):
        DeviceAggregator.__init__(self, model_wrapper, args)
        self.round = 0
        self.client_task_model_version = {}
        self.aggregation_denominator = 0


class DeviceCohortAggregator(DeviceCohortAggregatorMixin):
    """Standalone Auxo-style cohort state (tests / tools)."""

    def __init__(self, wrappers, tasks_round):
        self.model_wrapper = list(wrappers)
        self.tasks_round = list(tasks_round)
        self.model_in_update = [0] * len(self.model_wrapper)
        self.model_weights = [[] for _ in self.model_wrapper]

    def on_result(self, results, cohort_id):
        self.model_in_update[cohort_id] += 1  # examples/auxo/aggregator.py:307
        self.update_weight_aggregation(results, cohort_id)
