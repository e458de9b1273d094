"""Device server optimizer — drop-in for fedscale/cloud/aggregation/optimizers.py:5-108.

``TorchServerOptimizer(mode, args, device, sample_seed=233)`` keeps the reference constructor and
``update_round_gradient(last_model, current_model, target_model, client_training_results=None)``.

Accepted inputs:
  * the reference's types — ``last_model``/``current_model`` lists of tensors (CPU or device),
    ``target_model`` an ``nn.Module`` (or any object with state_dict/load_state_dict),
    ``client_training_results`` the list of result dicts retained by the aggregator; the tensors are
    flattened into HBM, the step runs as HIP kernels, and the module is loaded with the result;
  * the device types used by ``fedscale_amd``'s TorchModelAdapter — ``FlatState`` snapshots, the
    adapter itself as ``target_model`` and a ``DeviceRound`` as ``client_training_results``.

Modes (optimizers.py:43-108): ``"fed-yogi"`` -> YoGi step; ``"q-fedavg"`` -> q-FedAvg; anything else
(None, "fed-avg", "fed-prox") -> no-op (FedAvg was applied by the aggregator).
"""
from __future__ import annotations

import torch

from ... import kernels as kx
from ...bucket import BucketLayout
from ...round import DeviceRound
from ...state import FlatState


class TorchServerOptimizer(object):
    def __init__(self, mode, args, device, sample_seed=233):
        self.mode = mode
        self.args = args
        self.device = device
        if mode == "fed-yogi":
            from ...utils.optimizer.yogi import YoGi

            self.gradient_controller = YoGi(eta=args.yogi_eta, tau=args.yogi_tau, beta=args.yogi_beta,
                                            beta2=args.yogi_beta2)

    def for_shard(self, device) -> "TorchServerOptimizer":
        """The optimizer of one shard of a model sharded over the GPUs of this process: same mode and the
        same live ``args`` (optimizers.py:69 reads the learning rate at step time), its own YoGi state
        (m_t / v_t of the shard's parameters, yogi.py:11-19)."""
        return TorchServerOptimizer(self.mode, self.args, device)

    # ---------------------------------------------------------------------------------------------
    def _dev(self):
        d = self.device
        if d is None or (isinstance(d, str) and not d.startswith("cuda")) or (
                isinstance(d, torch.device) and d.type != "cuda"):
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device(d)

    def update_round_gradient(self, last_model, current_model, target_model, client_training_results=None):
        if self.mode not in ("fed-yogi", "q-fedavg"):
            return  # optimizers.py:106-108
        if isinstance(last_model, FlatState):
            return self._device_step(last_model, current_model, target_model, client_training_results)
        return self._list_step(last_model, current_model, target_model, client_training_results)

    # ---- device path (FlatState in, adapter out) -------------------------------------------------
    def _device_step(self, last: FlatState, current: FlatState, adapter, results):
        with adapter.dstream.joined():  # the adapter's GPU and stream (set_weights already entered them)
            self._device_step_on_stream(last, current, adapter, results)

    def _device_step_on_stream(self, last: FlatState, current: FlatState, adapter, results):
        lay = last.layout
        out_f, out_s = adapter._scratch_buffers()
        if self.mode == "fed-yogi":
            y = self.gradient_controller
            y.bind(lay, last.f32.device)
            kx.yogi_step(current.f32, last.f32, y.m, y.v, out_f, lay.P, init=not y.initialized,
                         **y.fp32_hparams())
            y.step_side(current.side, last.side, model=out_s)
            y.initialized = True
        else:
            rnd = results
            if not isinstance(rnd, DeviceRound):
                rnd = self._stage_results(lay, last, results, dstream=adapter.dstream)
            rnd.finalize_qfed(out=out_f, model_side=out_s, sqnorm_allreduce=adapter._sqnorm_allreduce())
        adapter._commit_scratch()

    def _stage_results(self, lay: BucketLayout, last: FlatState, results, dstream=None) -> DeviceRound:
        """q-FedAvg from the reference's retained list of result dicts (aggregator.py:466-467)."""
        from .aggregator import StagedUpload

        rnd = DeviceRound(lay, last.f32.device, len(results), "qfedavg", last_f32=last.f32, last_i64=last.side,
                          dstream=dstream)
        lr, q = self.args.learning_rate, self.args.qfed_q
        for res in results:
            if isinstance(res["update_weight"], StagedUpload):
                raise RuntimeError(
                    "a retained q-FedAvg result's update_weight was released after it was staged in HBM "
                    "(DeviceAggregatorMixin.device_release_uploads); only the device round can consume it — "
                    "set device_release_uploads = False to keep the host arrays for this set_weights path")
            rnd.add(res["update_weight"], loss=res["moving_loss"], learning_rate=lr, q=q)
        return rnd

    # ---- reference-typed path (lists + nn.Module) ------------------------------------------------
    def _list_step(self, last_model, current_model, target_model, results):
        from ..internal.torch_model_adapter import TorchModelAdapter

        if isinstance(target_model, TorchModelAdapter):
            raise TypeError("pass FlatState snapshots together with a fedscale_amd TorchModelAdapter")
        sd = target_model.state_dict()
        dev = self._dev()
        # a transient adapter over the module's layout runs the device step and loads the result back
        adapter = TorchModelAdapter(target_model, optimizer=None, device=dev, _load_from=last_model)
        lay = adapter.layout
        last = adapter._snapshot()
        cur_f = torch.zeros(lay.ld, dtype=torch.float32, device=dev)
        cur_s = torch.zeros(lay.ldq, dtype=torch.float64, device=dev)
        if current_model is not None:
            adapter._pack_values(list(current_model), cur_f, cur_s)
        self._device_step(last, FlatState(lay, cur_f, cur_s), adapter, results)
        new = adapter.get_weights()
        target_model.load_state_dict({n: t for n, t in zip(sd.keys(), new)})
