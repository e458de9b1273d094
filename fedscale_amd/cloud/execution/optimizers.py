"""Device ClientOptimizer — drop-in for fedscale/cloud/execution/optimizers.py:2-10.

``ClientOptimizer(sample_seed=233)`` and ``update_client_weight(conf, model, global_model=None)`` keep the
reference's names and argument meaning.  The reference runs the FedProx proximal step as one torch op
per parameter tensor after every local optimizer step (torch_client.py:238-240); here it is one
multi-tensor HIP launch over all of the model's parameters (``fa_prox_update``), bit-identical to the
reference's fp32 arithmetic:

    param.data += conf.learning_rate * conf.proxy_mu * (param.data - global_model[idx])

The parameters and ``global_model`` must live on the GPU (an executor training on the MI355X); there is
no CPU fallback.  Any ``gradient_policy`` other than ``'fed-prox'`` is a no-op, as in the reference.
"""
from __future__ import annotations

from ... import kernels as kx


class ClientOptimizer(object):
    def __init__(self, sample_seed=233):
        pass

    def update_client_weight(self, conf, model, global_model=None):
        if conf.gradient_policy == 'fed-prox':
            # the parameters themselves (not .data views: same storage, no per-step tensor objects); the
            # kernel writes in place outside autograd, like the reference's param.data update
            params = list(model.parameters())
            if global_model is None or len(global_model) != len(params):
                raise ValueError("fed-prox needs global_model: one tensor per model parameter")
            # the Python double lr*mu multiplies fp32 tensors, so torch rounds it to fp32 first
            kx.prox_update(params, global_model, float(conf.learning_rate * conf.proxy_mu))
