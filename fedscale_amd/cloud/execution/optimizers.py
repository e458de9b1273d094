"""Device ClientOptimizer — drop-in for fedscale/cloud/execution/optimizers.py:2-10.

``ClientOptimizer(sample_seed=233)`` and ``update_client_weight(conf, model, global_model=None)`` keep the
reference's names and argument meaning.  The reference runs the FedProx proximal step as one torch op
per parameter tensor after every local optimizer step (torch_client.py:238-240); here it is one
multi-tensor HIP launch over all of the model's parameters (``fa_prox_update``), bit-identical to the
reference's fp32 arithmetic:

    param.data += conf.learning_rate * conf.proxy_mu * (param.data - global_model[idx])

``step_and_update(optimizer, conf, model, global_model)`` fuses the executor's preceding
``torch.optim.SGD.step()`` (torch_client.py:236) into the same pass (``fa_sgd_prox_step_groups``).

The parameters and ``global_model`` must live on the GPU (an executor training on the MI355X); there is
no CPU fallback.  Any ``gradient_policy`` other than ``'fed-prox'`` is a no-op, as in the reference.
"""
from __future__ import annotations

from ... import kernels as kx
from ..._native import FA_SGD_FIRST as kx_first, FA_SGD_NESTEROV as kx_nesterov

_NESTEROV = kx_nesterov


class _StepPlan:
    """The launch tables of one (optimizer, global_model) pair, built after a general step that validated
    every tensor: all of the optimizer's parameters had gradients and, where momentum != 0, momentum
    buffers.  A later step re-reads only what changes between local steps — the gradients' pointers and the
    groups' hyper-parameters — and checks by identity / pointer that nothing else moved; torch itself keeps
    a gradient's dtype, device and size equal to its parameter's.  Anything unexpected sends the step
    back to the general path, which rebuilds the plan."""

    # Only weak references to what the executor may drop between rounds (the optimizer with its momentum
    # buffers, the round's global model): a stale plan never keeps a model-sized buffer alive.
    __slots__ = ("opt", "state_id", "groups_id", "ngroups", "group_len", "params", "pptr", "pnumel", "gidx",
                 "has_mom", "bufs", "bptr", "glob_items", "glob_mptr", "globptr", "numel", "T", "stream_dev", "prox")

    def __init__(self, optimizer, params, gidx, bufs, glob_list, glob):
        import weakref

        import numpy as np

        self.opt = weakref.ref(optimizer)
        self.state_id, self.groups_id = id(optimizer.state), id(optimizer.param_groups)
        groups = optimizer.param_groups
        self.ngroups = len(groups)
        self.group_len = [len(g['params']) for g in groups]
        self.params = [weakref.ref(p) for p in params]
        self.pptr = [p.data_ptr() for p in params]
        self.pnumel = [p.numel() for p in params]
        self.gidx = np.asarray(gidx, dtype=np.int64)
        self.has_mom = [float(g['momentum']) != 0 for g in groups]
        self.bufs = [None if b is None else weakref.ref(b) for b in bufs]
        self.bptr = np.asarray([0 if b is None else b.data_ptr() for b in bufs], dtype=np.uint64)
        self.prox = glob_list is not None
        # the global model's tensors (model order), weakly; their pointers in the optimizer's order
        self.glob_items = None if glob_list is None else [weakref.ref(t) for t in glob_list]
        self.glob_mptr = None if glob_list is None else [t.data_ptr() for t in glob_list]
        self.globptr = None if glob is None else np.asarray([t.data_ptr() for t in glob], dtype=np.uint64)
        self.numel = np.asarray(self.pnumel, dtype=np.int64)
        self.T = len(params)
        self.stream_dev = params[0].device


class ClientOptimizer(object):
    def __init__(self, sample_seed=233):
        self._plan = None

    def update_client_weight(self, conf, model, global_model=None):
        if conf.gradient_policy == 'fed-prox':
            # the parameters themselves (not .data views: same storage, no per-step tensor objects); the
            # kernel writes in place outside autograd, like the reference's param.data update
            params = list(model.parameters())
            if global_model is None or len(global_model) != len(params):
                raise ValueError("fed-prox needs global_model: one tensor per model parameter")
            # the Python double lr*mu multiplies fp32 tensors, so torch rounds it to fp32 first
            kx.prox_update(params, global_model, float(conf.learning_rate * conf.proxy_mu))

    @staticmethod
    def _fused_ok(optimizer, gmap, prox) -> bool:
        """The fused launch covers plain torch.optim.SGD over dense, contiguous fp32 device tensors whose
        parameters are all the model's (and have a global counterpart under fed-prox). Anything else
        (AMP half params, channels_last, sparse grads, params outside model.parameters()) takes the two
        reference calls, which torch and update_client_weight handle as the reference does."""
        import torch

        if type(optimizer) is not torch.optim.SGD:
            return False
        dev = None
        for g in optimizer.param_groups:
            if g.get('maximize', False) or g.get('differentiable', False):
                return False
            for p in g['params']:
                if prox and id(p) not in gmap:
                    return False
                for t in (p, p.grad):
                    if t is None:
                        continue
                    if (t.layout != torch.strided or t.dtype != torch.float32 or t.device.type != 'cuda'
                            or not t.is_contiguous()):
                        return False
                    if dev is None:
                        dev = t.device
                    elif t.device != dev:
                        return False
                if prox:
                    w = gmap[id(p)]
                    if (not isinstance(w, torch.Tensor) or w.dtype != torch.float32 or w.device != p.device
                            or not w.is_contiguous() or w.shape != p.shape):
                        return False
        return True

    def _plan_step(self, optimizer, conf, global_model, fma) -> bool:
        """The step through the cached plan; False (nothing launched) when the plan does not apply."""
        import numpy as np
        import torch

        plan = getattr(self, "_plan", None)
        if plan is None or plan.opt() is not optimizer or id(optimizer.state) != plan.state_id \
                or id(optimizer.param_groups) != plan.groups_id or len(optimizer.param_groups) != plan.ngroups:
            return False
        prox = conf.gradient_policy == 'fed-prox'
        if prox != plan.prox:
            return False
        if prox and (global_model is None or len(global_model) != len(plan.glob_items)):
            return False
        groups = optimizer.param_groups
        lr, mom, damp, wd, nest = [], [], [], [], []
        i = 0
        for j, g in enumerate(groups):
            m = float(g['momentum'])
            if (m != 0) != plan.has_mom[j] or g.get('maximize', False) or g.get('differentiable', False):
                return False
            gp = g['params']
            if len(gp) != plan.group_len[j]:
                return False
            for p in gp:  # the same parameter objects, in the same order
                if p is not plan.params[i]():
                    return False
                i += 1
            lr.append(g['lr'])
            mom.append(m)
            damp.append(g['dampening'])
            wd.append(g['weight_decay'])
            nest.append(_NESTEROV if g['nesterov'] else 0)
        state, pptr, pnumel, bufs = optimizer.state, plan.pptr, plan.pnumel, plan.bufs
        gptr = []
        for i, pr in enumerate(plan.params):
            p = pr()
            gr = p.grad
            if gr is None or p.data_ptr() != pptr[i] or p.numel() != pnumel[i]:
                return False
            try:
                if gr.layout is not torch.strided or not gr.is_contiguous():
                    return False
            except RuntimeError:
                return False
            gptr.append(gr.data_ptr())
            b = bufs[i]
            if b is not None:
                buf, st = b(), state.get(p)
                if buf is None or st is None or st.get('momentum_buffer') is not buf:
                    return False
        if prox:  # the same global tensors (a new round hands a new list: the general path rebuilds)
            gl, gp = plan.glob_items, plan.glob_mptr
            for i, t in enumerate(global_model):
                if t is not gl[i]() or t.data_ptr() != gp[i]:
                    return False
        gi = plan.gidx
        if plan.ngroups == 1:
            T = plan.T
            lr_a, mom_a = np.full(T, lr[0], np.float32), np.full(T, mom[0], np.float32)
            damp_a, wd_a = np.full(T, damp[0], np.float64), np.full(T, wd[0], np.float32)
            fl_a = np.full(T, nest[0], np.int32)
        else:
            lr_a, mom_a = np.asarray(lr, np.float32)[gi], np.asarray(mom, np.float32)[gi]
            damp_a, wd_a = np.asarray(damp, np.float64)[gi], np.asarray(wd, np.float32)[gi]
            fl_a = np.asarray(nest, np.int32)[gi]
        c = float(conf.learning_rate * conf.proxy_mu) if prox else 0.0
        kx.sgd_prox_step_groups_raw(np.asarray(pptr, np.uint64), np.asarray(gptr, np.uint64), plan.bptr,
                                    plan.globptr, plan.numel, plan.T, lr_a, mom_a, damp_a, wd_a, fl_a, c, fma,
                                    torch.cuda.current_stream(plan.stream_dev).cuda_stream)
        return True

    def step_and_update(self, optimizer, conf, model, global_model=None, fma=True):
        """torch_client.py:236-240, ``optimizer.step()`` then ``update_client_weight(conf, model,
        global_model)``, as ONE multi-tensor launch over every parameter group (``fa_sgd_prox_step_groups``,
        the groups' lr / momentum / dampening / weight decay per tensor): one pass over param, grad,
        momentum buffer and global model instead of torch's SGD passes plus the proximal pass. ``optimizer`` is the ``torch.optim.SGD`` of get_optimizer (torch_client.py:95-130); its
        momentum buffers stay in ``optimizer.state``, so it can still be stepped directly. Any other
        optimizer (Adam for 'nlp', maximize / differentiable SGD) takes the two reference calls."""
        import torch

        if self._plan_step(optimizer, conf, global_model, fma):
            return
        self._plan = None
        prox = conf.gradient_policy == 'fed-prox'
        params = list(model.parameters())
        if prox and (global_model is None or len(global_model) != len(params)):
            raise ValueError("fed-prox needs global_model: one tensor per model parameter")
        gmap = {id(p): global_model[i] for i, p in enumerate(params)} if prox else {}
        if not self._fused_ok(optimizer, gmap, prox):
            optimizer.step()
            return self.update_client_weight(conf, model, global_model)
        c = float(conf.learning_rate * conf.proxy_mu) if prox else 0.0
        # every param group in ONE launch: per-tensor lr / momentum / dampening / weight decay / flags, as
        # torch.optim.SGD keeps them per group (the detection task makes one group per parameter)
        ps, grads, bufs, fresh, lr, mom, damp, wd, flags, gidx = [], [], [], [], [], [], [], [], [], []
        all_grads = True
        for j, group in enumerate(optimizer.param_groups):
            m = float(group['momentum'])
            nest = kx_nesterov if group['nesterov'] else 0
            for p in group['params']:
                if p.grad is None:
                    all_grads = False
                    continue
                gidx.append(j)
                buf = optimizer.state[p].get('momentum_buffer') if m != 0 else None
                first = m != 0 and buf is None
                if first:  # enters optimizer.state only once the launch has been accepted (below)
                    buf = torch.empty_like(p, memory_format=torch.contiguous_format)
                    fresh.append((p, buf))
                ps.append(p)
                grads.append(p.grad)
                bufs.append(buf)
                lr.append(group['lr'])
                mom.append(m)
                damp.append(group['dampening'])
                wd.append(group['weight_decay'])
                flags.append(nest | (kx_first if first else 0))
        if ps:
            kx.sgd_prox_step_groups(ps, grads, bufs, [gmap[id(p)] for p in ps] if prox else None, lr, mom, damp,
                                    wd, flags, c, fma=fma)
        for p, buf in fresh:
            optimizer.state[p]['momentum_buffer'] = buf
        stepped = {id(p) for p in ps}
        rest = []
        if prox:  # parameters without a gradient still take the proximal step (optimizers.py:8-10)
            rest = [(p, global_model[i]) for i, p in enumerate(params) if id(p) not in stepped]
            if rest:
                kx.prox_update([p for p, _ in rest], [g for _, g in rest], c)
        if ps and all_grads and not rest:  # the next steps can reuse these validated tables
            self._plan = _StepPlan(optimizer, ps, gidx, bufs, global_model if prox else None,
                                   [gmap[id(p)] for p in ps] if prox else None)
