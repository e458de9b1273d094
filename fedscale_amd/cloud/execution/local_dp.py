"""Local differential privacy on the device — drop-in for examples/differential_privacy.

Reference (paths relative to /root/reference):
* ``clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False)``
  examples/differential_privacy/clip_norm.py:12-52 -> ``clip_grad_norm_`` below (same signature and
  return value: the total norm as a 0-d tensor; the tensors are scaled in place when clip_coef < 1).
* the upload step of ``Customized_Client.train``, customized_client.py:51-63:

      delta = [p - last]; clip_grad_norm_(delta, clip_threshold); p = last + delta
      model_param = {name: state_dict[name] + torch.normal(0, noise_factor * clip_threshold)}

  -> ``privatize_update(model, last_model_params, clip_threshold, noise_factor, seed)``: two
  multi-tensor HIP passes over the model (norms, then recover + noise) and one D2H copy of the packed
  upload.  It returns the same ``model_param`` dict of numpy arrays (fp32 entries fp32, int64 entries
  float64, as numpy's int64 + float32 promotes) and leaves the clipped parameters in the model.

Numerics: the clip coefficient comes from fp64-accumulated squares (the reference accumulates in fp32 in
torch's order), so it agrees with the reference to ~1 ulp; the recovered parameters then agree to the
same relative error, and exactly when no clipping happens.  The noise is N(0, sigma) from a
counter-based generator keyed by (seed, element index in state_dict order): the reference's
distribution, a different stream than torch's CPU generator.
"""
from __future__ import annotations

import math
import weakref
from typing import Dict, Iterable, List, Optional, Union

import numpy as np
import torch

from ... import kernels as kx


def clip_grad_norm_(parameters: Union[torch.Tensor, Iterable[torch.Tensor]], max_norm: float,
                    norm_type: float = 2.0, error_if_nonfinite: bool = False) -> torch.Tensor:
    """clip_norm.py:12-52 on device tensors (one norm pass + one scale pass, whole list per launch)."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = list(parameters)
    max_norm, norm_type = float(max_norm), float(norm_type)
    if len(parameters) == 0:
        return torch.tensor(0.)
    if norm_type not in (2.0, math.inf):
        raise NotImplementedError("the device path implements norm_type 2 and inf (the DP example uses 2)")
    ts = [p.detach() for p in parameters]
    if norm_type == math.inf and any(t.numel() == 0 for t in ts):  # torch's max() of an empty tensor raises
        raise RuntimeError("max(): Expected reduction dim to be specified for input.numel() == 0.")
    coef = torch.empty(3, dtype=torch.float32, device=ts[0].device)
    kx.dp_clip_coef(ts, None, max_norm, norm_type == math.inf, coef)
    total = coef[0]
    if error_if_nonfinite and bool(torch.logical_or(total.isnan(), total.isinf())):
        raise RuntimeError(f"The total norm of order {norm_type} for gradients from `parameters` is non-finite, "
                           f"so it cannot be clipped.")
    kx.dp_apply(ts, None, None, None, coef, 0.0, 0, scale_only=True)
    return total.clone()


class _UploadLayout:
    """state_dict entries of a model, split into fp32 (packed into one device bucket) and int64 ones.
    Entry i is ``model.parameters()[param_index[i]]`` or ``model.buffers()[buffer_index[i]]``."""

    def __init__(self, model: torch.nn.Module):
        sd = model.state_dict(keep_vars=True)
        self.names = list(sd.keys())
        pids = {id(p): i for i, p in enumerate(model.parameters())}
        bids = {id(b): i for i, b in enumerate(model.buffers())}
        self.param_index = [pids.get(id(sd[n])) for n in self.names]  # position in model.parameters()
        self.buffer_index = [bids.get(id(sd[n])) for n in self.names]
        for n, pi, bi in zip(self.names, self.param_index, self.buffer_index):
            if pi is None and bi is None:
                raise NotImplementedError(f"{n}: state_dict entry is neither a parameter nor a buffer")
        self.shapes = [tuple(sd[n].shape) for n in self.names]
        self.dtypes = [sd[n].dtype for n in self.names]
        for n, d in zip(self.names, self.dtypes):
            if d not in (torch.float32, torch.int64):
                raise NotImplementedError(f"{n}: dtype {d}; the device path handles float32 and int64 entries")
        self.numel = [int(np.prod(s)) if len(s) else 1 for s in self.shapes]
        self.noise_off = np.concatenate([[0], np.cumsum(self.numel)[:-1]]).astype(np.int64).tolist()
        f = [i for i, d in enumerate(self.dtypes) if d == torch.float32]
        self.f_idx = f
        # fp32 bucket offsets, each entry 16-byte aligned so the float4 path applies
        offs, o = [], 0
        for i in f:
            offs.append(o)
            o += (self.numel[i] + 3) // 4 * 4
        self.f_off, self.f_total = offs, o


_LAYOUTS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _layout_of(model: torch.nn.Module):
    """The model's upload layout, rebuilt only when its parameter / buffer objects or shapes change."""
    params, bufs = list(model.parameters()), list(model.buffers())
    key = (tuple(map(id, params)), tuple(map(id, bufs)), tuple(p.shape for p in params),
           tuple(b.shape for b in bufs))
    ent = _LAYOUTS.get(model)
    if ent is None or ent[0] != key:
        ent = (key, _UploadLayout(model))
        _LAYOUTS[model] = ent
    return ent[1], params, bufs


def privatize_update(model: torch.nn.Module, last_model_params: List[torch.Tensor], clip_threshold: float,
                     noise_factor: float, seed: int = 0, as_numpy: bool = True):
    """customized_client.py:51-63 on the device; returns ``model_param`` ({name: array}) like the reference."""
    L, params, bufs = _layout_of(model)
    entry = [params[pi] if pi is not None else bufs[bi] for pi, bi in zip(L.param_index, L.buffer_index)]
    if len(last_model_params) != len(params):
        raise ValueError(f"{len(last_model_params)} last-model tensors for {len(params)} parameters")
    dev = entry[0].device
    last = [t.to(dev) if t.device != dev else t for t in last_model_params]
    coef = torch.empty(3, dtype=torch.float32, device=dev)
    if params:
        for i, (p, l) in enumerate(zip(params, last)):
            if p.shape != l.shape:
                raise ValueError(f"parameter {i}: shape {tuple(p.shape)} != last-model shape {tuple(l.shape)}")
        kx.dp_clip_coef(params, last, float(clip_threshold), False, coef)
    else:
        coef.zero_()
    sigma = float(noise_factor * clip_threshold)
    bucket = torch.empty(max(1, L.f_total), dtype=torch.float32, device=dev)
    src, lst, up, offs = [], [], [], []
    for i, o in zip(L.f_idx, L.f_off):
        pi = L.param_index[i]
        src.append(entry[i])
        lst.append(last[pi] if pi is not None else None)
        up.append(bucket[o:o + L.numel[i]])
        offs.append(L.noise_off[i])
    kx.dp_apply(src, lst, up, offs, coef, sigma, seed, write_param=True)
    side = {i: torch.empty(L.numel[i], dtype=torch.float64, device=dev)
            for i, d in enumerate(L.dtypes) if d == torch.int64}
    if side:
        kx.dp_noise_i64([entry[i].reshape(-1) for i in side], list(side.values()),
                        [L.noise_off[i] for i in side], sigma, seed)
    if not as_numpy:
        res = {}
        for i, o in zip(L.f_idx, L.f_off):
            res[L.names[i]] = bucket[o:o + L.numel[i]].view(L.shapes[i])
        for i, t in side.items():
            res[L.names[i]] = t.view(L.shapes[i])
        return {n: res[n] for n in L.names}
    host = bucket.to("cpu").numpy()  # one D2H of the packed upload
    res: Dict[str, np.ndarray] = {}
    for i, o in zip(L.f_idx, L.f_off):
        res[L.names[i]] = np.asarray(host[o:o + L.numel[i]].reshape(L.shapes[i]))
    for i, t in side.items():
        res[L.names[i]] = np.asarray(t.to("cpu").numpy().reshape(L.shapes[i]))
    return {n: res[n] for n in L.names}
