"""HeteroFL sub-model combination on the device — drop-in for the HeteroFL plugin's
``Customized_Aggregator.combine_models`` (examples/heterofl/customized_aggregator.py:78-119).

A client at model rate r trains the sub-model ``split_model(global, r)`` (examples/heterofl/
customized_fllibs.py:73-95) whose index sets (``make_param_idx``, :25-70) are always prefixes: for a
tensor of shape (O, I, *S) the client holds the box [0:o) x [0:i) x S (1-D tensors: [0:o)).  The
reference scatter-adds every client's box into an fp32 zero tensor, counts the covering clients, and
overwrites the global elements with count > 0 by sum / count.  Here the boxes are read straight from the
clients' uploads by one HIP kernel (``fa_prefix_box_combine``) that, per global element, walks the
clients in order — the same fp32 operations in the same order, so the result is bit-identical.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from ... import _native as N

HB_ELEMS = 1024


def _dims(shape):
    shape = tuple(int(v) for v in shape)
    O = shape[0] if len(shape) >= 1 else 1
    I = shape[1] if len(shape) >= 2 else 1
    S = int(np.prod(shape[2:])) if len(shape) >= 3 else 1
    return O, I, S


def combine_prefix_boxes(global_state, local_states: Sequence, device=None) -> None:
    """In place: global_state (an ordered name -> tensor mapping, e.g. ``model.state_dict()``) takes the
    HeteroFL combination of ``local_states`` (per client: mapping name -> prefix-box tensor/array)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    names = list(global_state.keys())
    T, K = len(names), len(local_states)
    if K == 0:
        return
    tens = np.zeros((T, 4), dtype=np.int64)
    goff = 0
    for k, n in enumerate(names):
        v = global_state[n]
        if v.dtype != torch.float32:
            raise NotImplementedError(f"{n}: HeteroFL combination supports float32 entries (got {v.dtype})")
        O, I, S = _dims(v.shape)
        tens[k] = (goff, O, I, S)
        goff += O * I * S
    desc = np.zeros((K, T, 3), dtype=np.int64)
    sizes = []
    off = 0
    for m, loc in enumerate(local_states):
        for k, n in enumerate(names):
            a = loc[n]
            shp = tuple(a.shape)
            gshape = tuple(global_state[n].shape)
            O, I, S = _dims(gshape)
            o, i, s = _dims(shp)
            if len(shp) != len(gshape) or shp[2:] != gshape[2:] or o > O or i > I:
                raise ValueError(f"client {m} {n}: shape {shp} is not a prefix box of {gshape}")
            desc[m, k] = (off, o, i)
            off += o * i * S
            sizes.append(o * i * S)
    xs_host = torch.empty(max(off, 1), dtype=torch.float32, pin_memory=True)
    xv = xs_host.numpy()
    pos = 0
    for loc in local_states:
        for n in names:
            a = loc[n]
            a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            if a.dtype != np.float32:
                raise TypeError(f"{n}: local dtype {a.dtype}, expected float32")
            xv[pos:pos + a.size] = a.reshape(-1)
            pos += a.size
    glob_host = torch.cat([global_state[n].detach().reshape(-1).cpu() for n in names]) if T else torch.zeros(0)
    ck_t, ck_f = [], []
    for k in range(T):
        n_el = int(tens[k, 1] * tens[k, 2] * tens[k, 3])
        for f in range(0, n_el, HB_ELEMS):
            ck_t.append(k)
            ck_f.append(f)
    xs = xs_host.to(dev, non_blocking=True)
    glob = glob_host.to(dev)
    d_desc = torch.from_numpy(desc.reshape(-1)).to(dev)
    d_tens = torch.from_numpy(tens.reshape(-1)).to(dev)
    d_ct = torch.tensor(ck_t, dtype=torch.int32, device=dev)
    d_cf = torch.tensor(ck_f, dtype=torch.int64, device=dev)
    N.call("fa_prefix_box_combine", xs.data_ptr(), d_desc.data_ptr(), K, d_tens.data_ptr(), T, d_ct.data_ptr(),
           d_cf.data_ptr(), len(ck_t), glob.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    out = glob.cpu()
    for k, n in enumerate(names):
        v = global_state[n]
        v.copy_(out[int(tens[k, 0]):int(tens[k, 0]) + v.numel()].view(v.shape))


class DeviceHeteroFLMixin:
    """Overrides ``combine_models`` of a HeteroFL aggregator (customized_aggregator.py:78): the global
    model ``self.model`` and the round's ``self.client_training_results`` (each with 'local_parameters')
    keep their reference meaning; the combination runs on the GPU."""

    def combine_models(self):
        combine_prefix_boxes(self.model.state_dict(),
                             [r["local_parameters"] for r in self.client_training_results])
