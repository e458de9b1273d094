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
ROW_MODE_MIN = 256  # rows at least this long get one workgroup per (row, 1024 columns)


def _dims(shape):
    shape = tuple(int(v) for v in shape)
    O = shape[0] if len(shape) >= 1 else 1
    I = shape[1] if len(shape) >= 2 else 1
    S = int(np.prod(shape[2:])) if len(shape) >= 3 else 1
    return O, I, S


class PrefixBoxPlan:
    """Device-side launch plan for one combination: global tensor dims, per-(client, tensor) box
    descriptors into the concatenated uploads, and the workgroup -> (tensor, first element) chunk list.

    Upload layout (``xs``): client after client, tensor after tensor.  The box of a ROW-mode tensor (global
    rows of >= ROW_MODE_MIN elements) starts 16-byte aligned and its rows are padded to a multiple of 4
    elements, so the kernel reads 4 columns per dwordx4 load; ELEMENT-mode boxes are packed densely."""

    def __init__(self, global_shapes: Sequence, local_shapes: Sequence[Sequence], device):
        self.device = torch.device(device)
        T, K = len(global_shapes), len(local_shapes)
        tens = np.zeros((T, 4), dtype=np.int64)
        goff = 0
        row_mode = []
        for k, gs in enumerate(global_shapes):
            O, I, S = _dims(gs)
            tens[k] = (goff, O, I, S)
            goff += O * I * S
            row_mode.append(I * S >= ROW_MODE_MIN)
        desc = np.zeros((K, T, 4), dtype=np.int64)
        off = data = 0
        for m, shapes in enumerate(local_shapes):
            for k, (ls, gs) in enumerate(zip(shapes, global_shapes)):
                ls, gs = tuple(ls), tuple(gs)
                O, I, S = _dims(gs)
                o, i, _ = _dims(ls)
                if len(ls) != len(gs) or ls[2:] != gs[2:] or o > O or i > I:
                    raise ValueError(f"client {m} tensor {k}: shape {ls} is not a prefix box of {gs}")
                L = i * S
                if row_mode[k]:
                    off = (off + 3) // 4 * 4
                    ld = (L + 3) // 4 * 4
                else:
                    ld = L
                desc[m, k] = (off, o, L, ld)
                off += o * ld
                data += o * L
        ck_t, ck_f = [], []  # ck_t holds (tensor, row) pairs; row -1 = element mode
        for k in range(T):
            O, RL = int(tens[k, 1]), int(tens[k, 2] * tens[k, 3])
            if row_mode[k]:
                for o in range(O):
                    for f in range(0, RL, HB_ELEMS):
                        ck_t += [k, o]
                        ck_f.append(f)
            else:
                for f in range(0, O * RL, HB_ELEMS):
                    ck_t += [k, -1]
                    ck_f.append(f)
        self.K, self.T, self.P = K, T, goff
        self.upload_elems = (off + 3) // 4 * 4  # xs size including the row padding
        self.upload_data_elems = data           # the clients' actual parameters
        self.desc_host = desc
        self.tens_host = tens
        self.d_desc = torch.from_numpy(desc.reshape(-1)).to(self.device)
        self.d_tens = torch.from_numpy(tens.reshape(-1)).to(self.device)
        self.d_ct = torch.tensor(ck_t, dtype=torch.int32, device=self.device)
        self.d_cf = torch.tensor(ck_f, dtype=torch.int64, device=self.device)
        self.nchunks = len(ck_f)

    def pack(self, m: int, k: int, a: np.ndarray, xv: np.ndarray) -> None:
        """Copy client m's box of tensor k into the upload buffer xv at its (padded) place."""
        off, o, L, ld = (int(v) for v in self.desc_host[m, k])
        if a.size != o * L:
            raise ValueError(f"client {m} tensor {k}: {a.size} elements, the plan expects {o * L}")
        if ld == L:
            xv[off:off + o * L] = a.reshape(-1)
        else:
            xv[off:off + o * ld].reshape(o, ld)[:, :L] = a.reshape(o, L)

    def run(self, xs: torch.Tensor, glob: torch.Tensor) -> None:
        """glob (fp32 [P], device) <- HeteroFL combination of the uploads xs (fp32, device, plan layout)."""
        if xs.numel() < self.upload_elems or glob.numel() < self.P:
            raise ValueError("PrefixBoxPlan.run: buffers smaller than the plan")
        for t, n in ((xs, "xs"), (glob, "glob")):
            if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"PrefixBoxPlan.run: {n} must be a contiguous fp32 tensor on {self.device}")
        if xs.data_ptr() % 16:
            raise ValueError("PrefixBoxPlan.run: xs must be 16-byte aligned")
        N.call("fa_prefix_box_combine", xs.data_ptr(), self.d_desc.data_ptr(), self.K, self.d_tens.data_ptr(),
               self.T, self.d_ct.data_ptr(), self.d_cf.data_ptr(), self.nchunks, glob.data_ptr(),
               torch.cuda.current_stream(self.device).cuda_stream)


def combine_prefix_boxes(global_state, local_states: Sequence, device=None) -> None:
    """In place: global_state (an ordered name -> tensor mapping, e.g. ``model.state_dict()``) takes the
    HeteroFL combination of ``local_states`` (per client: mapping name -> prefix-box tensor/array)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    names = list(global_state.keys())
    if not local_states:
        return
    for n in names:
        if global_state[n].dtype != torch.float32:
            raise NotImplementedError(f"{n}: HeteroFL combination supports float32 entries "
                                      f"(got {global_state[n].dtype})")
    plan = PrefixBoxPlan([tuple(global_state[n].shape) for n in names],
                         [[tuple(loc[n].shape) for n in names] for loc in local_states], dev)
    xs_host = torch.zeros(max(plan.upload_elems, 4), dtype=torch.float32, pin_memory=True)
    xv = xs_host.numpy()
    for m, loc in enumerate(local_states):
        for k, n in enumerate(names):
            a = loc[n]
            a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            if a.dtype != np.float32:
                raise TypeError(f"{n}: local dtype {a.dtype}, expected float32")
            plan.pack(m, k, a, xv)
    glob = torch.cat([global_state[n].detach().reshape(-1).cpu() for n in names]).to(dev)
    plan.run(xs_host.to(dev, non_blocking=True), glob)
    out = glob.cpu()
    for k, n in enumerate(names):
        v = global_state[n]
        v.copy_(out[int(plan.tens_host[k, 0]):int(plan.tens_host[k, 0]) + v.numel()].view(v.shape))


class DeviceHeteroFLMixin:
    """Overrides ``combine_models`` of a HeteroFL aggregator (customized_aggregator.py:78): the global
    model ``self.model`` and the round's ``self.client_training_results`` (each with 'local_parameters')
    keep their reference meaning; the combination runs on the GPU."""

    def combine_models(self):
        combine_prefix_boxes(self.model.state_dict(),
                             [r["local_parameters"] for r in self.client_training_results])
