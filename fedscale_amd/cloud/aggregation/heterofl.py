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
from ...bucket import default_pack_workers

HB_ELEMS = 1024
FLAT_ELEMS = 8192   # FLAT mode: elements per workgroup (HB_FLAT_J x 1024 in fedagg.hip)
ROW_MODE_MIN = 256  # rows at least this long get one workgroup per (row, 1024 columns)
#: FLAT mode for tensors whose rows are a multiple of 4 long (False: the previous ROW / ELEMENT plan,
#: kept for A/B timing in tools/heterofl_bench.py)
USE_FLAT = True


def _dims(shape):
    shape = tuple(int(v) for v in shape)
    O = shape[0] if len(shape) >= 1 else 1
    I = shape[1] if len(shape) >= 2 else 1
    S = int(np.prod(shape[2:])) if len(shape) >= 3 else 1
    return O, I, S


def _box_desc(global_dims, row_mode, local_shapes, global_shapes, off: int, m: int = 0):
    """Upload descriptors {offset, o, L, ld} of ONE client's boxes starting at element ``off`` of the
    upload buffer; returns (desc rows, next offset, data elements).  Boxes of tensors read with float4
    loads (``row_mode[k]``: ROW or FLAT mode) start 16-byte aligned with rows padded to a multiple of 4
    elements; the others are packed densely."""
    rows, data = [], 0
    for k, (ls, gs) in enumerate(zip(local_shapes, global_shapes)):
        ls, gs = tuple(int(v) for v in ls), tuple(int(v) for v in gs)
        O, I, S = global_dims[k]
        o, i, _ = _dims(ls)
        if len(ls) != len(gs) or ls[2:] != gs[2:] or o > O or i > I:
            raise ValueError(f"client {m} tensor {k}: shape {ls} is not a prefix box of {gs}")
        L = i * S
        if row_mode[k]:
            off = (off + 3) // 4 * 4
            ld = (L + 3) // 4 * 4
        else:
            ld = L
        rows.append((off, o, L, ld))
        off += o * ld
        data += o * L
    return rows, off, data


def _flat_ok(I, S):
    return (I * S) % 4 == 0 and I * S >= 4


def _global_dims(global_shapes):
    """Per tensor (O, I, S) and whether its boxes use the padded 16-byte-row layout (ROW or FLAT mode)."""
    dims = [_dims(gs) for gs in global_shapes]
    return dims, [I * S >= ROW_MODE_MIN or _flat_ok(I, S) for (_, I, S) in dims]


_DTYPES = (torch.float32, torch.int64)  # int64 entries (BatchNorm num_batches_tracked) go through fp32
_CHUNKS: dict = {}


def _chunk_list(global_shapes: tuple, device):
    """Workgroup -> (tensor, row | -1 | -2) and first element, for a set of global shapes (cached on the
    device: it depends on the model only).  FLAT mode (-2, rows a multiple of 4 long): one chunk per
    FLAT_ELEMS elements of the flattened tensor; ROW mode (other rows of >= 256): one chunk per (row, 1024
    columns); ELEMENT mode (-1): one chunk per 1024 elements of the flattened tensor."""
    key = (global_shapes, str(device), USE_FLAT, FLAT_ELEMS)
    hit = _CHUNKS.get(key)
    if hit is not None:
        return hit
    dims, _ = _global_dims(global_shapes)
    cts, cfs = [], []
    for k, (O, I, S) in enumerate(dims):
        RL = I * S
        if USE_FLAT and _flat_ok(I, S):
            n = (O * RL + FLAT_ELEMS - 1) // FLAT_ELEMS
            cts.append(np.stack([np.full(n, k, dtype=np.int32), np.full(n, -2, dtype=np.int32)], axis=1).reshape(-1))
            cfs.append(np.arange(n, dtype=np.int64) * FLAT_ELEMS)
        elif RL >= ROW_MODE_MIN:
            nch = (RL + HB_ELEMS - 1) // HB_ELEMS
            rows = np.repeat(np.arange(O, dtype=np.int32), nch)
            cts.append(np.stack([np.full(O * nch, k, dtype=np.int32), rows], axis=1).reshape(-1))
            cfs.append(np.tile(np.arange(nch, dtype=np.int64) * HB_ELEMS, O))
        else:
            n = (O * RL + HB_ELEMS - 1) // HB_ELEMS
            cts.append(np.stack([np.full(n, k, dtype=np.int32), np.full(n, -1, dtype=np.int32)], axis=1).reshape(-1))
            cfs.append(np.arange(n, dtype=np.int64) * HB_ELEMS)
    ct = np.concatenate(cts) if cts else np.zeros(0, np.int32)
    cf = np.concatenate(cfs) if cfs else np.zeros(0, np.int64)
    hit = (len(cf), torch.from_numpy(ct).to(device), torch.from_numpy(cf).to(device))
    if len(_CHUNKS) > 16:
        _CHUNKS.clear()
    _CHUNKS[key] = hit
    return hit


class PrefixBoxPlan:
    """Device-side launch plan for one combination: global tensor dims, per-(client, tensor) box
    descriptors into the concatenated uploads, and the workgroup -> (tensor, first element) chunk list.

    Upload layout (``xs``): client after client, tensor after tensor.  The box of a ROW-mode tensor (global
    rows of >= ROW_MODE_MIN elements) starts 16-byte aligned and its rows are padded to a multiple of 4
    elements, so the kernel reads 4 columns per dwordx4 load; ELEMENT-mode boxes are packed densely."""

    def __init__(self, global_shapes: Sequence, local_shapes: Sequence[Sequence], device, desc_rows=None):
        """``desc_rows`` (per client: the rows ``_box_desc`` made for it, consecutive from offset 0) skips
        recomputing the layout when the uploads were staged already."""
        self.device = torch.device(device)
        T, K = len(global_shapes), len(local_shapes)
        tens = np.zeros((T, 4), dtype=np.int64)
        dims, row_mode = _global_dims(global_shapes)
        goff = 0
        for k, (O, I, S) in enumerate(dims):
            tens[k] = (goff, O, I, S)
            goff += O * I * S
        if desc_rows is not None:
            desc = np.asarray(desc_rows, dtype=np.int64).reshape(K, T, 4)
            off = int((desc[:, :, 0] + desc[:, :, 1] * desc[:, :, 3]).max(initial=0))
            data = int((desc[:, :, 1] * desc[:, :, 2]).sum())
        else:
            desc = np.zeros((K, T, 4), dtype=np.int64)
            off = data = 0
            for m, shapes in enumerate(local_shapes):
                rows, off, d = _box_desc(dims, row_mode, shapes, global_shapes, off, m)
                desc[m] = np.asarray(rows, dtype=np.int64).reshape(T, 4)
                data += d
        self.nchunks, self.d_ct, self.d_cf = _chunk_list(tuple(tuple(int(v) for v in gs) for gs in global_shapes),
                                                         self.device)
        self.K, self.T, self.P = K, T, goff
        self.upload_elems = (off + 3) // 4 * 4  # xs size including the row padding
        self.upload_data_elems = data           # the clients' actual parameters
        self.desc_host = desc
        self.tens_host = tens
        self.d_desc = torch.from_numpy(desc.reshape(-1)).to(self.device)
        self.d_tens = torch.from_numpy(tens.reshape(-1)).to(self.device)

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
        if global_state[n].dtype not in _DTYPES:
            raise NotImplementedError(f"{n}: HeteroFL combination supports float32 and int64 entries "
                                      f"(got {global_state[n].dtype})")
    st = PrefixBoxStaging([tuple(global_state[n].shape) for n in names], len(local_states), dev)
    for loc in local_states:
        st.add(names, loc)
    st.combine(global_state)


def _gather_boxes(rows, arrays, start: int, dst_ptr: int, workers: int) -> None:
    """Copy one client's boxes into a pinned row at their plan offsets (relative to ``start``) with the
    native multi-threaded host gather (fa_host_gather): a box is one piece, or one piece per row when its
    rows are padded."""
    srcs, offs, sizes, keep = [], [], [], []
    for (off, o, L, ld), a in zip(rows, arrays):
        if o * L == 0:
            continue
        a = np.ascontiguousarray(a, dtype=np.float32)
        if a.size != o * L:
            raise ValueError(f"box of {a.size} elements, the plan expects {o} x {L}")
        keep.append(a)
        base = a.ctypes.data
        if ld == L:
            srcs.append(np.asarray([base], dtype=np.uint64))
            offs.append(np.asarray([4 * (off - start)], dtype=np.int64))
            sizes.append(np.asarray([4 * o * L], dtype=np.int64))
        else:
            r = np.arange(o, dtype=np.int64)
            srcs.append((base + 4 * L * r).astype(np.uint64))
            offs.append(4 * (off - start + ld * r))
            sizes.append(np.full(o, 4 * L, dtype=np.int64))
    if not srcs:
        return
    ps, po, pn = np.concatenate(srcs), np.concatenate(offs), np.concatenate(sizes)
    N.call("fa_host_gather", dst_ptr, ps.ctypes.data, po.ctypes.data, pn.ctypes.data, len(ps), int(workers))
    del keep


_PINNED: list = []  # [pinned fp32 row, event of its last H2D]
_PINNED_MAX = 4


class PrefixBoxStaging:
    """Device staging of a round's HeteroFL uploads AS THEY ARRIVE: each client's boxes are packed into
    a pinned host row in the plan's layout and copied H2D asynchronously on the current stream, so the
    ingress overlaps the arrivals (as ``ClientStaging`` does for FedAvg); ``combine`` then runs on the
    resident uploads.  Capacity: K clients x the full model (each box is at most its global tensor)."""

    def __init__(self, global_shapes: Sequence, K: int, device):
        self.device = torch.device(device)
        self.global_shapes = [tuple(int(v) for v in gs) for gs in global_shapes]
        self.dims, self.row_mode = _global_dims(self.global_shapes)
        per_client = sum(O * ((I * S + 3) // 4 * 4) + 4 for (O, I, S) in self.dims) + 64
        self.capacity = max(4, int(K) * per_client)
        # padding and alignment gaps are never counted by the kernel, so the buffer needs no clearing
        self.xs = torch.empty(self.capacity, dtype=torch.float32, device=self.device)
        self.local_shapes: List[List[tuple]] = []
        self.rows: list = []  # per client: its _box_desc rows
        self.off = 0
        self.pack_workers = default_pack_workers()

    def _pinned(self, n):
        """A pinned host row of >= n floats whose last H2D has completed, from a pool shared by every
        staging object (pinning is expensive: rows are kept across rounds)."""
        for slot in _PINNED:
            if slot[0].numel() >= n and (slot[1] is None or slot[1].query()):
                return slot
        if len(_PINNED) >= _PINNED_MAX:  # bounded pool: wait for the oldest large-enough row
            for slot in _PINNED:
                if slot[0].numel() >= n:
                    slot[1].synchronize()
                    return slot
        slot = [torch.empty(max(n, 4), dtype=torch.float32, pin_memory=True), None]
        _PINNED.append(slot)
        return slot

    def add(self, names: Sequence[str], local_parameters) -> None:
        m = len(self.local_shapes)
        arrays = []
        for n in names:
            a = local_parameters[n]
            a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
            if a.dtype == np.int64:
                # the reference's fp32 tmp_v += int64 local converts element-wise (customized_aggregator.py:114)
                a = a.astype(np.float32)
            elif a.dtype != np.float32:
                raise TypeError(f"{n}: local dtype {a.dtype}, expected float32 (or int64)")
            arrays.append(a)
        shapes = [tuple(a.shape) for a in arrays]
        start = (self.off + 63) // 64 * 64  # each client's H2D lands 256-byte aligned
        rows, end, _ = _box_desc(self.dims, self.row_mode, shapes, self.global_shapes, start, m)
        if end > self.capacity:
            raise RuntimeError("PrefixBoxStaging: more uploads than the round's capacity")
        slot = self._pinned(end - start)
        _gather_boxes(rows, arrays, start, slot[0].data_ptr(), self.pack_workers)
        self.xs[start:end].copy_(slot[0][:end - start], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        slot[1] = ev
        self.local_shapes.append(shapes)
        self.rows.append(rows)
        self.off = end

    def combine(self, global_state) -> None:
        """global_state (name -> tensor, in place) <- the combination of the staged uploads."""
        names = list(global_state.keys())
        plan = PrefixBoxPlan(self.global_shapes, self.local_shapes, self.device, desc_rows=self.rows)
        glob = torch.cat([global_state[n].detach().reshape(-1).to(torch.float32).cpu() for n in names]).to(
            self.device)
        plan.run(self.xs, glob)
        out = glob.cpu()
        for k, n in enumerate(names):
            v = global_state[n]
            # v[count > 0] = tmp_v[...].to(v.dtype): an int64 entry takes the fp32 mean truncated
            v.copy_(out[int(plan.tens_host[k, 0]):int(plan.tens_host[k, 0]) + v.numel()].view(v.shape))


class DeviceHeteroFLMixin:
    """Device HeteroFL for a Customized_Aggregator (examples/heterofl/customized_aggregator.py):

    * ``client_completion_handler`` (:55-71) stages each result's ``local_parameters`` on the GPU as it
      arrives, then runs the reference handler (which appends the result, counts it and, at the K-th
      result, calls ``combine_models``);
    * ``combine_models`` (:78-119) combines on the GPU: from the staged uploads when they are exactly
      this round's ``client_training_results``, otherwise by packing ``client_training_results`` then.
    ``self.model`` and ``self.client_training_results`` keep their reference meaning."""

    def _hetero_names(self):
        sd = self.model.state_dict()
        for n, v in sd.items():
            if v.dtype not in _DTYPES:
                raise NotImplementedError(f"{n}: HeteroFL combination supports float32 and int64 entries "
                                          f"(got {v.dtype})")
        return list(sd.keys()), [tuple(v.shape) for v in sd.values()]

    def client_completion_handler(self, results):
        st = getattr(self, "_hetero_staging", None)
        if st is None or len(self.client_training_results) == 0:
            names, shapes = self._hetero_names()
            dev = torch.device("cuda", torch.cuda.current_device())
            st = self._hetero_staging = PrefixBoxStaging(shapes, max(1, int(getattr(self, "tasks_round", 1))), dev)
            st.names = names
        st.add(st.names, results["local_parameters"])
        st.results = getattr(st, "results", []) + [results]
        sup = getattr(super(), "client_completion_handler", None)
        if sup is not None:
            return sup(results)

    def combine_models(self):
        st = getattr(self, "_hetero_staging", None)
        res = self.client_training_results
        if st is not None and len(getattr(st, "results", [])) == len(res) and all(
                a is b for a, b in zip(st.results, res)):
            st.combine(self.model.state_dict())
            self._hetero_staging = None
            return
        combine_prefix_boxes(self.model.state_dict(), [r["local_parameters"] for r in res])
