"""Device-resident YoGi server optimizer — drop-in for fedscale/utils/optimizer/yogi.py:5-36.

State (m_t, v_t) persists across rounds in the object, as in the reference (yogi.py:11-19), but lives
in HBM as flat buckets: fp32 entries in one vector (``m``/``v``), the float64 entries that come from
int64 state_dict buffers (int64 - float64 promotes, optimizers.py:53) in a small fp64 side table
(``ms``/``vs``).  ``m_t`` / ``v_t`` expose per-tensor views in the reference's list form.

Two ways in:
  * ``update(gradients)`` — the reference API: list of gradient tensors -> list of step tensors
    (``fa_yogi_step`` / ``fa_side_yogi`` with last = 0);
  * the fused aggregation path (TorchModelAdapter.apply_round) passes ``fused_args()`` into
    ``fa_reduce_yogi`` so the mean, the YoGi step and the new model come out of one pass over HBM.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from ... import kernels as kx
from ...bucket import BucketLayout


def _f32(x: float) -> float:
    return float(np.float32(x))


class YoGi:
    def __init__(self, eta=1e-2, tau=1e-3, beta=0.9, beta2=0.99):
        self.eta = eta
        self.tau = tau
        self.beta = beta
        self.beta2 = beta2
        self.layout: Optional[BucketLayout] = None
        self.m = self.v = self.ms = self.vs = None
        self.initialized = False  # becomes True after the first step (yogi.py:17-19 lazy init)

    def __getstate__(self):
        """Pickle the hyper-parameters and (host copies of) the m/v state, like the reference object."""
        st = {k: self.__dict__[k] for k in ("eta", "tau", "beta", "beta2", "initialized")}
        st["_layout_args"] = None
        st["_state"] = None
        if self.layout is not None:
            L = self.layout
            st["_layout_args"] = (L.names, [e.shape for e in L.entries], [e.dtype for e in L.entries], L.rank, L.world)
            st["_state"] = tuple(t.cpu() for t in (self.m, self.v, self.ms, self.vs))
        return st

    def __setstate__(self, st):
        self.__init__(st["eta"], st["tau"], st["beta"], st["beta2"])
        if st.get("_layout_args") is not None:
            self.bind(BucketLayout(*st["_layout_args"]), torch.device("cuda", torch.cuda.current_device()))
            for dst, src in zip((self.m, self.v, self.ms, self.vs), st["_state"]):
                dst.copy_(src)
        self.initialized = st["initialized"]

    # ---- state ----------------------------------------------------------------------------------
    def bind(self, layout: BucketLayout, device):
        """Allocate m/v for ``layout`` (idempotent for the same layout)."""
        if self.layout is not None:
            if (self.layout.names == layout.names and self.layout.P == layout.P and self.layout.Q == layout.Q
                    and self.layout.p0 == layout.p0):
                return
            raise ValueError("YoGi state is bound to a different model layout")
        self.layout = layout
        dev = torch.device(device)
        self.m = torch.zeros(layout.ld, dtype=torch.float32, device=dev)
        self.v = torch.zeros(layout.ld, dtype=torch.float32, device=dev)
        self.ms = torch.zeros(layout.ldq, dtype=torch.float64, device=dev)
        self.vs = torch.zeros(layout.ldq, dtype=torch.float64, device=dev)

    def fp32_hparams(self) -> dict:
        """Scalars as torch rounds them for fp32 tensors (Python double -> fp32; 1-beta in double first)."""
        return dict(eta=_f32(self.eta), tau=_f32(self.tau), beta=_f32(self.beta), omb=_f32(1.0 - self.beta),
                    omb2=_f32(1.0 - self.beta2))

    def fp64_hparams(self) -> dict:
        return dict(eta=float(self.eta), tau=float(self.tau), beta=float(self.beta), omb=1.0 - self.beta,
                    omb2=1.0 - self.beta2)

    def fused_args(self, last_f32: torch.Tensor) -> dict:
        return dict(last=last_f32, m=self.m, v=self.v, init=not self.initialized, **self.fp32_hparams())

    def step_side(self, cur_side: torch.Tensor, last_side: Optional[torch.Tensor], *, step=None, model=None):
        kx.side_yogi(cur_side, last_side, self.ms, self.vs, self.layout.Q, step=step, model=model,
                     init=not self.initialized, **self.fp64_hparams())

    @property
    def m_t(self) -> List[torch.Tensor]:
        return self._views(self.m, self.ms)

    @property
    def v_t(self) -> List[torch.Tensor]:
        return self._views(self.v, self.vs)

    def _views(self, f, s):
        if not self.initialized or self.layout is None:
            return []
        if self.layout.world != 1:
            raise RuntimeError("per-tensor views of a sharded YoGi state are not available; use .m/.v")
        return self.layout.unpack(f, s)

    # ---- reference API --------------------------------------------------------------------------
    def update(self, gradients):
        """yogi.py:15-36: returns the list of steps ``(eta / (sqrt(v)+tau)) * m`` per tensor."""
        gradients = list(gradients)
        if len(gradients) == 0:
            return gradients
        dev = gradients[0].device if gradients[0].device.type == "cuda" else torch.device("cuda",
                                                                                             torch.cuda.current_device())
        names = [str(i) for i in range(len(gradients))]
        # float64 gradients (from int64 buffers) form the side table
        dtypes = [torch.int64 if g.dtype == torch.float64 else g.dtype for g in gradients]
        layout = BucketLayout(names, [tuple(g.shape) for g in gradients], dtypes)
        self.bind(layout, dev)
        cur = torch.zeros(layout.ld, dtype=torch.float32, device=dev)
        cur_s = torch.zeros(layout.ldq, dtype=torch.float64, device=dev)
        for e in layout.entries:
            src = gradients[e.index].detach().reshape(-1).to(dev)
            if e.kind == "f":
                cur[e.offset:e.offset + e.numel].copy_(src)
            else:
                cur_s[e.offset:e.offset + e.numel].copy_(src)
        zero = torch.zeros_like(cur)
        step = torch.empty_like(cur)
        step_s = torch.zeros_like(cur_s)
        kx.yogi_step(cur, zero, self.m, self.v, step, layout.P, init=not self.initialized, **self.fp32_hparams())
        self.step_side(cur_s, None, step=step_s)
        self.initialized = True
        out = layout.unpack(step, step_s)
        return [o.to(gradients[i].device) for i, o in enumerate(out)]
