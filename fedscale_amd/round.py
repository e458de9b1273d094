"""One aggregation round on the device: staging of arriving client updates + chunked in-order reduction.

A ``DeviceRound`` is the device-side state that replaces the reference's ``self.model_weights`` running
sum (aggregator.py:497-503 / async_aggregator.py:129-133) and, for q-FedAvg, its retained
``client_training_results`` (aggregator.py:466-467, consumed by optimizers.py:73-98).  Updates are
staged into a [capacity, ld] device buffer; whenever it fills before the round ends, the chunk is
folded into the running state by one kernel launch (the same per-element chain continues, so chunking
never changes a bit of the result).  The last chunk is reduced by ``finalize_*`` with the server step
fused in.

With a client-mode ``ShardGroup`` (``state.py``) the round is spread over ranks by arrival index: each
rank stages and folds only its own contiguous block of arrivals (its chain starts from its first client),
the partial chains / q-FedAvg deltas / side-table sums meet in one RCCL all-reduce, and the finishing
epilogue (divide, fused FedYoGi, q-FedAvg hs + step) runs replicated on the summed vector.
"""
from __future__ import annotations

import functools
from typing import Optional

import numpy as np
import torch

from . import kernels as kx
from .bucket import BucketLayout, ClientStaging
from .bucket import _NULL_CTX as _NULL
from .state import DeviceStream, ShardGroup

POLICIES = ("fedavg", "fedbuff", "qfedavg")


def default_capacity(layout: BucketLayout, K: int, device, budget_fraction: float = 0.5,
                     hard_cap: Optional[int] = None) -> int:
    """Clients per chunk: all K when they fit in ``budget_fraction`` of the free HBM."""
    free, _ = torch.cuda.mem_get_info(device)
    per_client = layout.ld * 4 + layout.ldq * 8
    cap = max(1, int(free * budget_fraction) // max(1, per_client))
    cap = min(cap, max(1, K))
    if hard_cap:
        cap = min(cap, hard_cap)
    return cap


def on_stream(fn):
    """Run a method under ``self.dstream`` (its GPU and HIP stream current), unless that DeviceStream is
    already the innermost one on this thread; without a dstream, on the caller's current stream."""

    @functools.wraps(fn)
    def run(self, *a, **k):
        ds = self.dstream
        if ds is None or DeviceStream.current() is ds:
            return fn(self, *a, **k)
        with ds:
            return fn(self, *a, **k)

    return run


class DeviceRound:
    def __init__(self, layout: BucketLayout, device, K: int, policy: str, *, capacity: Optional[int] = None,
                 staging: Optional[ClientStaging] = None, last_f32: Optional[torch.Tensor] = None,
                 last_i64: Optional[torch.Tensor] = None, clients: Optional[ShardGroup] = None,
                 mean_chain: bool = False, dstream: Optional[DeviceStream] = None):
        """``mean_chain`` (q-FedAvg): fuse the plain FedAvg chain into the phase-1 kernel, so the round's
        mean (the reference's model_weights, aggregator.py:497-507) exists however many chunks the round
        spans (fa_qfed_accumulate's ``chain``: +1 add per element, measured 9 % on the kernel).
        ``dstream``: the DeviceStream of the owning adapter; every kernel and copy of the round is issued on
        it (None: the caller's current stream)."""
        self.dstream = dstream
        self._init(layout, device, K, policy, capacity, staging, last_f32, last_i64, clients, mean_chain)

    def _on(self):
        """Context for GPU work of this round: its dstream unless already current (or none)."""
        ds = self.dstream
        return _NULL if ds is None or DeviceStream.current() is ds else ds

    def _init(self, layout, device, K, policy, capacity, staging, last_f32, last_i64, clients, mean_chain):
        """(steady-state FedAvg / FedBuff rounds reuse the staging and its side-table scratch: no GPU work,
        so no device context is entered; allocations are made on the dstream)"""
        if policy not in POLICIES:
            raise ValueError(f"policy {policy!r} not in {POLICIES}")
        if K < 1:
            raise ValueError("a round needs K >= 1 client results")
        self.layout, self.device, self.K, self.policy = layout, torch.device(device), int(K), policy
        self.cg = clients if clients is not None and clients.shards_clients else None
        if self.cg is not None and layout.world != 1:
            raise ValueError("client-mode rounds need the unsharded (whole-model) layout")
        # [k_begin, k_end): the arrival indices this rank reduces (all of them unless client-sharded)
        self.k_begin, self.k_end = self.cg.client_block(self.K) if self.cg is not None else (0, self.K)
        K_local = max(1, self.k_end - self.k_begin)
        if policy == "qfedavg":
            qmax = kx.qfed_max_chunk()
            implicit = capacity is None
            capacity = min(capacity or qmax, qmax)  # phase-1 calls take at most fa_qfed_max_chunk() clients
        else:
            implicit = False
        if staging is not None and (capacity is None or staging.capacity >= min(capacity, K_local)):
            self.staging = staging
        else:
            cap = capacity or default_capacity(layout, K_local, self.device)
            if implicit:  # ... and no more than fit the free HBM (a 100 M-parameter model: ~360, not 2048)
                cap = min(cap, default_capacity(layout, K_local, self.device))
            self.staging = ClientStaging(layout, self.device, min(cap, K_local), dstream=self.dstream)
        self.cap = min(self.staging.capacity, capacity or self.staging.capacity)
        self.staging.generation += 1  # a new round takes the staging slots over
        self.generation = self.staging.generation
        self.n = 0  # results received (all ranks' arrivals)
        self.n_local = 0  # results staged by this rank
        self.slot = 0  # staged in the current chunk
        self.chunks_done = 0
        dev, L = self.device, layout
        self.acc = None  # running fp32 chain across chunks
        # int64 / float64 side sums: the first chunk's accumulate overwrites them, so no memset is needed
        # unless a client-mode rank may contribute nothing to the cross-rank sum
        if self.cg is None and policy in ("fedavg", "fedbuff"):
            # consumed by finalize_mean before the next round can begin: one pair per staging, reused
            if self.staging.side_scratch is None:
                with self._on():
                    self.staging.side_scratch = (torch.empty(L.ldq, dtype=torch.int64, device=dev),
                                                 torch.empty(L.ldq, dtype=torch.float64, device=dev))
            self.acc_i, self.acc_d = self.staging.side_scratch
        else:  # q-FedAvg keeps them for the round's lazily computed mean (mean_from_staging)
            alloc = torch.zeros if self.cg is not None else torch.empty
            with self._on():
                self.acc_i = alloc(L.ldq, dtype=torch.int64, device=dev)
                self.acc_d = alloc(L.ldq, dtype=torch.float64, device=dev)
        self._w32 = np.zeros(self.cap, dtype=np.float32)  # per-slot weights of the current chunk
        self._w64 = np.zeros(self.cap, dtype=np.float64)
        self.last_f32, self.last_i64 = last_f32, last_i64
        if policy == "qfedavg":
            if last_f32 is None or last_i64 is None:
                raise ValueError("q-FedAvg needs the round's starting model (last_f32 / last_i64)")
            with self._on():
                self._init_qfed(L, dev)
        self.chain = None
        if policy == "qfedavg" and mean_chain and self.cg is None:
            with self._on():
                self.chain = torch.zeros(L.ld, dtype=torch.float32, device=dev)
        self.head = 0  # arrivals [0, head) already reduced into head_acc by the head launch (_launch_head)
        self.head_acc = None
        self._split_at = self._head_split()
        # FedAvg rounds of a whole-model layout staged in a pinned mirror take add()'s short path
        self._small = (policy == "fedavg" and self.cg is None and self.staging.bulk
                       and self.staging._views is not None)

    #: small zero-copy FedAvg rounds (config 1) reduce their first arrivals while the rest are still arriving
    #: (``_launch_head``); False: one finishing launch over every row
    SPLIT_SMALL_ROUNDS = True
    #: the share of the K arrivals the head launch reduces (the rest: the finishing launch).  Config 1 (K = 10) per
    #: round: 0.5 81.3-82.9 us, 0.7 76.7-78.3, 0.8 77.3-81.2, 0.9 79.6-84.6 (profiles/r06_c1_profile_split2.log): the
    #: head kernel's PCIe reads finish behind the last arrivals' staging, and the finishing launch reads less
    SPLIT_FRACTION = 0.7

    def _head_split(self):
        """The arrival count after which the head launch goes out (None: this round takes no head launch): FedAvg
        rounds of K >= 4 that fit one chunk of a zero-copy staging mirror (ClientStaging.host_rows: its kernels read
        the pinned rows over PCIe), on the adapter's own stream, with no int64 entries."""
        st, L = self.staging, self.layout
        if (not self.SPLIT_SMALL_ROUNDS or self.policy != "fedavg" or self.cg is not None or self.K < 4
                or self.cap < self.K or self.dstream is None or L.Q or not st.bulk or st._views is None
                or self.K * (L.ld * 4 + L.ldq * 8) > st.ZERO_COPY_MAX_BYTES):
            return None
        return min(self.K - 1, max(1, int(self.K * self.SPLIT_FRACTION)))

    def _launch_head(self):
        """Reduce the arrivals staged so far, [0, slot), straight out of the pinned mirror into ``head_acc`` (the
        raw fp32 chain, not divided), on the round's stream: the GPU reads these rows over PCIe while the host
        stages the rest, and the finishing launch continues the same per-element chain from ``head_acc`` over the
        remaining rows (aggregator.py:500-503 in arrival order; the bits of one launch over all rows).  The rows are
        not rewritten before the round's finishing launch has run (release_host_rows)."""
        st, L, n = self.staging, self.layout, self.slot
        zc = st.host_rows(n)
        if zc is None:
            return
        acc = st.head_acc
        if acc is None:
            with self._on():
                acc = st.head_acc = torch.empty(L.ld, dtype=torch.float32, device=self.device)
        x = zc[0]
        key = (x.data_ptr(), n, acc.data_ptr())
        if st._head_key != key:  # the wrapper's checks, once per (rows, count, accumulator)
            kx._check_x(x, n, L.P, host_ok=True)
            kx._dev(acc, torch.float32, "out", kx._cols(L.P))
            st._head_key = key
        kx.call("fa_reduce", key[0], x.shape[1], n, L.P, None, None, key[2], 1.0, 0, self.dstream.handle)
        self.head, self.head_acc = n, acc

    def _init_qfed(self, L, dev):
        self.delta = torch.zeros(L.ld, dtype=torch.float32, device=dev)
        self.delta_s = torch.zeros(L.ldq, dtype=torch.float32, device=dev)
        self.sqnorm = torch.zeros(self.K, dtype=torch.float64, device=dev)       # fp32 bucket part (per shard)
        self.sqnorm_side = torch.zeros(self.K, dtype=torch.float64, device=dev)  # side table part (replicated)
        self.workspace = kx.qfed_workspace(self.cap, dev, L.ld, L.P)
        self.alpha = np.zeros(self.K, dtype=np.float32)
        self.c1 = np.zeros(self.K, dtype=np.float32)
        self.c2 = np.zeros(self.K, dtype=np.float32)
        self.lr = None

    # ---------------------------------------------------------------------------------------------
    def add(self, update, *, weight: Optional[float] = None, loss: Optional[float] = None,
            learning_rate: Optional[float] = None, q: Optional[float] = None):
        """Stage one arriving client update (in arrival order)."""
        if self._small and type(update) is dict and self.n < self.K and self.slot < self.cap:
            # a small FedAvg round's upload straight into its slot of the pinned mirror (config 1; anything the
            # native copy does not take, or an error, goes on below and is handled — or raised — as before)
            slot = self.slot
            if self.staging.put_small(slot, update):
                self.slot = slot + 1
                self.n += 1
                self.n_local += 1
                if self.slot == self._split_at:
                    self._launch_head()
                return
        if self.n >= self.K:
            raise RuntimeError(f"round already has its K={self.K} results")
        if not (self.k_begin <= self.n < self.k_end):  # another rank's client (client mode)
            if self.policy == "qfedavg":
                self._qfed_scalars(self.n, loss, learning_rate, q)  # hs needs every client's scalars
            self.n += 1
            return
        if self.slot == self.cap:
            self._fold_chunk()
        self.staging.put(self.slot, update)
        if self.policy == "fedbuff":
            self._w32[self.slot] = np.float32(weight)  # fp32 array * Python float: scalar rounds to fp32
            self._w64[self.slot] = float(weight)       # int64 array * Python float: float64
        elif self.policy == "qfedavg":
            self._qfed_scalars(self.n, loss, learning_rate, q)
        self.slot += 1
        self.n += 1
        self.n_local += 1
        if self.slot == self._split_at:
            self._launch_head()

    def adopt_resident(self, n: int):
        """Bench hook (FedAvg): take ``n`` arrivals whose updates are ALREADY in the staging slots
        [slot, slot + n), written there on the device (``synth.fill`` on ``staging.x``), as ``add`` would have
        staged them — the device-resident round ``fedscale_amd.inproc_bench`` times, without host ingress (the
        same resident-input convention as bench.py's SPMD workload).  Their side-table rows are the staging's
        (zero unless written)."""
        if self.policy != "fedavg" or self.cg is not None:
            raise ValueError("adopt_resident: FedAvg rounds of a whole-model or parameter-sharded layout only")
        if n < 0 or self.slot + n > self.cap or self.n + n > self.K:
            raise ValueError(f"adopt_resident: {n} arrivals do not fit (slot {self.slot} of {self.cap}, "
                             f"{self.n} of K={self.K})")
        self.slot += n
        self.n += n
        self.n_local += n

    def _qfed_scalars(self, k, loss, lr, q):
        """Per-client scalars of optimizers.py:87-98, computed in double exactly as the reference does."""
        base = loss + 1e-10
        a = np.float_power(base, q)
        self.alpha[k] = np.float32(a)                         # a * grad: scalar rounded to fp32
        self.c1[k] = np.float32(q * np.float_power(base, q - 1))
        self.c2[k] = np.float32((1.0 / lr) * a)
        if self.lr is None:
            self.lr = lr
        elif lr != self.lr:
            raise RuntimeError("learning_rate changed in the middle of a q-FedAvg round")

    def _chunk_weights(self):
        n = self.slot
        a32 = torch.from_numpy(self._w32[:n].copy()).to(self.device, non_blocking=True)
        a64 = torch.from_numpy(self._w64[:n].copy()).to(self.device, non_blocking=True)
        return a32, a64

    @on_stream
    def _fold_chunk(self):
        """Fold the staged chunk into the running state (not the last chunk of the round)."""
        self.staging.drain()
        L, st, n = self.layout, self.staging, self.slot
        first = self.chunks_done == 0
        if self.policy in ("fedavg", "fedbuff"):
            if self.acc is None:
                self.acc = torch.zeros(L.ld, dtype=torch.float32, device=self.device)
            a32 = a64 = None
            if self.policy == "fedbuff":
                a32, a64 = self._chunk_weights()
            kx.reduce(st.x, n, L.P, self.acc, a=a32, acc_in=None if first else self.acc)
            kx.side_accumulate(st.xi, n, L.Q, 0 if self.policy == "fedavg" else 1, w=a64, acc_i=self.acc_i,
                               acc_d=self.acc_d, accumulate=not first)
        else:
            k0 = self.k_begin + self.n_local - n  # arrival index of the chunk's first client
            alpha = torch.from_numpy(self.alpha[k0:k0 + n].copy()).to(self.device, non_blocking=True)
            if L.P > 0:
                kx.qfed_accumulate(st.x, n, L.P, last=self.last_f32, alpha=alpha, lr=self.lr, delta=self.delta,
                                   sqnorm=self.sqnorm[k0:k0 + n], workspace=self.workspace, accumulate=not first,
                                   chain=self.chain)
            kx.side_qfed_accumulate(st.xi, n, L.Q, last=self.last_i64, alpha=alpha, lr=self.lr,
                                    delta_s=self.delta_s, sqnorm=self.sqnorm_side[k0:k0 + n], accumulate=not first)
            if self.chain is not None:  # the mean's int64 side sums (aggregator.py:500-503)
                kx.side_accumulate(st.xi, n, L.Q, 0, acc_i=self.acc_i, accumulate=not first)
        self.chunks_done += 1
        self.slot = 0

    def _check_complete(self):
        if self.n != self.K:
            raise RuntimeError(f"finalize with {self.n} of K={self.K} results")

    def _cross_rank_sum(self, *tensors):
        """Client mode: sum the per-rank partials (RCCL all-reduce over xGMI).  A rank that reduced no
        client contributes zeros."""
        for t in tensors:
            self.cg.all_reduce_sum(t)

    @on_stream
    def _finalize_mean_clients(self, denom32, denom64, out, cur_side, model_side, yogi):
        L = self.layout
        if self.slot:
            self._fold_chunk()
        if self.acc is None:
            self.acc = torch.zeros(L.ld, dtype=torch.float32, device=self.device)
        mode = 0 if self.policy == "fedavg" else 1
        self._cross_rank_sum(self.acc, self.acc_i if mode == 0 else self.acc_d)
        x1 = self.acc.view(1, L.ld)  # the summed chain as a one-client chunk: out = 1*sum / denom
        if yogi is None:
            kx.reduce(x1, 1, L.P, out, denom=denom32, finalize=True)
        else:
            kx.reduce_yogi(x1, 1, L.P, denom=denom32, out=out, **yogi)
        kx.side_close(L.Q, mode, denom64, acc_i=self.acc_i, acc_d=self.acc_d, cur=cur_side, model=model_side)

    # ---- FedAvg / FedBuff: mean (+ optional fused FedYoGi) --------------------------------------
    @on_stream
    def finalize_mean(self, denom32: float, denom64: float, *, out: torch.Tensor, cur_side: torch.Tensor,
                      model_side: Optional[torch.Tensor] = None, yogi: Optional[dict] = None,
                      mirror: Optional[torch.Tensor] = None):
        """Reduce the last chunk with the epilogue fused.

        out        <- fp32 mean (or, with ``yogi``, the new global model last + step)
        cur_side   <- float64 mean of the side table (np.divide of int64 sums)
        model_side <- int64(fp32(mean)) (what load_state_dict stores), when given
        yogi       -> dict(last=, m=, v=, eta=, tau=, beta=, omb=, omb2=, init=)
        mirror     <- (no ``yogi``) a second copy of the mean, e.g. a pinned host buffer (fa_reduce_mirror)

        A small single-chunk round whose updates are all still in the staging's pinned mirror is reduced
        straight from it (``ClientStaging.host_rows``): no H2D copy."""
        self._check_complete()
        if self.cg is not None:
            self.staging.drain()
            return self._finalize_mean_clients(denom32, denom64, out, cur_side, model_side, yogi)
        L, st, n = self.layout, self.staging, self.slot
        first = self.chunks_done == 0
        zc = st.host_rows(n) if (first and yogi is None) else None
        if zc is None:
            st.drain()
        x, xi = zc if zc is not None else (st.x, st.xi)
        a32 = a64 = None
        if self.policy == "fedbuff":
            a32, a64 = self._chunk_weights()
        acc_in = None if first else self.acc
        if self.head:  # the head launch reduced rows [0, head): continue its chain over the rest (FedAvg, Q == 0)
            x, n, acc_in = x[self.head:], n - self.head, self.head_acc
        mode = 0 if self.policy == "fedavg" else 1
        try:
            if yogi is not None:
                kx.reduce_yogi(x, n, L.P, a=a32, acc_in=acc_in, denom=denom32, out=out, **yogi)
            elif mirror is not None:
                kx.reduce_mirror(x, n, L.P, out, mirror, a=a32, acc_in=acc_in, denom=denom32)
            else:
                kx.reduce(x, n, L.P, out, a=a32, acc_in=acc_in, denom=denom32, finalize=True,
                          host_ok=zc is not None)
            kx.side_accumulate(xi, n, L.Q, mode, w=a64, acc_i=self.acc_i, acc_d=self.acc_d, accumulate=not first)
        finally:
            if zc is not None:  # the mirror's rows are rewritten only after the stream has passed these reads
                st.release_host_rows()
        kx.side_close(L.Q, mode, denom64, acc_i=self.acc_i, acc_d=self.acc_d, cur=cur_side, model=model_side)

    @on_stream
    def mean_from_staging(self, out: torch.Tensor, cur_side: torch.Tensor) -> bool:
        """The plain FedAvg mean of this round (aggregator.py:497-507), recomputed from the staged updates
        when they are all still resident (q-FedAvg rounds do not need it, but the reference keeps it in
        ``Aggregator.model_weights``).  Returns False when the staging was folded or reused."""
        if self.cg is not None:
            return False  # client mode: each rank holds only its block of the updates
        L = self.layout
        if self.chain is not None and self.n == self.K and self.slot == 0:  # the fused chain of every chunk
            kx.reduce(self.chain.view(1, L.ld), 1, L.P, out, denom=float(np.float32(self.K)), finalize=True)
            kx.side_close(L.Q, 0, float(self.K), acc_i=self.acc_i, cur=cur_side)
            return True
        if self.cap < self.K or self.staging.generation != self.generation or self.n != self.K:
            return False  # some updates were overwritten by later chunks, or the slots were reused
        self.staging.drain()
        st = self.staging
        kx.reduce(st.x, self.K, L.P, out, denom=float(np.float32(self.K)), finalize=True)
        acc_i = torch.zeros(L.ldq, dtype=torch.int64, device=self.device)
        kx.side_accumulate(st.xi, self.K, L.Q, 0, acc_i=acc_i, acc_d=None)
        kx.side_close(L.Q, 0, float(self.K), acc_i=acc_i, cur=cur_side)
        return True

    # ---- q-FedAvg --------------------------------------------------------------------------------
    @on_stream
    def finalize_qfed(self, *, out: torch.Tensor, model_side: torch.Tensor, sqnorm_allreduce=None):
        """Fold the last chunk, then hs (optimizers.py:96-98) and new = L - delta/(hs+1e-10) (:101-104).

        ``sqnorm_allreduce(t)`` sums the per-client partial squared norms across shards (RCCL) when the
        model is sharded over ranks; the side table contributes once, after the all-reduce."""
        self.qfed_fold()
        if self.cg is None and sqnorm_allreduce is not None:
            sqnorm_allreduce(self.sqnorm)
        self.qfed_finish(out=out, model_side=model_side)

    @on_stream
    def qfed_fold(self):
        """Phase 1 of the finish: fold the last chunk.  ``sqnorm`` then holds this shard's partial per-client
        squared norms (the fp32 bucket part; summed over the shards by the caller between the phases)."""
        self._check_complete()
        if self.slot:
            self._fold_chunk()
        if self.cg is not None:
            # each client's norms were computed on its owner rank only: the sum is a gather (exact);
            # delta and delta_s are per-rank partial chains
            self._cross_rank_sum(self.delta, self.delta_s, self.sqnorm, self.sqnorm_side)

    @on_stream
    def qfed_finish(self, *, out: torch.Tensor, model_side: torch.Tensor):
        """Phase 2: hs over the (shard-summed) norms and the step."""
        L = self.layout
        # side table: replicated on every rank, so it is added once, after the cross-shard sum
        self.sqnorm += self.sqnorm_side
        c1 = torch.from_numpy(self.c1).to(self.device, non_blocking=True)
        c2 = torch.from_numpy(self.c2).to(self.device, non_blocking=True)
        self.hs = torch.zeros(2, dtype=torch.float32, device=self.device)
        kx.qfed_hs(self.sqnorm, c1, c2, self.K, self.hs)
        kx.qfed_finalize(self.last_f32, self.delta, self.hs, out, L.P)
        kx.side_qfed_finalize(self.last_i64, self.delta_s, self.hs, model_side, L.Q)
