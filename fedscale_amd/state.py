"""Flat device snapshots of a model state and the multi-GPU (sharded) plumbing.

``FlatState`` is what the device path hands around instead of the reference's list-of-tensors:
``f32`` is this rank's slice of the fp32 bucket, ``side`` the replicated side table (int64 for a model
state, float64 for a FedAvg mean of int64 entries).

Two ways to spread a round over the GPUs of a node (one process per GPU, torch.distributed over RCCL;
SURVEY §8e):

* ``mode="params"`` (default): every rank owns an equal-size slice of the fp32 bucket and reduces its
  slice of every client update.  The only collectives are the all-gather that reassembles the global model
  for egress and, for q-FedAvg, one all-reduce of the K per-client squared norms.  The per-element chain
  is the reference's, so the result is bit-exact.
* ``mode="clients"``: every rank holds the whole model and reduces a contiguous block of the round's
  arrivals (rank r takes arrival indices [r*K/N, (r+1)*K/N)).  The per-rank partial sums meet in one RCCL
  all-reduce (the "final RCCL reduce" of the north star) and the server step then runs replicated, so
  egress needs no gather.  Summing per-rank partials re-associates the fp32 chain: the result is within
  the north-star tolerance (1e-5 relative), not bit-exact; int64 side-table sums stay exact.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from .bucket import BucketLayout


@dataclass
class FlatState:
    layout: BucketLayout
    f32: torch.Tensor
    side: torch.Tensor


MODES = ("params", "clients")


class ShardGroup:
    """rank/world of the GPUs sharing a round; ``None`` group = the default process group."""

    def __init__(self, rank: int = 0, world: int = 1, group=None, mode: str = "params"):
        if mode not in MODES:
            raise ValueError(f"shard mode {mode!r} not in {MODES}")
        self.rank, self.world, self.group, self.mode = rank, world, group, mode

    @classmethod
    def from_env(cls, group=None, mode: str = "params") -> "ShardGroup":
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_rank(group), dist.get_world_size(group), group, mode)
        return cls(mode=mode)

    @property
    def shards_params(self) -> bool:
        """The fp32 bucket is split across ranks (egress needs the all-gather)."""
        return self.world > 1 and self.mode == "params"

    @property
    def shards_clients(self) -> bool:
        """Each rank reduces a block of the round's clients over the whole model."""
        return self.world > 1 and self.mode == "clients"

    def client_block(self, K: int, rank: Optional[int] = None):
        """[k0, k1): the arrival indices rank ``rank`` reduces in client mode (contiguous, balanced)."""
        r = self.rank if rank is None else rank
        return r * K // self.world, (r + 1) * K // self.world

    def owner(self, k: int, K: int) -> int:
        """The rank that reduces arrival index k of a K-client round (client mode)."""
        return ((k + 1) * self.world - 1) // K

    def _host_staged(self, t: torch.Tensor) -> bool:
        """gloo (CPU tests, several ranks sharing one GPU) moves device tensors through the host."""
        import torch.distributed as dist

        return t.device.type == "cuda" and dist.get_backend(self.group) == "gloo"

    def all_gather(self, shard: torch.Tensor) -> torch.Tensor:
        """Concatenate the equal-size shards of every rank (RCCL all-gather over xGMI).  In client mode the
        model is replicated, so the local copy already is the whole model."""
        if not self.shards_params:
            return shard
        import torch.distributed as dist

        if self._host_staged(shard):
            return self.__class__.all_gather(self, shard.cpu()).to(shard.device)
        out = torch.empty(self.world * shard.numel(), dtype=shard.dtype, device=shard.device)
        if shard.device.type == "cpu" and dist.get_backend(self.group) == "gloo":
            parts = list(out.chunk(self.world))
            dist.all_gather(parts, shard.contiguous(), group=self.group)
            return torch.cat(parts)
        dist.all_gather_into_tensor(out, shard.contiguous(), group=self.group)
        return out

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks (RCCL all-reduce; the K per-client partial norms of q-FedAvg)."""
        if self.world == 1:
            return t
        import torch.distributed as dist

        if self._host_staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t
