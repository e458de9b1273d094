"""Flat device snapshots of a model state and the multi-GPU (sharded) plumbing.

``FlatState`` is what the device path hands around instead of the reference's list-of-tensors:
``f32`` is this rank's slice of the fp32 bucket, ``side`` the replicated side table (int64 for a model
state, float64 for a FedAvg mean of int64 entries).

Sharding (one process per GPU, torch.distributed over RCCL): every rank owns an equal-size slice of the
fp32 bucket, so the only collectives the path needs are the all-gather that reassembles the global model
for egress and, for q-FedAvg, one all-reduce of the K per-client squared norms.
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


class ShardGroup:
    """rank/world of the model shards; ``None`` group = single GPU, no collectives."""

    def __init__(self, rank: int = 0, world: int = 1, group=None):
        self.rank, self.world, self.group = rank, world, group

    @classmethod
    def from_env(cls, group=None) -> "ShardGroup":
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized():
            return cls(dist.get_rank(group), dist.get_world_size(group), group)
        return cls()

    def _host_staged(self, t: torch.Tensor) -> bool:
        """gloo (CPU tests, several ranks sharing one GPU) moves device tensors through the host."""
        import torch.distributed as dist

        return t.device.type == "cuda" and dist.get_backend(self.group) == "gloo"

    def all_gather(self, shard: torch.Tensor) -> torch.Tensor:
        """Concatenate the equal-size shards of every rank (RCCL all-gather over xGMI)."""
        if self.world == 1:
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
