"""One-process-per-GPU data parallelism over torch.distributed (RCCL on MI355X).

The reference's only parallelism is single-process `nn.DataParallel`
(models/utils.py:93): parameters broadcast on every forward and gradients
reduce-added to GPU 0.  Here:
  * sampling is batch-sharded: rank r owns global samples [r*B, (r+1)*B); the
    only exchange is a 2-float all-reduce per Langevin step (sampling.py:276-277)
    and an optional all-gather of the samples at the end;
  * training uses DistributedDataParallel: parameters are broadcast once, and the
    gradient buckets are all-reduced (RCCL over xGMI) while backward runs.
Backend "nccl" is RCCL on ROCm; "gloo" runs the same code on CPU for tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as tdist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    group: object = None

    @property
    def enabled(self):
        return self.world_size > 1

    def all_reduce_sum_(self, t):
        if self.world_size > 1:
            tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_max(self, value: float, device=None):
        if self.world_size == 1:
            return value
        t = torch.tensor([value], dtype=torch.float64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def all_gather_cat(self, t):
        if self.world_size == 1:
            return t
        parts = [torch.empty_like(t) for _ in range(self.world_size)]
        tdist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, 0)

    def barrier(self):
        if self.world_size > 1:
            if tdist.get_backend(self.group) == "nccl":
                tdist.barrier(group=self.group, device_ids=[self.local_rank])
            else:
                tdist.barrier(group=self.group)


def init_from_env(backend=None) -> DistContext:
    """Initialise from torchrun's RANK / WORLD_SIZE / LOCAL_RANK (single process if unset).
    Backend: `backend`, else $BPK_DIST_BACKEND, else nccl (RCCL) with a GPU and gloo
    without.  (gloo on GPU tensors lets several ranks share one device -- a rehearsal of
    the multi-GPU code paths on a one-GPU box.)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return DistContext()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = os.environ.get("BPK_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not tdist.is_initialized():
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        tdist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return DistContext(rank=rank, world_size=world, local_rank=local)


def shard(n_global: int, ctx: DistContext):
    """(offset, count) of this rank's slice of n_global items (equal shards required)."""
    if n_global % ctx.world_size:
        raise ValueError(f"batch {n_global} not divisible by world size {ctx.world_size}")
    per = n_global // ctx.world_size
    return ctx.rank * per, per
