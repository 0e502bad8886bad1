"""Multi-GPU control plane for the sharded batch hash (SURVEY.md §8 e).

Keys are independent, so a batch shards by contiguous index range (fixed
length) or by byte-balanced index range (variable length) with NO data-path
collective.  torch.distributed (gloo, CPU) only carries the barrier and the
max-over-ranks wall time used by bench.py.  One process per GPU, launched by
torch.distributed.run; MASTER_ADDR should be 127.0.0.1.
"""
from __future__ import annotations

import os
from typing import Tuple

from .workload import shard_range, shard_var  # noqa: F401


def env_ranks() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")


def barrier(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def reduce_max(x: float, world: int) -> float:
    if world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather(obj, world: int) -> list:
    """Every rank's `obj` (a small JSON-able value), in rank order."""
    if world <= 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def sum_int(x: int, world: int) -> int:
    if world <= 1:
        return int(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(x)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def finalize(world: int) -> None:
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
