"""One process per GPU: placement, barrier, max-over-ranks timing, host-side gather.

The path shards by stream: videos are independent, each
rank owns a contiguous block of streams and its own HIP device, and no tensor
crosses ranks.  torch.distributed is used only for control: the timing
barrier, the max of per-rank elapsed time, and gathering per-stream result
tuples on rank 0 (the equivalent of run_pool's res.get(), fm.py:1087).
Backend "nccl" (RCCL) on the GPU box, "gloo" in CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class Placement:
    rank: int
    world: int
    local_rank: int

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def placement_from_env() -> Placement:
    return Placement(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                     int(os.environ.get("LOCAL_RANK", "0")))


def rank_streams(p: Placement, streams_per_rank: int) -> list:
    """Global stream ids of this rank: stream s -> rank s // streams_per_rank."""
    return list(range(p.rank * streams_per_rank, (p.rank + 1) * streams_per_rank))


def init(p: Placement, backend: str, device=None, force: bool = False) -> bool:
    """Initialise the process group when world > 1 (rendezvous from MASTER_ADDR/PORT).

    `force` also builds a one-rank group, so that the RCCL calls an 8-GPU run makes (the
    `device_id` binding, barrier, all-reduce of a device tensor, gather_object) run on a
    one-GPU box too (bench.py's FM_BENCH_PG=1); RCCL refuses two ranks on one device.
    """
    if p.world <= 1 and not force:
        return False
    import torch.distributed as dist

    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    dist.init_process_group(backend, rank=p.rank, world_size=p.world, **kw)
    return True


def world_size(active: bool) -> int:
    """Ranks in the process group as the group itself reports them (1 without one)."""
    if not active:
        return 1
    import torch.distributed as dist

    return dist.get_world_size()


def barrier(active: bool) -> None:
    if active:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(value: float, active: bool, device="cpu") -> float:
    if not active:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_root(obj, p: Placement, active: bool):
    """List of every rank's obj on rank 0 (None elsewhere)."""
    if not active:
        return [obj]
    import torch.distributed as dist

    out = [None] * p.world if p.is_root else None
    dist.gather_object(obj, out, dst=0)
    return out


def finalize(active: bool) -> None:
    if active:
        import torch.distributed as dist

        dist.destroy_process_group()
