"""Multi-GPU request sharding: one process per GPU, no data-path collective.

The reference's DynamicBatchManager runs every request on one wgpu device
(src/dynamic_batch_manager.rs:409-476). Here requests shard across the GPUs of a node
(rank r takes every request whose index is r mod world), weights are broadcast once from
rank 0 over RCCL/xGMI (`nccl` backend) -- or gloo on CPU for tests -- and the only other
collectives are the timing/count reductions of a benchmark. Decode itself never communicates.
"""
from typing import List, Sequence, Tuple, TypeVar

T = TypeVar("T")


def shard(items: Sequence[T], rank: int, world: int) -> List[T]:
    """Round-robin shard: rank r gets items r, r + world, r + 2*world, ..."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return list(items[rank::world])


def unshard(parts: Sequence[Sequence[T]]) -> List[T]:
    """Inverse of shard over all ranks' result lists (rank-major input, original order out)."""
    world = len(parts)
    n = sum(len(p) for p in parts)
    out: List[T] = [None] * n  # type: ignore[list-item]
    for r, p in enumerate(parts):
        for j, x in enumerate(p):
            out[r + j * world] = x
    return out


def broadcast_blob(tensor, src: int = 0):
    """Broadcast a weight blob (a torch tensor, device or host) from `src` to every rank."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(tensor, src=src)
    return tensor


def reduce_run(elapsed_s: float, units: int, device=None) -> Tuple[float, int]:
    """Max wall time over ranks and the sum of processed units (the bench contract)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return elapsed_s, units
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    n = torch.tensor([units], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), int(n.item())
