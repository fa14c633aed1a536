"""Multi-GPU sharding of a proof set (one process per GPU, torch.distributed).

Per-proof verification has no exchange step: rank r verifies proofs [lo_r, hi_r) and
owns their statuses.  The RLC batch check reduces each shard to one 32-byte partial
point whose weights are keyed by the proofs' GLOBAL index, so the partials of all
shards sum to the single-GPU partial; the only collective is an all-gather of
world_size x 32 bytes (RCCL over xGMI with the "nccl" backend, gloo on CPU), after
which every rank can combine them (cpz_combine_partials) and decide the batch.
"""
from __future__ import annotations

from typing import List, Tuple

BLOCK = 256  # shard boundaries align to the RLC prepare block (block sums of a_i s_i)


def shard_range(n_total: int, world: int, rank: int, align: int = BLOCK) -> Tuple[int, int]:
    """Contiguous [lo, hi) of rank `rank`; boundaries are multiples of `align` except the end."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    units = (n_total + align - 1) // align
    lo_u = (units * rank) // world
    hi_u = (units * (rank + 1)) // world
    return min(lo_u * align, n_total), min(hi_u * align, n_total)


def all_gather_partials(partial: bytes, group=None) -> List[bytes]:
    """All-gather every rank's 32-byte partial (in rank order)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    mine = torch.tensor(list(partial), dtype=torch.uint8, device=dev)
    outs = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    return [bytes(o.cpu().tolist()) for o in outs]
