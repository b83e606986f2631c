"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo in CPU tests).

The reference parallelises only over points inside one process (rayon,
lib.rs:194-199); every (key, point) evaluation is independent.  Here the points
(or keys) are split into contiguous per-rank slices with NO collective on the
data path.  The only exchanges are:
  * broadcast of the key material (correction-word block + seeds) from the rank
    that ran gen, once, before evaluation;
  * an optional gather of output shares onto one rank when the caller needs
    them on one device.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def point_slice(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous slice [start, start + count) of `total` points for `rank`
    (strong scaling: the first total % world ranks get one extra point)."""
    if world_size <= 0 or not 0 <= rank < world_size:
        raise ValueError("bad world/rank")
    base, rem = divmod(total, world_size)
    start = rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def weak_slice(per_rank: int, rank: int) -> Tuple[int, int]:
    """Weak scaling: rank r owns global points [r * per_rank, (r + 1) * per_rank)."""
    return rank * per_rank, per_rank


def broadcast_key(tensors: List[torch.Tensor], src: int = 0) -> List[torch.Tensor]:
    """Broadcast key material (CWB, seeds, ...) from `src` to every rank, in place."""
    ws, _ = world()
    if ws > 1:
        for t in tensors:
            dist.broadcast(t, src=src)
    return tensors


def gather_shares(ys: torch.Tensor, dst: int = 0) -> Optional[torch.Tensor]:
    """Gather every rank's equally-sized output slice onto `dst` (rank order =
    global point order).  Returns the concatenation on dst, None elsewhere."""
    ws, rank = world()
    if ws == 1:
        return ys
    parts = [torch.empty_like(ys) for _ in range(ws)] if rank == dst else None
    dist.gather(ys, gather_list=parts, dst=dst)
    return torch.cat(parts, 0) if rank == dst else None
