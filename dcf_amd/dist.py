"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo in CPU tests).

The reference parallelises only over points inside one process (rayon,
lib.rs:194-199); every (key, point) evaluation is independent.  Here the points
(or keys) are split into contiguous per-rank slices with NO collective on the
data path.  The only exchanges are:
  * broadcast of the key material (correction-word block + seeds) from the rank
    that ran gen, once, before evaluation;
  * an optional gather of output shares onto one rank when the caller needs
    them on one device (the reference writes every output into the caller's
    `ys`, lib.rs:163,196-198).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def active() -> bool:
    """A process group is up (possibly of world size 1: the RCCL path still runs then)."""
    return dist.is_available() and dist.is_initialized()


def world() -> Tuple[int, int]:
    if active():
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
    """Broadcast key material (CWB, seeds, ...) from `src` to every rank, in place.  Runs
    the collective whenever a process group is up, also at world size 1 (so a one-GPU run
    exercises the same RCCL broadcast an 8-GPU run does)."""
    if active():
        for t in tensors:
            dist.broadcast(t, src=src)
    return tensors


def _host_collectives(t: torch.Tensor) -> bool:
    """gloo's gather / all_gather of row counts take host tensors only."""
    return t.is_cuda and dist.get_backend() == "gloo"


def gather_shares(ys: torch.Tensor, dst: int = 0, counts: Optional[Sequence[int]] = None) -> Optional[torch.Tensor]:
    """Gather every rank's output slice onto `dst` in rank order (= global point order
    for the contiguous slices of point_slice / weak_slice).  Slices may differ in length
    (point_slice gives the first total % world ranks one extra point): the row counts are
    all-gathered (or taken from `counts`), every slice is padded to the longest for the
    collective, and dst trims the padding.  Returns the concatenation (on ys's device)
    on dst, None elsewhere.  With a process group up the collectives run at any world
    size, 1 included; without one the slice is the whole output."""
    if not active():
        return ys
    ws, rank = world()
    dev = ys.device
    host = _host_collectives(ys)
    if counts is None:
        n = torch.tensor([ys.shape[0]], dtype=torch.int64, device="cpu" if host else dev)
        got = [torch.zeros_like(n) for _ in range(ws)]
        dist.all_gather(got, n)
        counts = [int(c.item()) for c in got]
    counts = [int(c) for c in counts]
    if len(counts) != ws or counts[rank] != ys.shape[0]:
        raise ValueError(f"counts {counts} do not match this rank's {ys.shape[0]} rows")
    rows = max(counts)
    src = ys.cpu() if host else ys
    if src.shape[0] < rows:  # pad to the longest slice (the collective needs equal shapes)
        pad = torch.zeros((rows,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        pad[:src.shape[0]] = src
        src = pad
    parts = [torch.empty_like(src) for _ in range(ws)] if rank == dst else None
    dist.gather(src.contiguous(), gather_list=parts, dst=dst)
    if rank != dst:
        return None
    return torch.cat([p[:c] for p, c in zip(parts, counts)], 0).to(dev)
