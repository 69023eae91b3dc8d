"""Multi-GPU sharding of the decode path: one process per GPU.

Frames are independent given their byte offsets and STREAMINFO, so a batch is split into
contiguous frame ranges balanced by output samples (variable blocksizes make equal frame
counts unequal work).  Decode needs no exchange; the only collective is the optional
final gather of each rank's PCM bytes to rank 0 (C5's "RCCL gather", which RCCL has no
gatherv for: sizes are exchanged first, then point-to-point send/recv).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def partition(samples_per_frame: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) frame ranges, one per rank, balanced by samples.

    Rank r's range starts at the first frame whose cumulative sample start reaches
    r/world of the total; ranges cover every frame exactly once, in order.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    spf = np.asarray(samples_per_frame, dtype=np.int64)
    n = int(spf.size)
    starts = np.concatenate([[0], np.cumsum(spf)[:-1]]) if n else np.zeros(0, dtype=np.int64)
    total = int(spf.sum())
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cuts.append(int(np.searchsorted(starts, target, side="left")) if n else 0)
    cuts.append(n)
    for r in range(1, len(cuts)):
        cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def gather_bytes(local, group=None, dst: int = 0):
    """Gather variable-length uint8 tensors to rank `dst` (concatenated in rank order).

    Returns the concatenation on `dst`, None elsewhere.  Works with the gloo (CPU tensors)
    and nccl/RCCL (device tensors) backends.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    if rank == dst:
        parts = []
        for r in range(world):
            if r == rank:
                parts.append(local)
            else:
                buf = torch.empty(sizes[r], dtype=local.dtype, device=local.device)
                if sizes[r]:
                    dist.recv(buf, src=r, group=group)
                parts.append(buf)
        return torch.cat(parts)
    if local.numel():
        dist.send(local, dst=dst, group=group)
    return None
