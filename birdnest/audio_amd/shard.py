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

    Sizes go first (all_gather of one int64); then `dst` posts every receive at once and
    the other ranks send, as one batch of point-to-point ops (dist.batch_isend_irecv: a
    grouped ncclSend/ncclRecv under RCCL), so the peers' transfers run concurrently over
    their own xGMI links instead of one link at a time.  RCCL has no gatherv.
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
    glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
    if rank == dst:
        parts = [local if r == rank else torch.empty(sizes[r], dtype=local.dtype, device=local.device)
                 for r in range(world)]
        ops = [dist.P2POp(dist.irecv, parts[r], glob(r), group) for r in range(world) if r != rank and sizes[r]]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return torch.cat(parts)
    if local.numel():
        for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, local.contiguous(), glob(dst), group)]):
            req.wait()
    return None


def gather_sizes(local, group=None):
    """Every rank's byte count (one all_gather of an int64), for gather_post."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    return [int(x.item()) for x in sizes]


def gather_post(local, sizes, group=None, dst: int = 0, parts=None):
    """Post one gather of `local` to `dst` (sizes from gather_sizes) without waiting: returns
    (works, parts).  On `dst`, parts are the receive buffers in rank order (pass the previous
    call's to reuse them; parts[dst] is `local` itself); elsewhere None.  Under RCCL the ops
    run on the communicator's stream, ordered after the work already enqueued on the current
    stream (the decode of `local`) and concurrent with work enqueued after them (the next
    step's decode into another buffer): bench.py's C5 flow overlaps step s's gather with step
    s + 1's decode this way.  work.wait() orders the current stream after the transfer."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
    if rank == dst:
        if parts is None:
            parts = [None] * world
            for r in range(world):
                if r != rank:
                    parts[r] = torch.empty(sizes[r], dtype=local.dtype, device=local.device)
        parts[rank] = local
        ops = [dist.P2POp(dist.irecv, parts[r], glob(r), group) for r in range(world) if r != rank and sizes[r]]
        return (dist.batch_isend_irecv(ops) if ops else []), parts
    if local.numel():
        return dist.batch_isend_irecv([dist.P2POp(dist.isend, local.contiguous(), glob(dst), group)]), None
    return [], None


def gather_group_sizes(group_sizes, group=None, device=None):
    """Every rank's per-group byte counts (all_gather of a fixed-width int64 vector, padded
    with -1), for GroupGather: a rank's output is the concatenation of its groups.  device:
    where the collective's tensors live (the GPU under RCCL, the CPU under gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([len(group_sizes)], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    width = max(int(x.item()) for x in ns)
    mine = torch.full((max(width, 1),), -1, dtype=torch.int64, device=device)
    if len(group_sizes):
        mine[:len(group_sizes)] = torch.tensor(list(group_sizes), dtype=torch.int64, device=device)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    return [[int(v) for v in a.tolist() if v >= 0] for a in allv]


class GroupGather:
    """A gather of every rank's output to `dst` that starts while the ranks are still decoding
    ("overlap the gather chunk-wise with decode").  A rank decodes its
    files in groups into consecutive slices of its output buffer and calls post(g, slice) as
    soon as group g is enqueued; `dst` posted every receive up front, straight into the final
    buffer at the rank-major, group-minor offset, so nothing is concatenated afterwards.
    Under RCCL each post runs on the communicator's stream after the work already enqueued on
    the current stream (that group's decode) and beside the decode of the next group; per
    peer, sends and receives match in group order.  wait() completes everything; on `dst`
    `out` then holds all ranks' bytes in rank order."""

    def __init__(self, sizes, like, group=None, dst: int = 0, out=None):
        import torch
        import torch.distributed as dist

        self.dist, self.group, self.dst = dist, group, dst
        self.rank = dist.get_rank(group)
        world = dist.get_world_size(group)
        self.glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
        self.sizes = sizes
        self.works = []
        self.order = []  # (rank, group) of every post made by this rank, in post order
        self.out = None
        if self.rank == dst:
            total = sum(sum(s) for s in sizes)
            self.out = out if out is not None else torch.empty(total, dtype=like.dtype, device=like.device)
            self.base = []
            off = 0
            for r in range(world):
                row = []
                for s in sizes[r]:
                    row.append(off)
                    off += s
                self.base.append(row)
            ops = []
            for r in range(world):
                if r == self.rank:
                    continue
                for g, s in enumerate(sizes[r]):
                    if s:
                        ops.append(dist.P2POp(dist.irecv, self.out[self.base[r][g]:self.base[r][g] + s], self.glob(r), group))
                        self.order.append(("recv", r, g))
            if ops:
                self.works += dist.batch_isend_irecv(ops)

    def post(self, g, part):
        """Group g of this rank (its bytes, in this rank's output order) is enqueued: send it
        (or, on `dst`, copy it into place)."""
        if self.rank == self.dst:
            if part.numel():
                self.out[self.base[self.rank][g]:self.base[self.rank][g] + part.numel()].copy_(part, non_blocking=True)
            self.order.append(("copy", self.rank, g))
            return
        if part.numel():
            self.works += self.dist.batch_isend_irecv([self.dist.P2POp(self.dist.isend, part.contiguous(),
                                                                       self.glob(self.dst), self.group)])
        self.order.append(("send", self.rank, g))

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
        return self.out
