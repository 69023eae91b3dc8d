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
    output in groups (files, or frame ranges of a file) into consecutive slices of its output
    buffer and calls post(g, slice) as soon as group g is enqueued.  Every post is one
    batch_isend_irecv on every side, and the two sides post the same groups in the same order:
    a sender posts its group g alone; `dst`, at its own post(g), posts the receives of group g
    from every peer that has one (into the final buffer at the rank-major, group-minor offset,
    so nothing is concatenated afterwards) and copies its own slice into place.  Groups `dst`
    does not have are posted by wait(), before it waits.  Under RCCL each post runs on the
    communicator's stream after the work already enqueued on the current stream (that group's
    decode) and beside the decode of the next group; per peer, sends and receives pair up one
    grouped call against one grouped call, in group order.  wait() completes everything; on
    `dst` `out` then holds all ranks' bytes in rank order."""

    def __init__(self, sizes, like, group=None, dst: int = 0, out=None):
        import torch
        import torch.distributed as dist

        self.dist, self.group, self.dst = dist, group, dst
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
        self.sizes = sizes
        self.ngroups = max((len(x) for x in sizes), default=0)
        self.works = []
        self.order = []  # every op this rank posted, in post order: ("recv"|"send"|"copy", rank, group)
        self.posted = 0  # dst: groups whose receives are posted (0 .. posted-1)
        self.out = None
        if self.rank == dst:
            total = sum(sum(x) for x in sizes)
            self.out = out if out is not None else torch.empty(total, dtype=like.dtype, device=like.device)
            self.base = []
            off = 0
            for r in range(self.world):
                row = []
                for n in sizes[r]:
                    row.append(off)
                    off += n
                self.base.append(row)

    def _post_recvs(self, g):
        """dst: one grouped call with the receives of group g from every peer that has it."""
        dist = self.dist
        ops = []
        for r in range(self.world):
            if r != self.rank and g < len(self.sizes[r]) and self.sizes[r][g]:
                b, n = self.base[r][g], self.sizes[r][g]
                ops.append(dist.P2POp(dist.irecv, self.out[b:b + n], self.glob(r), self.group))
                self.order.append(("recv", r, g))
        if ops:
            self.works += dist.batch_isend_irecv(ops)

    def post(self, g, part):
        """Group g of this rank (its bytes, in this rank's output order) is enqueued: send it
        (on `dst`: receive every peer's group g and copy this one into place)."""
        if self.rank == self.dst:
            while self.posted <= g:
                self._post_recvs(self.posted)
                self.posted += 1
            if part.numel():
                b = self.base[self.rank][g]
                self.out[b:b + part.numel()].copy_(part, non_blocking=True)
            self.order.append(("copy", self.rank, g))
            return
        if part.numel():
            self.works += self.dist.batch_isend_irecv([self.dist.P2POp(self.dist.isend, part.contiguous(),
                                                                       self.glob(self.dst), self.group)])
        self.order.append(("send", self.rank, g))

    def wait(self):
        if self.rank == self.dst:
            while self.posted < self.ngroups:
                self._post_recvs(self.posted)
                self.posted += 1
        for w in self.works:
            w.wait()
        self.works = []
        return self.out


def frame_groups(nframes_per_file, groups_per_file):
    """Frame ranges [f0, f1) for GroupGather groups: each file's frames cut into up to
    `groups_per_file` near-equal contiguous ranges (a file with fewer frames gets fewer), in
    file order; returns (ranges, file index of each range)."""
    out, owner, f0 = [], [], 0
    for i, n in enumerate(nframes_per_file):
        k = max(1, min(int(groups_per_file), int(n))) if n else 1
        cuts = [f0 + (n * j) // k for j in range(k + 1)]
        for a, b in zip(cuts, cuts[1:]):
            if b > a or n == 0:
                out.append((a, b))
                owner.append(i)
        f0 += n
    return out, owner
