"""N>1 path on CPU: contiguous frame sharding + gather of PCM to rank 0 (world size 2, gloo).

The device decode is stood in for by the oracle here (test infrastructure, no GPU): each
rank decodes only its own frame range, rank 0 gathers the packed PCM and checks it against
a whole-stream decode -- the property bench.py's multi-GPU path relies on.
"""
import os
import socket

import numpy as np
import pytest

from birdnest.audio_amd import shard


def test_partition_balanced_and_complete():
    spf = [4096] * 100 + [192] * 50 + [16384] * 10
    for world in (1, 2, 3, 8):
        parts = shard.partition(spf, world)
        assert parts[0][0] == 0 and parts[-1][1] == len(spf)
        assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
        loads = [sum(spf[s:e]) for s, e in parts]
        assert max(loads) - min(loads) <= max(spf) * 2
    assert shard.partition([], 4) == [(0, 0)] * 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame_pcm(oracle, data, off):
    """Interleaved int32 [bs, ch] of the frame at byte `off` (oracle, planar -> interleaved)."""
    rc, res, planar = oracle.decode_frame_at(data, off, None)
    assert rc == 0 and res.error < 0 and res.crc_ok == 1
    bs, ch = int(res.blocksize), int(res.channels)
    return planar[: bs * ch].reshape(ch, bs).T.reshape(-1)


def _worker(rank, world, port, data, offsets, blocksizes, result_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import torch
    import torch.distributed as dist
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        start, end = shard.partition(blocksizes, world)[rank]
        pcm = []
        for f in range(start, end):
            pcm.append(_frame_pcm(oracle, data, int(offsets[f])))
        local = np.concatenate(pcm).astype("<i2").view(np.uint8) if pcm else np.zeros(0, np.uint8)
        got = shard.gather_bytes(torch.from_numpy(local.copy()))
        if rank == 0:
            result_q.put(got.numpy().tobytes())
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_matches_whole_stream():
    import torch.multiprocessing as mp
    from birdnest.audio_amd import synth
    import oracle
    p = synth.config("C4", nframes=24, seed=11)
    s = synth.encode(p)
    data = s.data.tobytes()
    offs = [int(o) for o in s.frame_offsets]
    bss = [len(_frame_pcm(oracle, data, o)) // p.channels for o in offs]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, data, offs, bss, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert got == s.pcm.astype("<i2").tobytes()


def _gather_worker(rank, world, port, sizes, result_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        local = torch.full((sizes[rank],), rank + 1, dtype=torch.uint8)
        got = shard.gather_bytes(local)
        if rank == 0:
            result_q.put(got.numpy().tobytes())
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_concurrent_gather_three_ranks_ragged():
    """shard.gather_bytes posts every receive at once (batch_isend_irecv): ragged sizes,
    one rank with nothing to send, concatenated in rank order on rank 0."""
    import torch.multiprocessing as mp
    sizes = [5, 0, 70001]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 3, port, sizes, q)) for r in range(3)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert got == bytes([1] * 5 + [3] * 70001)


def _pipeline_worker(rank, world, port, steps, result_q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1000 + 37 * rank  # unequal shards
        bufs = [torch.zeros(n, dtype=torch.uint8), torch.zeros(n, dtype=torch.uint8)]
        sizes = shard.gather_sizes(bufs[0])
        pend, parts = [[], []], [None, None]
        for st in range(steps):
            b = st % 2
            for w in pend[b]:
                w.wait()
            bufs[b].copy_(torch.arange(n, dtype=torch.int64).add(rank * 7 + st * 13).remainder(251).to(torch.uint8))
            pend[b], parts[b] = shard.gather_post(bufs[b], sizes, parts=parts[b])
        for b in (0, 1):
            for w in pend[b]:
                w.wait()
        if rank == 0:
            result_q.put(torch.cat(parts[(steps - 1) % 2]).numpy().tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_overlapped_gather_pipeline(world):
    """bench.py's overlapped C5 flow: two output buffers, step s's gather posted
    (shard.gather_post) while step s + 1 fills the other buffer; rank 0 ends with the last
    step's bytes of every rank, in rank order."""
    import torch
    import torch.multiprocessing as mp
    steps = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    st = steps - 1
    ref = b"".join(torch.arange(1000 + 37 * r, dtype=torch.int64).add(r * 7 + st * 13).remainder(251).to(torch.uint8)
                   .numpy().tobytes() for r in range(world))
    assert got == ref


def _group_worker(rank, world, port, groups, result_q):
    """One rank "decodes" its files in groups (bytes derived from rank, group and position) and
    posts each group as soon as it is written; rank 0 checks the gathered bytes and the post
    order (receives posted first, then this rank's groups in decode order)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = groups[rank]
        out = torch.zeros(sum(mine), dtype=torch.uint8)
        sizes = shard.gather_group_sizes(mine)
        assert sizes == groups
        gg = shard.GroupGather(sizes, out)
        off = 0
        for g, n in enumerate(mine):
            part = out[off:off + n]
            part.copy_(torch.arange(n, dtype=torch.int64).add(rank * 31 + g * 7).remainder(253).to(torch.uint8))
            gg.post(g, part)
            off += n
        got = gg.wait()
        if rank == 0:
            result_q.put((got.numpy().tobytes(), gg.order))
        else:
            assert got is None
            assert gg.order == [("send", rank, g) for g in range(len(mine))]
    finally:
        dist.destroy_process_group()


def _run_group_gather(groups):
    import torch.multiprocessing as mp
    world = len(groups)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, groups, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got, order = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    want = b"".join(bytes((i + r * 31 + g * 7) % 253 for i in range(n)) for r, gs in enumerate(groups)
                    for g, n in enumerate(gs))
    assert got == want
    return order


def test_group_gather_overlaps_decode_three_ranks():
    """shard.GroupGather (the C5 flow's in-job overlap): every rank posts its groups as they
    are decoded, each group as one grouped call on both sides: rank 0's post(g) receives group
    g from every peer that has one (into the final buffer at the rank-major, group-minor
    offsets) and copies its own.  Ragged groups, an empty group, a rank with one group."""
    order = _run_group_gather([[300, 0, 1201], [4096, 17], [999]])
    assert order == [("recv", 1, 0), ("recv", 2, 0), ("copy", 0, 0), ("recv", 1, 1), ("copy", 0, 1), ("copy", 0, 2)]


def test_group_gather_dst_with_fewer_groups_two_ranks():
    """Sub-file groups of uneven counts: rank 0 has one group, rank 1 four (frame ranges of its
    file); wait() posts the receives of the groups rank 0 never reached, in group order."""
    order = _run_group_gather([[512], [100, 100, 0, 37]])
    assert order == [("recv", 1, 0), ("copy", 0, 0), ("recv", 1, 1), ("recv", 1, 3)]


def test_frame_groups_cover_every_frame_in_order():
    for nf, k in (([469] * 3, 4), ([5, 0, 1], 3), ([7], 1), ([2], 8)):
        ranges, owner = shard.frame_groups(nf, k)
        flat = [f for a, b in ranges for f in range(a, b)]
        assert flat == list(range(sum(nf)))
        starts = [0] + list(np.cumsum(nf))
        for (a, b), i in zip(ranges, owner):
            assert starts[i] <= a <= b <= starts[i + 1]
        assert all(sum(1 for o in owner if o == i) <= max(1, k) for i in range(len(nf)))
