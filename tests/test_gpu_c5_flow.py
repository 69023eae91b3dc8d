"""C5's data path end to end on one GPU (world size 1): bench.c5_job shards the files
(shard.partition), indexes each on the GPU (bnflac_index_stream), decodes all of the rank's
frames in one k_parse + decode launch into FLACFileReader 24-bit PCM, and gathers to rank 0
-- the same code the driver's multi-GPU C5 run takes, here with one rank.  Bit-exact against
the generator's source PCM (lossless round trip)."""
import argparse

import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu


def test_c5_flow_world1():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    import bench
    from birdnest.audio_amd import libflac, synth
    dev = torch.device("cuda:0")
    dec = libflac.BatchDecoder(0)
    args = argparse.Namespace(batches=2, steps=1, warmup=1)
    r = bench.c5_job(args, torch, None, dev, libflac, synth, dec, 1, 0)
    assert r["ok"] and r["files"] == 2
    p = synth.config("C5")
    assert r["samples"] == 2 * (468 * 4096 + p.last_blocksize) * 8
