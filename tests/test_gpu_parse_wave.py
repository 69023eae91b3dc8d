"""k_parse_wave (one wave per frame, wave-cooperative Rice boundary scan) against k_parse
(one lane per frame, serial walk): identical 128-byte records for every sync candidate.

Candidates are every frame-sync pattern in the stream (frame_sync_'s test, LibFlac.dll
@0x1001187c), so most records of corrupted streams are errors: header errors, LOST_SYNC in
a subframe header, reserved types, truncation.  The records carry the header fields, the
subframe start bits found by the walk (sub_start), the status / error / resume bit and the
decode class, and the decode of every frame reads them.  The scan's correctness is therefore
pinned against the lane walk, which the rest of the suite pins against the oracle.
"""
import json
import os

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(GOLD_DIR, "golden.json")))


@pytest.fixture(scope="module")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from birdnest.audio_amd import libflac
    L = libflac.load()
    yield torch, libflac, libflac.BatchDecoder(0), L
    L.bnflac_debug_set_parse_wave(-1)


def _sp(libflac, data):
    if data[:4] != b"fLaC":
        return libflac.StreamParams(0, 0, 0, 0, 2, 16, 0)  # a bare frame: no STREAMINFO (the API needs a channel count)
    si = data[8:42]
    x = int.from_bytes(si[10:18], "big")
    return libflac.StreamParams(1, int.from_bytes(si[0:2], "big"), int.from_bytes(si[2:4], "big"), x >> 44,
                                ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1, x & ((1 << 36) - 1))


def _candidates(data):
    b = np.frombuffer(data, dtype=np.uint8)
    if len(b) < 2:
        return np.zeros(0, np.int64)
    return np.nonzero((b[:-1] == 0xFF) & ((b[1:] >> 2) == 0x3E))[0].astype(np.int64)


def _records(gpu, data, offs, mode, nbytes=None):
    torch, libflac, dec, L = gpu
    dev = torch.device("cuda:0")
    n = len(data) if nbytes is None else nbytes
    d_bytes = torch.zeros((len(data) + 15) // 16 * 16 + 32, dtype=torch.uint8, device=dev)
    d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_info = torch.full((len(offs) * libflac.FRAME_INFO_BYTES,), 0x5A, dtype=torch.uint8, device=dev)
    L.bnflac_debug_set_parse_wave(mode)
    dec.parse_frames(d_bytes, n, d_offs, len(offs), _sp(libflac, data), d_info)
    torch.cuda.synchronize()
    L.bnflac_debug_set_parse_wave(-1)
    return d_info.cpu().numpy()


def _same(gpu, data, offs=None, nbytes=None):
    offs = _candidates(data) if offs is None else np.asarray(offs, dtype=np.int64)
    if nbytes is not None:
        offs = offs[offs < nbytes]
    if len(offs) == 0:
        return 0
    a = _records(gpu, data, offs, 0, nbytes)
    b = _records(gpu, data, offs, 1, nbytes)
    if not np.array_equal(a, b):
        _, libflac, _, _ = gpu
        ia, ib = libflac.info_array(a), libflac.info_array(b)
        bad = np.nonzero((a.reshape(len(offs), -1) != b.reshape(len(offs), -1)).any(axis=1))[0]
        i = int(bad[0])
        raise AssertionError(f"{len(bad)} of {len(offs)} records differ; first at offset {offs[i]}:\n"
                             f"lane walk {ia[i]}\nwave scan {ib[i]}")
    return len(offs)


@pytest.mark.parametrize("name", sorted(GOLD))
def test_fixture_candidates_identical(gpu, name):
    data = open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read()
    _same(gpu, data)


@pytest.mark.parametrize("cfg,kw", [("C1", dict(nframes=10)), ("C2", dict(nframes=64)),
                                    ("C3", dict(nframes=12)), ("C4", dict(nframes=60)),
                                    ("C5", dict(nframes=6, last_blocksize=0)),
                                    ("C4", dict(nframes=40, rice2=1, escape_permille=150, seed=11)),
                                    ("C2", dict(nframes=16, partition_order=0, seed=5)),
                                    ("C2", dict(nframes=16, partition_order=8, order=4, seed=6))])
def test_config_streams_identical(gpu, cfg, kw):
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config(cfg, **kw))
    data = s.data.tobytes()
    n = _same(gpu, data, s.frame_offsets.astype(np.int64))
    assert n == len(s.frame_offsets)
    _same(gpu, data)  # every candidate, false syncs included
    _same(gpu, data, nbytes=len(data) * 2 // 3)  # truncated: frames that run past the end


def test_corrupted_streams_identical(gpu):
    """Random byte flips in 40 streams of mixed configs: the records of every candidate match."""
    from birdnest.audio_amd import synth
    rng = np.random.default_rng(1234)
    total = 0
    for i in range(40):
        cfg = ["C1", "C2", "C3", "C4", "C5"][i % 5]
        kw = dict(nframes=int(rng.integers(3, 12)), seed=100 + i)
        if cfg == "C5":
            kw["last_blocksize"] = 0
        s = synth.encode(synth.config(cfg, **kw))
        data = bytearray(s.data.tobytes())
        for _ in range(int(rng.integers(1, 6))):
            p = int(rng.integers(42, len(data)))
            data[p] ^= int(rng.integers(1, 256))
        total += _same(gpu, bytes(data))
    assert total > 100


def test_reader_sized_stream_identical_and_decodes(gpu):
    """One whole C2 stream (the reader's launch): identical records, and the decode of the
    wave scan's records is the source PCM."""
    from birdnest.audio_amd import synth
    torch, libflac, dec, L = gpu
    s = synth.encode(synth.config("C2", nframes=1024))
    data = s.data.tobytes()
    _same(gpu, data, s.frame_offsets.astype(np.int64))
    dev = torch.device("cuda:0")
    d_bytes = torch.zeros((len(data) + 15) // 16 * 16 + 32, dtype=torch.uint8, device=dev)
    d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    offs = torch.tensor(s.frame_offsets.astype(np.int64), device=dev)
    sp = _sp(libflac, data)
    d_out = torch.zeros(s.nsamples * 4, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(1024 * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    L.bnflac_debug_set_parse_wave(1)
    dec.decode_frames(d_bytes, len(data), offs, 1024, sp, libflac.OUT_FLACDECODER, d_out, d_info)
    torch.cuda.synchronize()
    L.bnflac_debug_set_parse_wave(-1)
    assert d_out.cpu().numpy().tobytes() == s.pcm.astype("<i2").tobytes()
