"""k_decode_wave (one wave per frame: wave-cooperative Rice decode into LDS rows, lane-per-
channel restore, 64-lane CRC-16 and coalesced output) against the lane kernels (k_decode_st,
k_decode<W>), which the rest of the suite pins against the oracle: identical records and
identical PCM for every frame that decodes (status OK, CRC-failed frames zero-filled in both).
A frame whose decode ends TRUNC / ERROR gets the same record; its PCM is unspecified (the lane
kernels have written part of it, the wave kernel writes none), so it is not compared."""
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
    L.bnflac_debug_set_decode_wave(-1)


def _sp(libflac, data, max_bs=None):
    if data[:4] != b"fLaC":
        return libflac.StreamParams(0, 0, 0, 0, 2, 16, 0)
    si = data[8:42]
    x = int.from_bytes(si[10:18], "big")
    mx = int.from_bytes(si[2:4], "big") if max_bs is None else max_bs
    return libflac.StreamParams(1, int.from_bytes(si[0:2], "big"), mx, x >> 44,
                                ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1, x & ((1 << 36) - 1))


def _decode(gpu, data, offs, fmt, mode, sp):
    torch, libflac, dec, L = gpu
    dev = torch.device("cuda:0")
    d_bytes = torch.zeros((len(data) + 15) // 16 * 16 + 32, dtype=torch.uint8, device=dev)
    d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.tensor([int(o) for o in offs], dtype=torch.int64, device=dev)
    total = max(sp.total_samples, 1) if sp.has_stream_info else 1 << 20
    stride = libflac.out_stride(fmt, sp)
    d_out = torch.full((total * stride + 64,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(len(offs) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    L.bnflac_debug_set_decode_wave(mode)
    dec.decode_frames(d_bytes, len(data), d_offs, len(offs), sp, fmt, d_out, d_info)
    torch.cuda.synchronize()
    L.bnflac_debug_set_decode_wave(-1)
    return libflac.info_array(d_info.cpu().numpy()), d_out.cpu().numpy(), stride


FIELDS = ["status", "err", "frame_off", "resume_bit", "blocksize", "channels", "assignment", "bps",
          "out_sample", "crc16_calc", "crc16_read", "crc_ok"]


def _same(gpu, data, offs, fmt, max_bs=None):
    torch, libflac, _, _ = gpu
    sp = _sp(libflac, data, max_bs)
    a, oa, stride = _decode(gpu, data, offs, fmt, 0, sp)
    b, ob, _ = _decode(gpu, data, offs, fmt, 1, sp)
    for k in FIELDS:
        bad = np.nonzero(a[k] != b[k])[0]
        assert len(bad) == 0, f"{k} differs at frame {bad[0]} (offset {offs[bad[0]]}): lane {a[bad[0]]} wave {b[bad[0]]}"
    assert np.array_equal(a["flags"] & 6, b["flags"] & 6)
    n = 0
    for i in np.nonzero(a["status"] == 0)[0]:
        s0 = int(a["out_sample"][i]) * stride
        nb = int(a["blocksize"][i]) * (stride if fmt != libflac.OUT_PLANAR32 else 4 * int(a["channels"][i]))
        if fmt == libflac.OUT_FLACDECODER:
            nb = int(a["blocksize"][i]) * (4 if a["channels"][i] == 2 else 2)
            s0 = int(a["out_sample"][i]) * (4 if a["channels"][i] == 2 else 2)
        assert np.array_equal(oa[s0:s0 + nb], ob[s0:s0 + nb]), f"PCM of frame {i} (offset {offs[i]}) differs"
        n += 1
    return n


def _offsets(s):
    return [int(x) for x in s.frame_offsets]


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "roundtrip"])
def test_fixtures_identical(gpu, name):
    torch, libflac, _, _ = gpu
    data = open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read()
    assert _same(gpu, data, GOLD[name]["frame_offsets"], libflac.OUT_INTERLEAVED32) == len(GOLD[name]["frame_offsets"])


@pytest.mark.parametrize("fmt_name", ["OUT_PLANAR32", "OUT_INTERLEAVED32", "OUT_FLACDECODER", "OUT_FILEREADER"])
@pytest.mark.parametrize("cfg,kw", [("C1", {}), ("C2", {}), ("C2", {"stereo_mode": 3}), ("C3", {}), ("C4", {"nframes": 60}),
                                    ("C5", {"nframes": 6}), ("C2", {"partition_order": 0, "seed": 5}),
                                    ("C4", {"nframes": 40, "rice2": 1, "escape_permille": 150, "seed": 11}),
                                    ("C2", {"order": 32, "qlp_precision": 15, "prec_clamp": 0, "partition_order": -1,
                                            "seed": 7}),
                                    ("C2", {"channels": 1, "seed": 9})])
def test_configs_identical(gpu, fmt_name, cfg, kw):
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    fmt = getattr(libflac, fmt_name)
    s = synth.encode(synth.config(cfg, **({"nframes": 12, "last_blocksize": 0} | kw)))
    data = s.data.tobytes()
    _same(gpu, data, _offsets(s), fmt)


def test_wave_matches_source_pcm(gpu):
    """The wave path alone, end to end: the generator's PCM (FLACDecoder layout)."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C2", nframes=64))
    data = s.data.tobytes()
    info, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_FLACDECODER, 1, _sp(libflac, data))
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert out[:s.nsamples * 4].tobytes() == s.pcm.astype("<i2").tobytes()


def test_damaged_and_truncated_identical(gpu):
    """Byte flips (CRC failures, damaged residuals and headers) and a cut stream: same records,
    same PCM for every frame that decodes, CRC-failed frames zero-filled."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    rng = np.random.default_rng(77)
    for i in range(12):
        cfg = ["C1", "C2", "C3", "C4"][i % 4]
        s = synth.encode(synth.config(cfg, nframes=int(rng.integers(4, 16)), last_blocksize=0, seed=200 + i))
        data = bytearray(s.data.tobytes())
        offs = _offsets(s)
        for _ in range(int(rng.integers(1, 5))):
            p = int(rng.integers(offs[0] + 4, len(data)))
            data[p] ^= int(rng.integers(1, 256))
        if i % 3 == 2:
            data = data[:len(data) * 3 // 4]
            offs = [o for o in offs if o < len(data)]
        _same(gpu, bytes(data), offs, libflac.OUT_INTERLEAVED32)


def test_frames_wider_than_streaminfo_handed_back(gpu):
    """STREAMINFO's max blocksize below the frames' (C4's variable sizes): k_decode_wave hands
    the wide frames to the lane kernels (BNF_FL_WAVE_REDO); every frame still decodes."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C4", nframes=50, seed=3))
    data = s.data.tobytes()
    n = _same(gpu, data, _offsets(s), libflac.OUT_FLACDECODER, max_bs=1024)
    assert n == 50
    info, _, _ = _decode(gpu, data, _offsets(s), libflac.OUT_FLACDECODER, 1, _sp(libflac, data, 1024))
    assert (info["flags"] & 512).any() and not (info["flags"][info["blocksize"] <= 1024] & 512).any()


@pytest.mark.parametrize("order,stereo", [(2, 3), (4, 1), (3, 0)])
def test_fixed_24bit_side_leaves_24_bits(gpu, order, stereo):
    """FIXED subframes of 24-bit stereo (the side channel has 25 bits): the wave restore's
    24-bit MACs see history values past 24 bits, restore those groups again with 64-bit MACs,
    and stay identical to the lane kernels."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C3", nframes=6, last_blocksize=0, subframe_mode=synth.SUB_FIXED, order=order,
                                  stereo_mode=stereo, level=0.95, noise=0.3, wasted_bits_max=0, seed=40 + order))
    data = s.data.tobytes()
    assert _same(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32) == 6
    info, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32, 1, _sp(libflac, data))
    assert np.array_equal(out[:s.nsamples * 8].view("<i4").reshape(-1, 2), s.pcm)
