"""k_decode_sys (a producer wave decoding Rice residuals lane-per-subframe, restore waves running
the LPC / FIXED recurrence as a systolic lane quad per subframe, coalesced CRC-16) against the
lane kernels (k_decode_st, k_decode_sw, k_decode<W>), which the rest of the suite pins against
the oracle: identical records and identical PCM for every frame that decodes (status OK,
CRC-failed frames zero-filled in both).  Frames k_decode_sys hands back (errors, truncation, an
MMX16 subframe leaving int16, a 64-bit shift >= 32) go through k_decode_list, the exact lane
kernel, so their records are the lane path's too.  A frame that ends TRUNC / ERROR has its range
zero-filled by k_fill_bad in both paths (include/bnflac.h), so the whole output buffer must match."""
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
    L.bnflac_debug_set_decode_sys(-1)


def _sp(libflac, data):
    if data[:4] != b"fLaC":
        return libflac.StreamParams(0, 0, 0, 0, 2, 16, 0)
    si = data[8:42]
    x = int.from_bytes(si[10:18], "big")
    return libflac.StreamParams(1, int.from_bytes(si[0:2], "big"), int.from_bytes(si[2:4], "big"), x >> 44,
                                ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1, x & ((1 << 36) - 1))


def _decode(gpu, data, offs, fmt, sys_on, sp, out_frac=None):
    """out_frac: pass only that fraction of the output buffer as out_bytes (frames past it SKIPPED)"""
    torch, libflac, dec, L = gpu
    dev = torch.device("cuda:0")
    d_bytes = torch.zeros((len(data) + 15) // 16 * 16 + 32, dtype=torch.uint8, device=dev)
    d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.tensor([int(o) for o in offs], dtype=torch.int64, device=dev)
    total = max(sp.total_samples, 1) if sp.has_stream_info else 1 << 20
    stride = libflac.out_stride(fmt, sp)
    d_out = torch.full((total * stride + 64,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(len(offs) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    L.bnflac_debug_set_decode_sys(1 if sys_on else 0)
    try:
        out_bytes = None if out_frac is None else int(total * stride * out_frac)
        dec.decode_frames(d_bytes, len(data), d_offs, len(offs), sp, fmt, d_out, d_info, out_bytes=out_bytes)
        torch.cuda.synchronize()
    finally:
        L.bnflac_debug_set_decode_sys(-1)
    return libflac.info_array(d_info.cpu().numpy()), d_out.cpu().numpy(), stride


FIELDS = ["status", "err", "frame_off", "resume_bit", "blocksize", "channels", "assignment", "bps",
          "out_sample", "crc16_calc", "crc16_read", "crc_ok"]


def _frame_range(libflac, fmt, info, i, stride):
    C = int(info["channels"][i])
    bs = int(info["blocksize"][i])
    os_ = int(info["out_sample"][i])
    if fmt == libflac.OUT_FLACDECODER:
        w = 4 if C == 2 else 2
        return os_ * w, bs * w
    if fmt == libflac.OUT_PLANAR32:  # k_fill_bad stops at the batch's channel count (stride / 4)
        return os_ * stride, bs * 4 * min(C, stride // 4)
    return os_ * stride, bs * stride


def _same(gpu, data, offs, fmt, out_frac=None):
    """lane kernels vs k_decode_sys: records, and the PCM of every frame that decodes"""
    torch, libflac, _, _ = gpu
    sp = _sp(libflac, data)
    a, oa, stride = _decode(gpu, data, offs, fmt, False, sp, out_frac)
    b, ob, _ = _decode(gpu, data, offs, fmt, True, sp, out_frac)
    for k in FIELDS:
        bad = np.nonzero(a[k] != b[k])[0]
        assert len(bad) == 0, f"{k} differs at frame {bad[0]} (offset {offs[bad[0]]}): lane {a[bad[0]]} sys {b[bad[0]]}"
    assert np.array_equal(a["flags"] & 6, b["flags"] & 6)
    n = 0
    for i in np.nonzero(a["status"] == 0)[0]:
        s0, nb = _frame_range(libflac, fmt, a, i, stride)
        assert np.array_equal(oa[s0:s0 + nb], ob[s0:s0 + nb]), f"PCM of frame {i} (offset {offs[i]}) differs"
        n += 1
    for i in np.nonzero((a["status"] == 1) | (a["status"] == 2))[0]:  # k_fill_bad: zeros, or untouched
        s0, nb = _frame_range(libflac, fmt, a, i, stride)
        if a["sub_start"][i][0] != 0 and s0 + nb <= len(oa) - 64:
            assert not oa[s0:s0 + nb].any(), f"non-OK frame {i} (offset {offs[i]}) not zero-filled"
    assert oa.tobytes() == ob.tobytes()
    return n, b


def _oracle_interleaved(data, out, nsamples, channels):
    """the batch output of a valid stream in INTERLEAVED32 equals the oracle's decode"""
    import oracle
    ev, opcm = oracle.run(data)
    pcm = out[:nsamples * 4 * channels].view("<i4").reshape(-1, channels)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm)), "differs from the oracle"


def _offsets(s):
    return [int(x) for x in s.frame_offsets]


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "roundtrip"])
def test_fixtures_identical(gpu, name):
    torch, libflac, _, _ = gpu
    data = open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read()
    n, _ = _same(gpu, data, GOLD[name]["frame_offsets"], libflac.OUT_INTERLEAVED32)
    assert n == len(GOLD[name]["frame_offsets"])
    sp = _sp(libflac, data)
    if sp.has_stream_info and sp.total_samples:
        _, out, _ = _decode(gpu, data, GOLD[name]["frame_offsets"], libflac.OUT_INTERLEAVED32, True, sp)
        _oracle_interleaved(data, out, sp.total_samples, sp.channels)


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
    _same(gpu, s.data.tobytes(), _offsets(s), fmt)
    if fmt == libflac.OUT_INTERLEAVED32:  # anchored on the oracle, not only on the lane kernels
        data = s.data.tobytes()
        _, out, _ = _decode(gpu, data, _offsets(s), fmt, True, _sp(libflac, data))
        _oracle_interleaved(data, out, s.nsamples, s.pcm.shape[1])


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4", "C5"])
def test_sys_matches_source_pcm(gpu, cfg):
    """The systolic path alone, end to end: the generator's PCM, no frame handed back."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    p = synth.config(cfg, nframes={"C4": 96, "C5": 16}.get(cfg, 40), last_blocksize=0)
    s = synth.encode(p)
    data = s.data.tobytes()
    info, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32, True, _sp(libflac, data))
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert not (info["flags"] & 512).any(), "a valid stream's frame was handed back"
    assert np.array_equal(out[:s.nsamples * 4 * p.channels].view("<i4").reshape(-1, p.channels), s.pcm)


@pytest.mark.parametrize("order,prec,stereo", [(1, 15, 0), (2, 15, 0), (3, 0, 3), (4, 12, 0), (5, 13, 1), (8, 15, 1),
                                                (8, 0, 2), (9, 14, 0), (12, 15, 3), (16, 0, 0), (17, 12, 2), (24, 15, 1),
                                                (32, 15, 3), (32, 0, 0)])
def test_lpc_restore_paths(gpu, order, prec, stereo):
    """Every libFLAC restore path (MMX16, ia32, 64-bit; prec 0 = unclamped, forcing the 64-bit
    path at high orders) and every slot count of the quad (orders 1..32): source PCM and the
    lane kernels' bytes."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    p = synth.config("C2", nframes=10, order=order, qlp_precision=prec, stereo_mode=stereo, prec_clamp=0,
                     partition_order=-1 if order > 16 else 4, seed=100 + order)
    s = synth.encode(p)
    data = s.data.tobytes()
    n, info = _same(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32)
    assert n == 10
    _, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32, True, _sp(libflac, data))
    pcm = out[:s.nsamples * 8].view("<i4").reshape(-1, 2)
    assert np.array_equal(pcm, s.pcm)
    ev, opcm = oracle.run(data)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm))


@pytest.mark.parametrize("order,stereo", [(2, 3), (4, 1), (3, 0)])
def test_fixed_24bit_side_leaves_24_bits(gpu, order, stereo):
    """FIXED subframes of 24-bit stereo (the side channel has 25 bits, its FIXED sums wrap in
    32 bits): identical to the lane kernels and the generator's PCM."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C3", nframes=6, last_blocksize=0, subframe_mode=synth.SUB_FIXED, order=order,
                                  stereo_mode=stereo, level=0.95, noise=0.3, wasted_bits_max=0, seed=40 + order))
    data = s.data.tobytes()
    assert _same(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32)[0] == 6
    _, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32, True, _sp(libflac, data))
    assert np.array_equal(out[:s.nsamples * 8].view("<i4").reshape(-1, 2), s.pcm)


@pytest.mark.parametrize("fmt_name", ["OUT_INTERLEAVED32", "OUT_PLANAR32", "OUT_FLACDECODER", "OUT_FILEREADER"])
def test_damaged_and_truncated_identical(gpu, fmt_name):
    """Byte flips (CRC failures, damaged residuals and headers) and cut streams: same records,
    same PCM for every frame that decodes, CRC-failed frames zero-filled, ERROR / TRUNC frames
    zero-filled within their own slot (k_fill_bad) in every layout."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    fmt = getattr(libflac, fmt_name)
    rng = np.random.default_rng(91)
    for i in range(16):
        cfg = ["C1", "C2", "C3", "C4", "C5"][i % 5]
        s = synth.encode(synth.config(cfg, nframes=int(rng.integers(4, 16)), last_blocksize=0, seed=300 + i))
        data = bytearray(s.data.tobytes())
        offs = _offsets(s)
        for _ in range(int(rng.integers(1, 5))):
            p = int(rng.integers(offs[0] + 4, len(data)))
            data[p] ^= int(rng.integers(1, 256))
        if i % 3 == 2:
            data = data[:len(data) * 3 // 4]
            offs = [o for o in offs if o < len(data)]
        _same(gpu, bytes(data), offs, fmt)


@pytest.mark.parametrize("cfg", ["C3", "C5"])
def test_unsupported_and_short_buffer_flags(gpu, cfg):
    """24-bit frames into the 16-bit FLACDecoder layout (unsupported, flag bit 2) with an output
    buffer cut to 60% (the later frames also end past out_bytes, bit 1): both outcome bits are
    set independently, the same on k_decode_sys and the lane kernels (decode_block)."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config(cfg, nframes=10, last_blocksize=0))
    n, b = _same(gpu, s.data.tobytes(), _offsets(s), libflac.OUT_FLACDECODER, out_frac=0.6)
    assert n == 0 and (b["status"] == 3).all()
    fl = b["flags"] & 6
    assert (fl & 4).all() and (fl == 6).any() and (fl == 4).any()


def test_crc_mismatch_zero_filled(gpu):
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C2", nframes=6))
    d = bytearray(s.data.tobytes())
    o = _offsets(s)
    d[o[2] + 100] ^= 0x40
    info, out, _ = _decode(gpu, bytes(d), o, libflac.OUT_INTERLEAVED32, True, _sp(libflac, bytes(d)))
    pcm = out[:s.nsamples * 8].view("<i4").reshape(-1, 2)
    assert info["crc_ok"].tolist() == [1, 1, 0, 1, 1, 1]
    assert not pcm[2 * 4096: 3 * 4096].any()
    assert np.array_equal(np.delete(pcm, np.s_[2 * 4096: 3 * 4096], axis=0),
                          np.delete(s.pcm, np.s_[2 * 4096: 3 * 4096], axis=0))


@pytest.mark.parametrize("stereo_mode", [0, 1, 3])
def test_mmx16_leaving_int16_handed_back(gpu, stereo_mode):
    """Loud, weakly correlated stereo: samples of MMX16-path subframes leave int16 (libFLAC's
    saturated history then differs from the exact sum); k_decode_sys hands those frames to
    k_decode_list and the bytes equal the lane kernels' and the oracle's."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    s = synth.encode(synth.config("C2", nframes=8, level=0.999, noise=0.9, stereo_mode=stereo_mode, seed=61 + stereo_mode))
    data = s.data.tobytes()
    n, info = _same(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32)
    ev, opcm = oracle.run(data)
    _, out, _ = _decode(gpu, data, _offsets(s), libflac.OUT_INTERLEAVED32, True, _sp(libflac, data))
    assert np.array_equal(out[:s.nsamples * 8].view("<i4").reshape(-1, 2), oracle.interleave(ev, opcm))


@pytest.mark.parametrize("cfg", ["C2", "C3", "C5"])
def test_full_size_batches(gpu, cfg):
    """BASELINE configs at full size (C2 1024 frames, C3 1024 frames, C5 one 469-frame file)."""
    from birdnest.audio_amd import synth
    torch, libflac, _, _ = gpu
    p = synth.config(cfg)
    s = synth.encode(p)
    data = s.data.tobytes()
    fmt = libflac.OUT_FLACDECODER if cfg == "C2" else libflac.OUT_FILEREADER
    info, out, stride = _decode(gpu, data, _offsets(s), fmt, True, _sp(libflac, data))
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert not (info["flags"] & 512).any()
    if cfg == "C2":
        ref = s.pcm.astype("<i2").tobytes()
    else:
        ref = np.ascontiguousarray(s.pcm.astype("<i4")).view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    assert out[:len(ref)].tobytes() == ref
