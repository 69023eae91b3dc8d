"""k_decode_sw: one lane per stereo frame above 16 bits (C3's fast path).

Every case decodes the same batch twice, with k_decode_sw (default) and without it
(BNFLAC_ABLATE bit 0x10000: k_decode<16> alone), and requires identical output bytes and
identical frame records, plus the generator's source PCM for intact streams (the lossless
round trip).  Cases cover the stereo assignments, 20- and 24-bit streams, wasted bits, LPC
orders 1..12 on the 64-bit and the 32-bit restore paths, partition orders, escaped
partitions, RICE2, blocksizes that are not a multiple of the 32-sample chunk, variable
blocksizes, and damaged frames (CRC mismatch -> hand-back -> zero fill).
"""
import numpy as np
import pytest

from tests.test_gpu_parity import _decode_batch, gpu  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu

FL_REDO = 64
FL_SW = 1024
NO_SW = 0x10000


def _both(gpu, data, offsets, fmt):
    torch, libflac, dec = gpu
    out_a, info_a, sp = _decode_batch(gpu, data, offsets, fmt)
    dec.L.bnflac_debug_set_ablate(NO_SW)
    try:
        out_b, info_b, _ = _decode_batch(gpu, data, offsets, fmt)
    finally:
        dec.L.bnflac_debug_set_ablate(0)
    keep = [n for n in info_a.dtype.names if n != "flags"]
    for n in keep:
        assert np.array_equal(info_a[n], info_b[n]), n
    # the whole output: OK frames' PCM (CRC mismatches zero-filled), non-OK frames whose header
    # parsed zero-filled by k_fill_bad, the rest untouched (include/bnflac.h)
    assert out_a.tobytes() == out_b.tobytes()
    return out_a, info_a, sp


def _expect(libflac, fmt, pcm, info, bps):
    if fmt == libflac.OUT_INTERLEAVED32:
        return pcm.astype("<i4").tobytes()
    if fmt == libflac.OUT_PLANAR32:
        parts = []
        for fr in range(len(info)):
            bs, st = int(info["blocksize"][fr]), int(info["out_sample"][fr])
            parts.append(np.ascontiguousarray(pcm[st: st + bs].T).astype("<i4").tobytes())
        return b"".join(parts)
    v = pcm.astype(np.int64).reshape(-1)
    if bps == 24:
        b = np.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], axis=1).astype(np.uint8)
        return b.tobytes()
    return (v & 0xFFFF).astype("<u2").tobytes()


FMTS = ["OUT_FILEREADER", "OUT_INTERLEAVED32", "OUT_PLANAR32"]

CASES = {
    "c3": dict(),
    "indep": dict(stereo_mode=0),
    "left_side": dict(stereo_mode=1),
    "right_side": dict(stereo_mode=2),
    "cycle": dict(stereo_mode=4, wasted_bits_max=2),
    "order1": dict(order=1),
    "order5": dict(order=5, partition_order=4),
    "order12_po8": dict(partition_order=8, blocksize=4096),
    "narrow_path": dict(qlp_precision=3, order=4),
    "tail_1000": dict(last_blocksize=1000),
    "odd_bs": dict(blocksize=4100, last_blocksize=0, partition_order=0),
    "escape": dict(escape_permille=150, partition_order=3),
    "rice2": dict(rice2=1, partition_order=2),
    "bps20": dict(bps=20),
    "varbs": dict(variable_blocksize=1, bs_min=192, bs_max=8192, partition_order=-1),
}


@pytest.mark.parametrize("fmt_name", FMTS)
@pytest.mark.parametrize("case", sorted(CASES))
def test_sw_matches_handback_and_source(gpu, case, fmt_name):
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    fmt = getattr(libflac, fmt_name)
    kw = dict(nframes=24, last_blocksize=0)
    kw.update(CASES[case])
    p = synth.config("C3", **kw)
    if fmt == libflac.OUT_FILEREADER and p.bps != 24:
        pytest.skip("FLACFileReader packs 16 or 24 bits only")
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _both(gpu, data, s.frame_offsets, fmt)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert out.tobytes() == _expect(libflac, fmt, s.pcm, info, p.bps)
    if case in ("c3", "indep", "left_side", "right_side", "cycle", "order5", "order12_po8", "bps20"):
        # regular LPC streams: k_decode_sw decodes every frame itself
        assert (info["flags"] & FL_SW).all(), info["flags"]
        assert not (info["flags"] & FL_REDO).any(), info["flags"]


def test_sw_c3_full_frames_no_handback(gpu):
    """A C3 batch at its own frame shape (8192-sample M/S LPC-12 frames with wasted bits):
    all frames are k_decode_sw's and none is handed back."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C3", nframes=130)
    s = synth.encode(p)
    out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, libflac.OUT_FILEREADER)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_SW).all() and not (info["flags"] & FL_REDO).any()
    assert out.tobytes() == _expect(libflac, libflac.OUT_FILEREADER, s.pcm, info, 24)


@pytest.mark.parametrize("seed", [11, 12])
def test_sw_damaged_frames(gpu, seed):
    """Flipped bytes inside some frames: the CRC-16 mismatch (or a parse error) hands the
    frame back; the record and the output (zero fill on a CRC mismatch) equal the path
    without k_decode_sw, and the intact frames still decode to the source PCM."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C3", nframes=20, last_blocksize=0, blocksize=4096)
    s = synth.encode(p)
    data = bytearray(s.data.tobytes())
    rng = np.random.default_rng(seed)
    offs = [int(o) for o in s.frame_offsets]
    bad = sorted(rng.choice(np.arange(1, 19), size=5, replace=False).tolist())
    for fr in bad:
        a, b = offs[fr] + 40, offs[fr + 1] - 8
        for pos in rng.integers(a, b, size=2):
            data[int(pos)] ^= 0x5A
    for fmt in (libflac.OUT_INTERLEAVED32, libflac.OUT_FILEREADER):
        out, info, sp = _both(gpu, bytes(data), s.frame_offsets, fmt)
        good = [fr for fr in range(p.nframes) if fr not in bad]
        assert (info["crc_ok"][good] == 1).all()
        assert not (info["crc_ok"][bad] == 1).all()
        if fmt == libflac.OUT_INTERLEAVED32:
            got = out.view("<i4").reshape(-1, 2)
            for fr in good:
                st, bs = int(info["out_sample"][fr]), int(info["blocksize"][fr])
                assert np.array_equal(got[st: st + bs], s.pcm[st: st + bs])
