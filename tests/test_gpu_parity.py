"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and golden vectors.

Bar: bit-exact PCM, identical libFLAC callback sequences, identical C#-surface bytes and
exception messages.  Full-size configs are checked through the lossless round trip
(decoded PCM == generator source PCM, CRC-16 ok on every frame).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(GOLD_DIR, "golden.json")))


def _read(name):
    return open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read()


def _sha(pcm):
    return hashlib.sha256(np.ascontiguousarray(pcm, dtype="<i4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from birdnest.audio_amd import libflac
    return torch, libflac, libflac.BatchDecoder(0)


@pytest.fixture
def decode_mode(request, gpu):
    """The decode kernels for one test: 0 the lane kernels (k_decode_st / k_decode_sw /
    k_decode<W>), 2 k_decode_sys (systolic restore, every frame class; its hand-backs through
    k_decode_list).  Auto (-1) afterwards."""
    torch, libflac, _ = gpu
    L = libflac.load()
    L.bnflac_debug_set_decode_sys(1 if request.param == 2 else 0)
    yield request.param
    L.bnflac_debug_set_decode_sys(-1)


LANE = pytest.mark.parametrize("decode_mode", [0], indirect=True)  # tests of the lane kernels' own paths


def _stream_params(libflac, data: bytes):
    """STREAMINFO -> StreamParams (host parse of the 34-byte block, like MetadataCallback)."""
    si = data[8:42]
    minbs = int.from_bytes(si[0:2], "big")
    maxbs = int.from_bytes(si[2:4], "big")
    x = int.from_bytes(si[10:18], "big")
    sr = x >> 44
    ch = ((x >> 41) & 7) + 1
    bps = ((x >> 36) & 31) + 1
    total = x & ((1 << 36) - 1)
    return libflac.StreamParams(1, minbs, maxbs, sr, ch, bps, total)


def _decode_batch(gpu, data: bytes, offsets, fmt, out_sample=None):
    torch, libflac, dec = gpu
    sp = _stream_params(libflac, data)
    dev = torch.device("cuda:0")
    n = len(data)
    d_bytes = torch.zeros((n + 3) // 4 * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    offs = torch.tensor([int(o) for o in offsets], dtype=torch.int64, device=dev)
    nf = len(offsets)
    total = sp.total_samples
    stride = libflac.out_stride(fmt, sp)
    d_out = torch.full((total * stride + 64,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    d_os = None
    if out_sample is not None:
        d_os = torch.tensor(out_sample, dtype=torch.int64, device=dev)
    dec.decode_frames(d_bytes, n, offs, nf, sp, fmt, d_out, d_info, d_out_sample=d_os)
    torch.cuda.synchronize()
    info = libflac.info_array(d_info.cpu().numpy())
    return d_out.cpu().numpy()[: total * stride], info, sp


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "roundtrip"])
def test_batch_roundtrip_interleaved32(gpu, name):
    torch, libflac, _ = gpu
    g = GOLD[name]
    data = _read(name)
    out, info, sp = _decode_batch(gpu, data, g["frame_offsets"], libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all(), info[["status", "err"]]
    assert (info["crc_ok"] == 1).all()
    pcm = out.view("<i4").reshape(-1, sp.channels)
    assert _sha(pcm) == g["pcm_sha256"]


def test_rfc9639_example1_gpu(gpu):
    torch, libflac, _ = gpu
    data = _read("rfc9639_ex1")
    out, info, sp = _decode_batch(gpu, data, [data.index(b"\xff\xf8")], libflac.OUT_INTERLEAVED32)
    assert info["crc_ok"][0] == 1
    assert out.view("<i4").reshape(-1, 2).tolist() == GOLD["rfc9639_ex1"]["pcm"]


def test_rfc9639_example2_frame1_gpu(gpu):
    torch, libflac, dec = gpu
    g = GOLD["rfc9639_ex2_frame1"]
    fr = _read("rfc9639_ex2_frame1")
    data = b"fLaC" + b"\x80\x00\x00\x22" + bytes.fromhex("00100010000017000044") + \
        bytes.fromhex("0ac442f000000013") + bytes(16) + fr
    out, info, sp = _decode_batch(gpu, data, [42], libflac.OUT_PLANAR32)
    assert info["crc_ok"][0] == 1 and info["blocksize"][0] == 16 and info["assignment"][0] == 2
    pcm = out.view("<i4")[:32].reshape(2, 16).T
    assert _sha(pcm) == g["pcm_sha256_oracle"]


@pytest.mark.parametrize("decode_mode", [0, 2], indirect=True)
@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4", "C5"])
def test_config_batch_vs_oracle_and_source(gpu, cfg, decode_mode):
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config(cfg, nframes={"C4": 64}.get(cfg, 12), last_blocksize=0)
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    pcm = out.view("<i4").reshape(-1, p.channels)
    assert np.array_equal(pcm, s.pcm)
    ev, opcm = oracle.run(data)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm))


_C4_FULL = {}


def _c4_full():
    """BASELINE C4 at its full shape: 4,096 frames, variable blocksize 192-16,384, CONSTANT /
    VERBATIM / FIXED / LPC up to order 32 (the generator takes ~15 s: encoded once per module)."""
    if not _C4_FULL:
        from birdnest.audio_amd import synth
        p = synth.config("C4")
        assert p.nframes == 4096 and p.bs_max == 16384
        _C4_FULL["s"] = synth.encode(p)
    return _C4_FULL["s"]


@pytest.mark.parametrize("fmt_name", ["FLACDECODER", "INTERLEAVED32"])
def test_c4_full_size_vs_source(gpu, fmt_name):
    """C4 as the bench decodes it (default dispatch: k_decode_st, k_decode<8|16|32> by class,
    the W16/W32 side grids), at full size: every record OK with a checked CRC-16, and the PCM
    equal to the generator's source, including the 16,384-sample LPC-32 frames at the long tail
    of the decode order."""
    torch, libflac, _ = gpu
    s = _c4_full()
    data = s.data.tobytes()
    assert int(np.diff(np.asarray(s.frame_offsets)).max()) > 0
    fmt = getattr(libflac, "OUT_" + fmt_name)
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, fmt)
    assert len(info) == 4096
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert int(info["blocksize"].max()) == 16384 and int(info["blocksize"].min()) <= 256
    if fmt_name == "FLACDECODER":
        assert out.tobytes() == s.pcm.astype("<i2").tobytes()
    else:
        assert np.array_equal(out.view("<i4").reshape(-1, 2), s.pcm)


@pytest.mark.parametrize("order,prec,stereo", [(2, 15, 0), (3, 0, 3), (4, 12, 0), (8, 15, 1), (8, 0, 2),
                                                (12, 15, 3), (16, 0, 0), (32, 15, 3), (32, 0, 0)])
@pytest.mark.parametrize("decode_mode", [0, 2], indirect=True)
def test_lpc_restore_paths_16bit(gpu, order, prec, stereo, decode_mode):
    """Every libFLAC restore path on 16-bit input (MMX for order >= 4 at <= 32 bits, ia32
    for low orders, the 64-bit path when bps + precision + log2(order) > 32 -- no encoder
    precision clamp here), in both k_decode instances (orders <= 8 and above)."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C2", nframes=10, order=order, qlp_precision=prec, stereo_mode=stereo, prec_clamp=0,
                     partition_order=-1 if order > 16 else 4, seed=100 + order)
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    pcm = out.view("<i4").reshape(-1, 2)
    assert np.array_equal(pcm, s.pcm)
    ev, opcm = oracle.run(data)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm))


def test_flacdecoder_format_vs_oracle(gpu):
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    for cfg, kw in (("C1", {}), ("C2", {}), ("C4", {"nframes": 40}), ("C2", {"channels": 1, "seed": 9})):
        p = synth.config(cfg, **({"nframes": 10, "last_blocksize": 0} | kw))
        s = synth.encode(p)
        data = s.data.tobytes()
        out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_FLACDECODER)
        rc, ref, msg, _ = oracle.flacdecoder_copyto(data)
        assert rc == 0, msg
        assert out.tobytes() == ref, cfg


def test_filereader_format_24bit_vs_oracle(gpu):
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    for cfg in ("C3", "C5"):
        p = synth.config(cfg, nframes=4, last_blocksize=0)
        s = synth.encode(p)
        data = s.data.tobytes()
        out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_FILEREADER)
        rc, ref, msg = oracle.filereader_readall(data, buf_len=p.blocksize * p.channels * 3)
        assert rc == 0, msg
        assert out.tobytes() == ref, cfg


def test_index_frames_matches_numpy_scan(gpu):
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config("C2", nframes=64))
    data = s.data.tobytes()
    arr = np.frombuffer(data, dtype=np.uint8)
    ref = np.nonzero((arr[:-1] == 0xFF) & ((arr[1:] >> 2) == 0x3E))[0]
    assert set(int(x) for x in s.frame_offsets) <= set(int(x) for x in ref)
    dev = torch.device("cuda:0")
    n = len(data)
    d_bytes = torch.zeros((n + 3) // 4 * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.from_numpy(arr.copy()).to(dev)
    d_off = torch.zeros(len(ref) + 16, dtype=torch.int64, device=dev)
    d_cnt = torch.zeros(4, dtype=torch.int32, device=dev)
    dec.index_frames(d_bytes, n, d_off, d_cnt)
    torch.cuda.synchronize()
    cnt = int(d_cnt[0].item())
    assert cnt == len(ref)
    assert np.array_equal(d_off[:cnt].cpu().numpy(), ref)


def test_full_c2_batch_lossless(gpu):
    """BASELINE config C2 at full size: 1024 frames x 4096 x 2ch, LPC-8, RPO 4."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C2")
    s = synth.encode(p)
    out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, libflac.OUT_FLACDECODER)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert out.tobytes() == s.pcm.astype("<i2").tobytes()


def test_crc_mismatch_zero_filled_in_batch(gpu):
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C2", nframes=6))
    d = bytearray(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    d[o[2] + 100] ^= 0x40
    out, info, sp = _decode_batch(gpu, bytes(d), o, libflac.OUT_INTERLEAVED32)
    pcm = out.view("<i4").reshape(-1, 2)
    assert info["crc_ok"].tolist() == [1, 1, 0, 1, 1, 1]
    assert not pcm[2 * 4096: 3 * 4096].any()
    assert np.array_equal(np.delete(pcm, np.s_[2 * 4096: 3 * 4096], axis=0),
                          np.delete(s.pcm, np.s_[2 * 4096: 3 * 4096], axis=0))


def test_crc_mismatch_and_junk_gap(gpu):
    """A CRC-corrupted frame, junk bytes between two frames (the footer no longer ends at the
    next offset) and the last frame of the batch: every CRC-16 is checked by the decode
    kernels, the corrupted frame alone fails it and is zero-filled."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    for cfg in ("C2", "C3", "C4"):
        s = synth.encode(synth.config(cfg, nframes=8, last_blocksize=0))
        d = bytearray(s.data.tobytes())
        o = [int(x) for x in s.frame_offsets]
        d[o[2] + 100] ^= 0x40                       # frame 2: CRC mismatch
        junk = bytes([0x5A, 0x00, 0x13] * 7)         # 21 bytes of junk between frames 5 and 6
        d = d[: o[6]] + junk + d[o[6]:]
        o = o[:6] + [x + len(junk) for x in o[6:]]
        out, info, sp = _decode_batch(gpu, bytes(d), o, libflac.OUT_INTERLEAVED32)
        assert info["crc_ok"].tolist() == [1, 1, 0, 1, 1, 1, 1, 1], cfg
        assert (info["status"] == 0).all(), cfg
        pcm = out.view("<i4").reshape(-1, s.pcm.shape[1])
        bs = s.params.blocksize if not s.params.variable_blocksize else None
        if bs:
            assert not pcm[2 * bs: 3 * bs].any(), cfg
            assert np.array_equal(np.delete(pcm, np.s_[2 * bs: 3 * bs], axis=0),
                                  np.delete(s.pcm, np.s_[2 * bs: 3 * bs], axis=0)), cfg


@pytest.fixture
def crc_mode(request, gpu):
    """Who computes the CRC-16 hand-off for one test (bnflac_debug_set_crc_mode), with the
    lane-per-frame k_parse forced (small batches otherwise take k_parse_wave, which hands
    nothing over); the defaults after."""
    torch, libflac, _ = gpu
    L = libflac.load()
    L.bnflac_debug_set_crc_mode(request.param)
    L.bnflac_debug_set_parse_wave(0)
    yield request.param
    L.bnflac_debug_set_parse_wave(-1)
    L.bnflac_debug_set_crc_mode(-1)


@LANE
@pytest.mark.parametrize("crc_mode", [0, 1, 2], indirect=True)
@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_crc_handoff_paths(gpu, cfg, decode_mode, crc_mode):
    """k_parse's CRC-16 hand-off to the stereo decode tails (include/bnflac.h), on each of its
    paths, with damage past the part k_parse folds while walking channel 0: a frame that ends
    at the next frame's offset (k_parse's verdict), one followed by junk and the batch's last
    frame (its prefix continued by the tail).  A second decode of the same parsed records has
    no hand-off (the whole frame again) and must give the same records and PCM."""
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config(cfg, nframes=8, last_blocksize=0))
    d = bytearray(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    ends = o[1:] + [len(d)]
    d[ends[3] - 1] ^= 0x01                       # frame 3: its footer (verdict path)
    d[ends[5] - 40] ^= 0x08                      # frame 5: channel 1's bytes, junk after it
    d[ends[7] - 40] ^= 0x08                      # frame 7, the last: channel 1's bytes
    junk = bytes([0x5A, 0x00, 0x13] * 7)
    d = d[: o[6]] + junk + d[o[6]:]
    o = o[:6] + [x + len(junk) for x in o[6:]]
    fmt = libflac.OUT_INTERLEAVED32
    sp = _stream_params(libflac, bytes(d))
    dev = torch.device("cuda:0")
    n = len(d)
    d_bytes = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev)
    offs = torch.tensor(o, dtype=torch.int64, device=dev)
    stride = libflac.out_stride(fmt, sp)
    outs, infos = [], []
    d_info = torch.zeros(len(o) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec.parse_frames(d_bytes, n, offs, len(o), sp, d_info)
    parsed = d_info.clone()
    for _ in range(2):
        d_info.copy_(parsed)
        d_out = torch.full((sp.total_samples * stride + 64,), 0xAB, dtype=torch.uint8, device=dev)
        dec.decode_parsed(d_bytes, n, len(o), sp, fmt, d_out, d_info)
        torch.cuda.synchronize()
        outs.append(d_out[: sp.total_samples * stride].cpu().numpy())
        infos.append(libflac.info_array(d_info.cpu().numpy()))
    for info in infos:
        good = (info["status"] == 0) & (info["crc_ok"] == 1)
        assert good.tolist() == [True, True, True, False, True, False, True, False], cfg
        assert info["crc_ok"][3] == 0 and info["status"][3] == 0, cfg
    assert np.array_equal(outs[0], outs[1]), cfg
    assert np.array_equal(infos[0], infos[1]), cfg
    pcm = outs[0].view("<i4").reshape(-1, s.pcm.shape[1])
    bs = s.params.blocksize
    keep = np.ones(len(pcm), bool)
    for f in (3, 5, 7):
        keep[f * bs:(f + 1) * bs] = False
        if infos[0]["status"][f] == 0:
            assert not pcm[f * bs:(f + 1) * bs].any(), (cfg, f)
    assert np.array_equal(pcm[keep], s.pcm[keep]), cfg


@LANE
@pytest.mark.parametrize("crc_mode", [1], indirect=True)
def test_crc_handoff_contract(gpu, decode_mode, crc_mode):
    """The hand-off's contract (include/bnflac.h): it belongs to the context's last
    bnflac_parse_frames batch and the next decode takes it (used or not: a decode of other
    records gets none and checks whole frames); bnflac_index_stream drops it.  Every path
    decodes the same records."""
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config("C2", nframes=12, last_blocksize=0, seed=17))
    d = bytes(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    fmt = libflac.OUT_FLACDECODER
    sp = _stream_params(libflac, d)
    dev = torch.device("cuda:0")
    n = len(d)
    d_bytes = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev)
    offs = torch.tensor(o, dtype=torch.int64, device=dev)
    nf = len(o)
    stride = libflac.out_stride(fmt, sp)
    want = s.pcm.astype("<i2").tobytes()

    def decode(d_info):
        d_out = torch.zeros(sp.total_samples * stride, dtype=torch.uint8, device=dev)
        dec.decode_parsed(d_bytes, n, nf, sp, fmt, d_out, d_info)
        torch.cuda.synchronize()
        info = libflac.info_array(d_info.cpu().numpy())
        assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
        assert d_out.cpu().numpy().tobytes() == want
        return info

    d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec.parse_frames(d_bytes, n, offs, nf, sp, d_info)
    h = dec.crc_handoff(nf)
    assert (h[:, 2] != 0).sum() >= nf - 1          # prefixes were handed over
    ref = decode(d_info)                              # ... and used
    with pytest.raises(RuntimeError):                 # used once
        dec.crc_handoff(nf)
    # another records buffer than the parse wrote: no hand-off, same result, and the pending
    # one is gone
    dec.parse_frames(d_bytes, n, offs, nf, sp, d_info)
    other = d_info.clone()
    assert np.array_equal(decode(other), ref)
    with pytest.raises(RuntimeError):
        dec.crc_handoff(nf)
    # bnflac_index_stream on the context drops it
    dec.parse_frames(d_bytes, n, offs, nf, sp, d_info)
    dec.crc_handoff(nf)
    dec.index_stream(d_bytes, n, o[0], sp, nf + 16)
    with pytest.raises(RuntimeError):
        dec.crc_handoff(nf)
    assert np.array_equal(decode(d_info), ref)


_T15 = (1 << 15) | 3  # T = x^15 + x + 1: P = (x + 1) T (the tails' zero test, bnflac_kernels.hip)


def _gf2_mod(a: int, m: int) -> int:
    dm = m.bit_length() - 1
    while a and a.bit_length() - 1 >= dm:
        a ^= m << (a.bit_length() - 1 - dm)
    return a


@pytest.mark.parametrize("crc_mode", [1, 2], indirect=True)
def test_crc_handoff_against_oracle(gpu, crc_mode):
    """The hand-off itself (bnflac_debug_crc_handoff) against the oracle: each prefix holds the
    remainder mod T and the parity of the frame's whole lines before channel 1, and each
    verdict (mode 2) is the zero test of the CRC-16 over [offset, next offset) (frame + footer,
    or + junk)."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config("C2", nframes=10, last_blocksize=0, seed=13))
    d = bytearray(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    d[o[2] + 100] ^= 0x40
    d[o[4 + 1] - 30] ^= 0x02
    junk = bytes([0x77, 0x01] * 9)
    d = d[: o[7]] + junk + d[o[7]:]
    o = o[:7] + [x + len(junk) for x in o[7:]]
    d = bytes(d)
    sp = _stream_params(libflac, d)
    dev = torch.device("cuda:0")
    n = len(d)
    d_bytes = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).to(dev)
    nf = len(o)
    d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec.parse_frames(d_bytes, n, torch.tensor(o, dtype=torch.int64, device=dev), nf, sp, d_info)
    h = dec.crc_handoff(nf).astype(np.int64)
    spans = prefixes = 0
    for f in range(nf):
        if h[f, 4]:
            assert crc_mode == 2, f
            nx = o[f + 1]
            assert h[f, 4] == nx - o[f] and h[f, 6] == o[f] & 0xFFFFFFFF, f
            assert h[f, 5] == int(oracle.crc16(d[o[f]:nx]) == 0), f
            spans += 1
        if h[f, 2]:
            assert h[f, 3] == o[f] & 0xFFFFFFFF, f
            end = ((o[f] >> 6) + int(h[f, 2]) - 1) * 64
            m = int.from_bytes(d[o[f]:end], "big")
            r = ((int(h[f, 1]) & 0x0FFFFFFF) << 32) | int(h[f, 0])
            assert _gf2_mod(r, _T15) == _gf2_mod(m, _T15), f
            assert (int(h[f, 1]) >> 31) == bin(m).count("1") & 1, f
            prefixes += 1
    assert h[nf - 1, 4] == 0                    # the last frame: no next offset
    # frame 2's damage may end k_parse's walk early (no hand-off for it)
    assert prefixes >= nf - 1
    if crc_mode == 2:
        assert spans >= nf - 2 and h[2, 5] == 0
        assert h[4, 4] and h[4, 5] == 0 and h[6, 4] and h[6, 5] == 0 and h[0, 4] and h[0, 5] == 1


# ---------------------------------------------------------- libFLAC API parity
STREAM_CASES =[k for k, v in GOLD.items() if v["kind"] in ("roundtrip", "error", "rfc")]


@pytest.mark.parametrize("name", STREAM_CASES)
def test_stream_api_event_parity(gpu, name):
    import oracle
    from birdnest.audio_amd import harness
    data = _read(name)
    for driver in (0, 1):
        ev, pcm = harness.run(data, driver=driver)
        oev, opcm = oracle.run(data, driver=driver)
        assert ev == harness.oracle_events_as_tuples(oev), (name, driver)
        assert np.array_equal(pcm, opcm), (name, driver)


def test_stream_api_write_abort_state(gpu):
    import oracle
    from birdnest.audio_amd import harness
    data = _read("c2_lpc8")
    ev, _ = harness.run(data, write_abort_at=2)
    oev, _ = oracle.run(data, write_abort_at=2)
    assert ev == harness.oracle_events_as_tuples(oev)
    assert ev[-1][1:3] == (0, 3)  # process_single false, state READ_FRAME


@pytest.mark.parametrize("name", STREAM_CASES)
def test_flacdecoder_mirror_vs_oracle_replay(gpu, name):
    import oracle
    from birdnest.audio_amd import flac_decoder
    data = _read(name)
    rc, pk, msg, fmt = flac_decoder.copy_to_bytes(data)
    orc, opk, omsg, ofmt = oracle.flacdecoder_copyto(data)
    assert (rc, msg) == (orc, omsg)
    assert pk == opk
    if rc == 0:
        assert fmt == ofmt[:4]


def test_stream_api_large_c2_windows(gpu):
    """Multi-window read-ahead (small windows force re-decode at window ends)."""
    import oracle
    from birdnest.audio_amd import harness, synth
    s = synth.encode(synth.config("C2", nframes=96))
    os.environ["BNFLAC_READ_AHEAD_MB"] = "1"
    try:
        ev, pcm = harness.run(s.data.tobytes(), driver=1, read_chunk=16384)
    finally:
        del os.environ["BNFLAC_READ_AHEAD_MB"]
    oev, opcm = oracle.run(s.data.tobytes(), driver=1)
    assert ev == harness.oracle_events_as_tuples(oev)
    assert np.array_equal(pcm, opcm)


# ---------------------------------------------- frame chain indexer
def _first_frame_offset(data: bytes) -> int:
    """Byte after the last metadata block (what read_metadata_ leaves the reader at)."""
    assert data[:4] == b"fLaC"
    p = 4
    while True:
        hdr = data[p]
        p += 4 + int.from_bytes(data[p + 1:p + 4], "big")
        if hdr & 0x80:
            return p


def _crc16(b: bytes) -> int:
    c = 0
    for x in b:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _index(gpu, data: bytes, sp=None, first=None, cap=None):
    torch, libflac, dec = gpu
    sp = sp or _stream_params(libflac, data)
    n = len(data)
    d_bytes = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device="cuda:0")
    d_bytes[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")
    first = _first_frame_offset(data) if first is None else first
    cap = cap or (n // 16 + 16)
    offs, os_, info, nf = dec.index_stream(d_bytes, n, first, sp, cap)
    return d_bytes, sp, offs, os_, info, nf


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "roundtrip"])
def test_index_stream_golden(gpu, name):
    """Chain == the generator's frame offsets; the records it returns decode bit-exactly."""
    torch, libflac, dec = gpu
    g = GOLD[name]
    data = _read(name)
    d_bytes, sp, offs, os_, info, nf = _index(gpu, data)
    assert nf == len(g["frame_offsets"])
    assert offs[:nf].cpu().tolist() == list(g["frame_offsets"])
    rec = libflac.info_array(info[: nf * libflac.FRAME_INFO_BYTES].cpu().numpy())
    bs = rec["blocksize"].astype(np.int64)
    assert os_[:nf].cpu().tolist() == np.concatenate([[0], np.cumsum(bs)[:-1]]).tolist()
    assert int(bs.sum()) == sp.total_samples
    d_out = torch.zeros(sp.total_samples * sp.channels * 4 + 64, dtype=torch.uint8, device="cuda:0")
    dec.decode_parsed(d_bytes, len(data), nf, sp, libflac.OUT_INTERLEAVED32, d_out, info)
    torch.cuda.synchronize()
    pcm = d_out[: sp.total_samples * sp.channels * 4].cpu().numpy().view("<i4").reshape(-1, sp.channels)
    assert _sha(pcm) == g["pcm_sha256"]


@pytest.mark.parametrize("cfg,kw", [("C2", {}), ("C4", {"nframes": 600}), ("C5", {"nframes": 40}),
                                    ("C3", {"nframes": 64})])
def test_index_stream_synth_configs(gpu, cfg, kw):
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config(cfg, **kw))
    data = s.data.tobytes()
    d_bytes, sp, offs, os_, info, nf = _index(gpu, data)
    assert nf == len(s.frame_offsets)
    assert np.array_equal(offs[:nf].cpu().numpy(), s.frame_offsets.astype(np.int64))
    # trailing junk (an ID3v1-style tag holding a sync code) changes nothing
    tail = b"TAG" + b"\xff\xf8\xc9\x18" + bytes(range(121))
    _, _, offs2, _, _, nf2 = _index(gpu, data + tail)
    assert nf2 == nf and torch.equal(offs2[:nf], offs[:nf])


def test_index_stream_eos_rule_and_head(gpu):
    torch, libflac, dec = gpu
    g = GOLD["c4_mixed_varbs"]
    data = _read("c4_mixed_varbs")
    sp = _stream_params(libflac, data)
    # STREAMINFO total_samples ending inside frame k: frames from k+1 on are past the end
    _, _, offs, os_, info, nf = _index(gpu, data)
    os_ = os_[:nf].cpu().numpy()
    k = nf // 2
    sp2 = libflac.StreamParams(1, sp.min_blocksize, sp.max_blocksize, sp.sample_rate, sp.channels, sp.bps,
                               int(os_[k]) + 1)
    _, _, _, _, _, nf2 = _index(gpu, data, sp=sp2)
    assert nf2 == k + 1
    # a first_offset inside frame 0 starts the chain at the next frame
    _, _, offs3, _, _, nf3 = _index(gpu, data, first=g["frame_offsets"][0] + 1)
    assert nf3 == nf - 1 and offs3[0].item() == g["frame_offsets"][1]


def test_index_stream_stops_at_damage(gpu):
    """A frame whose bytes fail CRC-16 has no successor: the chain ends with it."""
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config("C2", nframes=12))
    d = bytearray(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    d[o[6] - 10] ^= 0x10  # inside the last subframe: the header and the k_parse walk stay valid
    assert _crc16(bytes(d[o[5]:o[6]])) != 0
    _, _, offs, _, _, nf = _index(gpu, bytes(d))
    assert nf == 6 and offs[:nf].cpu().tolist() == o[:6]


# ------------------------------------------------ MD5 verification
MD5_CASES = [k for k, v in GOLD.items() if v["kind"] in ("roundtrip", "rfc")]


@pytest.mark.parametrize("name", MD5_CASES)
def test_md5_checking_passes_on_golden(gpu, name):
    """set_md5_checking(true): finish() is true when the decoded PCM hashes to STREAMINFO's
    md5sum (rfc9639_ex1's sum is the RFC's own), and checking changes no callback."""
    from birdnest.audio_amd import harness
    data = _read(name)
    assert data[26:42].hex() == GOLD[name]["md5"]
    ev, pcm = harness.run(data, driver=1)
    ev2, pcm2, ok = harness.run(data, driver=1, md5_check=True)
    assert ok is True
    assert ev2 == ev and np.array_equal(pcm2, pcm)


def test_md5_checking_detects_mismatch(gpu):
    from birdnest.audio_amd import harness
    data = bytearray(_read("c3_lpc12_ms_wasted"))
    data[30] ^= 0x01  # STREAMINFO md5sum byte 4
    ev, pcm, ok = harness.run(bytes(data), driver=0, md5_check=True)
    assert ok is False
    # checking off (the default): finish is true whatever the sum says
    d = bytearray(data)
    ev_off, _ = harness.run(bytes(d), driver=0)
    assert ev_off == ev
    data[26:42] = bytes(16)  # all-zero sum: nothing to check
    assert harness.run(bytes(data), driver=0, md5_check=True)[2] is True


def test_md5_checking_hashes_zeroed_crc_frames(gpu):
    """A CRC-16 mismatch frame is written as silence and hashed as such (libFLAC), so the
    stream's true sum no longer matches."""
    from birdnest.audio_amd import harness
    data = _read("err_crc16_mismatch")
    ev, pcm, ok = harness.run(data, driver=1, md5_check=True)
    assert any(e[0] == harness.EV_ERROR for e in ev)
    si_md5 = data[26:42]
    if si_md5 != bytes(16):
        assert ok is False


def test_md5_checking_off_after_seek(gpu, tmp_path):
    """seek_absolute turns MD5 checking off: a wrong sum no longer fails finish()."""
    import ctypes
    torch, libflac, _ = gpu
    L = libflac.load()
    data = bytearray(_read("c2_lpc8"))
    data[26] ^= 0xFF
    path = tmp_path / "bad_md5.flac"
    path.write_bytes(bytes(data))
    wr = libflac.DecoderWriteCallbackWithStatus(lambda *a: 0)
    er = libflac.Decoder_ErrorCallback(lambda *a: None)
    md = libflac.Decoder_MetadataCallback()
    for seek in (False, True):
        d = L.FLAC__stream_decoder_new()
        assert L.FLAC__stream_decoder_set_md5_checking(d, 1)
        assert L.FLAC__stream_decoder_init_file(d, str(path).encode(), wr, md, er, None) == 0
        assert not L.FLAC__stream_decoder_set_md5_checking(d, 0)  # refused once initialised
        assert L.FLAC__stream_decoder_process_until_end_of_metadata(d)
        if seek:
            assert L.FLAC__stream_decoder_seek_absolute(d, ctypes.c_uint64(5000))
        assert L.FLAC__stream_decoder_process_until_end_of_stream(d)
        assert bool(L.FLAC__stream_decoder_finish(d)) is seek
        assert L.FLAC__stream_decoder_get_md5_checking(d) == 0  # finish restores defaults
        L.FLAC__stream_decoder_delete(d)


def test_md5_helper_on_batch_output(gpu):
    """Batch path: interleaved32 output hashed by bnflac_md5_interleaved32 == STREAMINFO sum."""
    torch, libflac, _ = gpu
    for name in ("c2_lpc8", "c5_lpc32_8ch", "mono_8bit_fixed"):
        data = _read(name)
        out, info, sp = _decode_batch(gpu, data, GOLD[name]["frame_offsets"], libflac.OUT_INTERLEAVED32)
        assert libflac.md5_interleaved32(out.view("<i4"), sp.channels, sp.bps) == data[26:42], name


# ------------------------------------------------ stereo fast path (k_decode_st)
FL_ST, FL_REDO = 32, 64


@pytest.mark.parametrize("fmt_name", ["OUT_FLACDECODER", "OUT_INTERLEAVED32", "OUT_PLANAR32", "OUT_FILEREADER"])
@pytest.mark.parametrize("cfg,kw", [("C1", {}), ("C2", {}), ("C2", {"stereo_mode": 1}), ("C2", {"stereo_mode": 2}),
                                    ("C2", {"stereo_mode": 3}), ("C2", {"partition_order": 0}),
                                    ("C2", {"blocksize": 1152}), ("C1", {"blocksize": 4000})])
@LANE
def test_stereo_fast_path_layouts(gpu, fmt_name, cfg, kw, decode_mode):
    """k_decode_st (one lane per stereo frame) writes every layout bit-exactly, and takes
    the frames itself (BNF_FL_ST set, no hand-back) on regular streams -- including a
    blocksize that is not a multiple of its 32-sample chunk (general path for the tail)."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    fmt = getattr(libflac, fmt_name)
    p = synth.config(cfg, nframes=70, last_blocksize=0, **kw)
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, fmt)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_ST).all(), info["flags"]
    assert not (info["flags"] & FL_REDO).any(), info["flags"]
    pcm = s.pcm.astype(np.int64)
    if fmt == libflac.OUT_INTERLEAVED32:
        assert np.array_equal(out.view("<i4").reshape(-1, 2), s.pcm)
    elif fmt == libflac.OUT_PLANAR32:
        got = out.view("<i4")
        o = 0
        for fr in range(p.nframes):
            bs = int(info["blocksize"][fr])
            st = int(info["out_sample"][fr])
            assert np.array_equal(got[o: o + 2 * bs].reshape(2, bs).T, s.pcm[st: st + bs])
            o += 2 * bs
    else:
        assert out.tobytes() == (pcm & 0xFFFF).astype("<u2").tobytes()
    ev, opcm = oracle.run(data)
    assert np.array_equal(s.pcm, oracle.interleave(ev, opcm))


@pytest.mark.parametrize("fmt_name", ["OUT_FLACDECODER", "OUT_INTERLEAVED32"])
@LANE
def test_long_rice_prefixes_small_parameters(gpu, fmt_name, decode_mode):
    """Impulses in a C2-shaped stream (Rice parameters ~8, so k_parse takes its bulk instance):
    unary prefixes of ~100 bits, far beyond a 32-bit window, where a pair of codewords does
    not fit -- k_parse's bulk steps hand the lane to the generic reader, k_decode_st's fused
    pairs take st_rare_pair.  Bit-exact against the source and the oracle, every frame kept by
    k_decode_st, and its slow-codeword counter (ablation 0x100's stats) nonzero."""
    import ctypes
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    fmt = getattr(libflac, fmt_name)
    p = synth.config("C2", nframes=70, last_blocksize=0, impulse_permille=2)
    s = synth.encode(p)
    data = s.data.tobytes()
    buf = (ctypes.c_uint64 * 16)()
    dec.L.bnflac_debug_stats(buf, 1)
    dec.L.bnflac_debug_set_ablate(0x100)
    try:
        out, info, sp = _decode_batch(gpu, data, s.frame_offsets, fmt)
    finally:
        dec.L.bnflac_debug_set_ablate(0)
    dec.L.bnflac_debug_stats(buf, 1)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_ST).all() and not (info["flags"] & FL_REDO).any(), info["flags"]
    assert buf[3] > 0, list(buf)
    if fmt == libflac.OUT_INTERLEAVED32:
        assert np.array_equal(out.view("<i4").reshape(-1, 2), s.pcm)
    else:
        assert out.tobytes() == (s.pcm.astype(np.int64) & 0xFFFF).astype("<u2").tobytes()
    ev, opcm = oracle.run(data)
    assert np.array_equal(s.pcm, oracle.interleave(ev, opcm))


@pytest.mark.parametrize("cfg", ["C1", "C2", "C4"])
@LANE
def test_stereo_handback_matches(gpu, cfg, decode_mode):
    """With k_decode_st disabled (ablation 0x400) every stereo frame goes to k_decode<8>;
    both routes give identical PCM and frame records."""
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    p = synth.config(cfg, nframes={"C4": 64}.get(cfg, 16), last_blocksize=0)
    s = synth.encode(p)
    data = s.data.tobytes()
    out_a, info_a, _ = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_FLACDECODER)
    dec.L.bnflac_debug_set_ablate(0x400)
    try:
        out_b, info_b, _ = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_FLACDECODER)
    finally:
        dec.L.bnflac_debug_set_ablate(0)
    assert out_a.tobytes() == out_b.tobytes()
    keep = [n for n in info_a.dtype.names if n != "flags"]
    assert all(np.array_equal(info_a[n], info_b[n]) for n in keep)


@pytest.mark.parametrize("stereo_mode", [1, 2, 3])
@LANE
def test_stereo_side_beyond_int16_handed_back(gpu, stereo_mode, decode_mode):
    """k_decode_st's dot2 predictor is exact only while samples fit int16.  Loud,
    weakly correlated channels push the 17-bit side channel past that: those frames must be
    handed back (BNF_FL_REDO) and come out of k_decode<8> bit-exact."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C2", nframes=40, stereo_mode=stereo_mode, level=0.9, noise=0.5)
    s = synth.encode(p)
    side = s.pcm[:, 0].astype(np.int64) - s.pcm[:, 1]
    assert np.abs(side).max() > 32767  # the fixture does leave int16
    out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_REDO).any(), info["flags"]
    assert np.array_equal(out.view("<i4").reshape(-1, 2), s.pcm)


# ------------------------------------------------- streaming reader
@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] in ("roundtrip", "rfc")])
def test_reader_matches_flacdecoder_copyto(gpu, name):
    """bnflac_reader yields the bytes FLACDecoder.CopyTo yields (the libFLAC-API mirror),
    read in OpenAL-sized 16 KiB pieces."""
    from birdnest.audio_amd import flac_decoder
    torch, libflac, _ = gpu
    data = _read(name)
    rc, pk, msg, fmt = flac_decoder.copy_to_bytes(data)
    if rc != 0 or fmt[2] != 16:
        # FLACDecoder aborts on these (FLACDecoder.cs:526-530); FLACFileReader is the
        # reference's reader for them: its Read semantics against the oracle's replay
        _filereader_vs_oracle(libflac, data)
        return
    r = libflac.Reader(data, libflac.OUT_FLACDECODER, window_frames=5)
    try:
        assert r.total_bytes == len(pk)
        assert r.read_all(16384) == pk
    finally:
        r.close()


def _filereader_vs_oracle(libflac, data, windows=(3,)):
    """bnflac_reader in FLACFileReader mode == oracle.filereader_readall, byte for byte and
    exception for exception, over buffer lengths that hit the reader's quirks: one frame,
    half a frame (carry-over between calls), a length that is not a whole number of samples
    (IndexOutOfRange), and Read(buf, 0, n) with n far below buf.Length (overfill)."""
    import oracle
    si = data[8:42]
    x = int.from_bytes(si[10:18], "big")
    ch, bps = ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1
    maxbs = int.from_bytes(si[2:4], "big")
    sf = ch * (3 if bps == 24 else 2)
    cases = [(maxbs * sf, None), (maxbs * sf // 2 + sf, None), (sf * 100 + 1, None), (maxbs * sf * 3, 7),
             (sf * 37, None)]
    for win in windows:
        for buf_len, nb in cases:
            rc, ref, msg = oracle.filereader_readall(data, buf_len, nb)
            r = libflac.Reader(data, libflac.OUT_FILEREADER, window_frames=win)
            try:
                grc, got, gmsg = r.filereader_read_all(buf_len, nb)
            finally:
                r.close()
            assert (grc, gmsg) == (rc, msg), (buf_len, nb)
            assert got == ref, (buf_len, nb, len(got), len(ref))


def test_filereader_mode_quirks_24bit(gpu):
    """FLACFileReader surface on the 24-bit configs (its only reference path, FLACFileReader.cs:
    230-237): a short last frame (stale tail: m_samplesPerChannel fixed by the first frame),
    variable blocksizes (truncation), carry-over, overfill and IndexOutOfRange, all against
    the oracle's replay."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    for cfg, kw in (("C3", dict(nframes=5, last_blocksize=3000)), ("C5", dict(nframes=4, last_blocksize=1500)),
                    ("C4", dict(nframes=30, bps=24, seed=7)), ("C1", dict(nframes=6, last_blocksize=100))):
        s = synth.encode(synth.config(cfg, **kw))
        _filereader_vs_oracle(libflac, s.data.tobytes(), windows=(2, 64))


@pytest.mark.parametrize("name", ["mono_8bit_fixed", "odd_headers_20bit"])
def test_filereader_mode_unsupported_depth_offset_at_end(gpu, tmp_path, name):
    """NotSupported is thrown from CopyFlacBufferToNAudioBuffer's sample loop
    (FLACFileReader.cs:214-240), which never runs with the offset at buffer.Length: Read then
    returns 0 per frame and ProcessSingle runs to the end of the stream.  The native compat
    mode must agree with the C# mirror over the libFLAC-compatible API (and throw as soon as
    the offset is inside the buffer)."""
    from birdnest.audio_amd import flac_file_reader
    torch, libflac, _ = gpu
    data = _read(name)
    path = os.path.join(str(tmp_path), name + ".flac")
    open(path, "wb").write(data)
    buf = bytearray(4096)
    mirror = flac_file_reader.FLACFileReader(path)
    try:
        want = [mirror.Read(buf, len(buf), 64), mirror.Read(buf, len(buf), 64)]
    finally:
        mirror.Dispose()
    mirror = flac_file_reader.FLACFileReader(path)
    try:
        with pytest.raises(flac_file_reader.NotSupportedException):
            mirror.Read(buf, 0, 64)
    finally:
        mirror.Dispose()
    r = libflac.Reader(data, libflac.OUT_FILEREADER, window_frames=3)
    try:
        got = [r.ReadFileReader(buf, len(buf), 64), r.ReadFileReader(buf, len(buf), 64)]
    finally:
        r.close()
    assert got == want == [0, 0]
    r = libflac.Reader(data, libflac.OUT_FILEREADER, window_frames=3)
    try:
        with pytest.raises(RuntimeError, match="bit depth is not supported"):
            r.ReadFileReader(buf, 0, 64)
    finally:
        r.close()


@pytest.mark.parametrize("window,chunk", [(256, 16384), (7, 1000), (1, 4096 * 4 + 3)])
def test_reader_c2_windows_and_chunks(gpu, window, chunk):
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C2", nframes=96))
    r = libflac.Reader(s.data.tobytes(), libflac.OUT_FLACDECODER, window_frames=window)
    try:
        assert r.nframes == 96
        got = r.read_all(chunk)
        assert got == s.pcm.astype("<i2").tobytes()
        buf = bytearray(10)
        assert r.Read(buf, 0, 10) == 0  # end of stream
    finally:
        r.close()
    r = libflac.Reader(s.data.tobytes(), libflac.OUT_INTERLEAVED32, window_frames=window)
    try:
        assert np.array_equal(np.frombuffer(r.read_all(chunk), dtype="<i4").reshape(-1, 2), s.pcm)
    finally:
        r.close()


def test_reader_more_frames_than_streaminfo_implies(gpu):
    """The reader sizes its frame records from STREAMINFO (total / minimum blocksize + 16).  A
    variable-blocksize stream whose STREAMINFO claims a larger minimum than its frames use
    overflows that guess: open re-indexes at the byte bound and still reads every frame."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C4", nframes=300))
    d = bytearray(s.data.tobytes())
    assert d[:4] == b"fLaC" and (d[4] & 0x7F) == 0  # STREAMINFO first: min/max blocksize at 8..11
    assert d[int(s.frame_offsets[0]) + 1] & 1  # variable-blocksize frames (sample-numbered)
    d[8:12] = (16384).to_bytes(2, "big") + (65535).to_bytes(2, "big")
    assert s.pcm.shape[0] // 16384 + 16 < 300  # the guess is short: the retry runs
    for win in (256, 7):
        r = libflac.Reader(bytes(d), libflac.OUT_FLACDECODER, window_frames=win)
        try:
            assert r.nframes == 300
            assert r.read_all(16384) == s.pcm.astype("<i2").tobytes()
        finally:
            r.close()


def test_reader_refuses_damaged_stream(gpu):
    torch, libflac, _ = gpu
    data = _read("err_crc16_mismatch")
    with pytest.raises(RuntimeError, match="damaged|covers"):
        r = libflac.Reader(data, libflac.OUT_FLACDECODER, window_frames=2)
        try:
            r.read_all(16384)
        finally:
            r.close()
    with pytest.raises(RuntimeError, match="fLaC"):
        libflac.Reader(b"not a flac stream at all", libflac.OUT_FLACDECODER)
    with pytest.raises(RuntimeError, match="16-bit"):
        libflac.Reader(_read("c3_lpc12_ms_wasted"), libflac.OUT_FLACDECODER)


def _zero_total(data: bytes) -> bytearray:
    """STREAMINFO total_samples := 0 (unknown length): the low 36 bits of bytes 21..25."""
    d = bytearray(data)
    d[21] &= 0xF0
    d[22:26] = bytes(4)
    return d


def test_reader_unknown_length_refuses_a_cut_chain(gpu):
    """total_samples 0: a damaged mid-stream header ends the GPU frame chain early with every
    chained frame intact -- the reader must refuse, not return a prefix; an
    intact stream with trailing non-frame bytes (an ID3v1 tag) still reads completely."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C2", nframes=12))
    d = _zero_total(s.data.tobytes())
    r = libflac.Reader(bytes(d) + b"TAG" + bytes(125), libflac.OUT_FLACDECODER, window_frames=4)
    try:
        assert r.read_all(16384) == s.pcm.astype("<i2").tobytes()
    finally:
        r.close()
    o = [int(x) for x in s.frame_offsets]
    d[o[5] + 4] ^= 0x55  # frame 5's header (its CRC-8 no longer matches)
    with pytest.raises(RuntimeError, match="damaged"):
        libflac.Reader(bytes(d), libflac.OUT_FLACDECODER, window_frames=4).close()


def test_reader_seek(gpu):
    """bnflac_reader_seek: the next read starts at the target sample (FLACFileReader.Position),
    across frame and window boundaries, mid-frame, and at the last sample."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C4", nframes=120))
    ref = s.pcm.astype("<i2").tobytes()
    n = s.pcm.shape[0]
    r = libflac.Reader(s.data.tobytes(), libflac.OUT_FLACDECODER, window_frames=9)
    try:
        buf = bytearray(5000)
        for target in (0, 1, 4095, n // 3, n // 2 + 7, n - 1, 12345):
            r.Seek(target)
            got = r.Read(buf, 0, len(buf))
            want = ref[target * 4: target * 4 + len(buf)]
            assert got == len(want) and bytes(buf[:got]) == want, target
        r.Seek(n - 100)
        assert r.read_all(64) == ref[(n - 100) * 4:]
        with pytest.raises(RuntimeError, match="past the end"):
            r.Seek(n)
    finally:
        r.close()


@pytest.mark.parametrize("seed", range(24))
def test_stereo_fast_path_random_sweep(gpu, seed):
    """Randomised 16-bit stereo streams through k_decode_st (and its hand-backs): blocksize,
    predictor type/order, partition order, RICE2, escapes, wasted bits, stereo mode, level
    and noise all drawn per seed; output must equal the generator's source PCM."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    rng = np.random.default_rng(1000 + seed)
    bs = int(rng.choice([1152, 2048, 4096, 4608, 576 * 7]))
    kw = dict(nframes=int(rng.integers(40, 140)), blocksize=bs, last_blocksize=int(rng.integers(64, bs)),
              subframe_mode=int(rng.choice([synth.SUB_LPC, synth.SUB_FIXED, synth.SUB_LPC])),
              order=int(rng.integers(1, 9)), partition_order=int(rng.choice([-1, 0, 2, 4, 6])),
              stereo_mode=int(rng.integers(0, 5)), rice2=int(rng.integers(0, 2)),
              escape_permille=int(rng.choice([0, 0, 20])), wasted_bits_max=int(rng.choice([0, 0, 3])),
              level=float(rng.uniform(0.05, 0.9)), noise=float(rng.choice([0.0005, 0.006, 0.05])),
              seed=50 + seed, prec_clamp=int(rng.integers(0, 2)))
    if kw["subframe_mode"] == synth.SUB_FIXED:
        kw["order"] = int(rng.integers(0, 5))
    s = synth.encode(synth.config("C2", **kw))
    for fmt in (libflac.OUT_FLACDECODER, libflac.OUT_INTERLEAVED32):
        out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, fmt)
        assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all(), kw
        if fmt == libflac.OUT_INTERLEAVED32:
            assert np.array_equal(out.view("<i4").reshape(-1, 2), s.pcm), kw
        else:
            assert out.tobytes() == (s.pcm.astype(np.int64) & 0xFFFF).astype("<u2").tobytes(), kw


@pytest.mark.parametrize("kw", [
    dict(channels=1, bps=16, blocksize=2048, nframes=79, last_blocksize=1591, subframe_mode=4, order=3,
         partition_order=-1, stereo_mode=0, level=0.0534, noise=0.3, seed=849887222, sample_rate=192000),
    dict(channels=6, bps=16, blocksize=4096, nframes=42, last_blocksize=1673, subframe_mode=4, order=1,
         partition_order=1, stereo_mode=0, level=0.374, noise=0.03, seed=455035102, sample_rate=8000),
])
def test_constant_last_subframe(gpu, kw):
    """Regression (found by tools/stress.py): a CONSTANT subframe in the last channel has no
    residual, so k_decode must not read a partition header after it (that misread the
    zero padding as LOST_SYNC on tiny constant frames)."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C2", **kw))
    out, info, sp = _decode_batch(gpu, s.data.tobytes(), s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all(), info[["status", "err", "flags"]]
    assert np.array_equal(out.view("<i4").reshape(-1, kw["channels"]), s.pcm)


@pytest.mark.parametrize("bps,ch,stereo", [(16, 2, 0), (16, 2, 3), (24, 2, 1), (12, 1, 0), (20, 8, 0)])
def test_loud_noisy_fixed4_escapes(gpu, bps, ch, stereo):
    """Loud, noisy FIXED-4 (residuals up to 16x the signal): escaped partitions dominate and
    partition boundaries fall anywhere -- the fused paths read partition headers and raw
    escaped values inline.  Bit-exact against the oracle and the source PCM."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C2", channels=ch, bps=bps, subframe_mode=synth.SUB_FIXED, order=4, level=0.95, noise=0.3,
                     stereo_mode=stereo, nframes=8, partition_order=-1, escape_permille=200, seed=40 + bps + ch)
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    pcm = out.view("<i4").reshape(-1, ch)
    ev, opcm = oracle.run(data)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm))
    assert np.array_equal(pcm, s.pcm)


@pytest.mark.gpu
@pytest.mark.parametrize("order,bs,porder", [(32, 512, 4), (32, 256, 3), (16, 256, 4), (8, 128, 4)])
def test_empty_first_partition(gpu, order, bs, porder):
    """LPC order == partition size: Rice partition 0 carries no samples, and the first
    residual of the subframe sits in partition 1 (found by tools/stress.py: the fused path
    must skip the empty partition's header).  Bit-exact against the oracle."""
    import oracle
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    p = synth.config("C2", channels=3, bps=16, subframe_mode=synth.SUB_LPC, order=order, blocksize=bs,
                     last_blocksize=bs // 2, partition_order=porder, nframes=12, seed=700 + order)
    s = synth.encode(p)
    data = s.data.tobytes()
    out, info, sp = _decode_batch(gpu, data, s.frame_offsets, libflac.OUT_INTERLEAVED32)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    pcm = out.view("<i4").reshape(-1, 3)
    ev, opcm = oracle.run(data)
    assert np.array_equal(pcm, oracle.interleave(ev, opcm))
    assert np.array_equal(pcm, s.pcm)


def test_reader_pool_reuse_across_sizes_and_layouts(gpu):
    """bnflac_reader_close keeps one reader's buffers per device and the next open reuses
    them, growing what is too small: alternate small and large streams, both layouts, two
    readers open at once (the second allocates afresh), a failed open in between."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    c2 = synth.encode(synth.config("C2", nframes=40, last_blocksize=0))
    c2b = synth.encode(synth.config("C2", nframes=300, last_blocksize=1000, seed=77))
    c3 = synth.encode(synth.config("C3", nframes=12))
    want_c2 = c2.pcm.astype("<i2").tobytes()
    want_c2b = c2b.pcm.astype("<i2").tobytes()
    for _ in range(2):
        for s, want in ((c2, want_c2), (c2b, want_c2b), (c2, want_c2)):
            r = libflac.Reader(s.data.tobytes(), libflac.OUT_FLACDECODER, window_frames=16)
            try:
                assert r.read_all(16384) == want
            finally:
                r.close()
        r = libflac.Reader(c3.data.tobytes(), libflac.OUT_FILEREADER, window_frames=4)
        try:
            got = r.read_all(49152)
        finally:
            r.close()
        pcm = c3.pcm.astype("<i4")
        ref = np.stack([(pcm >> 8 * k) & 0xFF for k in range(3)], axis=-1).astype(np.uint8).tobytes()
        assert got == ref
        with pytest.raises(RuntimeError):
            libflac.Reader(b"not a flac stream", libflac.OUT_FLACDECODER)
    a = libflac.Reader(c2b.data.tobytes(), libflac.OUT_FLACDECODER)
    b = libflac.Reader(c2.data.tobytes(), libflac.OUT_FLACDECODER)
    try:
        assert b.read_all(1000) == want_c2
        assert a.read_all(65536) == want_c2b
    finally:
        a.close()
        b.close()
    # one pooled set per device; releasing it frees it, and the next open allocates afresh
    L = libflac.load()
    assert L.bnflac_reader_pool_release(-1) == 1
    assert L.bnflac_reader_pool_release(-1) == 0
    r = libflac.Reader(c2.data.tobytes(), libflac.OUT_FLACDECODER, window_frames=16)
    try:
        assert r.read_all(16384) == want_c2
    finally:
        r.close()
    assert L.bnflac_reader_pool_release(0) == 1


def _crc_cases(gpu, data, offs, base=0):
    """Decode `data` placed at byte `base` of a device buffer; every stereo frame's CRC-16
    (k_decode_st computes it from its two bit-reader rings, channel 0's bytes and channel 1's
    combined by a GF(2) shift) against the CRC of the frame's bytes."""
    import oracle
    torch, libflac, dec = gpu
    sp = _stream_params(libflac, data)
    dev = torch.device("cuda:0")
    n = base + len(data)
    d_bytes = torch.zeros((n + 3) // 4 * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[base:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.tensor([base + int(o) for o in offs], dtype=torch.int64, device=dev)
    stride = libflac.out_stride(libflac.OUT_FLACDECODER, sp)
    d_out = torch.full((sp.total_samples * stride + 64,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(len(offs) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec.decode_frames(d_bytes, n, d_offs, len(offs), sp, libflac.OUT_FLACDECODER, d_out, d_info)
    torch.cuda.synchronize()
    info = libflac.info_array(d_info.cpu().numpy())
    del d_bytes
    for i, o in enumerate(offs):
        if info["status"][i] != 0:
            continue
        end = int(info["resume_bit"][i]) // 8 - base
        assert info["crc16_calc"][i] == oracle.crc16(data[int(o):end - 2]), (i, o)
        assert info["crc_ok"][i] == (oracle.crc16(data[int(o):end - 2]) == int.from_bytes(data[end - 2:end], "big"))
    return info, d_out[: sp.total_samples * stride].cpu().numpy()


def test_ring_crc_beyond_4gib(gpu):
    """Frames at byte offsets past 2^32 (the rings track bytes mod 2^32): CRCs computed
    right, PCM lossless, and a damaged frame zero-filled."""
    from birdnest.audio_amd import synth
    torch, libflac, _ = gpu
    s = synth.encode(synth.config("C2", nframes=24, seed=21))
    data = bytearray(s.data.tobytes())
    o = [int(x) for x in s.frame_offsets]
    info, out = _crc_cases(gpu, bytes(data), o, base=(1 << 32) + 4099)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert out.tobytes() == s.pcm.astype("<i2").tobytes()
    data[o[7] + 3000] ^= 0x10
    info, out = _crc_cases(gpu, bytes(data), o, base=(1 << 32) - 2000)
    assert info["crc_ok"][7] == 0 or info["status"][7] != 0
    pcm = out.view("<i2").reshape(-1, 2)
    assert not pcm[7 * 4096: 8 * 4096].any()


@pytest.mark.parametrize("cfg,kw", [("C2", {}), ("C2", {"partition_order": 0, "seed": 3}),
                                    ("C2", {"stereo_mode": 2, "seed": 4}), ("C1", {"seed": 5})])
def test_ring_crc_damage_positions(gpu, cfg, kw):
    """One flipped bit at 40 positions across a frame (header, channel 0, around the channel
    split, channel 1, the footer), each its own stream: every CRC-16 the decode computes is the
    CRC of the frame's bytes, and frames it rejects are zero-filled."""
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config(cfg, **({"nframes": 4, "last_blocksize": 0} | kw)))
    data = s.data.tobytes()
    o = [int(x) for x in s.frame_offsets]
    f = 1
    lo, hi = o[f], o[f + 1]
    rng = np.random.default_rng(7)
    pos = sorted(set(np.linspace(lo, hi - 1, 40).astype(int).tolist()))
    bad = 0
    for p in pos:
        d = bytearray(data)
        d[p] ^= 1 << int(rng.integers(0, 8))
        info, out = _crc_cases(gpu, bytes(d), o)
        ok = info["status"][f] == 0 and info["crc_ok"][f] == 1
        bad += not ok
        if info["status"][f] == 0 and info["crc_ok"][f] == 0:
            bs = int(info["blocksize"][f])
            assert not out.view("<i2")[f * bs * 2:(f + 1) * bs * 2].any()
    assert bad >= len(pos) - 2  # a flipped bit is (almost always) caught


@pytest.mark.parametrize("decode_mode", [0, 2], indirect=True)
@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_non_ok_frame_range_zero_filled(gpu, cfg, decode_mode):
    """The batch API's output for a frame that does not decode (include/bnflac.h): the last
    frame cut short inside its subframes (status TRUNC, header parsed) leaves zeros over its
    whole range, not the lane kernels' partial stores; a frame whose header fails (a broken
    sync code) leaves its range untouched; the other frames decode bit-exactly."""
    from birdnest.audio_amd import synth
    torch, libflac, dec = gpu
    s = synth.encode(synth.config(cfg, nframes=6, last_blocksize=0))
    data = bytearray(s.data.tobytes())
    offs = [int(o) for o in s.frame_offsets]
    data[offs[2] + 1] ^= 0x02  # frame 2: 0xFFF8 -> 0xFFFA, a header error (reserved bit)
    sp = _stream_params(libflac, bytes(data))
    fmt = libflac.OUT_INTERLEAVED32
    stride = libflac.out_stride(fmt, sp)
    dev = torch.device("cuda:0")
    cut = offs[5] + (len(data) - offs[5]) // 2  # frame 5 ends past nbytes
    d_bytes = torch.zeros((len(data) + 3) // 4 * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_os = torch.tensor([i * sp.max_blocksize for i in range(6)], dtype=torch.int64, device=dev)
    d_out = torch.full((sp.total_samples * stride,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(6 * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec.decode_frames(d_bytes, cut, d_offs, 6, sp, fmt, d_out, d_info, d_out_sample=d_os)
    torch.cuda.synchronize()
    info = libflac.info_array(d_info.cpu().numpy())
    out = d_out.cpu().numpy()
    bs = sp.max_blocksize * stride
    assert info["status"][5] == 2 and info["sub_start"][5][0] != 0
    assert not out[5 * bs:6 * bs].any()
    assert info["status"][2] == 1 and info["sub_start"][2][0] == 0
    assert (out[2 * bs:3 * bs] == 0xAB).all()
    pcm = out.view("<i4").reshape(-1, sp.channels)
    for i in (0, 1, 3, 4):
        assert info["status"][i] == 0 and info["crc_ok"][i] == 1
        n = sp.max_blocksize
        assert np.array_equal(pcm[i * n:(i + 1) * n], s.pcm[i * n:(i + 1) * n])
