"""Stream-API seeking on the GPU path against the oracle.

The reference's only seek pattern is FLACFileReader's: setting Position makes the NEXT
write callback copy its frame and then call FLAC__stream_decoder_seek_absolute from inside
itself (FLACFileReader.cs:125-136, 267-301); the trimmed target frame arrives through a
nested write callback and decoding continues after it.  harness.run(seeks=...) drives
libbnflac.so that way and oracle.run_seek drives the CPU restatement the same way; the
callback sequences (writes with blocksize and sample number, errors, metadata, every
process_* and seek_absolute return) and the delivered PCM must be identical.
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
    from birdnest.audio_amd import harness
    return harness


def _stream(cfg, **kw):
    from birdnest.audio_amd import synth
    p = synth.config(cfg, **kw)
    s = synth.encode(p)
    return s.data.tobytes(), s


def _compare(harness, data, seeks, read_chunk=16384):
    import oracle
    ev, pcm = harness.run(data, seeks=seeks, read_chunk=read_chunk)
    oev, opcm = oracle.run_seek(data, seeks, read_chunk=read_chunk)
    assert ev == harness.oracle_events_as_tuples(oev)
    assert np.array_equal(pcm, opcm)
    return ev, pcm


CASES = [
    ("C2", dict(nframes=24), [(3, 20000), (6, 4096 * 2)]),            # forward mid-frame, then backward to a frame start
    ("C2", dict(nframes=24), [(0, 0), (1, 24 * 4096 - 1)]),            # to the first and to the last sample
    ("C2", dict(nframes=24), [(-1, 50000)]),                           # right after the metadata pass
    ("C2", dict(nframes=24), [(-2, 12345)]),                           # before the metadata pass: no STREAMINFO callback
    ("C3", dict(nframes=12), [(2, 3 * 8192 + 17), (4, 100)]),          # 24-bit M/S + wasted bits
    ("C4", dict(nframes=40), [(5, 60000), (7, 5), (9, 150000)]),       # variable blocksize, mixed subframes
    ("C5", dict(nframes=6, last_blocksize=0), [(1, 4096 * 4 + 1000)]),  # 8 channels, LPC-32
]


@pytest.mark.parametrize("cfg,kw,seeks", CASES)
def test_seek_from_write_callback_matches_oracle(gpu, cfg, kw, seeks):
    data, s = _stream(cfg, **kw)
    ev, pcm = _compare(gpu, data, seeks)
    seek_ret = [e for e in ev if e[0] == gpu.EV_SEEK]
    assert len(seek_ret) == len(seeks) and all(e[1] == 1 for e in seek_ret)
    if seeks[0][0] == -2:
        assert not [e for e in ev if e[0] == gpu.EV_METADATA]  # suppressed while seeking


def test_seek_delivers_source_pcm(gpu):
    """After a seek the trimmed frame and everything after it equal the source PCM."""
    data, s = _stream("C2", nframes=20)
    target = 7 * 4096 + 1234
    ev, pcm = gpu.run(data, seeks=[(-1, target)])
    writes = [e for e in ev if e[0] == gpu.EV_WRITE]
    assert writes[0][8] == target and writes[0][3] == 4096 - 1234
    out = []
    off = 0
    for e in writes:
        bs, ch = e[3], e[5]
        out.append(pcm[off: off + bs * ch].reshape(ch, bs).T)
        off += bs * ch
    assert np.array_equal(np.concatenate(out), s.pcm[target:])


def test_seek_is_windowed_not_a_stream_walk(gpu):
    """A seek to the end of a 10 MB stream reads a few windows, not the stream: the client's
    seek callback positions the probes (interpolation over decoded windows)."""
    data, s = _stream("C2", nframes=1024)
    stats = {}
    target = 1020 * 4096 + 7
    ev, pcm = gpu.run(data, seeks=[(-1, target)], stats=stats)
    writes = [e for e in ev if e[0] == gpu.EV_WRITE]
    assert writes[0][8] == target
    assert stats["read_total"] < len(data) // 3, stats
    _compare(gpu, data, [(-1, target)])


def test_seek_refusals(gpu):
    """Past the end: false, no callbacks; no seek callback: false."""
    data, s = _stream("C2", nframes=8)
    ev, pcm = _compare(gpu, data, [(2, 8 * 4096)])
    assert [e for e in ev if e[0] == gpu.EV_SEEK][0][1] == 0


def _with_seektable(data, s, every, shift=0, placeholder=True):
    """The stream with a SEEKTABLE block after STREAMINFO (libFLAC's layout: sample number,
    byte offset from the first frame header, frame samples; 18 bytes a point, placeholders
    0xFFFFFFFFFFFFFFFF last).  shift moves every offset (a misleading table)."""
    bs = s.params.blocksize
    first = int(s.frame_offsets[0])
    pts = b""
    n = 0
    for i in range(0, len(s.frame_offsets), every):
        off = int(s.frame_offsets[i]) - first + shift
        pts += (i * bs).to_bytes(8, "big") + max(off, 0).to_bytes(8, "big") + bs.to_bytes(2, "big")
        n += 1
    if placeholder:
        pts += b"\xff" * 8 + bytes(10)
    assert data[:4] == b"fLaC" and data[4] & 0x7F == 0 and data[4] & 0x80  # STREAMINFO, last block
    head = data[:4] + bytes([data[4] & 0x7F]) + data[5:42]
    block = bytes([0x80 | 3]) + len(pts).to_bytes(3, "big") + pts
    return head + block + data[42:]


@pytest.mark.parametrize("cfg,kw,every,seeks", [
    ("C2", dict(nframes=600), 16, [(-1, 517 * 4096 + 77), (3, 40 * 4096), (5, 599 * 4096 + 1)]),
    ("C3", dict(nframes=60), 8, [(-1, 41 * 8192 + 5), (2, 7 * 8192)]),
    ("C5", dict(nframes=40, last_blocksize=0), 4, [(1, 33 * 4096 + 100)]),
])
def test_seektable_narrows_seek_and_matches_oracle(gpu, cfg, kw, every, seeks):
    """libFLAC reads a SEEKTABLE whatever the respond set (LibFLACSharp.cs:64 seek_absolute
    uses it): the points bracket the search, so a seek takes fewer client seeks, and the
    delivered callbacks and PCM are the oracle's, which ignores the table."""
    plain, s = _stream(cfg, **kw)
    data = _with_seektable(plain, s, every)
    _compare(gpu, data, seeks)
    st_tab, st_plain = {}, {}
    ev_t, pcm_t = gpu.run(data, seeks=seeks, stats=st_tab)
    ev_p, pcm_p = gpu.run(plain, seeks=seeks, stats=st_plain)
    assert np.array_equal(pcm_t, pcm_p)
    assert st_tab["seek_calls"] <= st_plain["seek_calls"], (st_tab, st_plain)
    if cfg == "C2":  # a window from the bracketing point, not centred on an estimate: fewer bytes read
        assert st_tab["read_total"] < st_plain["read_total"], (st_tab, st_plain)


def _vbr_stream(nframes=400):
    """A variable-bitrate C2-shaped stream: the first half of the frames from a near-silent
    encode, the second half from a loud, noisy one (same blocksize, so the spliced frames keep
    consecutive frame numbers and their own CRCs).  Byte position is then far from linear in
    the sample number, which is what a SEEKTABLE is for."""
    import types
    from birdnest.audio_amd import synth
    a = synth.encode(synth.config("C2", nframes=nframes, last_blocksize=0, level=0.0001, noise=0.000002, seed=21))
    b = synth.encode(synth.config("C2", nframes=nframes, last_blocksize=0, level=0.95, noise=0.3, seed=22))
    h = nframes // 2
    ca, cb = int(a.frame_offsets[h]), int(b.frame_offsets[h])
    data = a.data.tobytes()[:ca] + b.data.tobytes()[cb:]
    offs = np.concatenate([a.frame_offsets[:h], b.frame_offsets[h:] - cb + ca]).astype(np.uint64)
    pcm = np.concatenate([a.pcm[:h * 4096], b.pcm[h * 4096:]])
    return data, types.SimpleNamespace(params=a.params, frame_offsets=offs, pcm=pcm)


def test_seektable_reduces_probes_on_variable_bitrate(gpu):
    """On a stream whose bitrate changes about 8-fold half way, the table-free interpolation search
    guesses badly; with a SEEKTABLE libFLAC's search starts from the bracketing points and takes
    strictly fewer client seeks.  Output equals the oracle's (which ignores the table) and the
    source PCM either way."""
    plain, s = _vbr_stream()
    assert int(s.frame_offsets[-1] - s.frame_offsets[200]) > 6 * int(s.frame_offsets[200] - s.frame_offsets[0])
    data = _with_seektable(plain, s, 8)
    seeks = [(-1, 150 * 4096 + 33), (2, 330 * 4096 + 7), (4, 260 * 4096)]
    _compare(gpu, data, seeks)
    st_tab, st_plain = {}, {}
    ev_t, pcm_t = gpu.run(data, seeks=seeks, stats=st_tab)
    ev_p, pcm_p = gpu.run(plain, seeks=seeks, stats=st_plain)
    assert np.array_equal(pcm_t, pcm_p)
    assert st_tab["seek_calls"] < st_plain["seek_calls"], (st_tab, st_plain)
    assert st_tab["read_total"] < st_plain["read_total"], (st_tab, st_plain)


@pytest.mark.parametrize("shift", [-5000, 3, 1 << 40])
def test_misleading_seektable_same_output(gpu, shift):
    """A table whose offsets are wrong (before, inside or past the stream) costs a
    table-free search, never different output."""
    plain, s = _stream("C2", nframes=64)
    data = _with_seektable(plain, s, 8, shift=shift)
    _compare(gpu, data, [(-1, 50 * 4096 + 9), (2, 3 * 4096)])
