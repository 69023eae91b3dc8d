"""Decode-class split across streams (SURVEY.md 8a A10 dispatch; bnf_launch_decode).

k_decode_st -> k_decode<8> run on the caller's stream, and k_decode<16> / k_decode<32> each
on a side stream forked before k_decode_st (or after it, BNFLAC_DECODE_FORK=1).  k_decode<8>
takes k_decode_st's hand-backs (BNF_FL_REDO) also in blocks that belong to the other
instances, which never look at stereo fast-path frames.
These tests put hand-back-prone stereo frames, LPC-12 (W16) and LPC-32 (W32) frames into
one batch, so the decode order's 32-frame blocks mix the classes at their edges, and
compare with the generator's source PCM and with the serial order (BNFLAC_DECODE_SERIAL=1,
in a child process).  The batches here are small enough for k_decode_sys's auto range, so the
module pins the lane kernels.  When the previous decode order had no W16 / W32 frames, both
classes go through one small segment grid (k_decode_seg) instead of the side grids: the last
test decodes a batch without them first, so that its mixed batch takes that path.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FL_REDO = 16


@pytest.fixture(autouse=True)
def _lane_kernels():
    if not gpu_available():
        yield
        return
    from birdnest.audio_amd import libflac
    L = libflac.load()
    L.bnflac_debug_set_decode_sys(0)
    yield
    L.bnflac_debug_set_decode_sys(-1)


def _mixed_batch(n_each, class1=False):
    from birdnest.audio_amd import synth
    parts = [
        synth.encode(synth.config("C2", nframes=n_each, stereo_mode=3, level=0.9, noise=0.5, seed=41)),
        synth.encode(synth.config("C2", nframes=n_each, order=12, seed=42)),
        synth.encode(synth.config("C2", nframes=n_each, order=32, partition_order=-1, seed=43)),
        synth.encode(synth.config("C2", nframes=n_each, seed=44)),
    ]
    if class1:  # C4's subframe mix at a fixed blocksize: VERBATIM / CONSTANT frames (decode class 1)
        parts.append(synth.encode(synth.config("C2", nframes=n_each, subframe_mode=synth.SUB_MIXED,
                                               stereo_mode=synth.ST_CYCLE, partition_order=-1, seed=45)))
    data, offs, osmp, pcm = bytearray(), [], [], []
    base = 0
    for s in parts:
        fo = s.frame_offsets.astype(np.int64)
        offs.append(fo + len(data))
        nsamp = np.full(len(fo), 4096, dtype=np.int64)
        nsamp[-1] = s.nsamples - 4096 * (len(fo) - 1)
        osmp.append(base + np.concatenate([[0], np.cumsum(nsamp)[:-1]]))
        pcm.append(s.pcm)
        data += s.data.tobytes()
        base += s.nsamples
    # frame i of each part in turn, so the classes alternate before the decode order sorts them
    order = [(p, i) for i in range(n_each) for p in range(len(parts))]
    o = np.array([offs[p][i] for p, i in order], dtype=np.int64)
    os_ = np.array([osmp[p][i] for p, i in order], dtype=np.int64)
    return bytes(data), o, os_, np.concatenate(pcm), base


def _decode(data, offs, osmp, total):
    import torch
    from birdnest.audio_amd import libflac
    dev = torch.device("cuda:0")
    sp = libflac.StreamParams(1, 4096, 4096, 44100, 2, 16, total)
    n = len(data)
    d_bytes = torch.zeros((n + 3) // 4 * 4 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:n] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    d_offs = torch.from_numpy(offs).to(dev)
    d_os = torch.from_numpy(osmp).to(dev)
    stride = libflac.out_stride(libflac.OUT_INTERLEAVED32, sp)
    d_out = torch.full((total * stride,), 0xAB, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(len(offs) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    libflac.BatchDecoder(0).decode_frames(d_bytes, n, d_offs, len(offs), sp, libflac.OUT_INTERLEAVED32, d_out,
                                          d_info, d_out_sample=d_os)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), libflac.info_array(d_info.cpu().numpy())


@pytest.mark.skipif(not gpu_available(), reason="no GPU")
@pytest.mark.parametrize("n_each", [7, 20, 45])
def test_mixed_classes_with_handbacks(n_each):
    data, offs, osmp, pcm, total = _mixed_batch(n_each)
    out, info = _decode(data, offs, osmp, total)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_REDO).any(), "the batch should hold handed-back stereo frames"
    assert np.array_equal(out.view("<i4").reshape(-1, 2), pcm)


_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from tests.test_gpu_decode_classes import _mixed_batch, _decode
data, offs, osmp, pcm, total = _mixed_batch(20)
out, info = _decode(data, offs, osmp, total)
sys.stdout.buffer.write(out.tobytes())
"""


@pytest.mark.skipif(not gpu_available(), reason="no GPU")
@pytest.mark.parametrize("env", [{"BNFLAC_DECODE_SERIAL": "1"}, {"BNFLAC_DECODE_FORK": "1"}])
def test_side_stream_matches_other_orders(env):
    data, offs, osmp, pcm, total = _mixed_batch(20)
    out, _ = _decode(data, offs, osmp, total)
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=dict(os.environ, BNFLAC_DECODE_SYS="0", **env),
                       capture_output=True, timeout=100)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout == out.tobytes()


def _plain_c2(nframes):
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config("C2", nframes=nframes, seed=44))
    fo = s.frame_offsets.astype(np.int64)
    osmp = np.arange(len(fo), dtype=np.int64) * 4096
    return s.data.tobytes(), fo, osmp, s.pcm, s.nsamples


@pytest.mark.skipif(not gpu_available(), reason="no GPU")
@pytest.mark.parametrize("n_each", [7, 45])
def test_segment_grid_after_batch_without_w16_w32(n_each):
    from birdnest.audio_amd import libflac
    L = libflac.load()
    data, offs, osmp, pcm, total = _plain_c2(40)
    out, info = _decode(data, offs, osmp, total)  # records W16 = W32 = 0 for the next decode
    assert np.array_equal(out.view("<i4").reshape(-1, 2), pcm)
    data, offs, osmp, pcm, total = _mixed_batch(n_each)
    n0 = L.bnflac_debug_decode_seg_launches()
    out, info = _decode(data, offs, osmp, total)  # W16 + W32 through k_decode_seg
    assert L.bnflac_debug_decode_seg_launches() == n0 + 1
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert np.array_equal(out.view("<i4").reshape(-1, 2), pcm)
    out2, info2 = _decode(data, offs, osmp, total)  # this batch had both: the side grids again
    assert L.bnflac_debug_decode_seg_launches() == n0 + 1
    assert out2.tobytes() == out.tobytes() and info2.tobytes() == info.tobytes()


@pytest.mark.skipif(not gpu_available(), reason="no GPU")
@pytest.mark.parametrize("n_each", [9, 40])
def test_w8_split_launches(n_each):
    """k_decode<8> as two launches (the class-1 frames on a third side stream beside
    k_decode_st, the stereo hand-backs after it) once the previous decode order had class-1
    frames: the same bytes and records as the single launch (host bit 0x100000)."""
    from birdnest.audio_amd import libflac
    L = libflac.load()
    data, offs, osmp, pcm, total = _mixed_batch(n_each, class1=True)
    _decode(data, offs, osmp, total)  # records the class-1 count for the next decode
    out, info = _decode(data, offs, osmp, total)
    assert (info["status"] == 0).all() and (info["crc_ok"] == 1).all()
    assert (info["flags"] & FL_REDO).any(), "the batch should hold handed-back stereo frames"
    assert np.array_equal(out.view("<i4").reshape(-1, 2), pcm)
    L.bnflac_debug_set_ablate(0x100000)
    try:
        out1, info1 = _decode(data, offs, osmp, total)
    finally:
        L.bnflac_debug_set_ablate(0)
    assert out1.tobytes() == out.tobytes() and info1.tobytes() == info.tobytes()
