"""FLACFileReader on the GPU stream API (init_file + ProcessSingle + carry-over) against the
oracle's replay of the same C# code (FLACFileReader.cs:45-78, 145-254, 267-341).

birdnest.audio_amd.flac_file_reader mirrors the C# class member by member and drives
libbnflac.so's FLAC__stream_decoder_init_file / process_single exactly as the C# does;
oracle.filereader_readall replays the same C# over the CPU restatement.  Bytes returned,
exception type/message and the point where they occur must be identical -- including the
reader's quirks: m_samplesPerChannel fixed by the first frame (stale tail on a short last
frame, truncation of longer frames), carry-over between Read calls, copies that run to the
buffer's Length (overfill), IndexOutOfRange on a buffer that is not a whole number of samples,
NotSupported for depths other than 16/24, and libFLAC errors thrown from the error callback.
"""
import json
import os

import pytest

from tests.conftest import gpu_available

pytestmark = pytest.mark.gpu

GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(GOLD_DIR, "golden.json")))


@pytest.fixture(scope="module")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    from birdnest.audio_amd import flac_file_reader
    return flac_file_reader


def _cases(data):
    si = data[8:42] if data[:4] == b"fLaC" else bytes(34)
    x = int.from_bytes(si[10:18], "big")
    ch, bps = ((x >> 41) & 7) + 1, ((x >> 36) & 31) + 1
    maxbs = max(16, int.from_bytes(si[2:4], "big"))
    sf = ch * (3 if bps == 24 else 2)
    return [(maxbs * sf, None), (maxbs * sf // 2 + sf, None), (sf * 100 + 1, None), (maxbs * sf * 3, 7)]


def _check(fr, tmp_path, name, data):
    import oracle
    path = os.path.join(str(tmp_path), name + ".flac")
    with open(path, "wb") as f:
        f.write(data)
    for buf_len, nb in _cases(data):
        ref = oracle.filereader_readall(data, buf_len, nb)
        got = fr.read_all(path, buf_len, nb)
        assert (got[0], got[2]) == (ref[0], ref[2]), (name, buf_len, nb)
        assert got[1] == ref[1], (name, buf_len, nb, len(got[1]), len(ref[1]))


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] in ("roundtrip", "error")])
def test_filereader_fixture_vs_oracle(gpu, tmp_path, name):
    _check(gpu, tmp_path, name, open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read())


@pytest.mark.parametrize("cfg,kw", [("C3", dict(nframes=5, last_blocksize=3000)),
                                    ("C5", dict(nframes=3, last_blocksize=1500)),
                                    ("C4", dict(nframes=24, bps=24, seed=9)),
                                    ("C1", dict(nframes=8, last_blocksize=99))])
def test_filereader_configs_vs_oracle(gpu, tmp_path, cfg, kw):
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config(cfg, **kw))
    _check(gpu, tmp_path, cfg, s.data.tobytes())


def test_filereader_position_seek_from_write_callback(gpu, tmp_path):
    """Position: the next Read's write callback seeks from inside itself; the samples after the
    reposition point equal the source PCM (the first frame after a seek is copied with the
    reader's fixed m_samplesPerChannel, so only its well-defined prefix is compared)."""
    import numpy as np
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config("C3", nframes=8))
    path = os.path.join(str(tmp_path), "c3.flac")
    open(path, "wb").write(s.data.tobytes())
    r = gpu.FLACFileReader(path)
    try:
        ba = r.WaveFormat.BlockAlign
        buf = bytearray(8192 * ba)
        assert r.Read(buf, 0, len(buf)) == len(buf)
        target = 5 * 8192 + 100
        r.Position = target * ba
        n = r.Read(buf, 0, len(buf))
        assert n == len(buf)
        # the trimmed target frame: 8192 - 100 valid samples (the rest of the copy is past it)
        valid = (8192 - 100) * ba
        want = np.ascontiguousarray(s.pcm[target: target + 8192 - 100].astype("<i4")).view(np.uint8).reshape(-1, 4)[:, :3]
        assert bytes(buf[:valid]) == want.tobytes()
        assert r.Position == target * ba
        n = r.Read(buf, 0, len(buf))  # the frame after the target frame, complete
        want = np.ascontiguousarray(s.pcm[6 * 8192: 7 * 8192].astype("<i4")).view(np.uint8).reshape(-1, 4)[:, :3]
        assert bytes(buf[:n]) == want.tobytes()
    finally:
        r.Dispose()
