"""CPU: pin the oracle (oracle/flac_oracle.c) against the golden vectors.

The reference has no FLAC tests or fixtures; these tests pin the
CPU restatement with RFC 9639's known-answer stream, CRC-validated libFLAC-written
frames, lossless round trips, and the libFLAC/C# behaviours restated from the DLL.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from birdnest.audio_amd import synth

GOLD_DIR = os.path.join(os.path.dirname(__file__), "golden")
GOLD = json.load(open(os.path.join(GOLD_DIR, "golden.json")))


def _read(name):
    return open(os.path.join(GOLD_DIR, GOLD[name]["file"]), "rb").read()


def _sha(pcm):
    return hashlib.sha256(np.ascontiguousarray(pcm, dtype="<i4").tobytes()).hexdigest()


def test_crc_known_values():
    # CRC-8/0x07 and CRC-16/0x8005 (init 0) check values for "123456789"
    assert oracle.crc8(b"123456789") == 0xF4
    assert oracle.crc16(b"123456789") == 0xFEE8


def test_rfc9639_example1_known_answer():
    data = _read("rfc9639_ex1")
    ev, pcm = oracle.run(data)
    kinds = [e.kind for e in ev]
    assert oracle.EV_ERROR not in kinds  # CRC-8 and CRC-16 both verified
    got = oracle.interleave(ev, pcm)
    assert got.tolist() == GOLD["rfc9639_ex1"]["pcm"]
    assert hashlib.md5(got.astype("<i2").tobytes()).hexdigest() == GOLD["rfc9639_ex1"]["md5"]
    meta = [e for e in ev if e.kind == oracle.EV_METADATA][0]
    assert (meta.sample_rate, meta.channels, meta.bps, meta.sample_number) == (44100, 2, 16, 1)


def test_rfc9639_example2_frame1_crc_and_structure():
    g = GOLD["rfc9639_ex2_frame1"]
    data = _read("rfc9639_ex2_frame1")
    rc, res, planar = oracle.decode_frame_at(data, 0, oracle.StreamParams(*g["stream_params"]))
    assert rc == 0 and res.crc_ok == 1
    assert res.end_off == len(data) == g["end_off"]  # bit accounting lands exactly on the CRC-16
    assert (res.blocksize, res.channels, res.assignment, res.bps) == (16, 2, 2, 16)  # right-side stereo
    pcm = planar[: res.blocksize * 2].reshape(2, res.blocksize).T
    assert _sha(pcm) == g["pcm_sha256_oracle"]


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "roundtrip"])
def test_roundtrip_fixture(name):
    g = GOLD[name]
    data = _read(name)
    ev, pcm = oracle.run(data)
    assert not [e for e in ev if e.kind == oracle.EV_ERROR]
    got = oracle.interleave(ev, pcm)
    assert got.shape == (g["nsamples"], g["channels"])
    assert _sha(got) == g["pcm_sha256"]
    nbytes = (g["bps"] + 7) // 8
    b = np.ascontiguousarray(got, dtype="<i4").view(np.uint8).reshape(-1, 4)[:, :nbytes].tobytes()
    assert hashlib.md5(b).hexdigest() == g["md5"]  # STREAMINFO MD5 (libFLAC convention)


@pytest.mark.parametrize("name", [k for k, v in GOLD.items() if v["kind"] == "error"])
def test_error_fixture_sequences(name):
    g = GOLD[name]
    data = _read(name)
    ev, pcm = oracle.run(data)
    from tests.golden.make_golden import events_to_json  # same serialisation
    assert events_to_json(ev) == g["events"]
    rc, pk, msg, _ = oracle.flacdecoder_copyto(data)
    assert (rc, msg) == (g["flacdecoder_rc"], g["flacdecoder_msg"])


def test_crc_mismatch_zero_fills_and_reports_first():
    g = GOLD["err_crc16_mismatch"]
    ev, pcm = oracle.run(_read("err_crc16_mismatch"))
    i = [k for k, e in enumerate(ev) if e.kind == oracle.EV_ERROR][0]
    assert ev[i].status == 2  # FRAME_CRC_MISMATCH
    w = ev[i + 1]
    assert w.kind == oracle.EV_WRITE
    assert not pcm[w.pcm_offset: w.pcm_offset + w.blocksize * w.channels].any()


def test_write_abort_leaves_state_read_frame():
    # LibFlac.dll@0x10011bd3-0x10011be4: a non-CONTINUE write status returns false
    # without touching the state (SURVEY.md 8b's "Aborted" is corrected here).
    data = _read("c2_lpc8")
    ev, _ = oracle.run(data, write_abort_at=1)
    rets = [e for e in ev if e.kind == oracle.EV_RETURN]
    assert rets[-1].status == 0 and rets[-1].state == 3


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4", "C5"])
def test_config_roundtrip(cfg):
    p = synth.config(cfg, nframes=5, last_blocksize=0)
    s = synth.encode(p)
    ev, pcm = oracle.run(s.data.tobytes())
    assert not [e for e in ev if e.kind == oracle.EV_ERROR]
    assert np.array_equal(oracle.interleave(ev, pcm), s.pcm)


def test_long_rice_prefixes_roundtrip():
    """Impulses (generator impulse_permille): residuals whose unary prefixes run ~100 bits in
    partitions coded with small Rice parameters; the oracle's unary reader returns the source."""
    s = synth.encode(synth.config("C2", nframes=4, last_blocksize=0, impulse_permille=3))
    ev, pcm = oracle.run(s.data.tobytes())
    assert np.array_equal(oracle.interleave(ev, pcm), s.pcm)
    plain = synth.encode(synth.config("C2", nframes=4, last_blocksize=0))
    assert len(s.data) > len(plain.data)  # the impulses cost bits: they are in the stream


def test_flacdecoder_pack_rules():
    # FLACDecoder.cs:543-562 stereo: [L lo, L hi, R lo, R hi]
    s = synth.encode(synth.config("C2", nframes=3))
    rc, pk, msg, fmt = oracle.flacdecoder_copyto(s.data.tobytes(), copy_chunk=12345)
    assert rc == 0, msg
    assert pk == s.pcm.astype("<i2").tobytes()
    assert fmt[:3] == [2, 44100, 16]
    # >2 channels: channel 0 only (:564-577)
    s3 = synth.encode(synth.config("C2", channels=3, nframes=2, seed=7))
    rc, pk, msg, _ = oracle.flacdecoder_copyto(s3.data.tobytes())
    assert rc == 0 and pk == s3.pcm[:, 0].astype("<i2").tobytes()
    # 24-bit: WriteCallback aborts (:526-530) -> "Could not process single - ReadFrame!"
    s24 = synth.encode(synth.config("C3", nframes=2))
    rc, pk, msg, _ = oracle.flacdecoder_copyto(s24.data.tobytes())
    assert rc == 1 and msg == "FLAC: Could not process single - ReadFrame!" and pk == b""


def test_filereader_pack_rules_24bit_and_quirks():
    # FLACFileReader.cs:230-237: 3 bytes LE per sample, all channels interleaved
    s = synth.encode(synth.config("C3", nframes=3))
    rc, pk, msg = oracle.filereader_readall(s.data.tobytes(), buf_len=8192 * 6)
    assert rc == 0, msg
    want = np.ascontiguousarray(s.pcm, dtype="<i4").view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    assert pk == want
    # stale tail: a short last frame copies m_samplesPerChannel samples per channel
    p = synth.config("C1", nframes=3, last_blocksize=1000)
    s = synth.encode(p)
    rc, pk, msg = oracle.filereader_readall(s.data.tobytes(), buf_len=4096 * 4)
    assert rc == 0
    assert len(pk) == 3 * 4096 * 4  # 2 full frames + a "full" last frame
    assert pk[: (2 * 4096 + 1000) * 4] == s.pcm.astype("<i2").tobytes()


def test_generator_md5_and_determinism():
    p = synth.config("C2", nframes=3)
    a, b = synth.encode(p), synth.encode(p)
    assert np.array_equal(a.data, b.data) and np.array_equal(a.pcm, b.pcm)
    assert bytes(a.data[26:42]) == synth.md5(a.pcm.astype("<i2").tobytes())
    assert bytes(a.data[26:42]) == hashlib.md5(a.pcm.astype("<i2").tobytes()).digest()


def test_oracle_seek_from_write_callback_delivers_source_pcm():
    """oracle_seek_absolute (libFLAC 1.2.1 seek_absolute semantics) in FLACFileReader's
    pattern: the nested write delivers the target frame trimmed, decoding continues after
    it, every sample equals the generator's source PCM; a target past the end is refused."""
    import oracle
    from birdnest.audio_amd import synth
    s = synth.encode(synth.config("C4", nframes=30, seed=21))
    data = s.data.tobytes()
    n = s.pcm.shape[0]
    for seeks in ([(2, n // 2 + 11)], [(-1, 77), (4, n - 1)], [(-2, 5000)]):
        ev, pcm = oracle.run_seek(data, seeks)
        kinds = [e.kind for e in ev]
        assert kinds.count(oracle.EV_SEEK) == len(seeks)
        assert all(e.status == 1 for e in ev if e.kind == oracle.EV_SEEK)
        if seeks[0][0] == -2:
            assert oracle.EV_METADATA not in kinds
        # the writes after the last seek are the source PCM from its target on
        last = max(i for i, e in enumerate(ev) if e.kind == oracle.EV_SEEK)
        first_w = max(i for i, e in enumerate(ev[:last]) if e.kind == oracle.EV_WRITE)
        tail = [e for e in ev[first_w:] if e.kind == oracle.EV_WRITE]
        assert tail[0].sample_number == seeks[-1][1]
        got = np.concatenate([pcm[e.pcm_offset: e.pcm_offset + e.blocksize * e.channels]
                              .reshape(e.channels, e.blocksize).T for e in tail])
        assert np.array_equal(got, s.pcm[seeks[-1][1]:])
    ev, pcm = oracle.run_seek(data, [(1, n)])
    assert [e.status for e in ev if e.kind == oracle.EV_SEEK] == [0]
