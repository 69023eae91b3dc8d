"""Regenerate the golden fixtures in tests/golden/.

Sources of truth, strongest first:
  1. RFC 9639 Appendix D.1 "decoding example 1" (a complete 1-sample stereo stream):
     its STREAMINFO MD5, CRC-8 and CRC-16 were written by an independent encoder, and
     the decoded samples (25588, 10416) are stated in the RFC.
  2. RFC 9639 Appendix D.2, first frame (written by "reference libFLAC 1.3.3"):
     FIXED subframes, right-side stereo, partitioned Rice -- its CRC-8/CRC-16 pin the
     parser's bit accounting; the sample values are oracle-derived (regression only).
  3. Lossless round trips: streams from our generator (birdnest/audio_amd/csrc/synth);
     the generator's source PCM is the expected output, and its STREAMINFO MD5 covers it.
  4. Corrupted-stream cases: the expected libFLAC callback sequences come from the
     oracle (oracle/flac_oracle.c) -- regression pins of the restated behaviour.

The reference repository itself holds no FLAC fixtures and its
LibFlac.dll is never executed, so nothing here comes from running the reference.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from birdnest.audio_amd import synth  # noqa: E402

RFC_EX1 = ("664c614380000022100010000000 0f00000f0ac442f0000000013e84b41807dc69030758"
           "6a3dad1a2e0ffff869180000bf0358fd03128baa9a").replace(" ", "")
RFC_EX2_FRAME1 = ("fff86998000f9912086701623d1442998f5df70d6fe00c17caeb21000ee7a77a24a1590c1217b603097b784faa9a33d2"
                  "85e070ad5b1b4851b4010d99d2cd1a68f1e6b810")

# small round-trip streams per BASELINE config (config shape, few frames)
SYNTH_CASES = {
    "c1_fixed2": dict(base="C1", nframes=6, last_blocksize=2728),
    "c2_lpc8": dict(base="C2", nframes=4),
    "c3_lpc12_ms_wasted": dict(base="C3", nframes=3),
    "c4_mixed_varbs": dict(base="C4", nframes=24, bs_max=4096),
    "c5_lpc32_8ch": dict(base="C5", nframes=2, last_blocksize=0),
    "rice2_escape": dict(base="C2", nframes=4, rice2=1, escape_permille=150, seed=11),
    "mono_8bit_fixed": dict(base="C1", channels=1, bps=8, nframes=3, last_blocksize=0, subframe_mode=1, order=3,
                            seed=12),
    "odd_headers_20bit": dict(base="C2", bps=20, sample_rate=22222, nframes=4, odd_headers=1, stereo_mode=4,
                              seed=13),
    "verbatim_12bit_3ch": dict(base="C2", bps=12, channels=3, nframes=3, subframe_mode=2, seed=14),
    "lpc_orders_lowprec": dict(base="C2", nframes=4, order=3, qlp_precision=5, stereo_mode=4, seed=15),
}


def pcm_sha(pcm: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(pcm, dtype="<i4").tobytes()).hexdigest()


def events_to_json(ev):
    out = []
    for e in ev:
        if e.kind == oracle.EV_WRITE:
            out.append(["W", e.blocksize, e.channels, e.assignment, e.bps, e.sample_number])
        elif e.kind == oracle.EV_ERROR:
            out.append(["E", e.status, e.state])
        elif e.kind == oracle.EV_METADATA:
            out.append(["M", e.status])
        else:
            out.append(["R", e.status, e.state])
    return out


def corrupt_cases(data: bytes, offsets):
    """(name, bytes) corrupted variants of a 4-frame stream."""
    d = bytearray(data)
    o = [int(x) for x in offsets]
    cases = []
    x = bytearray(d); x[o[1] + 40] ^= 0x10; cases.append(("crc16_mismatch", bytes(x)))
    x = bytearray(d); x[o[2] + 4] ^= 0x01; cases.append(("header_crc8_bad", bytes(x)))
    x = bytearray(d); x[o[2]:o[2]] = b"\x00\x13\x37junk"; cases.append(("junk_lost_sync", bytes(x)))
    x = bytearray(d); x = x[: o[3] + (len(d) - o[3]) // 2]; cases.append(("truncated_last", bytes(x)))
    cases.append(("sync_in_header", bytes(d[: o[1] + 2]) + b"\xff" + bytes(d[o[1] + 3:])))
    x = bytearray(d); x[o[1] + 1] = 0xFA; cases.append(("reserved_bit_unparseable", bytes(x)))
    return cases


def main():
    gold = {}
    # 1. RFC 9639 D.1
    ex1 = bytes.fromhex(RFC_EX1)
    open(os.path.join(HERE, "rfc9639_ex1.flac"), "wb").write(ex1)
    gold["rfc9639_ex1"] = {"file": "rfc9639_ex1.flac", "kind": "rfc", "pcm": [[25588, 10416]],
                           "md5": "3e84b41807dc690307586a3dad1a2e0f"}
    # 2. RFC 9639 D.2 frame 1
    fr = bytes.fromhex(RFC_EX2_FRAME1)
    open(os.path.join(HERE, "rfc9639_ex2_frame1.bin"), "wb").write(fr)
    sp = oracle.StreamParams(1, 16, 16, 44100, 2, 16, 19)
    rc, res, planar = oracle.decode_frame_at(fr, 0, sp)
    assert rc == 0 and res.crc_ok == 1, (rc, res.error)
    pcm = planar[: res.blocksize * res.channels].reshape(res.channels, res.blocksize).T
    gold["rfc9639_ex2_frame1"] = {"file": "rfc9639_ex2_frame1.bin", "kind": "rfc_frame", "blocksize": res.blocksize,
                                  "assignment": res.assignment, "channels": res.channels, "bps": res.bps,
                                  "end_off": int(res.end_off), "pcm_sha256_oracle": pcm_sha(pcm),
                                  "stream_params": [1, 16, 16, 44100, 2, 16, 19]}
    # 3. synthetic round trips
    for name, kw in SYNTH_CASES.items():
        kw = dict(kw)
        base = kw.pop("base")
        p = synth.config(base, **kw)
        s = synth.encode(p)
        fn = name + ".flac"
        open(os.path.join(HERE, fn), "wb").write(s.data.tobytes())
        md5 = bytes(s.data[26:42]).hex()
        ev, opcm = oracle.run(s.data.tobytes())
        assert np.array_equal(oracle.interleave(ev, opcm), s.pcm), name
        gold[name] = {"file": fn, "kind": "roundtrip", "channels": p.channels, "bps": p.bps, "nframes": p.nframes,
                      "nsamples": int(s.nsamples), "pcm_sha256": pcm_sha(s.pcm), "md5": md5,
                      "frame_offsets": [int(x) for x in s.frame_offsets], "params": kw | {"base": base}}
    # 4. corrupted streams (oracle event sequences)
    p = synth.config("C2", nframes=4, blocksize=1024, seed=21)
    s = synth.encode(p)
    for name, data in corrupt_cases(s.data.tobytes(), s.frame_offsets):
        fn = "err_" + name + ".flac"
        open(os.path.join(HERE, fn), "wb").write(data)
        ev, opcm = oracle.run(data)
        rc, pk, msg, _ = oracle.flacdecoder_copyto(data)
        gold["err_" + name] = {"file": fn, "kind": "error", "events": events_to_json(ev),
                               "pcm_sha256_oracle": pcm_sha(opcm), "flacdecoder_rc": rc, "flacdecoder_msg": msg,
                               "flacdecoder_sha256": hashlib.sha256(pk).hexdigest()}
    json.dump(gold, open(os.path.join(HERE, "golden.json"), "w"), indent=1, sort_keys=True)
    print(f"wrote {len(gold)} fixtures")


if __name__ == "__main__":
    main()
