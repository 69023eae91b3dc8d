"""Callback-sequence driver for libbnflac.so's libFLAC API.

Drives FLAC__stream_decoder_* exactly like oracle/flac_oracle.c's ``oracle_run`` drives
the CPU restatement (same read-callback behaviour as FLACDecoder.ReadCallback,
FLACDecoder.cs:325-363), and records the same event tuples, so tests can compare the
GPU-backed decoder and the oracle event by event.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .libflac import (LibFLAC, DecoderEofCallback, DecoderReadCallback, DecoderWriteCallbackWithStatus,
                      Decoder_ErrorCallback, Decoder_MetadataCallback, load)

EV_METADATA, EV_WRITE, EV_ERROR, EV_RETURN, EV_SEEK = 1, 2, 3, 4, 5


def run(data: bytes, driver: int = 0, read_chunk: int = 16384, write_abort_at: int = -1, md5_check: bool = False,
        seeks=None, stats=None):
    """-> (events, pcm); with md5_check, MD5 checking is enabled before init and the
    result is (events, pcm, finish_ok) where finish_ok is FLAC__stream_decoder_finish's
    return (false on an MD5 mismatch).

    seeks: FLACFileReader's seek pattern (FLACFileReader.cs:125-136, 267-301) as oracle.run_seek
    drives it -- a list of (write_index | -1, target_sample): after copying write number
    write_index the write callback itself calls seek_absolute (the trimmed target frame
    arrives through a nested write callback); -1 seeks right after the metadata pass.  The
    stream then has memory seek/tell/length callbacks, and every seek_absolute return is an
    EV_SEEK event."""
    L = load()
    data = bytes(data)
    st = {"pos": 0, "eof": False, "frames": 0}
    events = []
    pcm_parts = []
    npcm = [0]
    dec = L.FLAC__stream_decoder_new()
    if md5_check and not L.FLAC__stream_decoder_set_md5_checking(dec, 1):
        L.FLAC__stream_decoder_delete(dec)
        raise RuntimeError("set_md5_checking refused before init")
    finish_ok = None

    def state():
        return int(L.FLAC__stream_decoder_get_state(dec))

    def rd(d, buf, nbytes, ud):
        want = nbytes[0]
        if want == 0:
            st["eof"] = True
            return 2
        length = min(want, read_chunk)
        chunk = data[st["pos"]: st["pos"] + length]
        n = len(chunk)
        st["read_total"] = st.get("read_total", 0) + n
        if n:
            ctypes.memmove(buf, chunk, n)
        st["pos"] += n
        nbytes[0] = n
        if n < length:
            st["eof"] = True
            return 1
        return 0

    def eof(d, ud):
        return 1 if st["eof"] else 0

    seeks = list(seeks or [])
    nxt = [0]

    def do_seek():
        target = seeks[nxt[0]][1]
        nxt[0] += 1
        r = int(L.FLAC__stream_decoder_seek_absolute(dec, target))
        events.append((EV_SEEK, r, state(), 0, 0, 0, 0, 0, 0, 0))

    def sk(d, off, ud):
        if off > len(data):
            return 1
        st["pos"] = int(off)
        st["eof"] = False
        st["seek_calls"] = st.get("seek_calls", 0) + 1
        return 0

    def tl(d, off, ud):
        off[0] = st["pos"]
        return 0

    def ln(d, n, ud):
        n[0] = len(data)
        return 0

    def wr(d, frame, buf, ud):
        raw = ctypes.string_at(frame, 40)
        bs, sr, ch, asg, bps, _nt = np.frombuffer(raw[:24], dtype="<u4")
        sn = int.from_bytes(raw[24:32], "little")
        events.append((EV_WRITE, 0, state(), int(bs), int(sr), int(ch), int(asg), int(bps), sn, npcm[0]))
        for c in range(int(ch)):
            pcm_parts.append(np.ctypeslib.as_array(buf[c], shape=(int(bs),)).copy())
            npcm[0] += int(bs)
        idx = st["frames"]
        st["frames"] += 1
        if nxt[0] < len(seeks) and seeks[nxt[0]][0] == idx:
            do_seek()
        return 1 if idx == write_abort_at else 0

    def md(d, m, ud):
        raw = ctypes.string_at(m, 72)
        mtype = int.from_bytes(raw[0:4], "little")
        ev = [EV_METADATA, mtype, state(), 0, 0, 0, 0, 0, 0, 0]
        if mtype == 0:
            ev[3] = int.from_bytes(raw[20:24], "little")
            ev[4] = int.from_bytes(raw[32:36], "little")
            ev[5] = int.from_bytes(raw[36:40], "little")
            ev[7] = int.from_bytes(raw[40:44], "little")
            ev[8] = int.from_bytes(raw[48:56], "little")
        events.append(tuple(ev))

    def er(d, status, ud):
        events.append((EV_ERROR, int(status), state(), 0, 0, 0, 0, 0, 0, 0))

    from .libflac import DecoderSeekCallback, DecoderTellCallback, DecoderLengthCallback
    cbs = (DecoderReadCallback(rd), DecoderEofCallback(eof), DecoderWriteCallbackWithStatus(wr),
           Decoder_MetadataCallback(md), Decoder_ErrorCallback(er), DecoderSeekCallback(sk), DecoderTellCallback(tl),
           DecoderLengthCallback(ln))
    if seeks:
        rc = L.FLAC__stream_decoder_init_stream(dec, cbs[0], cbs[5], cbs[6], cbs[7], cbs[1], cbs[2], cbs[3], cbs[4],
                                                None)
    else:
        rc = L.FLAC__stream_decoder_init_stream(dec, cbs[0], _null(0), _null(1), _null(2), cbs[1], cbs[2], cbs[3],
                                                cbs[4], None)
    if rc != 0:
        L.FLAC__stream_decoder_delete(dec)
        raise RuntimeError(f"init_stream failed rc={rc}: {L.bnflac_last_error().decode()}")
    try:
        while nxt[0] < len(seeks) and seeks[nxt[0]][0] == -2:  # right after init: before the metadata pass
            do_seek()
        if driver == 0:
            ok = int(L.FLAC__stream_decoder_process_until_end_of_metadata(dec))
            events.append((EV_RETURN, ok, state(), 0, 0, 0, 0, 0, 0, 0))
            while ok and nxt[0] < len(seeks) and seeks[nxt[0]][0] < 0:
                do_seek()
            if ok:
                for _ in range(50_000_000):
                    if state() >= 4:
                        break
                    ok = int(L.FLAC__stream_decoder_process_single(dec))
                    events.append((EV_RETURN, ok, state(), 0, 0, 0, 0, 0, 0, 0))
                    if not ok:
                        break
        else:
            ok = int(L.FLAC__stream_decoder_process_until_end_of_stream(dec))
            events.append((EV_RETURN, ok, state(), 0, 0, 0, 0, 0, 0, 0))
        if md5_check:
            finish_ok = bool(L.FLAC__stream_decoder_finish(dec))
    finally:
        L.FLAC__stream_decoder_delete(dec)
    if stats is not None:
        stats["read_total"] = st.get("read_total", 0)
        stats["seek_calls"] = st.get("seek_calls", 0)
    pcm = np.concatenate(pcm_parts) if pcm_parts else np.zeros(0, dtype=np.int32)
    if md5_check:
        return events, pcm, finish_ok
    return events, pcm


def _null(kind):
    from .libflac import DecoderSeekCallback, DecoderTellCallback, DecoderLengthCallback
    return [DecoderSeekCallback, DecoderTellCallback, DecoderLengthCallback][kind]()


def oracle_events_as_tuples(events):
    """oracle.Event list -> tuples comparable with run()'s."""
    out = []
    for e in events:
        if e.kind == EV_WRITE:
            out.append((e.kind, 0, e.state, e.blocksize, e.sample_rate, e.channels, e.assignment, e.bps,
                        e.sample_number, e.pcm_offset))
        elif e.kind == EV_METADATA:
            ev = [e.kind, e.status, e.state, 0, 0, 0, 0, 0, 0, 0]
            if e.status == 0:
                ev[3], ev[4], ev[5], ev[7], ev[8] = e.blocksize, e.sample_rate, e.channels, e.bps, e.sample_number
            out.append(tuple(ev))
        else:
            out.append((e.kind, e.status, e.state, 0, 0, 0, 0, 0, 0, 0))
    return out
