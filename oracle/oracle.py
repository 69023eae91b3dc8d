"""ctypes bindings for the CPU oracle (oracle/flac_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "liboracle.so")

EV_METADATA, EV_WRITE, EV_ERROR, EV_RETURN, EV_SEEK = 1, 2, 3, 4, 5


class Event(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("status", ctypes.c_int32), ("state", ctypes.c_int32),
                ("blocksize", ctypes.c_uint32), ("sample_rate", ctypes.c_uint32), ("channels", ctypes.c_uint32),
                ("assignment", ctypes.c_uint32), ("bps", ctypes.c_uint32), ("crc8", ctypes.c_uint32),
                ("sample_number", ctypes.c_uint64), ("pcm_offset", ctypes.c_uint64)]

    def as_tuple(self):
        return (self.kind, self.status, self.state, self.blocksize, self.sample_rate, self.channels,
                self.assignment, self.bps, self.sample_number)


class StreamParams(ctypes.Structure):
    _fields_ = [("has_stream_info", ctypes.c_int32), ("min_blocksize", ctypes.c_uint32),
                ("max_blocksize", ctypes.c_uint32), ("sample_rate", ctypes.c_uint32),
                ("channels", ctypes.c_uint32), ("bps", ctypes.c_uint32), ("total_samples", ctypes.c_uint64)]


class FrameResult(ctypes.Structure):
    _fields_ = [("error", ctypes.c_int32), ("crc_ok", ctypes.c_int32), ("blocksize", ctypes.c_uint32),
                ("sample_rate", ctypes.c_uint32), ("channels", ctypes.c_uint32), ("assignment", ctypes.c_uint32),
                ("bps", ctypes.c_uint32), ("number_type", ctypes.c_uint32), ("number", ctypes.c_uint64),
                ("end_off", ctypes.c_uint64), ("cached", ctypes.c_int32)]


def build() -> str:
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(
            os.path.getmtime(os.path.join(HERE, f)) for f in ("flac_oracle.c", "flac_oracle.h")):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return SO


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        _LIB.oracle_crc16.restype = ctypes.c_uint16
        _LIB.oracle_crc8.restype = ctypes.c_uint8
    return _LIB


def _buf(data):
    data = bytes(data)
    return ctypes.create_string_buffer(data, len(data)), len(data)


def run(data, driver=0, read_chunk=16384, write_abort_at=-1, max_events=None, max_pcm=None):
    """Decode a whole stream; returns (events, pcm) with pcm planar-per-frame int32."""
    b, n = _buf(data)
    max_events = max_events or 4096 + n // 8
    max_pcm = max_pcm or 1 << 22
    ev = (Event * max_events)()
    nev = ctypes.c_int()
    pcm = np.zeros(max_pcm, dtype=np.int32)
    npcm = ctypes.c_size_t()
    rc = lib().oracle_run(b, ctypes.c_size_t(n), driver, read_chunk, write_abort_at, ev, max_events,
                          ctypes.byref(nev), pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(max_pcm),
                          ctypes.byref(npcm))
    if rc != 0:
        raise RuntimeError(f"oracle_run rc={rc}")
    if npcm.value > max_pcm:
        return run(data, driver, read_chunk, write_abort_at, max_events, int(npcm.value))
    return list(ev[: nev.value]), pcm[: npcm.value].copy()


def run_seek(data, seeks, read_chunk=16384, max_events=None, max_pcm=None):
    """FLACFileReader's seek pattern (seek_absolute from inside the write callback): seeks is a
    list of (write_index | -1, target_sample); returns (events, pcm) like run()."""
    b, n = _buf(data)
    max_events = max_events or 4096 + n // 8
    max_pcm = max_pcm or 1 << 22
    ev = (Event * max_events)()
    nev = ctypes.c_int()
    pcm = np.zeros(max_pcm, dtype=np.int32)
    npcm = ctypes.c_size_t()
    arr = (ctypes.c_int64 * (2 * max(1, len(seeks))))(*[v for sk in seeks for v in sk])
    rc = lib().oracle_run_seek(b, ctypes.c_size_t(n), read_chunk, arr, len(seeks), ev, max_events, ctypes.byref(nev),
                               pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(max_pcm), ctypes.byref(npcm))
    if rc != 0:
        raise RuntimeError(f"oracle_run_seek rc={rc}")
    if npcm.value > max_pcm:
        return run_seek(data, seeks, read_chunk, max_events, int(npcm.value))
    return list(ev[: nev.value]), pcm[: npcm.value].copy()


def interleave(events, pcm):
    """Planar-per-frame oracle PCM -> interleaved [samples, channels] array."""
    out = []
    for e in events:
        if e.kind != EV_WRITE:
            continue
        n = e.blocksize * e.channels
        fr = pcm[e.pcm_offset: e.pcm_offset + n].reshape(e.channels, e.blocksize)
        out.append(fr.T)
    if not out:
        return np.zeros((0, 0), dtype=np.int32)
    return np.concatenate(out, axis=0)


def decode_frame_at(data, off, sp: StreamParams | None, planar_cap=8 * 65536):
    b, n = _buf(data)
    planar = np.zeros(planar_cap, dtype=np.int32)
    res = FrameResult()
    rc = lib().oracle_decode_frame_at(b, ctypes.c_size_t(n), ctypes.c_size_t(off),
                                      ctypes.byref(sp) if sp is not None else None,
                                      planar.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(planar_cap),
                                      ctypes.byref(res))
    return rc, res, planar


def flacdecoder_copyto(data, copy_chunk=81920):
    b, n = _buf(data)
    cap = n * 8 + (1 << 20)
    out = np.zeros(cap, dtype=np.uint8)
    olen = ctypes.c_size_t()
    fmt = (ctypes.c_int32 * 4)()
    msg = ctypes.create_string_buffer(512)
    rc = lib().oracle_flacdecoder_copyto(b, ctypes.c_size_t(n), copy_chunk, out.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.c_size_t(cap), ctypes.byref(olen), fmt, msg, 512)
    return rc, out[: olen.value].tobytes(), msg.value.decode(), list(fmt)


def filereader_readall(data, buf_len=4096 * 6, num_bytes=None):
    """FLACFileReader ctor + Read(buf, 0, num_bytes) on a buf_len-byte buffer until it returns
    0 (num_bytes defaults to buf_len).  -> (rc, bytes of every returned read, message)."""
    b, n = _buf(data)
    cap = n * 8 + (1 << 20)
    out = np.zeros(cap, dtype=np.uint8)
    olen = ctypes.c_size_t()
    msg = ctypes.create_string_buffer(512)
    rc = lib().oracle_filereader_readall_n(b, ctypes.c_size_t(n), buf_len, buf_len if num_bytes is None else num_bytes,
                                           out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap),
                                           ctypes.byref(olen), msg, 512)
    return rc, out[: olen.value].tobytes(), msg.value.decode()


def crc8(data) -> int:
    b, n = _buf(data)
    return int(lib().oracle_crc8(b, ctypes.c_size_t(n)))


def crc16(data) -> int:
    b, n = _buf(data)
    return int(lib().oracle_crc16(b, ctypes.c_size_t(n)))
