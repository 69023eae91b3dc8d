"""Synthetic FLAC workloads (ctypes over libbnflac_synth.so).

The generator is this repository's own encoder (csrc/synth/bnflac_synth.c); the reference
ships none.  ``CONFIGS`` maps BASELINE.json's configs to generator parameters
(SURVEY.md 8d).  Generating input is not the decode path.
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
from typing import Optional

import numpy as np

from ._lib import lib_path

SUB_LPC, SUB_FIXED, SUB_VERBATIM, SUB_CONSTANT, SUB_MIXED = 0, 1, 2, 3, 4
ST_INDEP, ST_LEFT_SIDE, ST_RIGHT_SIDE, ST_MID_SIDE, ST_CYCLE = 0, 1, 2, 3, 4


class _Params(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_uint32), ("channels", ctypes.c_uint32), ("bps", ctypes.c_uint32),
        ("blocksize", ctypes.c_uint32), ("nframes", ctypes.c_uint32), ("last_blocksize", ctypes.c_uint32),
        ("subframe_mode", ctypes.c_int32), ("order", ctypes.c_uint32), ("qlp_precision", ctypes.c_uint32),
        ("partition_order", ctypes.c_int32), ("stereo_mode", ctypes.c_int32),
        ("wasted_bits_max", ctypes.c_uint32), ("variable_blocksize", ctypes.c_int32),
        ("bs_min", ctypes.c_uint32), ("bs_max", ctypes.c_uint32), ("level", ctypes.c_double),
        ("noise", ctypes.c_double), ("seed", ctypes.c_uint64), ("rice2", ctypes.c_int32),
        ("escape_permille", ctypes.c_int32), ("write_header", ctypes.c_int32),
        ("force_sr_code", ctypes.c_int32), ("odd_headers", ctypes.c_int32),
        ("prec_clamp", ctypes.c_int32), ("impulse_permille", ctypes.c_int32),
    ]


@dataclasses.dataclass
class SynthParams:
    sample_rate: int = 44100
    channels: int = 2
    bps: int = 16
    blocksize: int = 4096
    nframes: int = 16
    last_blocksize: int = 0
    subframe_mode: int = SUB_LPC
    order: int = 8
    qlp_precision: int = 0
    partition_order: int = 4
    stereo_mode: int = ST_INDEP
    wasted_bits_max: int = 0
    variable_blocksize: int = 0
    bs_min: int = 192
    bs_max: int = 16384
    level: float = 0.5
    noise: float = 0.006
    seed: int = 1
    rice2: int = 0
    escape_permille: int = 0
    write_header: int = 1
    force_sr_code: int = -1
    odd_headers: int = 0
    prec_clamp: int = 0   # 1: libFLAC encoder's precision clamp (see bnflac_synth.c)
    impulse_permille: int = 0  # impulses of 0.4 x full scale per 1000 samples (long Rice prefixes)


@dataclasses.dataclass
class SynthStream:
    data: np.ndarray            # uint8 FLAC bytes
    pcm: np.ndarray             # int32 interleaved [samples, channels] -- the expected output
    frame_offsets: np.ndarray   # uint64 byte offset of each frame
    params: SynthParams

    @property
    def nsamples(self) -> int:
        return int(self.pcm.shape[0])


# BASELINE.json configs -> generator parameters
CONFIGS = {
    # C1: 44.1k/16/2ch, 10 s, bs 4096 (107 x 4096 + 2728), FIXED-2
    "C1": SynthParams(nframes=108, blocksize=4096, last_blocksize=441000 - 107 * 4096,
                      subframe_mode=SUB_FIXED, order=2, partition_order=-1, stereo_mode=ST_CYCLE, seed=1),
    # C2: 1024 frames x bs 4096, 44.1k/16/2ch, LPC-8, Rice partition order 4.  LPC precision
    # clamped the way libFLAC 1.2.1's encoder does for 16-bit input, so subframes use the
    # 32-bit restore paths as in real files; the unclamped 64-bit path is covered by tests.
    "C2": SynthParams(nframes=1024, blocksize=4096, subframe_mode=SUB_LPC, order=8,
                      partition_order=4, stereo_mode=ST_INDEP, seed=2, prec_clamp=1),
    # C3: 96k/24/2ch, LPC-12, bs 8192, wasted bits + mid/side (1024 frames)
    "C3": SynthParams(sample_rate=96000, bps=24, nframes=1024, blocksize=8192, subframe_mode=SUB_LPC,
                      order=12, partition_order=-1, stereo_mode=ST_MID_SIDE, wasted_bits_max=4,
                      noise=0.0004, seed=3),
    # C4: 4096 frames, variable bs 192-16384, mixed CONSTANT/VERBATIM/FIXED/LPC, 16/2ch
    "C4": SynthParams(nframes=4096, variable_blocksize=1, bs_min=192, bs_max=16384,
                      subframe_mode=SUB_MIXED, partition_order=-1, stereo_mode=ST_CYCLE, seed=4),
    # C5: 192k/24/8ch, LPC-32, bs 4096, 10 s per file (469 frames, last 3840)
    "C5": SynthParams(sample_rate=192000, bps=24, channels=8, nframes=469, blocksize=4096,
                      last_blocksize=1920000 - 468 * 4096, subframe_mode=SUB_LPC, order=32,
                      partition_order=-1, noise=0.0004, seed=5),
}


def _lib():
    lib = ctypes.CDLL(lib_path("libbnflac_synth.so"))
    lib.bnsyn_encode.restype = ctypes.c_int
    lib.bnsyn_max_bytes.restype = ctypes.c_size_t
    return lib


_LIB = None


def _get():
    global _LIB
    if _LIB is None:
        _LIB = _lib()
    return _LIB


def encode(p: SynthParams) -> SynthStream:
    lib = _get()
    cp = _Params(**dataclasses.asdict(p))
    cap = int(lib.bnsyn_max_bytes(ctypes.byref(cp)))
    out = np.zeros(cap, dtype=np.uint8)
    max_bs = p.bs_max if p.variable_blocksize else max(p.blocksize, p.last_blocksize)
    pcm_cap = int(p.nframes) * int(max_bs) * int(p.channels)
    pcm = np.zeros(pcm_cap, dtype=np.int32)
    offs = np.zeros(p.nframes, dtype=np.uint64)
    out_len = ctypes.c_size_t()
    pcm_len = ctypes.c_size_t()
    nfr = ctypes.c_uint32()
    rc = lib.bnsyn_encode(ctypes.byref(cp), out.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(cap),
                          ctypes.byref(out_len), pcm.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(pcm_cap),
                          ctypes.byref(pcm_len), offs.ctypes.data_as(ctypes.c_void_p),
                          ctypes.c_size_t(p.nframes), ctypes.byref(nfr))
    if rc != 0:
        raise RuntimeError(f"bnsyn_encode failed rc={rc}")
    data = out[: out_len.value].copy()
    pcm = pcm[: pcm_len.value].reshape(-1, p.channels).copy()
    return SynthStream(data=data, pcm=pcm, frame_offsets=offs, params=p)


def md5(buf: bytes) -> bytes:
    lib = _get()
    out = (ctypes.c_uint8 * 16)()
    lib.bnsyn_md5(ctypes.c_char_p(buf), ctypes.c_size_t(len(buf)), out)
    return bytes(out)


def config(name: str, **overrides) -> SynthParams:
    return dataclasses.replace(CONFIGS[name], **overrides)
