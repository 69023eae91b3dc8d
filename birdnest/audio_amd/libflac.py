"""ctypes binding of libbnflac.so -- the Python mirror of LibFLACSharp.

``LibFLAC`` mirrors ``Library/LibFLACSharp/LibFLACSharp.cs`` (class LibFLAC, :18): the same
decoder entry points (:42-85, :175-185), enums (:24-36, :89-173, :248-280) and callback
delegate shapes (:187-212), bound to the MI355X library instead of the Win32 LibFlac.dll.
``BatchDecoder`` wraps the device-pointer API (include/bnflac.h part 2).

The library is GPU-only: loading works anywhere (symbol checks run on CPU-only hosts);
decoding without a usable GPU fails loudly.
"""
from __future__ import annotations

import ctypes
import enum
from typing import Optional

import numpy as np

from ._lib import lib_path


class StreamDecoderState(enum.IntEnum):  # LibFLACSharp.cs:24-36
    SearchForMetadata = 0
    ReadMetadata = 1
    SearchForFrameSync = 2
    ReadFrame = 3
    EndOfStream = 4
    OggError = 5
    SeekError = 6
    Aborted = 7
    MemoryAllocationError = 8
    Uninitialized = 9


class StreamDecoderReadStatus(enum.IntEnum):  # :89-110
    ReadStatusContinue = 0
    ReadStatusEndOfStream = 1
    ReadStatusAbort = 2


class StreamDecoderSeekStatus(enum.IntEnum):  # :113-127
    SeekStatusOk = 0
    SeekStatusError = 1
    SeekStatusUnsupported = 2


class StreamDecoderTellStatus(enum.IntEnum):  # :130-144
    TellStatusOK = 0
    TellStatusError = 1
    TellStatusUnsupported = 2


class StreamDecoderLengthStatus(enum.IntEnum):  # :147-161
    LengthStatusOk = 0
    LengthStatusError = 1
    LengthStatusUnsupported = 2


class StreamDecoderWriteStatus(enum.IntEnum):  # :163-173
    WriteStatusContinue = 0
    WriteStatusAbort = 1


class DecodeError(enum.IntEnum):  # :262-268
    LostSync = 0
    BadHeader = 1
    FrameCrcMismatch = 2
    UnparsableStream = 3


class FLACMetaDataType(enum.IntEnum):  # :270-280
    StreamInfo = 0
    Padding = 1
    Application = 2
    Seekable = 3
    VorbisComment = 4
    CueSheet = 5
    Picture = 6
    Undefined = 7


class FrameHeader(ctypes.Structure):  # :224-234 (offsets 0/4/8/12/16/20/24/32)
    _fields_ = [("BlockSize", ctypes.c_int32), ("SampleRate", ctypes.c_int32), ("Channels", ctypes.c_int32),
                ("ChannelAssignment", ctypes.c_int32), ("BitsPerSample", ctypes.c_int32),
                ("NumberType", ctypes.c_int32), ("FrameOrSampleNumber", ctypes.c_int64), ("Crc", ctypes.c_uint8)]


class FLACMetaData(ctypes.Structure):  # :282-293 (Data[] marshalled from offset 12)
    _pack_ = 4
    _fields_ = [("MetaDataType", ctypes.c_int32), ("IsLast", ctypes.c_int32), ("Length", ctypes.c_int32),
                ("Data", ctypes.c_uint8 * 100)]


class FLACStreamInfo(ctypes.Structure):  # :295-319 explicit layout over FLACMetaData.Data
    _pack_ = 1
    _fields_ = [("_hdr", ctypes.c_int32), ("MinBlocksize", ctypes.c_int32), ("MaxBlocksize", ctypes.c_int32),
                ("min_framesize", ctypes.c_int32), ("max_framesize", ctypes.c_int32), ("SampleRate", ctypes.c_int32),
                ("Channels", ctypes.c_int32), ("BitsPerSample", ctypes.c_int32), ("TotalSamplesHi", ctypes.c_int32),
                ("TotalSamplesLo", ctypes.c_int32)]


_DEC = ctypes.c_void_p
DecoderReadCallback = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.POINTER(ctypes.c_uint8),
                                       ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p)
DecoderSeekCallback = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.c_uint64, ctypes.c_void_p)
DecoderTellCallback = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)
DecoderLengthCallback = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)
DecoderEofCallback = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.c_void_p)
DecoderWriteCallbackWithStatus = ctypes.CFUNCTYPE(ctypes.c_int, _DEC, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)), ctypes.c_void_p)
Decoder_WriteCallback = DecoderWriteCallbackWithStatus  # declared void in C# (:205-206); see init_file
Decoder_MetadataCallback = ctypes.CFUNCTYPE(None, _DEC, ctypes.c_void_p, ctypes.c_void_p)
Decoder_ErrorCallback = ctypes.CFUNCTYPE(None, _DEC, ctypes.c_int, ctypes.c_void_p)

DECODER_SYMBOLS = [
    "FLAC__stream_decoder_new", "FLAC__stream_decoder_finish", "FLAC__stream_decoder_delete",
    "FLAC__stream_decoder_init_file", "FLAC__stream_decoder_process_single",
    "FLAC__stream_decoder_process_until_end_of_metadata", "FLAC__stream_decoder_process_until_end_of_stream",
    "FLAC__stream_decoder_seek_absolute", "FLAC__stream_decoder_get_decode_position",
    "FLAC__stream_decoder_get_total_samples", "FLAC__stream_decoder_get_channels",
    "FLAC__stream_decoder_get_bits_per_sample", "FLAC__stream_decoder_get_sample_rate",
    "FLAC__stream_decoder_get_state", "FLAC__stream_decoder_reset", "FLAC__stream_decoder_init_stream",
    "FLAC__stream_decoder_set_md5_checking", "FLAC__stream_decoder_get_md5_checking",
]
BATCH_SYMBOLS = ["bnflac_ctx_create", "bnflac_ctx_destroy", "bnflac_last_error", "bnflac_device_count",
                 "bnflac_index_frames", "bnflac_decode_frames", "bnflac_parse_frames", "bnflac_decode_parsed",
                 "bnflac_out_stride", "bnflac_debug_set_ablate", "bnflac_debug_stats", "bnflac_debug_set_parse_wave", "bnflac_debug_parse_wave_stats",
                 "bnflac_debug_set_decode_sys", "bnflac_debug_decode_seg_launches", "bnflac_md5_interleaved32", "bnflac_index_stream",
                 "bnflac_debug_set_crc_mode", "bnflac_debug_crc_handoff"]
READER_SYMBOLS = ["bnflac_reader_open", "bnflac_reader_params", "bnflac_reader_read", "bnflac_reader_close",
                  "bnflac_reader_last_error", "bnflac_reader_seek", "bnflac_reader_read_filereader",
                  "bnflac_reader_pool_release"]

_LIB = None


def load() -> ctypes.CDLL:
    """Load libbnflac.so and declare signatures (no GPU work)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    L = ctypes.CDLL(lib_path("libbnflac.so"))
    b, u, i, p = ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_void_p
    L.FLAC__stream_decoder_new.restype = p
    for n in ("finish", "delete", "process_single", "process_until_end_of_metadata",
              "process_until_end_of_stream", "reset"):
        f = getattr(L, "FLAC__stream_decoder_" + n)
        f.restype, f.argtypes = b, [p]
    L.FLAC__stream_decoder_init_file.restype = i
    L.FLAC__stream_decoder_init_file.argtypes = [p, ctypes.c_char_p, Decoder_WriteCallback,
                                                 Decoder_MetadataCallback, Decoder_ErrorCallback, p]
    L.FLAC__stream_decoder_init_stream.restype = i
    L.FLAC__stream_decoder_init_stream.argtypes = [p, DecoderReadCallback, DecoderSeekCallback, DecoderTellCallback,
                                                   DecoderLengthCallback, DecoderEofCallback,
                                                   DecoderWriteCallbackWithStatus, Decoder_MetadataCallback,
                                                   Decoder_ErrorCallback, p]
    L.FLAC__stream_decoder_seek_absolute.restype, L.FLAC__stream_decoder_seek_absolute.argtypes = b, [p, ctypes.c_uint64]
    L.FLAC__stream_decoder_get_decode_position.restype = b
    L.FLAC__stream_decoder_get_decode_position.argtypes = [p, ctypes.POINTER(ctypes.c_uint64)]
    L.FLAC__stream_decoder_get_total_samples.restype = ctypes.c_uint64
    L.FLAC__stream_decoder_get_total_samples.argtypes = [p]
    for n in ("get_channels", "get_bits_per_sample", "get_sample_rate", "get_state"):
        f = getattr(L, "FLAC__stream_decoder_" + n)
        f.restype, f.argtypes = u, [p]
    L.bnflac_last_error.restype = ctypes.c_char_p
    L.bnflac_ctx_create.restype, L.bnflac_ctx_create.argtypes = i, [i, ctypes.POINTER(p)]
    L.bnflac_ctx_destroy.argtypes = [p]
    L.bnflac_index_frames.restype = i
    L.bnflac_index_frames.argtypes = [p, p, ctypes.c_uint64, p, ctypes.c_uint32, p, p]
    L.bnflac_decode_frames.restype = i
    L.bnflac_decode_frames.argtypes = [p, p, ctypes.c_uint64, p, ctypes.c_uint32, p, p, ctypes.c_uint64, i, p,
                                       ctypes.c_uint64, p, p]
    L.bnflac_parse_frames.restype = i
    L.bnflac_parse_frames.argtypes = [p, p, ctypes.c_uint64, p, ctypes.c_uint32, p, p, ctypes.c_uint64, p, p]
    L.bnflac_decode_parsed.restype = i
    L.bnflac_decode_parsed.argtypes = [p, p, ctypes.c_uint64, ctypes.c_uint32, p, i, p, ctypes.c_uint64, p, p]
    L.bnflac_debug_set_ablate.argtypes = [ctypes.c_uint32]
    L.bnflac_debug_set_parse_wave.argtypes = [ctypes.c_int]
    L.bnflac_debug_set_decode_sys.argtypes = [ctypes.c_int]
    L.bnflac_debug_set_crc_mode.argtypes = [ctypes.c_int]
    L.bnflac_debug_crc_handoff.restype = i
    L.bnflac_debug_crc_handoff.argtypes = [p, p, ctypes.c_uint32]
    L.bnflac_debug_decode_seg_launches.restype, L.bnflac_debug_decode_seg_launches.argtypes = ctypes.c_uint64, []
    L.bnflac_debug_parse_wave_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.bnflac_debug_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.bnflac_debug_stats.restype = ctypes.c_int
    L.bnflac_out_stride.restype = ctypes.c_uint32
    L.bnflac_out_stride.argtypes = [i, p]
    L.FLAC__stream_decoder_set_md5_checking.restype = b
    L.FLAC__stream_decoder_set_md5_checking.argtypes = [p, b]
    L.FLAC__stream_decoder_get_md5_checking.restype = b
    L.FLAC__stream_decoder_get_md5_checking.argtypes = [p]
    L.bnflac_index_stream.restype = i
    L.bnflac_index_stream.argtypes = [p, p, ctypes.c_uint64, ctypes.c_uint64, p, p, p, p, ctypes.c_uint32, p, p]
    L.bnflac_reader_open.restype = i
    L.bnflac_reader_open.argtypes = [i, p, ctypes.c_uint64, i, ctypes.c_uint32, ctypes.POINTER(p)]
    L.bnflac_reader_params.restype = i
    L.bnflac_reader_params.argtypes = [p, p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]
    L.bnflac_reader_read.restype = ctypes.c_int64
    L.bnflac_reader_read.argtypes = [p, p, ctypes.c_uint64]
    L.bnflac_reader_close.argtypes = [p]
    L.bnflac_reader_pool_release.argtypes = [ctypes.c_int]
    L.bnflac_reader_pool_release.restype = ctypes.c_int
    L.bnflac_reader_read_filereader.restype = ctypes.c_int64
    L.bnflac_reader_read_filereader.argtypes = [p, p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    L.bnflac_reader_seek.restype = i
    L.bnflac_reader_seek.argtypes = [p, ctypes.c_uint64]
    L.bnflac_reader_last_error.restype = ctypes.c_char_p
    L.bnflac_md5_interleaved32.restype = i
    L.bnflac_md5_interleaved32.argtypes = [p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, p]
    _LIB = L
    return L


class LibFLAC:
    """Static-style facade named like the C# class (LibFLACSharp.cs:18)."""

    @staticmethod
    def _l():
        return load()

    @staticmethod
    def FLAC__stream_decoder_new():
        return LibFLAC._l().FLAC__stream_decoder_new()

    @staticmethod
    def FLAC__stream_decoder_finish(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_finish(ctx))

    @staticmethod
    def FLAC__stream_decoder_delete(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_delete(ctx))

    @staticmethod
    def FLAC__stream_decoder_init_file(ctx, filename, write, metadata, error, user):
        fn = filename.encode() if isinstance(filename, str) else filename
        return LibFLAC._l().FLAC__stream_decoder_init_file(ctx, fn, write, metadata, error, user)

    @staticmethod
    def FLAC__stream_decoder_init_stream(ctx, read, seek, tell, length, eof, write, metadata, error, user):
        return LibFLAC._l().FLAC__stream_decoder_init_stream(ctx, read, seek, tell, length, eof, write, metadata,
                                                             error, user)

    @staticmethod
    def FLAC__stream_decoder_process_single(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_process_single(ctx))

    @staticmethod
    def FLAC__stream_decoder_process_until_end_of_metadata(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_process_until_end_of_metadata(ctx))

    @staticmethod
    def FLAC__stream_decoder_process_until_end_of_stream(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_process_until_end_of_stream(ctx))

    @staticmethod
    def FLAC__stream_decoder_seek_absolute(ctx, sample):
        return bool(LibFLAC._l().FLAC__stream_decoder_seek_absolute(ctx, sample))

    @staticmethod
    def FLAC__stream_decoder_get_total_samples(ctx):
        return int(LibFLAC._l().FLAC__stream_decoder_get_total_samples(ctx))

    @staticmethod
    def FLAC__stream_decoder_get_state(ctx):
        return StreamDecoderState(LibFLAC._l().FLAC__stream_decoder_get_state(ctx))

    @staticmethod
    def FLAC__stream_decoder_get_channels(ctx):
        return int(LibFLAC._l().FLAC__stream_decoder_get_channels(ctx))

    @staticmethod
    def FLAC__stream_decoder_get_bits_per_sample(ctx):
        return int(LibFLAC._l().FLAC__stream_decoder_get_bits_per_sample(ctx))

    @staticmethod
    def FLAC__stream_decoder_get_sample_rate(ctx):
        return int(LibFLAC._l().FLAC__stream_decoder_get_sample_rate(ctx))

    @staticmethod
    def FLAC__stream_decoder_reset(ctx):
        return int(LibFLAC._l().FLAC__stream_decoder_reset(ctx))

    @staticmethod
    def FLAC__stream_decoder_set_md5_checking(ctx, value):
        return bool(LibFLAC._l().FLAC__stream_decoder_set_md5_checking(ctx, 1 if value else 0))

    @staticmethod
    def FLAC__stream_decoder_get_md5_checking(ctx):
        return bool(LibFLAC._l().FLAC__stream_decoder_get_md5_checking(ctx))


# ------------------------------------------------------------------ batch API
OUT_PLANAR32, OUT_INTERLEAVED32, OUT_FLACDECODER, OUT_FILEREADER = 0, 1, 2, 3
FRAME_INFO_BYTES = 128
ST_OK, ST_ERROR, ST_TRUNC, ST_SKIPPED = 0, 1, 2, 3

FRAME_INFO_DTYPE = np.dtype([
    ("status", "<u4"), ("err", "<i4"), ("frame_off", "<u8"), ("resume_bit", "<u8"), ("cached", "<i4"),
    ("blocksize", "<u4"), ("sample_rate", "<u4"), ("channels", "<u4"), ("assignment", "<u4"), ("bps", "<u4"),
    ("number_type", "<u4"), ("unparseable", "<u4"), ("number", "<u8"), ("out_sample", "<u8"), ("crc8", "<u4"),
    ("crc16_calc", "<u4"), ("crc16_read", "<u4"), ("crc_ok", "<u4"), ("sub_start", "<u4", (8,)), ("flags", "<u4"),
    ("reserved", "<u4")])
assert FRAME_INFO_DTYPE.itemsize == FRAME_INFO_BYTES


class StreamParams(ctypes.Structure):
    _fields_ = [("has_stream_info", ctypes.c_int32), ("min_blocksize", ctypes.c_uint32),
                ("max_blocksize", ctypes.c_uint32), ("sample_rate", ctypes.c_uint32), ("channels", ctypes.c_uint32),
                ("bps", ctypes.c_uint32), ("total_samples", ctypes.c_uint64)]

    @classmethod
    def from_synth(cls, p, total_samples=0):
        bs = p.blocksize
        mn = p.bs_min if p.variable_blocksize else bs
        mx = p.bs_max if p.variable_blocksize else bs
        return cls(1, mn, mx, p.sample_rate, p.channels, p.bps, total_samples)


def out_stride(fmt: int, sp: StreamParams) -> int:
    return int(load().bnflac_out_stride(fmt, ctypes.byref(sp)))


def md5_interleaved32(pcm: np.ndarray, channels: int, bps: int) -> bytes:
    """STREAMINFO md5sum of interleaved int32 PCM (host), libFLAC's byte convention."""
    a = np.ascontiguousarray(pcm, dtype=np.int32).reshape(-1)
    if a.size % channels:
        raise ValueError("pcm size is not a multiple of channels")
    out = (ctypes.c_uint8 * 16)()
    rc = load().bnflac_md5_interleaved32(a.ctypes.data if a.size else None, a.size // channels, channels, bps, out)
    if rc != 0:
        raise RuntimeError(load().bnflac_last_error().decode())
    return bytes(out)


class BatchDecoder:
    """Device-pointer batch decode (bnflac_decode_frames) over torch CUDA tensors."""

    def __init__(self, device: int = 0):
        self.L = load()
        self.device = device
        h = ctypes.c_void_p()
        rc = self.L.bnflac_ctx_create(device, ctypes.byref(h))
        if rc != 0:
            raise RuntimeError("bnflac_ctx_create failed: " + self.L.bnflac_last_error().decode())
        self.ctx = h

    def close(self):
        if self.ctx:
            self.L.bnflac_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _stream(stream):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def index_frames(self, d_bytes, nbytes: int, d_offsets, d_count, stream=None):
        rc = self.L.bnflac_index_frames(self.ctx, ctypes.c_void_p(d_bytes.data_ptr()), nbytes,
                                        ctypes.c_void_p(d_offsets.data_ptr()), d_offsets.numel(),
                                        ctypes.c_void_p(d_count.data_ptr()), self._stream(stream))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())

    def index_stream(self, d_bytes, nbytes: int, first_offset: int, sp: StreamParams, cap: int, stream=None):
        """Frame chain of a whole stream in HBM (bnflac_index_stream).
        -> (d_offsets int64[cap], d_out_sample int64[cap], d_info uint8[cap*128], nframes)."""
        import torch
        dev = d_bytes.device
        d_offs = torch.zeros(max(cap, 1), dtype=torch.int64, device=dev)
        d_os = torch.zeros(max(cap, 1), dtype=torch.int64, device=dev)
        d_info = torch.zeros(max(cap, 1) * FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        d_n = torch.zeros(1, dtype=torch.int32, device=dev)
        rc = self.L.bnflac_index_stream(self.ctx, ctypes.c_void_p(d_bytes.data_ptr()), nbytes, first_offset,
                                        ctypes.byref(sp), ctypes.c_void_p(d_offs.data_ptr()),
                                        ctypes.c_void_p(d_os.data_ptr()), ctypes.c_void_p(d_info.data_ptr()), cap,
                                        ctypes.c_void_p(d_n.data_ptr()), self._stream(stream))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())
        s = stream if stream is not None else torch.cuda.current_stream()
        s.synchronize()
        return d_offs, d_os, d_info, int(d_n.item())

    def decode_frames(self, d_bytes, nbytes: int, d_offsets, nframes: int, sp: StreamParams, fmt: int, d_out,
                      d_info, d_out_sample=None, base_sample: int = 0, stream=None, out_bytes=None):
        """out_bytes: the output size passed to the library (default: all of d_out)"""
        nout = d_out.numel() * d_out.element_size()
        rc = self.L.bnflac_decode_frames(
            self.ctx, ctypes.c_void_p(d_bytes.data_ptr()), nbytes, ctypes.c_void_p(d_offsets.data_ptr()), nframes,
            ctypes.byref(sp), ctypes.c_void_p(d_out_sample.data_ptr()) if d_out_sample is not None else None,
            base_sample, fmt, ctypes.c_void_p(d_out.data_ptr()), nout if out_bytes is None else min(out_bytes, nout),
            ctypes.c_void_p(d_info.data_ptr()), self._stream(stream))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())


    def parse_frames(self, d_bytes, nbytes: int, d_offsets, nframes: int, sp: StreamParams, d_info,
                     d_out_sample=None, base_sample: int = 0, stream=None):
        rc = self.L.bnflac_parse_frames(
            self.ctx, ctypes.c_void_p(d_bytes.data_ptr()), nbytes, ctypes.c_void_p(d_offsets.data_ptr()), nframes,
            ctypes.byref(sp), ctypes.c_void_p(d_out_sample.data_ptr()) if d_out_sample is not None else None,
            base_sample, ctypes.c_void_p(d_info.data_ptr()), self._stream(stream))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())

    def decode_parsed(self, d_bytes, nbytes: int, nframes: int, sp: StreamParams, fmt: int, d_out, d_info,
                      stream=None):
        rc = self.L.bnflac_decode_parsed(self.ctx, ctypes.c_void_p(d_bytes.data_ptr()), nbytes, nframes,
                                         ctypes.byref(sp), fmt, ctypes.c_void_p(d_out.data_ptr()),
                                         d_out.numel() * d_out.element_size(), ctypes.c_void_p(d_info.data_ptr()),
                                         self._stream(stream))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())

    def crc_handoff(self, nframes: int) -> np.ndarray:
        """Debug: the CRC-16 hand-off of the last parse_frames call, [nframes, 8] uint32."""
        a = np.zeros(8 * nframes, np.uint32)
        if self.L.bnflac_debug_crc_handoff(self.ctx, a.ctypes.data_as(ctypes.c_void_p), nframes) != 0:
            raise RuntimeError(self.L.bnflac_last_error().decode())
        return a.reshape(nframes, 8)


class Reader:
    """Streaming PCM reader (include/bnflac.h part 3): Read(buffer, offset, count) like
    FLACDecoder.Read (FLACDecoder.cs:124-205), backed by GPU decode-ahead."""

    def __init__(self, data: bytes, out_format: int = OUT_FLACDECODER, window_frames: int = 0, device: int = 0):
        self.L = load()
        self._data = np.frombuffer(bytes(data), dtype=np.uint8)
        h = ctypes.c_void_p()
        rc = self.L.bnflac_reader_open(device, self._data.ctypes.data, self._data.size, out_format, window_frames,
                                       ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(self.L.bnflac_reader_last_error().decode())
        self.h = h
        sp = StreamParams()
        tb, nf = ctypes.c_uint64(), ctypes.c_uint32()
        self.L.bnflac_reader_params(self.h, ctypes.byref(sp), ctypes.byref(tb), ctypes.byref(nf))
        self.stream_params, self.total_bytes, self.nframes = sp, int(tb.value), int(nf.value)

    def Read(self, buffer: bytearray, offset: int, count: int) -> int:
        if offset < 0 or count < 0 or offset + count > len(buffer):
            raise ValueError("offset/count outside the buffer")
        view = (ctypes.c_uint8 * len(buffer)).from_buffer(buffer)
        n = self.L.bnflac_reader_read(self.h, ctypes.addressof(view) + offset, count)
        if n < 0:
            raise RuntimeError(self.L.bnflac_reader_last_error().decode())
        return int(n)

    def ReadFileReader(self, buffer: bytearray, offset: int, count: int) -> int:
        """FLACFileReader.Read(buffer, offset, numBytes) semantics (bnflac_reader_read_filereader):
        copies may run past offset + count up to len(buffer); C# exceptions raise RuntimeError."""
        if offset < 0 or count < 0:
            raise ValueError("negative offset/count")
        view = (ctypes.c_uint8 * len(buffer)).from_buffer(buffer) if len(buffer) else None
        n = self.L.bnflac_reader_read_filereader(self.h, ctypes.addressof(view) if view is not None else None, offset,
                                                 count, len(buffer))
        if n < 0:
            raise RuntimeError(self.L.bnflac_reader_last_error().decode())
        return int(n)

    def filereader_read_all(self, buf_len: int, num_bytes: int = None):
        """Read(buf, 0, num_bytes) on a buf_len-byte buffer until 0, like
        oracle.filereader_readall -> (rc, bytes, message)."""
        num_bytes = buf_len if num_bytes is None else num_bytes
        out = bytearray()
        buf = bytearray(buf_len)
        try:
            while True:
                n = self.ReadFileReader(buf, 0, num_bytes)
                if n == 0:
                    return 0, bytes(out), ""
                out += buf[:n]
        except RuntimeError as e:
            return 1, bytes(out), str(e)

    def Seek(self, sample: int):
        """Next Read starts at this sample (per channel): FLACFileReader.Position."""
        if self.L.bnflac_reader_seek(self.h, sample) != 0:
            raise RuntimeError(self.L.bnflac_reader_last_error().decode())

    def read_all(self, chunk: int = 16384) -> bytes:
        out = bytearray()
        buf = bytearray(chunk)
        while True:
            n = self.Read(buf, 0, chunk)
            if n == 0:
                return bytes(out)
            out += buf[:n]

    def close(self):
        if getattr(self, "h", None):
            self.L.bnflac_reader_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def info_array(raw: np.ndarray) -> np.ndarray:
    """View a uint8 buffer of frame records as a structured array."""
    return np.frombuffer(np.ascontiguousarray(raw).tobytes(), dtype=FRAME_INFO_DTYPE)
