"""Python mirror of BirdNest.Audio's NAudio-style FLACFileReader, running on libbnflac.so.

Follows ``Library/BirdNest.Audio.UnitTests/FLACFileReader.cs`` member by member: the
constructor opens the file through ``FLAC__stream_decoder_init_file`` and reads the
metadata (:45-78), ``Read`` drains leftover samples and then calls ProcessSingle + copy
until ``numBytes`` are reached (:145-174), the write callback copies ``m_samplesPerChannel``
samples per channel, a value fixed by the first frame (:267-301), the copy interleaves 2 or
3 little-endian bytes per sample up to the buffer's Length (:208-254), and ``Position``
requests a seek that the next write callback issues from inside itself (:109-137, 295-299).
It is the only reference reader for the 24-bit configs.  Same names, argument meaning and
exception messages, so tests read like the reference's usage; the GPU stream API is what it
drives.  C# exceptions thrown in callbacks are recorded and raised when the native call
returns (ctypes cannot unwind through C), as in flac_decoder.py.
"""
from __future__ import annotations

import ctypes

import numpy as np

from .flac_decoder import ApplicationException
from .libflac import (LibFLAC, DecodeError, Decoder_ErrorCallback, Decoder_MetadataCallback, Decoder_WriteCallback,
                      FLACMetaDataType, FrameHeader, StreamDecoderState)


class IndexOutOfRangeException(Exception):
    """System.IndexOutOfRangeException."""

    def __init__(self):
        super().__init__("Index was outside the bounds of the array.")


class NotSupportedException(Exception):
    """System.NotSupportedException."""


class WaveInformation:  # WaveInformation.cs:15-62, BlockAlign :78
    def __init__(self, rate: int, bits: int, channels: int):
        self.SampleRate, self.BitsPerSample, self.Channels = rate, bits, channels
        self.BlockAlign = channels * (bits // 8)


class FLACFileReader:
    """FLACFileReader.cs:41-455 (a System.IO.Stream over a FLAC file)."""

    def __init__(self, flacFileName: str):
        self.m_repositionRequested = False
        self.m_flacReposition = 0
        self.m_lastSampleNumber = 0
        self.m_flacSamples = None
        self.m_samplesPerChannel = 0
        self.m_flacSampleIndex = 0
        self.m_totalSamples = 0
        self.m_NAudioSampleBuffer = None
        self.m_playbackBufferOffset = 0
        self._pending = None
        self.m_channels = self.m_bits = self.m_rate = 0
        self.m_decoderContext = LibFLAC.FLAC__stream_decoder_new()
        if not self.m_decoderContext:
            raise ApplicationException("FLAC: Could not initialize stream decoder!")
        self.m_writeCallback = Decoder_WriteCallback(self.FLAC_WriteCallback)
        self.m_metadataCallback = Decoder_MetadataCallback(self.FLAC_MetadataCallback)
        self.m_errorCallback = Decoder_ErrorCallback(self.FLAC_ErrorCallback)
        if LibFLAC.FLAC__stream_decoder_init_file(self.m_decoderContext, flacFileName, self.m_writeCallback,
                                                  self.m_metadataCallback, self.m_errorCallback, None) != 0:
            raise ApplicationException("FLAC: Could not open stream for reading!")
        self.FLACCheck(LibFLAC.FLAC__stream_decoder_process_until_end_of_metadata(self.m_decoderContext),
                       "Could not process until end of metadata")
        self.m_waveFormat = WaveInformation(self.m_rate, self.m_bits, self.m_channels)

    # ---- properties (:85-137)
    @property
    def Length(self) -> int:
        return self.m_totalSamples * self.m_waveFormat.BlockAlign

    @property
    def WaveFormat(self) -> WaveInformation:
        return self.m_waveFormat

    @property
    def Position(self) -> int:
        return self.m_lastSampleNumber * self.m_waveFormat.BlockAlign

    @Position.setter
    def Position(self, value: int):
        self.m_flacSampleIndex = 0
        self.m_repositionRequested = True
        self.m_flacReposition = value // self.m_waveFormat.BlockAlign
        self.m_lastSampleNumber = self.m_flacReposition

    # ---- Read (:145-174)
    def Read(self, playbackSampleBuffer: bytearray, offset: int, numBytes: int) -> int:
        flacBytesCopied = 0
        self.m_NAudioSampleBuffer = playbackSampleBuffer
        self.m_playbackBufferOffset = offset
        if self.m_flacSampleIndex > 0:
            flacBytesCopied = self.CopyFlacBufferToNAudioBuffer()
        while flacBytesCopied < numBytes:
            self.ProcessSingle()
            if LibFLAC.FLAC__stream_decoder_get_state(self.m_decoderContext) == StreamDecoderState.EndOfStream:
                break
            flacBytesCopied += self.CopyFlacBufferToNAudioBuffer()
        return flacBytesCopied

    def ProcessSingle(self):  # :177-181 (the bool result is ignored)
        LibFLAC.FLAC__stream_decoder_process_single(self.m_decoderContext)
        self._raise_pending()

    def FLACCheck(self, result: bool, operation: str):  # :188-195
        self._raise_pending()
        if not result:
            state = LibFLAC.FLAC__stream_decoder_get_state(self.m_decoderContext)
            raise ApplicationException(f"FLAC: Could not {operation} - {state.name}!")

    def _raise_pending(self):
        if self._pending is not None:
            e, self._pending = self._pending, None
            raise e

    # ---- CopyFlacBufferToNAudioBuffer (:208-254)
    def CopyFlacBufferToNAudioBuffer(self) -> int:
        buf = self.m_NAudioSampleBuffer
        start = self.m_playbackBufferOffset
        full = self.m_playbackBufferOffset >= len(buf)
        spc, C = self.m_samplesPerChannel, self.m_channels
        while self.m_flacSampleIndex < spc and not full:
            ch = 0
            while ch < C and not full:
                sample = int(self.m_flacSamples[self.m_flacSampleIndex + ch * spc])
                if self.m_bits == 16:
                    nb = 2
                elif self.m_bits == 24:
                    nb = 3
                else:
                    raise NotSupportedException("Input FLAC bit depth is not supported!")
                for k in range(nb):
                    if self.m_playbackBufferOffset >= len(buf):
                        raise IndexOutOfRangeException()
                    buf[self.m_playbackBufferOffset] = (sample >> (8 * k)) & 0xFF
                    self.m_playbackBufferOffset += 1
                full = self.m_playbackBufferOffset >= len(buf)
                ch += 1
            self.m_flacSampleIndex += 1
        if self.m_flacSampleIndex >= spc:
            self.m_flacSampleIndex = 0
        return self.m_playbackBufferOffset - start

    # ---- callbacks (:267-341)
    def FLAC_WriteCallback(self, context, frame, buffer, clientData):
        try:
            hdr = FrameHeader.from_address(frame)
            if self.m_flacSamples is None:
                self.m_samplesPerChannel = hdr.BlockSize
                self.m_flacSamples = np.zeros(self.m_samplesPerChannel * self.m_channels, dtype=np.int32)
                self.m_flacSampleIndex = 0
            spc = self.m_samplesPerChannel
            for ch in range(self.m_channels):  # Marshal.Copy of m_samplesPerChannel values per channel
                self.m_flacSamples[ch * spc:(ch + 1) * spc] = np.ctypeslib.as_array(buffer[ch], shape=(spc,))
            self.m_lastSampleNumber = hdr.FrameOrSampleNumber
            if self.m_repositionRequested:
                self.m_repositionRequested = False
                ok = LibFLAC.FLAC__stream_decoder_seek_absolute(self.m_decoderContext, self.m_flacReposition)
                self.FLACCheck(ok, "Could not seek absolute: " + str(self.m_flacReposition))
        except Exception as e:  # thrown through the native frames in C#
            if self._pending is None:
                self._pending = e
        return 0  # declared void in C# (LibFLACSharp.cs:205-206): treated as CONTINUE

    def FLAC_MetadataCallback(self, context, metadata, userData):
        raw = ctypes.string_at(metadata, 52)
        if int.from_bytes(raw[0:4], "little") == FLACMetaDataType.StreamInfo:
            self.m_rate = int.from_bytes(raw[32:36], "little")
            self.m_channels = int.from_bytes(raw[36:40], "little")
            self.m_bits = int.from_bytes(raw[40:44], "little")
            hi = int.from_bytes(raw[44:48], "little", signed=True)  # FieldOffset 32: padding (LibFLACSharp.cs:315)
            lo = int.from_bytes(raw[48:52], "little", signed=True)
            self.m_totalSamples = hi + lo  # (long)(hi << 32) == hi in C#: int shift counts are masked to 5 bits

    def FLAC_ErrorCallback(self, context, status, userData):
        state = LibFLAC.FLAC__stream_decoder_get_state(self.m_decoderContext)
        if self._pending is None:
            self._pending = ApplicationException(
                f"FLAC: Could not decode frame: {DecodeError(status).name} - {state.name}!")

    # ---- Dispose (:350-381)
    def Dispose(self):
        if self.m_decoderContext:
            self.FLACCheck(LibFLAC.FLAC__stream_decoder_finish(self.m_decoderContext), "finalize stream decoder")
            self.FLACCheck(LibFLAC.FLAC__stream_decoder_delete(self.m_decoderContext),
                           "dispose of stream decoder instance")
            self.m_decoderContext = None

    def close(self):
        self.Dispose()


def read_all(path: str, buf_len: int, num_bytes: int = None):
    """FLACFileReader(path) + Read(buf, 0, num_bytes) on a buf_len-byte buffer until 0, like
    oracle.filereader_readall -> (rc, bytes, message)."""
    num_bytes = buf_len if num_bytes is None else num_bytes
    out = bytearray()
    r = None
    try:
        r = FLACFileReader(path)
        buf = bytearray(buf_len)
        while True:
            n = r.Read(buf, 0, num_bytes)
            if n == 0:
                break
            out += buf[:n]
        return 0, bytes(out), ""
    except Exception as e:
        return 1, bytes(out), str(e)
    finally:
        if r is not None:
            try:
                r.Dispose()
            except Exception:
                pass
