"""Python mirror of BirdNest.Audio's decode surface, running on libbnflac.so.

``FLACDecoder`` follows ``Library/BirdNest.Audio/FLACDecoder.cs`` (a Stream whose Read pulls
frames through libFLAC callbacks, 16-bit mono/stereo packets), ``FLACPacket`` /
``FLACPacketQueue`` / ``EmptyStubLogger`` follow FLACPacket.cs, FLACPacketQueue.cs and
EmptyStubLogger.cs.  Same names, argument meaning and exception messages, so the parity
tests read like the reference's usage (OpenALDemo/Program.cs:26-38).

C# exceptions thrown inside native callbacks unwind through libFLAC; ctypes cannot
unwind through C, so a callback that must throw records the exception, makes the
decoder stop at its next callback (ABORT), and the pending exception is raised when the
native call returns -- the bytes handed out before the exception are identical.
"""
from __future__ import annotations

import collections
import ctypes
import datetime
import io
from typing import Optional

from .libflac import (LibFLAC, DecoderEofCallback, DecoderLengthCallback, DecoderReadCallback, DecoderSeekCallback,
                      DecoderTellCallback, DecoderWriteCallbackWithStatus, Decoder_ErrorCallback,
                      Decoder_MetadataCallback, DecodeError, FLACMetaDataType, FrameHeader, StreamDecoderLengthStatus,
                      StreamDecoderReadStatus, StreamDecoderSeekStatus, StreamDecoderState, StreamDecoderTellStatus,
                      StreamDecoderWriteStatus)


class ApplicationException(Exception):
    """System.ApplicationException."""


class FLACPacket:  # FLACPacket.cs:3-10
    __slots__ = ("SampleRate", "Channels", "BlockSize", "Data", "Offset")

    def __init__(self):
        self.SampleRate = self.Channels = self.BlockSize = self.Offset = 0
        self.Data = b""


class IFLACPacketQueue:  # IFLACPacketQueue.cs:3-9
    def Enqueue(self, p): raise NotImplementedError
    def TryPeek(self): raise NotImplementedError
    def TryDequeue(self): raise NotImplementedError
    def IsEmpty(self): raise NotImplementedError


class FLACPacketQueue(IFLACPacketQueue):  # FLACPacketQueue.cs:5-36 (ConcurrentQueue, used single-threaded)
    def __init__(self):
        self._q = collections.deque()

    def Enqueue(self, p):
        self._q.append(p)

    def TryPeek(self):
        return (True, self._q[0]) if self._q else (False, None)

    def TryDequeue(self):
        return (True, self._q.popleft()) if self._q else (False, None)

    def IsEmpty(self):
        return not self._q


class IFLACDecoderLogger:  # IFLACDecoderLogger.cs:3-6
    def Warning(self, message: str): raise NotImplementedError


class EmptyStubLogger(IFLACDecoderLogger):  # EmptyStubLogger.cs:3-13
    def Warning(self, message: str):
        pass


def _al_format(channels: int, bits: int) -> Optional[str]:
    if bits == 16:
        return "Stereo16" if channels == 2 else "Mono16"
    if bits == 8:
        return "Stereo8" if channels == 2 else "Mono8"
    return None


class FLACDecoder(io.RawIOBase):
    """FLACDecoder.cs:14-598."""

    DEFAULT_MAX_BUFFER_SIZE = 16384  # :21

    def __init__(self, stream, queue: IFLACPacketQueue, logger: IFLACDecoderLogger, buffer: Optional[bytearray] = None):
        super().__init__()
        self.mStream = stream
        self.mPacketQueue = queue
        self.mLogger = logger
        self.mInstreamBuffer = buffer if buffer is not None else bytearray(self.DEFAULT_MAX_BUFFER_SIZE)
        self.mHitEOFYet = False
        self._pending: Optional[BaseException] = None
        self.Format = None
        self.Channels = self.SampleRate = self.BitsPerSample = 0
        self.Duration = datetime.timedelta(0)
        self.mBlockAlign = 0
        self.mTotalSamples = 0
        self.mFLACLength = 0
        self.mIsDisposed = False
        self._SetupDecoder()
        self._SetupCallbacks()
        self._SetupFLACStream()
        self._SetupStreamInfo()

    # ---- setup (:37-70)
    def _SetupCallbacks(self):
        self.mReadCallback = DecoderReadCallback(self._ReadCallback)
        self.mSeekCallback = DecoderSeekCallback(self._SeekCallback)
        self.mTellCallback = DecoderTellCallback(self._TellCallback)
        self.mLengthCallback = DecoderLengthCallback(self._LengthCallback)
        self.mEOFCallback = DecoderEofCallback(self._EOFCallback)
        self.mWriteCallback = DecoderWriteCallbackWithStatus(self._WriteCallback)
        self.mMetadataCallback = Decoder_MetadataCallback(self._MetadataCallback)
        self.mErrorCallback = Decoder_ErrorCallback(self._ErrorCallback)

    def _SetupDecoder(self):
        self.mDecoderContext = LibFLAC.FLAC__stream_decoder_new()
        if not self.mDecoderContext:
            raise ApplicationException("FLAC: Could not initialize stream decoder!")

    def _SetupFLACStream(self):
        if LibFLAC.FLAC__stream_decoder_init_stream(self.mDecoderContext, self.mReadCallback, self.mSeekCallback,
                                                    self.mTellCallback, self.mLengthCallback, self.mEOFCallback,
                                                    self.mWriteCallback, self.mMetadataCallback, self.mErrorCallback,
                                                    None) != 0:
            raise ApplicationException("FLAC: Could not open stream for reading!")

    def _SetupStreamInfo(self):
        self._FLACCheck(self._native(LibFLAC.FLAC__stream_decoder_process_until_end_of_metadata),
                        "Could not process until end of metadata")

    def _native(self, fn):
        r = fn(self.mDecoderContext)
        if self._pending is not None:
            e, self._pending = self._pending, None
            raise e
        return r

    def _FLACCheck(self, result: bool, operation: str):  # :98-105
        if not result:
            state = LibFLAC.FLAC__stream_decoder_get_state(self.mDecoderContext)
            raise ApplicationException(f"FLAC: Could not {operation} - {state.name}!")

    # ---- Stream members
    def readable(self):
        return True

    @property
    def CanSeek(self):
        return False

    @property
    def Length(self):
        return self.mFLACLength

    def Read(self, buffer: bytearray, offset: int, count: int) -> int:  # :124-205
        localOffset = offset
        spaceRemaining = count
        bytesRead = 0
        while spaceRemaining > 0:
            self._RequestAnotherFLACPacket()
            ok, current = self.mPacketQueue.TryPeek()
            if ok:
                bytesLeft = len(current.Data) - current.Offset
                if bytesLeft > spaceRemaining:
                    buffer[localOffset:localOffset + spaceRemaining] = current.Data[current.Offset:current.Offset + spaceRemaining]
                    current.Offset += spaceRemaining
                    bytesRead += spaceRemaining
                    spaceRemaining = 0
                elif 0 < bytesLeft <= spaceRemaining:
                    buffer[localOffset:localOffset + bytesLeft] = current.Data[current.Offset:]
                    localOffset += bytesLeft
                    spaceRemaining -= bytesLeft
                    bytesRead += bytesLeft
                    self._PopTopOffQueue()
            else:
                break
        return bytesRead

    def _RequestAnotherFLACPacket(self):  # :207-224
        if self.mPacketQueue.IsEmpty():
            state = LibFLAC.FLAC__stream_decoder_get_state(self.mDecoderContext)
            if state < StreamDecoderState.EndOfStream:
                self._FLACCheck(self._native(LibFLAC.FLAC__stream_decoder_process_single), "process single")
            elif state >= StreamDecoderState.OggError:
                raise ApplicationException(f"FLAC: Decoding returned with critical state: {state.name}")

    def _PopTopOffQueue(self):  # :226-233
        ok, _ = self.mPacketQueue.TryDequeue()
        if not ok:
            raise Exception("FLAC - queue error")

    def CopyTo(self, dest, buffer_size: int = 81920):
        """System.IO.Stream.CopyTo (OpenALDemo/Program.cs:33)."""
        buf = bytearray(buffer_size)
        while True:
            n = self.Read(buf, 0, buffer_size)
            if n == 0:
                break
            dest.write(bytes(buf[:n]))

    def Dispose(self):  # :285-319
        if self.mIsDisposed:
            return
        self.mHitEOFYet = False
        if self.mDecoderContext:
            self._FLACCheck(LibFLAC.FLAC__stream_decoder_finish(self.mDecoderContext), "finalize stream decoder")
            self._FLACCheck(LibFLAC.FLAC__stream_decoder_delete(self.mDecoderContext),
                            "dispose of stream decoder instance")
            self.mDecoderContext = None
        try:
            self.mStream.close()
        except Exception:
            pass
        self.mIsDisposed = True

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.Dispose()

    # ---- callbacks (:325-594)
    def _ReadCallback(self, context, buffer, nbytes, userData):
        if self._pending is not None:
            return StreamDecoderReadStatus.ReadStatusAbort
        if self.mInstreamBuffer is None:
            return StreamDecoderReadStatus.ReadStatusAbort
        noOfBytes = nbytes[0]
        if noOfBytes > 0:
            length = min(noOfBytes, len(self.mInstreamBuffer))
            data = self.mStream.read(length)
            count = len(data)
            if count:
                ctypes.memmove(buffer, data, count)
            if count < length:
                self.mHitEOFYet = True
                nbytes[0] = count
                return StreamDecoderReadStatus.ReadStatusEndOfStream
            nbytes[0] = count
            return StreamDecoderReadStatus.ReadStatusContinue
        self.mHitEOFYet = True
        return StreamDecoderReadStatus.ReadStatusAbort

    def _SeekCallback(self, context, absoluteByteOffset, userData):
        try:
            if not self.mStream.seekable():
                return StreamDecoderSeekStatus.SeekStatusUnsupported
            self.mStream.seek(absoluteByteOffset)
            return StreamDecoderSeekStatus.SeekStatusOk
        except Exception:
            return StreamDecoderSeekStatus.SeekStatusError

    def _TellCallback(self, context, absoluteByteOffset, userData):
        try:
            absoluteByteOffset[0] = self.mStream.tell()
            return StreamDecoderTellStatus.TellStatusOK
        except Exception:
            return StreamDecoderTellStatus.TellStatusError

    def _LengthCallback(self, context, streamLength, userData):
        try:
            cur = self.mStream.tell()
            end = self.mStream.seek(0, io.SEEK_END)
            self.mStream.seek(cur)
            streamLength[0] = end
            return StreamDecoderLengthStatus.LengthStatusOk
        except Exception:
            return StreamDecoderLengthStatus.LengthStatusError

    def _MetadataCallback(self, context, metadata, userData):  # :431-473
        raw = ctypes.string_at(metadata, 112)
        mtype = int.from_bytes(raw[0:4], "little")
        if mtype == FLACMetaDataType.StreamInfo:
            data = raw[12:112]
            i32 = lambda o: int.from_bytes(data[o:o + 4], "little", signed=True)
            self.BitsPerSample = i32(28)
            self.Channels = i32(24)
            self.SampleRate = i32(20)
            self.mBlockAlign = self.Channels * (self.BitsPerSample // 8)
            self.mTotalSamples = i32(32) + i32(36)  # (long)(Hi << 32) + (long)Lo, C# masks the shift
            self.mFLACLength = self.mBlockAlign * self.mTotalSamples
            self.Duration = datetime.timedelta(seconds=self.mTotalSamples / self.SampleRate) if self.SampleRate else 0
            fmt = _al_format(self.Channels, self.BitsPerSample)
            if fmt is not None:
                self.Format = fmt
            else:
                self.mLogger.Warning(f"FLAC: Unsupported sample bit size: {self.BitsPerSample}\n")

    def _EOFCallback(self, context, userData):
        return 1 if self.mHitEOFYet else 0

    def _WriteCallback(self, context, frame, buffer, clientData):  # :520-580
        if self._pending is not None:
            return StreamDecoderWriteStatus.WriteStatusAbort
        hdr = FrameHeader.from_address(frame)
        if hdr.BitsPerSample != 16:
            self.mLogger.Warning(f"FLAC: Unsupported bit-rate: {hdr.BitsPerSample}")
            return StreamDecoderWriteStatus.WriteStatusAbort
        import numpy as np
        packet = FLACPacket()
        packet.Channels = hdr.Channels
        packet.SampleRate = hdr.SampleRate
        packet.BlockSize = hdr.BlockSize
        packet.Offset = 0
        bs = packet.BlockSize
        ch0 = np.ctypeslib.as_array(buffer[0], shape=(bs,))
        if packet.Channels == 2:
            ch1 = np.ctypeslib.as_array(buffer[1], shape=(bs,))
            out = np.empty((bs, 2), dtype="<u2")
            out[:, 0] = ch0.astype(np.uint32) & 0xFFFF
            out[:, 1] = ch1.astype(np.uint32) & 0xFFFF
            packet.Data = out.tobytes()
        else:
            packet.Data = (ch0.astype(np.uint32) & 0xFFFF).astype("<u2").tobytes()
        self.mPacketQueue.Enqueue(packet)
        return StreamDecoderWriteStatus.WriteStatusContinue

    def _ErrorCallback(self, context, status, userData):  # :590-594
        state = LibFLAC.FLAC__stream_decoder_get_state(context)
        if self._pending is None:
            self._pending = ApplicationException(
                f"FLAC: Could not decode frame: {DecodeError(status).name} - {state.name}!")


def copy_to_bytes(data: bytes, copy_chunk: int = 81920):
    """OpenALDemo path (Program.cs:26-35): FLACDecoder over a byte stream, CopyTo a
    MemoryStream.  Returns (rc, pcm_bytes, message, [channels, rate, bits, total])."""
    out = io.BytesIO()
    try:
        with FLACDecoder(io.BytesIO(data), FLACPacketQueue(), EmptyStubLogger()) as reader:
            fmt = [reader.Channels, reader.SampleRate, reader.BitsPerSample, reader.mTotalSamples]
            reader.CopyTo(out, copy_chunk)
        return 0, out.getvalue(), "", fmt
    except ApplicationException as e:
        return 1, out.getvalue(), str(e), None
