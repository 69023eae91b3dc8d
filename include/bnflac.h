/*
 * bnflac.h -- C ABI of libbnflac.so, the MI355X FLAC decoder behind BirdNest.Audio.
 *
 * Part 1: the libFLAC 1.2.1 stream-decoder entry points that BirdNest.Audio's P/Invoke
 * layer binds ([DllImport("LibFlac", CallingConvention = Cdecl)],
 * Library/LibFLACSharp/LibFLACSharp.cs:22).  Same names, argument meaning, return
 * conventions and callback order as libFLAC, so FLACDecoder / FLACFileReader /
 * OpenALDemo run unchanged when this library is loaded under the name "LibFlac"
 * (INTEGRATION.md).  Frame decode runs on the GPU; metadata and the libFLAC state
 * machine replay run on the host.
 *
 * Part 2: a batched, device-pointer API (bnflac_*) for callers that keep compressed
 * frames and PCM resident in HBM -- the path bench.py measures.
 *
 * Only plain C types cross this boundary (no torch, no HIP types: a HIP stream is
 * passed as void*).
 */
#ifndef BNFLAC_H
#define BNFLAC_H

#include "FLAC_compat.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define BNFLAC_API __attribute__((visibility("default")))
#else
#define BNFLAC_API
#endif

/* ===================== Part 1: libFLAC-compatible stream decoder ===================== */

/* LibFLACSharp.cs:42-43 */
BNFLAC_API FLAC__StreamDecoder *FLAC__stream_decoder_new(void);
/* LibFLACSharp.cs:45-46 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_finish(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:48-49 declares `bool` where libFLAC returns void; this export returns
 * true so FLACDecoder.cs:299-301's FLACCheck passes (SURVEY.md 8b hazard 1). */
BNFLAC_API FLAC__bool FLAC__stream_decoder_delete(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:51-52.  The C# write delegate is declared void (:205-206); its
 * return value is ignored for decoders initialised through init_file (hazard 2). */
BNFLAC_API int FLAC__stream_decoder_init_file(FLAC__StreamDecoder *decoder, const char *filename,
                                              FLAC__StreamDecoderWriteCallback write_callback,
                                              FLAC__StreamDecoderMetadataCallback metadata_callback,
                                              FLAC__StreamDecoderErrorCallback error_callback,
                                              void *client_data);
/* LibFLACSharp.cs:54-55 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_process_single(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:57-58 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_process_until_end_of_metadata(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:60-61 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_process_until_end_of_stream(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:63-64 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_seek_absolute(FLAC__StreamDecoder *decoder, FLAC__uint64 sample);
/* LibFLACSharp.cs:66-67 */
BNFLAC_API FLAC__bool FLAC__stream_decoder_get_decode_position(const FLAC__StreamDecoder *decoder,
                                                               FLAC__uint64 *position);
/* LibFLACSharp.cs:69-70 */
BNFLAC_API FLAC__uint64 FLAC__stream_decoder_get_total_samples(const FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:72-79 */
BNFLAC_API unsigned FLAC__stream_decoder_get_channels(const FLAC__StreamDecoder *decoder);
BNFLAC_API unsigned FLAC__stream_decoder_get_bits_per_sample(const FLAC__StreamDecoder *decoder);
BNFLAC_API unsigned FLAC__stream_decoder_get_sample_rate(const FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:81-82 */
BNFLAC_API FLAC__StreamDecoderState FLAC__stream_decoder_get_state(const FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:84-85 (declared int in C#; libFLAC returns FLAC__bool) */
BNFLAC_API FLAC__bool FLAC__stream_decoder_reset(FLAC__StreamDecoder *decoder);
/* LibFLACSharp.cs:175-185 */
BNFLAC_API int FLAC__stream_decoder_init_stream(FLAC__StreamDecoder *decoder,
                                                FLAC__StreamDecoderReadCallback read_callback,
                                                FLAC__StreamDecoderSeekCallback seek_callback,
                                                FLAC__StreamDecoderTellCallback tell_callback,
                                                FLAC__StreamDecoderLengthCallback length_callback,
                                                FLAC__StreamDecoderEofCallback eof_callback,
                                                FLAC__StreamDecoderWriteCallback write_callback,
                                                FLAC__StreamDecoderMetadataCallback metadata_callback,
                                                FLAC__StreamDecoderErrorCallback error_callback,
                                                void *client_data);
/* libFLAC stream_decoder.h (not bound by LibFLACSharp.cs; BirdNest leaves MD5 checking
 * off).  Only while UNINITIALIZED; finish() then returns false when the MD5 of the
 * decoded PCM differs from STREAMINFO's non-zero md5sum.  A seek turns checking off. */
BNFLAC_API FLAC__bool FLAC__stream_decoder_set_md5_checking(FLAC__StreamDecoder *decoder, FLAC__bool value);
BNFLAC_API FLAC__bool FLAC__stream_decoder_get_md5_checking(const FLAC__StreamDecoder *decoder);

/* ========================= Part 2: batched device-pointer API ========================= */

typedef struct {
    int32_t has_stream_info;
    uint32_t min_blocksize, max_blocksize;
    uint32_t sample_rate, channels, bps;
    uint64_t total_samples;
} bnflac_stream_params;

/* Per-frame result record (128 bytes), device-resident. */
typedef struct {
    uint32_t status;        /* 0 ok, 1 libFLAC error (err), 2 truncated, 3 skipped */
    int32_t err;            /* FLAC__StreamDecoderErrorStatus, -1 none */
    uint64_t frame_off;
    uint64_t resume_bit;
    int32_t cached;
    uint32_t blocksize, sample_rate, channels, assignment, bps;
    uint32_t number_type, unparseable;
    uint64_t number;
    uint64_t out_sample;
    uint32_t crc8, crc16_calc, crc16_read, crc_ok;
    uint32_t sub_start[8];
    uint32_t flags;         /* bit 1: past out_bytes (status 3), bit 2: layout cannot carry it (status 3); the other
                               bits record the decode path (which kernel, hand-backs) and differ between paths */
    uint32_t reserved;      /* 0 */
} bnflac_frame_info;

enum {
    BNFLAC_OUT_PLANAR32 = 0,      /* int32, per frame channel-major (libFLAC write buffers) */
    BNFLAC_OUT_INTERLEAVED32 = 1, /* int32 [sample][channel] */
    BNFLAC_OUT_FLACDECODER = 2,   /* FLACDecoder.WriteCallback packing (FLACDecoder.cs:543-577) */
    BNFLAC_OUT_FILEREADER = 3     /* FLACFileReader packing (FLACFileReader.cs:220-237) */
};

typedef struct bnflac_ctx bnflac_ctx;

/* 0 on success, else a negative bnflac error code. */
BNFLAC_API int bnflac_ctx_create(int device, bnflac_ctx **out);
BNFLAC_API void bnflac_ctx_destroy(bnflac_ctx *ctx);
BNFLAC_API const char *bnflac_last_error(void);
BNFLAC_API int bnflac_device_count(void);

/* Find every frame-sync candidate (0xFF, then a byte with top 6 bits 111110) in
 * d_bytes[0, nbytes), in stream order.  d_bytes must be 4-byte aligned and its
 * allocation at least round_up(nbytes, 4) bytes.  *d_count (device) receives the total
 * (which may exceed cap; only cap offsets are written).  Asynchronous on hip_stream. */
BNFLAC_API int bnflac_index_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                   uint64_t *d_offsets, uint32_t cap, uint32_t *d_count, void *hip_stream);

/* Frame chain resolution: the frames of a whole FLAC stream resident in
 * d_bytes (16-byte aligned, allocation >= round_up(nbytes, 16)), in stream order, without
 * decoding them.  Sync scan -> header, CRC-8 and subframe walk of every candidate ->
 * successor of each valid frame = the first later valid candidate at which the CRC-16 of
 * the bytes from the frame start is zero (the CRC-16 footer zeroes it; this is where
 * libFLAC's frame_sync_ finds the next frame in an intact stream) -> the chain from the
 * first valid candidate at or after first_offset (the byte after the metadata blocks).
 * Frames at or past STREAMINFO total_samples are dropped (frame_sync_'s end-of-stream
 * rule).  Writes d_frame_offsets, d_out_sample (running sample count; may be NULL) and,
 * when d_info != NULL, the parsed records ready for bnflac_decode_parsed.  *d_nframes
 * (device) = chain length (only cap entries are written).  A damaged stream ends the
 * chain at the damage; the libFLAC stream API handles resync.  Synchronises hip_stream
 * once (candidate count); otherwise asynchronous. */
BNFLAC_API int bnflac_index_stream(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, uint64_t first_offset,
                                   const bnflac_stream_params *sp, uint64_t *d_frame_offsets, uint64_t *d_out_sample,
                                   bnflac_frame_info *d_info, uint32_t cap, uint32_t *d_nframes, void *hip_stream);

/* Decode nframes frames starting at d_frame_offsets (byte offsets into d_bytes).
 * Output position of each frame: d_out_sample[i] if non-NULL, else the header's
 * sample number (frame number x STREAMINFO blocksize for fixed-blocksize streams) minus
 * base_sample.  Frames that would end past out_bytes are not written (status 3,
 * flags bit 1).  d_info receives one record per frame.  A frame whose status is not OK
 * (an error or truncation inside a subframe; libFLAC writes nothing for it) has its output
 * range zero-filled when its header parsed (sub_start[0] != 0), and is not written when the
 * header itself failed (no range).  A CRC-16 mismatch is status OK with crc_ok 0 and a
 * zero-filled frame, as libFLAC writes it.  Asynchronous on hip_stream. */
BNFLAC_API int bnflac_decode_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                    const uint64_t *d_frame_offsets, uint32_t nframes,
                                    const bnflac_stream_params *sp, const uint64_t *d_out_sample,
                                    uint64_t base_sample, int out_format, uint8_t *d_out, uint64_t out_bytes,
                                    bnflac_frame_info *d_info, void *hip_stream);

/* The two phases of bnflac_decode_frames, for callers that time or overlap them:
 * parse = frame headers + subframe cursor walk (k_parse), decode = subframe decode,
 * decorrelation, packing and CRC-16 (k_decode).  decode must follow parse on the same
 * stream with the same arguments.  The parse also does part of the CRC-16 work of 2-channel
 * frames and hands it to the next bnflac_decode_parsed call on the same ctx with the same
 * d_bytes, nbytes, d_info and nframes (used once; bnflac_index_stream drops it): the frame
 * bytes must not change between the two calls (bnflac_debug_set_crc_mode). */
BNFLAC_API int bnflac_parse_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                   const uint64_t *d_frame_offsets, uint32_t nframes,
                                   const bnflac_stream_params *sp, const uint64_t *d_out_sample,
                                   uint64_t base_sample, bnflac_frame_info *d_info, void *hip_stream);
BNFLAC_API int bnflac_decode_parsed(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, uint32_t nframes,
                                    const bnflac_stream_params *sp, int out_format, uint8_t *d_out,
                                    uint64_t out_bytes, bnflac_frame_info *d_info, void *hip_stream);

/* Timing experiments only: skip parts of the kernels (bit0 CRC-16, bit1 PCM stores,
 * bit2 restore, bit3 Rice decode, bit4 subframe walk).  Output is wrong while set.
 * Exception: bit 0x800 only routes every k_decode chunk through the generic path (exact).
 * Bit 0x10000000 aims k_decode_st's / k_decode_sw's PCM stores at a 513 KB window at the
 * start of d_out (an L2-resident footprint); it is ignored when out_bytes < 1 MiB. */
BNFLAC_API void bnflac_debug_set_ablate(uint32_t flags);
/* Development / test switch: parse kernel (-1 auto, 0 lane-per-frame k_parse, 1 wave-per-frame
 * k_parse_wave); both write identical records. */
BNFLAC_API void bnflac_debug_set_parse_wave(int mode);
/* Development / test switch: k_decode_sys, the systolic-restore decode of every frame class
 * (-1 auto: env BNFLAC_DECODE_SYS, else k_decode_sys for launches below 1024 subframe waves of
 * the lane kernels; 0 the lane kernels by class; 1 always); identical PCM and records. */
BNFLAC_API void bnflac_debug_set_decode_sys(int mode);
/* Development / test switch: who computes the CRC-16 hand-off bnflac_parse_frames passes to
 * bnflac_decode_parsed (-1 env BNFLAC_CRC_MODE, default 3; 0 none: the decode reads every frame
 * again; 1 k_parse's prefix: the lines before channel 1; 2 and its verdict over the span to
 * the next frame's offset; 3 the prefix, except for a 16-bit stream after a decode on the
 * device whose frames were a quarter or more LPC above order 8); identical PCM and records. */
BNFLAC_API void bnflac_debug_set_crc_mode(int mode);
/* Debug: the hand-off of ctx's last bnflac_parse_frames call (8 words per frame: prefix
 * remainder r0, r1 | parity << 31, its lines + 1, frame_off low word; span to the next
 * offset, verdict over it, frame_off low word, 0), synchronously.  0, or -1 when none. */
BNFLAC_API int bnflac_debug_crc_handoff(bnflac_ctx *ctx, uint32_t *out, uint32_t nframes);
/* Debug: how many decodes of this process took the W16 / W32 classes through one small
 * segment grid (k_decode_seg: the previous decode order on the device had neither class)
 * instead of the two full-size side grids. */
BNFLAC_API uint64_t bnflac_debug_decode_seg_launches(void);
/* Debug: k_parse_wave's counters, collected while BNFLAC_PW_STATS is set in the environment
 * (passes, splice rounds, serial fallbacks, partitions, frames, scan / window-wait / splice
 * wave-cycles).  out8 holds 8 values; reset != 0 clears them.  0 or -1. */
BNFLAC_API int bnflac_debug_parse_wave_stats(uint64_t *out8, int reset);
/* Debug: k_decode event counters collected while ablate bit 0x100 is set: [0..5] fused
 * chunks, generic chunks, DMA landing waits, slow Rice codewords, refills, waves (wave-level
 * events); [8..12] shader-clock cycles summed over waves in setup, chunk decode, refill,
 * pack, tail.  out16 holds 16 values.  Synchronous; reset != 0 clears them. */
BNFLAC_API int bnflac_debug_stats(uint64_t *out16, int reset);

/* Bytes of one sample frame (all channels of one sample index) in out_format. */
BNFLAC_API uint32_t bnflac_out_stride(int out_format, const bnflac_stream_params *sp);

/* Host helper: STREAMINFO md5sum of nsamples interleaved int32 sample frames (host
 * memory, e.g. a BNFLAC_OUT_INTERLEAVED32 result copied back), hashed as libFLAC does:
 * each sample as (bps + 7) / 8 little-endian bytes.  0 on success. */
BNFLAC_API int bnflac_md5_interleaved32(const int32_t *pcm, uint64_t nsamples, uint32_t channels, uint32_t bps,
                                        uint8_t out_md5[16]);

/* ======================== Part 3: streaming reader ======================= */

/* The fast path under FLACDecoder.Read (FLACDecoder.cs:124-205) and OpenAL's buffer fill
 * (OpenALDemo/Program.cs:33-38): a whole FLAC stream in host memory in, packed PCM out in
 * caller-sized pieces.  open() copies the stream to HBM once, indexes its frames on the GPU
 * (bnflac_index_stream) and starts decoding ahead in windows of `window_frames` frames
 * (0: 256) into a two-slot pinned host ring; read() copies from the ring while the next
 * window decodes.  The bytes are those of out_format (BNFLAC_OUT_FLACDECODER: what
 * FLACDecoder.CopyTo yields).  Intact streams only: open() or read() returns -1 at the
 * first sign of damage (frame chain short of STREAMINFO's total, CRC failure), with the
 * reason in bnflac_reader_last_error(); the libFLAC stream API (part 1) handles those. */
typedef struct bnflac_reader bnflac_reader;
BNFLAC_API int bnflac_reader_open(int device, const uint8_t *bytes, uint64_t nbytes, int out_format,
                                  uint32_t window_frames, bnflac_reader **out);
/* STREAMINFO, total PCM bytes the reader will return, frames found.  Any pointer may be NULL. */
BNFLAC_API int bnflac_reader_params(const bnflac_reader *reader, bnflac_stream_params *sp, uint64_t *total_bytes,
                                    uint32_t *nframes);
/* Up to count bytes into buf; returns the number copied (0: end of stream) or -1. */
BNFLAC_API int64_t bnflac_reader_read(bnflac_reader *reader, uint8_t *buf, uint64_t count);
/* Position the reader so the next read starts at `sample` (per channel), like
 * FLACFileReader.Position / seek_absolute (FLACFileReader.cs:109-137,295-299).  0 or -1
 * (sample past the end, or damage in the target window). */
BNFLAC_API int bnflac_reader_seek(bnflac_reader *reader, uint64_t sample);
/* FLACFileReader.Read(buffer, offset, numBytes) (FLACFileReader.cs:145-254) replayed with
 * buffer.Length = buffer_length, on a reader opened with BNFLAC_OUT_FILEREADER: samples left
 * over from the previous call first, then whole frames until numBytes are reached; every copy
 * runs to the buffer's end (the return may exceed num_bytes), m_samplesPerChannel is the first
 * frame's blocksize (shorter frames leave earlier samples behind, longer ones are cut).
 * Returns the bytes copied, 0 at the end, -1 with the C# exception's message in
 * bnflac_reader_last_error() ("Index was outside the bounds of the array." / "Input FLAC bit
 * depth is not supported!").  Not mixed with bnflac_reader_read / bnflac_reader_seek. */
BNFLAC_API int64_t bnflac_reader_read_filereader(bnflac_reader *reader, uint8_t *buffer, uint64_t offset,
                                                 uint64_t num_bytes, uint64_t buffer_length);
BNFLAC_API void bnflac_reader_close(bnflac_reader *reader);
/* A closed reader's stream, events and small buffers stay pooled per device for the next
 * open (buffers above BNFLAC_READER_POOL_CAP bytes, default 64 MiB, are freed on close;
 * BNFLAC_READER_POOL=0 turns pooling off).  This frees every pooled resource of `device`
 * (-1: of every device), e.g. before handing the GPU's memory to another user.  Returns the
 * number of pooled reader sets freed. */
BNFLAC_API int bnflac_reader_pool_release(int device);
BNFLAC_API const char *bnflac_reader_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* BNFLAC_H */
