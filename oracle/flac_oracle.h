/*
 * flac_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's decode path, used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  Nothing in
 * the product (birdnest/audio_amd, libbnflac.so) links or calls it.
 *
 * What it restates:
 *   - libFLAC 1.2.1 ("reference libFLAC 1.2.1 20070917"), which BirdNest.Audio ships
 *     prebuilt as Library/BirdNest.Audio/LibFLACDLL/LibFlac.dll.  No libFLAC source is
 *     present in the reference; the behaviour followed is pinned to the DLL's code
 *     addresses listed in SURVEY.md section 8a (read as disassembly text, never run).
 *   - The BirdNest.Audio C# surfaces on top of it: FLACDecoder.Read/WriteCallback
 *     (Library/BirdNest.Audio/FLACDecoder.cs:124-233, 520-580) and
 *     FLACFileReader.Read/CopyFlacBufferToNAudioBuffer/FLAC_WriteCallback
 *     (Library/BirdNest.Audio.UnitTests/FLACFileReader.cs:145-254, 267-301).
 *
 * Parity pinning: the reference holds no FLAC fixtures or golden vectors (SURVEY.md
 * section 4) and LibFlac.dll is prebuilt machine code that is never executed here.  The
 * oracle is pinned by (a) the RFC 9639 Appendix D known-answer stream (CRC-8, CRC-16
 * and the STREAMINFO MD5 written by an independent encoder), and (b) lossless
 * round trips from tests/golden (PCM in == PCM out, MD5 match).  See DESIGN.md
 * "Parity" for what that does and does not pin.
 */
#ifndef BNFLAC_ORACLE_H
#define BNFLAC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/FLAC_compat.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_decoder oracle_decoder;

/* libFLAC-shaped API (same argument meaning and return conventions as
 * FLAC__stream_decoder_*; the decoder pointer handed to callbacks is the oracle_decoder). */
oracle_decoder *oracle_new(void);
void oracle_delete(oracle_decoder *d);
int oracle_init_stream(oracle_decoder *d, FLAC__StreamDecoderReadCallback read,
                       FLAC__StreamDecoderSeekCallback seek, FLAC__StreamDecoderTellCallback tell,
                       FLAC__StreamDecoderLengthCallback length, FLAC__StreamDecoderEofCallback eof,
                       FLAC__StreamDecoderWriteCallback write,
                       FLAC__StreamDecoderMetadataCallback metadata,
                       FLAC__StreamDecoderErrorCallback error, void *client);
FLAC__bool oracle_finish(oracle_decoder *d);
FLAC__bool oracle_process_single(oracle_decoder *d);
FLAC__bool oracle_process_until_end_of_metadata(oracle_decoder *d);
FLAC__bool oracle_process_until_end_of_stream(oracle_decoder *d);
FLAC__bool oracle_seek_absolute(oracle_decoder *d, FLAC__uint64 sample);
FLAC__StreamDecoderState oracle_get_state(const oracle_decoder *d);
FLAC__uint64 oracle_get_total_samples(const oracle_decoder *d);
unsigned oracle_get_channels(const oracle_decoder *d);
unsigned oracle_get_bits_per_sample(const oracle_decoder *d);
unsigned oracle_get_sample_rate(const oracle_decoder *d);

/* ---- test drivers ------------------------------------------------------------------ */

enum { ORACLE_EV_METADATA = 1, ORACLE_EV_WRITE = 2, ORACLE_EV_ERROR = 3, ORACLE_EV_RETURN = 4, ORACLE_EV_SEEK = 5 };

typedef struct {
    int32_t kind;        /* ORACLE_EV_* */
    int32_t status;      /* error status / process_* return value */
    int32_t state;       /* decoder state right after the event */
    uint32_t blocksize, sample_rate, channels, assignment, bps;
    uint32_t crc8;
    uint64_t sample_number;
    uint64_t pcm_offset; /* for WRITE: offset (in int32 units) of this frame's planar PCM */
} oracle_event;

/* Decode an in-memory stream through the restated state machine.  The read callback
 * mimics FLACDecoder.ReadCallback (FLACDecoder.cs:325-363: at most read_chunk bytes per
 * call, END_OF_STREAM on a short read, EOF callback = "hit EOF yet").
 * driver 0: process_until_end_of_metadata, then process_single while state < EOS and
 *           the call returns true (the FLACDecoder.RequestAnotherFLACPacket loop);
 * driver 1: process_until_end_of_stream.
 * write_abort_at: frame index whose write callback returns ABORT (-1: never).
 * Planar int32 PCM of every written frame is appended channel-major to pcm. */
int oracle_run(const uint8_t *data, size_t len, int driver, int read_chunk, int write_abort_at,
               oracle_event *ev, int ev_cap, int *n_ev, int32_t *pcm, size_t pcm_cap,
               size_t *n_pcm);

/* FLACFileReader's seek pattern: seek_absolute issued from inside the write callback after
 * write seeks[2i] (-1: after the metadata pass), to sample seeks[2i+1]; a SEEK event carries
 * each seek_absolute return.  See flac_oracle.c. */
int oracle_run_seek(const uint8_t *data, size_t len, int read_chunk, const int64_t *seeks, int nseeks,
                    oracle_event *ev, int ev_cap, int *n_ev, int32_t *pcm, size_t pcm_cap, size_t *n_pcm);

/* One frame, decoded as read_frame_ would after frame_sync_ matched at byte `off`.
 * Returns 0 when a frame was produced (crc_ok tells whether the CRC-16 matched; on a
 * mismatch libFLAC zero-fills, and so does this), otherwise the first error status + 1.
 * *end_off receives the byte offset where libFLAC's reader stands afterwards. */
typedef struct {
    int32_t has_stream_info;
    uint32_t min_blocksize, max_blocksize, sample_rate, channels, bps;
    uint64_t total_samples;
} oracle_stream_params;

typedef struct {
    int32_t error;            /* -1 none, else FLAC__StreamDecoderErrorStatus */
    int32_t crc_ok;
    uint32_t blocksize, sample_rate, channels, assignment, bps;
    uint32_t number_type;     /* as parsed (before frame->sample conversion) */
    uint64_t number;
    uint64_t end_off;         /* byte offset just past the frame (or where the error left the reader) */
    int32_t cached;           /* lookahead byte cached by the header parser (-1 none) */
} oracle_frame_result;

int oracle_decode_frame_at(const uint8_t *data, size_t len, size_t off,
                           const oracle_stream_params *sp, int32_t *planar, size_t planar_cap,
                           oracle_frame_result *res);

/* BirdNest.Audio C# replays (exceptions become a non-zero return + message). */
/* FLACDecoder ctor + Stream.CopyTo(ms) with copy_chunk-byte Read calls
 * (FLACDecoder.cs:72-88, 124-233, 431-473, 520-580; OpenALDemo/Program.cs:26-35). */
int oracle_flacdecoder_copyto(const uint8_t *data, size_t len, int copy_chunk, uint8_t *out,
                              size_t cap, size_t *out_len, int32_t *fmt4, char *msg, int msg_cap);
/* FLACFileReader ctor + repeated Read(buf, 0, buf_len) until it returns 0
 * (FLACFileReader.cs:45-78, 145-254, 267-329). */
int oracle_filereader_readall(const uint8_t *data, size_t len, int buf_len, uint8_t *out,
                              size_t cap, size_t *out_len, char *msg, int msg_cap);
/* ... with Read(buf, 0, num_bytes) on a buf_len-byte buffer (num_bytes <= buf_len: overfill) */
int oracle_filereader_readall_n(const uint8_t *data, size_t len, int buf_len, int num_bytes, uint8_t *out,
                                size_t cap, size_t *out_len, char *msg, int msg_cap);

/* CRC helpers (poly 0x07 / 0x8005, init 0) -- exported for the generator tests. */
uint8_t oracle_crc8(const uint8_t *p, size_t n);
uint16_t oracle_crc16(const uint8_t *p, size_t n);

#ifdef __cplusplus
}
#endif

#endif
