/*
 * bnflac_device.h -- device-side data contracts shared by the HIP kernels and the host
 * runtime (bnflac_runtime.cpp).  Plain structs, no torch types.
 */
#ifndef BNFLAC_DEVICE_H
#define BNFLAC_DEVICE_H

#include <stdint.h>

/* Per-candidate frame record, written by k_parse (header + subframes 0..C-2) and
 * completed by k_decode (last subframe, padding, CRC-16).  128 bytes. */
enum {
    BNF_ST_OK = 0,        /* frame decoded (crc_ok tells whether the CRC-16 matched) */
    BNF_ST_ERROR = 1,     /* libFLAC error callback status in `err`, reader at resume_bit */
    BNF_ST_TRUNC = 2,     /* ran past the end of the buffered data: libFLAC would block on read */
    BNF_ST_SKIPPED = 3    /* not processed (e.g. beyond the batch) */
};

typedef struct {
    uint32_t status;        /* BNF_ST_* */
    int32_t err;            /* FLAC__StreamDecoderErrorStatus when status == ERROR, else -1 */
    uint64_t frame_off;     /* byte offset of the 0xFF sync byte */
    uint64_t resume_bit;    /* absolute bit position of libFLAC's reader after the frame / error */
    int32_t cached;         /* lookahead byte cached by the header parser (-1 none) */
    uint32_t blocksize;
    uint32_t sample_rate;
    uint32_t channels;
    uint32_t assignment;
    uint32_t bps;
    uint32_t number_type;   /* as coded in the header (0 frame number, 1 sample number) */
    uint32_t unparseable;   /* header decoded but libFLAC flags it UNPARSEABLE_STREAM */
    uint64_t number;        /* frame or sample number as coded */
    uint64_t out_sample;    /* first output sample (per channel) of this frame in the batch output */
    uint32_t crc8;
    uint32_t crc16_calc;
    uint32_t crc16_read;
    uint32_t crc_ok;
    uint32_t sub_start[8];  /* bit offset of each subframe header, relative to frame_off*8 */
    uint32_t flags;         /* BNF_FL_* */
    uint32_t reserved;      /* 0 (the 128-byte record's last word) */
} bnf_frame_info;

enum {
    BNF_FL_NEEDS_SLOW = 1u,
    BNF_FL_OUT_OF_BOUNDS = 2u, /* set by k_decode: frame would end past out_bytes (SKIPPED) */
    BNF_FL_UNSUPPORTED = 4u,   /* set by k_decode: the output format cannot carry the frame (SKIPPED) */
    BNF_FL_W32 = 16u,          /* set by k_parse: an LPC order > 16 (decoded by k_decode<32>) */
    BNF_FL_ST = 32u,           /* set by k_parse: 2-channel frame, LPC orders <= 8 (k_decode_st's candidates) */
    BNF_FL_REDO = 64u,         /* set by k_decode_st: declined (rare case), decoded again by k_decode<8> */
    BNF_FL_W16 = 128u,         /* set by k_parse: LPC orders 9..16, or LPC above 16 bits (k_decode<16>) */
    BNF_FL_WAVE_REDO = 512u,   /* set by k_decode_sys: handed back, decoded again by k_decode_list */
    BNF_FL_SW = 1024u          /* set by k_parse: 2-channel W16 frame of 17..24 bits, LPC orders <= 12 (k_decode_sw's candidates) */
};

/* Output formats of k_decode */
enum {
    BNF_OUT_PLANAR32 = 0,     /* libFLAC write-callback buffers: per frame, channel-major int32 */
    BNF_OUT_INTERLEAVED32 = 1,/* int32 [sample][channel] */
    BNF_OUT_FLACDECODER = 2,  /* FLACDecoder.WriteCallback pack: 16-bit LE, stereo L/R or ch0 only */
    BNF_OUT_FILEREADER = 3    /* FLACFileReader pack: 2 or 3 bytes LE per sample, all channels */
};

typedef struct {
    int32_t has_stream_info;
    uint32_t min_blocksize, max_blocksize;
    uint32_t sample_rate, channels, bps;
    uint64_t total_samples;
} bnf_stream_params;

/* How k_decode positions frames in the output buffer. */
enum {
    BNF_POS_BY_NUMBER = 0,   /* out_sample = header sample number - base (libFLAC's own positioning) */
    BNF_POS_BY_SCAN = 1      /* out_sample precomputed by the caller/scan (compact, per candidate) */
};

#endif
