/*
 * bnflac_synth.h -- deterministic synthetic FLAC stream generator.
 *
 * Produces the workloads named in BASELINE.json (configs C1-C5) and the coverage
 * corpus for the parity tests.  It is an encoder written for this repository (the
 * reference ships none, and no flac/libFLAC binary exists in the image): it emits
 * spec-conformant FLAC frames whose residuals are computed with exactly the
 * arithmetic the libFLAC 1.2.1 decoder uses to restore them, so PCM in == PCM out is
 * a lossless round-trip golden vector ("Golden vectors" (1)).
 *
 * This is input generation, not the decode path; the GPU decoder never calls it.
 */
#ifndef BNFLAC_SYNTH_H
#define BNFLAC_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    BNSYN_SUB_LPC = 0,      /* LPC of `order` (1..32) */
    BNSYN_SUB_FIXED = 1,    /* FIXED of `order` (0..4) */
    BNSYN_SUB_VERBATIM = 2,
    BNSYN_SUB_CONSTANT = 3,
    BNSYN_SUB_MIXED = 4     /* per-subframe random type/order (config C4) */
};

enum {
    BNSYN_STEREO_INDEPENDENT = 0,
    BNSYN_STEREO_LEFT_SIDE = 1,
    BNSYN_STEREO_RIGHT_SIDE = 2,
    BNSYN_STEREO_MID_SIDE = 3,
    BNSYN_STEREO_CYCLE = 4  /* frame i uses assignment i % 4 */
};

typedef struct {
    uint32_t sample_rate;
    uint32_t channels;          /* 1..8 */
    uint32_t bps;               /* 4..24 (frame header codes); up to 32 via STREAMINFO */
    uint32_t blocksize;         /* fixed-blocksize streams */
    uint32_t nframes;
    uint32_t last_blocksize;    /* 0: same as blocksize; else the short final frame */
    int32_t subframe_mode;      /* BNSYN_SUB_* */
    uint32_t order;             /* LPC (1..32) or FIXED (0..4) order */
    uint32_t qlp_precision;     /* 0: random in [12,15]; else 1..15 */
    int32_t partition_order;    /* >= 0 fixed (clamped to what the frame allows), -1 best */
    int32_t stereo_mode;        /* BNSYN_STEREO_* */
    uint32_t wasted_bits_max;   /* per frame, w uniform in [0, max] */
    int32_t variable_blocksize; /* 1: blocking-strategy bit set, bs random over legal codes */
    uint32_t bs_min, bs_max;    /* for variable blocksize */
    double level;               /* target peak level as a fraction of full scale (0.5 = -6 dBFS) */
    double noise;               /* excitation noise std as a fraction of full scale */
    uint64_t seed;
    int32_t rice2;              /* 1: partitioned RICE2 (5-bit parameters) */
    int32_t escape_permille;    /* probability of forcing an escape partition */
    int32_t write_header;       /* 1: "fLaC" + STREAMINFO (+ optional padding block) */
    int32_t force_sr_code;      /* -1 auto; else the 4-bit sample-rate code to use when valid */
    int32_t odd_headers;        /* 1: use 8/16-bit explicit blocksize and explicit-rate codes */
    int32_t prec_clamp;         /* 1: clamp LPC precision like libFLAC's encoder (<= 17-bit subframes
                                 * stay on the 32-bit restore path); 0: any precision (64-bit path) */
    int32_t impulse_permille;   /* probability per sample of an impulse of 0.4 x full scale: residuals far
                                 * above the partition's Rice parameter (unary prefixes beyond a
                                 * 32-bit window); 0 leaves the signal (and its random stream) as before */
} bnsyn_params;

void bnsyn_default_params(bnsyn_params *p);

/* Encode.  out: FLAC bytes (cap bytes).  pcm (optional): interleaved int32 source
 * samples, i.e. the expected decoder output.  frame_offsets (optional): byte offset of
 * every frame.  Returns 0 on success, <0 on error (-1 capacity, -2 bad params). */
int bnsyn_encode(const bnsyn_params *p, uint8_t *out, size_t cap, size_t *out_len, int32_t *pcm,
                 size_t pcm_cap, size_t *pcm_len, uint64_t *frame_offsets, size_t offsets_cap,
                 uint32_t *nframes_out);

/* Upper bound on the encoded size for the given parameters (bytes). */
size_t bnsyn_max_bytes(const bnsyn_params *p);

/* MD5 (RFC 1321) of buf, for STREAMINFO checks. */
void bnsyn_md5(const uint8_t *buf, size_t n, uint8_t out[16]);

#ifdef __cplusplus
}
#endif

#endif
