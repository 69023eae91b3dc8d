/*
 * flac_oracle.c -- CPU ORACLE, test infrastructure only (see flac_oracle.h).
 *
 * Restates libFLAC 1.2.1's stream decoder as shipped in the reference's
 * Library/BirdNest.Audio/LibFLACDLL/LibFlac.dll.  Function-level anchors are the DLL
 * virtual addresses catalogued in SURVEY.md section 8a (A1-A14); where this file
 * depends on a detail the survey does not state, the address it was read from is cited.
 * The C# pack rules (A15-A18) follow BirdNest.Audio's own sources, cited file:line.
 *
 * Plain scalar C on purpose: clarity over speed.  Never linked into the product.
 */
#include "flac_oracle.h"

#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- CRCs (A3, A4) */
/* CRC-8 poly x^8+x^2+x+1 (0x07), init 0: FLAC__crc8 @0x10002f90.
 * CRC-16 poly x^16+x^15+x^2+1 (0x8005), init 0: bitreader crc16 @0x10001270. */
static uint8_t crc8_tab[256];
static uint16_t crc16_tab[256];
static int crc_ready;

static void crc_init(void) {
    if (crc_ready) return;
    for (int i = 0; i < 256; i++) {
        uint8_t c = (uint8_t)i;
        for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
        crc8_tab[i] = c;
        uint16_t w = (uint16_t)(i << 8);
        for (int b = 0; b < 8; b++) w = (uint16_t)((w & 0x8000) ? (w << 1) ^ 0x8005 : (w << 1));
        crc16_tab[i] = w;
    }
    crc_ready = 1;
}

uint8_t oracle_crc8(const uint8_t *p, size_t n) {
    crc_init();
    uint8_t c = 0;
    for (size_t i = 0; i < n; i++) c = crc8_tab[c ^ p[i]];
    return c;
}

static uint16_t crc16_update(uint16_t crc, const uint8_t *p, size_t n) {
    crc_init();
    for (size_t i = 0; i < n; i++) crc = (uint16_t)((crc << 8) ^ crc16_tab[(crc >> 8) ^ p[i]]);
    return crc;
}

uint16_t oracle_crc16(const uint8_t *p, size_t n) { return crc16_update(0, p, n); }

/* ------------------------------------------------------------------ decoder state */
struct oracle_decoder {
    FLAC__StreamDecoderState state;
    FLAC__StreamDecoderReadCallback read_cb;
    FLAC__StreamDecoderSeekCallback seek_cb;
    FLAC__StreamDecoderTellCallback tell_cb;
    FLAC__StreamDecoderLengthCallback length_cb;
    FLAC__StreamDecoderEofCallback eof_cb;
    FLAC__StreamDecoderWriteCallback write_cb;
    FLAC__StreamDecoderMetadataCallback metadata_cb;
    FLAC__StreamDecoderErrorCallback error_cb;
    void *client;

    /* bit reader: every byte handed over by the read callback is kept; bitpos is the
     * consumed position (libFLAC's consumed_words/consumed_bits). */
    uint8_t *buf;
    size_t len, cap;
    uint64_t bitpos;
    size_t crc_from;   /* CRC-16 runs over buf[crc_from .. consumed) */
    uint16_t crc_seed;

    int cached;
    uint8_t lookahead;
    uint8_t header_warmup[2];

    int has_stream_info;
    FLAC__StreamMetadata stream_info;
    uint64_t samples_decoded;
    unsigned fixed_block_size, next_fixed_block_size;

    FLAC__Frame frame;
    uint32_t raw_number_type;  /* header number before frame->sample conversion */
    uint64_t raw_number;
    int32_t *output[FLAC__MAX_CHANNELS];
    int32_t *residual[FLAC__MAX_CHANNELS];
    unsigned output_capacity, output_channels;
    unsigned rice_params[FLAC__MAX_CHANNELS][1u << 15];
    unsigned rice_raw[FLAC__MAX_CHANNELS][1u << 15];
    FLAC__EntropyCodingMethod_PartitionedRiceContents rice_contents[FLAC__MAX_CHANNELS];

    /* seeking (seek_absolute / seek_to_absolute_sample_) */
    int is_seeking;
    uint64_t first_frame_offset, target_sample;

    /* FLAC__StreamDecoderProtected */
    unsigned channels, bits_per_sample, sample_rate, blocksize;
    FLAC__ChannelAssignment channel_assignment;
    unsigned read_request;
};

/* --------------------------------------------------------------------- bit reader */
/* read_callback_ (stream_decoder.c) semantics: eof callback first, abort/EOS handling
 * exactly as libFLAC 1.2.1 (SURVEY.md 8b "ReadCallback"). */
static int br_fill(oracle_decoder *d) {
    for (int spins = 0; spins < 1000000; spins++) {
        if (d->eof_cb && d->eof_cb((const FLAC__StreamDecoder *)d, d->client)) {
            d->state = FLAC__STREAM_DECODER_END_OF_STREAM;
            return 0;
        }
        size_t bytes = d->read_request ? d->read_request : 8192;
        if (d->len + bytes > d->cap) {
            size_t nc = d->cap ? d->cap * 2 : 65536;
            while (nc < d->len + bytes) nc *= 2;
            d->buf = (uint8_t *)realloc(d->buf, nc + 8);
            d->cap = nc;
        }
        FLAC__StreamDecoderReadStatus st =
            d->read_cb((const FLAC__StreamDecoder *)d, d->buf + d->len, &bytes, d->client);
        if (st == FLAC__STREAM_DECODER_READ_STATUS_ABORT) {
            d->state = FLAC__STREAM_DECODER_ABORTED;
            return 0;
        }
        if (bytes == 0) {
            if (st == FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM ||
                (d->eof_cb && d->eof_cb((const FLAC__StreamDecoder *)d, d->client))) {
                d->state = FLAC__STREAM_DECODER_END_OF_STREAM;
                return 0;
            }
            continue; /* libFLAC retries */
        }
        d->len += bytes;
        return 1;
    }
    d->state = FLAC__STREAM_DECODER_ABORTED;
    return 0;
}

static int br_need(oracle_decoder *d, uint64_t bits) {
    while ((uint64_t)d->len * 8u - d->bitpos < bits)
        if (!br_fill(d)) return 0;
    return 1;
}

/* up to 32 bits at the cursor, MSB first (libFLAC's bitreader works on whole 32-bit
 * words; this reads the 5 bytes that can hold them).  Bytes past len read as 0: callers
 * have already checked availability with br_need. */
static uint32_t br_peek_bits(const oracle_decoder *d, unsigned bits) { /* 1..32 */
    const uint64_t byte = d->bitpos >> 3;
    uint64_t w = 0;
    for (unsigned i = 0; i < 5; i++) w = (w << 8) | (byte + i < d->len ? d->buf[byte + i] : 0u);
    w <<= 24 + (d->bitpos & 7);           /* cursor bit at bit 63 */
    return (uint32_t)(w >> (64 - bits));
}

/* FLAC__bitreader_read_raw_uint32: bits == 0 yields 0. */
static int br_u32(oracle_decoder *d, uint32_t *v, unsigned bits) {
    if (bits == 0) { *v = 0; return 1; }
    if (!br_need(d, bits)) return 0;
    *v = br_peek_bits(d, bits);
    d->bitpos += bits;
    return 1;
}

/* FLAC__bitreader_read_raw_int32: sign extension by (x << (32-bits)) >> (32-bits); x86
 * masks the count, so bits == 0 gives 0. */
static int br_i32(oracle_decoder *d, int32_t *v, unsigned bits) {
    uint32_t u;
    if (!br_u32(d, &u, bits)) return 0;
    unsigned s = (32u - bits) & 31u;
    *v = (int32_t)(u << s) >> s;
    return 1;
}

static int br_u64(oracle_decoder *d, uint64_t *v, unsigned bits) {
    uint32_t hi = 0, lo = 0;
    if (bits > 32) {
        if (!br_u32(d, &hi, bits - 32)) return 0;
        if (!br_u32(d, &lo, 32)) return 0;
        *v = ((uint64_t)hi << 32) | lo;
    } else {
        if (!br_u32(d, &lo, bits)) return 0;
        *v = lo;
    }
    return 1;
}

/* FLAC__bitreader_read_unary_unsigned @0x10001960 */
static int br_unary(oracle_decoder *d, uint32_t *v) {
    uint32_t n = 0;
    for (;;) {
        uint64_t avail = (uint64_t)d->len * 8u - d->bitpos;
        if (avail == 0) {
            if (!br_need(d, 1)) return 0;
            continue;
        }
        unsigned take = avail >= 32 ? 32u : (unsigned)avail;
        uint32_t w = br_peek_bits(d, take) << (32 - take);
        if (w) {
            unsigned z = (unsigned)__builtin_clz(w);
            d->bitpos += z + 1;
            *v = n + z;
            return 1;
        }
        n += take;
        d->bitpos += take;
    }
}

/* FLAC__bitreader_read_rice_signed_block: C @0x10001b30 / asm-bswap @0x1001aed0.
 * u = (q << k) | lsbs in 32-bit unsigned arithmetic, r = (u >> 1) ^ -(u & 1). */
static int br_rice_block(oracle_decoder *d, int32_t *vals, unsigned n, unsigned k) {
    for (unsigned i = 0; i < n; i++) {
        uint32_t q, lsb;
        /* fast path: one 64-bit big-endian window holds the whole codeword */
        if ((uint64_t)d->len * 8u - d->bitpos >= 64) {
            const uint8_t *p = d->buf + (d->bitpos >> 3);
            uint64_t w = 0;
            for (int b = 0; b < 8; b++) w = (w << 8) | p[b];
            const unsigned sh = (unsigned)(d->bitpos & 7u);
            w <<= sh;
            if (w) {
                const unsigned z = (unsigned)__builtin_clzll(w);
                if (z + 1u + k <= 64u - sh) {
                    lsb = k ? (uint32_t)((w << (z + 1)) >> (64 - k)) : 0u;
                    d->bitpos += z + 1u + k;
                    const uint32_t u = (k ? ((uint32_t)z << k) : (uint32_t)z) | lsb;
                    vals[i] = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1u)));
                    continue;
                }
            }
        }
        if (!br_unary(d, &q)) return 0;
        if (!br_u32(d, &lsb, k)) return 0;
        uint32_t u = (k ? (q << k) : q) | lsb;
        vals[i] = (int32_t)((u >> 1) ^ (uint32_t)(-(int32_t)(u & 1u)));
    }
    return 1;
}

static int br_aligned(const oracle_decoder *d) { return (d->bitpos & 7u) == 0; }

static int br_skip_bytes(oracle_decoder *d, uint32_t n) {
    if (!br_need(d, (uint64_t)n * 8u)) return 0;
    d->bitpos += (uint64_t)n * 8u;
    return 1;
}

static int br_read_bytes(oracle_decoder *d, uint8_t *dst, uint32_t n) {
    if (!br_need(d, (uint64_t)n * 8u)) return 0;
    memcpy(dst, d->buf + (d->bitpos >> 3), n);
    d->bitpos += (uint64_t)n * 8u;
    return 1;
}

/* FLAC__bitreader_read_utf8_uint32 @0x10001e20 -- note libFLAC's truthiness tests
 * ("x & 0xC0 && !(x & 0x20)"), which accept some continuation bytes as lead bytes. */
static int br_utf8_u32(oracle_decoder *d, uint32_t *val, uint8_t *raw, unsigned *rawlen) {
    uint32_t v = 0, x;
    unsigned i;
    if (!br_u32(d, &x, 8)) return 0;
    raw[(*rawlen)++] = (uint8_t)x;
    if (!(x & 0x80)) { v = x; i = 0; }
    else if ((x & 0xC0) && !(x & 0x20)) { v = x & 0x1F; i = 1; }
    else if ((x & 0xE0) && !(x & 0x10)) { v = x & 0x0F; i = 2; }
    else if ((x & 0xF0) && !(x & 0x08)) { v = x & 0x07; i = 3; }
    else if ((x & 0xF8) && !(x & 0x04)) { v = x & 0x03; i = 4; }
    else if ((x & 0xFC) && !(x & 0x02)) { v = x & 0x01; i = 5; }
    else { *val = 0xffffffffu; return 1; }
    for (; i; i--) {
        if (!br_u32(d, &x, 8)) return 0;
        raw[(*rawlen)++] = (uint8_t)x;
        if (!(x & 0x80) || (x & 0x40)) { *val = 0xffffffffu; return 1; }
        v <<= 6;
        v |= (x & 0x3F);
    }
    *val = v;
    return 1;
}

/* FLAC__bitreader_read_utf8_uint64 @0x10001f60 */
static int br_utf8_u64(oracle_decoder *d, uint64_t *val, uint8_t *raw, unsigned *rawlen) {
    uint64_t v = 0;
    uint32_t x;
    unsigned i;
    if (!br_u32(d, &x, 8)) return 0;
    raw[(*rawlen)++] = (uint8_t)x;
    if (!(x & 0x80)) { v = x; i = 0; }
    else if ((x & 0xC0) && !(x & 0x20)) { v = x & 0x1F; i = 1; }
    else if ((x & 0xE0) && !(x & 0x10)) { v = x & 0x0F; i = 2; }
    else if ((x & 0xF0) && !(x & 0x08)) { v = x & 0x07; i = 3; }
    else if ((x & 0xF8) && !(x & 0x04)) { v = x & 0x03; i = 4; }
    else if ((x & 0xFC) && !(x & 0x02)) { v = x & 0x01; i = 5; }
    else if ((x & 0xFE) && !(x & 0x01)) { v = 0; i = 6; }
    else { *val = 0xffffffffffffffffull; return 1; }
    for (; i; i--) {
        if (!br_u32(d, &x, 8)) return 0;
        raw[(*rawlen)++] = (uint8_t)x;
        if (!(x & 0x80) || (x & 0x40)) { *val = 0xffffffffffffffffull; return 1; }
        v <<= 6;
        v |= (x & 0x3F);
    }
    *val = v;
    return 1;
}

static void send_error(oracle_decoder *d, FLAC__StreamDecoderErrorStatus st) { /* send_error_to_client_ */
    if (d->error_cb && !d->is_seeking) d->error_cb((const FLAC__StreamDecoder *)d, st, d->client);
}

/* ------------------------------------------------------------------ restore kernels */
/* FLAC__fixed_restore_signal @0x10003810 (orders at @0x10003827/839/863/896/8cc);
 * 32-bit wrapping arithmetic. */
static void fixed_restore(const int32_t *res, unsigned n, unsigned order, int32_t *data) {
    uint32_t *o = (uint32_t *)data;
    const uint32_t *r = (const uint32_t *)res;
    for (unsigned i = 0; i < n; i++) {
        uint32_t v;
        switch (order) {
        case 0: v = r[i]; break;
        case 1: v = r[i] + o[(int)i - 1]; break;
        case 2: v = r[i] + (o[(int)i - 1] << 1) - o[(int)i - 2]; break;
        case 3: v = r[i] + (((o[(int)i - 1] - o[(int)i - 2]) << 1) + (o[(int)i - 1] - o[(int)i - 2])) + o[(int)i - 3]; break;
        default: v = r[i] + ((o[(int)i - 1] + o[(int)i - 3]) << 2) - ((o[(int)i - 2] << 2) + (o[(int)i - 2] << 1)) - o[(int)i - 4]; break;
        }
        o[i] = v;
    }
}

static int32_t sat16(int32_t x) { return x > 32767 ? 32767 : (x < -32768 ? -32768 : x); }
static int32_t trunc16(int32_t x) { return (int32_t)(int16_t)(uint16_t)(uint32_t)x; }

/* 32-bit restore through the ia32 asm routine @0x1001be10 (imul wrap, sar %cl: the
 * shift count is masked to 5 bits).  Also what the C routine @0x10005a00 computes for
 * non-negative shifts. */
static void lpc_restore_32(const int32_t *res, unsigned n, const int32_t *c, unsigned order,
                           int shift, int32_t *data) {
    for (unsigned i = 0; i < n; i++) {
        uint32_t sum = 0;
        for (unsigned j = 0; j < order; j++) sum += (uint32_t)c[j] * (uint32_t)data[(int)i - 1 - (int)j];
        data[i] = (int32_t)((uint32_t)res[i] + (uint32_t)((int32_t)sum >> (shift & 31)));
    }
}

/* 16-bit path on MMX CPUs, @0x1001c000, for order >= 4 (order < 4 jumps to the ia32
 * routine at @0x1001be2c).  Coefficients as int16, pmaddwd/paddd wrap in 32 bits.  The
 * four most recent history words live in mm4: seeded from the warm-up with packssdw
 * (saturation) and refilled with the low 16 bits of each new sample (psllq $0x30);
 * older groups are reloaded from memory with packssdw each step.  psrad takes a 64-bit
 * count: a negative shift (>= 32 as unsigned) fills with the sign bit. */
static void lpc_restore_16_mmx(const int32_t *res, unsigned n, const int32_t *c, unsigned order,
                               int shift, int32_t *data) {
    int32_t hs[FLAC__MAX_LPC_ORDER + 4]; /* scratch: per-tap history words */
    for (unsigned i = 0; i < n; i++) {
        uint32_t sum = 0;
        for (unsigned j = 0; j < order; j++) {
            int idx = (int)i - 1 - (int)j;
            /* taps 0..3 come from mm4: low 16 bits of computed samples, saturated
             * warm-ups; older taps are reloaded from memory with packssdw */
            hs[j] = (j < 4 && idx >= 0) ? trunc16(data[idx]) : sat16(data[idx]);
        }
        for (unsigned j = 0; j < order; j++) sum += (uint32_t)((int32_t)(int16_t)c[j] * hs[j]);
        int32_t sh = ((uint32_t)shift >= 32u) ? ((int32_t)sum >> 31) : ((int32_t)sum >> shift);
        data[i] = (int32_t)((uint32_t)res[i] + (uint32_t)sh);
    }
}

/* FLAC__lpc_restore_signal_wide @0x10006120: exact int64 sum, MSVC _allshr @0x1001d080
 * (count = low byte of the shift; >= 64 fills with the sign bit), truncated to int32. */
static void lpc_restore_64(const int32_t *res, unsigned n, const int32_t *c, unsigned order,
                           int shift, int32_t *data) {
    for (unsigned i = 0; i < n; i++) {
        int64_t sum = 0;
        for (unsigned j = 0; j < order; j++) sum += (int64_t)c[j] * (int64_t)data[(int)i - 1 - (int)j];
        unsigned cnt = (unsigned)shift & 0xFFu;
        int64_t q = (cnt >= 64) ? (sum >> 63) : (sum >> cnt);
        data[i] = (int32_t)((uint32_t)res[i] + (uint32_t)(int32_t)q);
    }
}

static unsigned ilog2u(unsigned v) { /* FLAC__bitmath_ilog2 @0x10001000 */
    unsigned l = 0;
    while (v >>= 1) l++;
    return l;
}

/* ---------------------------------------------------------------- frame decoding */
static int allocate_output(oracle_decoder *d, unsigned size, unsigned channels) {
    if (size <= d->output_capacity && channels <= d->output_channels) return 1;
    for (unsigned i = 0; i < FLAC__MAX_CHANNELS; i++) {
        free(d->output[i] ? d->output[i] - 4 : NULL);
        free(d->residual[i]);
        d->output[i] = d->residual[i] = NULL;
    }
    for (unsigned i = 0; i < channels; i++) {
        /* libFLAC mallocs (uninitialised); zero here so the stale-tail quirk is defined */
        d->output[i] = (int32_t *)calloc(size + 4, sizeof(int32_t)) + 4;
        d->residual[i] = (int32_t *)calloc(size ? size : 1, sizeof(int32_t));
    }
    d->output_capacity = size;
    d->output_channels = channels;
    return 1;
}

/* read_residual_partitioned_rice_ @0x10012da0 */
static int read_residual(oracle_decoder *d, unsigned pred_order, unsigned porder, int ch,
                         int32_t *residual, int is_extended) {
    const unsigned partitions = 1u << porder;
    const unsigned bs = d->frame.header.blocksize;
    const unsigned psamples = porder > 0 ? bs >> porder : bs - pred_order;
    const unsigned plen = is_extended ? 5 : 4;
    const unsigned pesc = is_extended ? 31 : 15;
    if (porder == 0) {
        if (bs < pred_order) { /* @0x10012e41 */
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
    } else if (psamples < pred_order) { /* @0x10012e1e */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    if (porder > 0 && (bs & (partitions - 1u))) {
        /* libFLAC 1.2.1 restores over stale residual memory here; both this oracle and
         * the GPU path reject the (RFC-invalid) layout instead. */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    unsigned sample = 0;
    for (unsigned p = 0; p < partitions; p++) {
        uint32_t k;
        if (!br_u32(d, &k, plen)) return 0;
        d->rice_params[ch][p] = k;
        if (k < pesc) {
            d->rice_raw[ch][p] = 0;
            unsigned u = (porder == 0 || p > 0) ? psamples : psamples - pred_order;
            if (!br_rice_block(d, residual + sample, u, k)) return 0;
            sample += u;
        } else {
            uint32_t nb;
            if (!br_u32(d, &nb, 5)) return 0;
            d->rice_raw[ch][p] = nb;
            for (unsigned u = (porder == 0 || p > 0) ? 0 : pred_order; u < psamples; u++, sample++) {
                int32_t x;
                if (!br_i32(d, &x, nb)) return 0;
                residual[sample] = x;
            }
        }
    }
    return 1;
}

static int read_entropy_header(oracle_decoder *d, FLAC__EntropyCodingMethod *m, int ch) {
    uint32_t u;
    if (!br_u32(d, &u, 2)) return 0;
    m->type = (FLAC__EntropyCodingMethodType)u;
    if (u > 1) { /* FIXED @0x100127ed, LPC @0x10012a99 */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    if (!br_u32(d, &u, 4)) return 0;
    m->data.partitioned_rice.order = u;
    d->rice_contents[ch].parameters = d->rice_params[ch];
    d->rice_contents[ch].raw_bits = d->rice_raw[ch];
    d->rice_contents[ch].capacity_by_order = u;
    m->data.partitioned_rice.contents = &d->rice_contents[ch];
    return 1;
}

/* read_subframe_constant_ @0x10012690 */
static int read_subframe_constant(oracle_decoder *d, int ch, unsigned bps) {
    FLAC__Subframe *sf = &d->frame.subframes[ch];
    int32_t x;
    sf->type = FLAC__SUBFRAME_TYPE_CONSTANT;
    if (!br_i32(d, &x, bps)) return 0;
    sf->data.constant.value = x;
    for (unsigned i = 0; i < d->frame.header.blocksize; i++) d->output[ch][i] = x;
    return 1;
}

/* read_subframe_verbatim_ @0x10012ce0 */
static int read_subframe_verbatim(oracle_decoder *d, int ch, unsigned bps) {
    FLAC__Subframe *sf = &d->frame.subframes[ch];
    sf->type = FLAC__SUBFRAME_TYPE_VERBATIM;
    sf->data.verbatim.data = d->residual[ch];
    for (unsigned i = 0; i < d->frame.header.blocksize; i++) {
        int32_t x;
        if (!br_i32(d, &x, bps)) return 0;
        d->residual[ch][i] = x;
    }
    memcpy(d->output[ch], d->residual[ch], sizeof(int32_t) * d->frame.header.blocksize);
    return 1;
}

/* read_subframe_fixed_ @0x10012720 */
static int read_subframe_fixed(oracle_decoder *d, int ch, unsigned bps, unsigned order) {
    FLAC__Subframe *sf = &d->frame.subframes[ch];
    FLAC__Subframe_Fixed *fx = &sf->data.fixed;
    sf->type = FLAC__SUBFRAME_TYPE_FIXED;
    fx->residual = d->residual[ch];
    fx->order = order;
    for (unsigned u = 0; u < order; u++) {
        int32_t x;
        if (!br_i32(d, &x, bps)) return 0;
        fx->warmup[u] = x;
    }
    if (!read_entropy_header(d, &fx->entropy_coding_method, ch)) return 0;
    if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    if (!read_residual(d, order, fx->entropy_coding_method.data.partitioned_rice.order, ch,
                       d->residual[ch], fx->entropy_coding_method.type == FLAC__ENTROPY_CODING_METHOD_PARTITIONED_RICE2))
        return 0;
    if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    memcpy(d->output[ch], fx->warmup, sizeof(int32_t) * order);
    fixed_restore(d->residual[ch], d->frame.header.blocksize - order, order, d->output[ch] + order);
    return 1;
}

/* read_subframe_lpc_ @0x10012900, restore dispatch @0x10012b7a-0x10012c9f */
static int read_subframe_lpc(oracle_decoder *d, int ch, unsigned bps, unsigned order) {
    FLAC__Subframe *sf = &d->frame.subframes[ch];
    FLAC__Subframe_LPC *lp = &sf->data.lpc;
    uint32_t u32;
    int32_t i32;
    sf->type = FLAC__SUBFRAME_TYPE_LPC;
    lp->residual = d->residual[ch];
    lp->order = order;
    for (unsigned u = 0; u < order; u++) {
        if (!br_i32(d, &i32, bps)) return 0;
        lp->warmup[u] = i32;
    }
    if (!br_u32(d, &u32, 4)) return 0;
    if (u32 == 15) {
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    lp->qlp_coeff_precision = u32 + 1;
    if (!br_i32(d, &i32, 5)) return 0;
    lp->quantization_level = i32; /* negative values are not rejected by 1.2.1 */
    for (unsigned u = 0; u < order; u++) {
        if (!br_i32(d, &i32, lp->qlp_coeff_precision)) return 0;
        lp->qlp_coeff[u] = i32;
    }
    if (!read_entropy_header(d, &lp->entropy_coding_method, ch)) return 0;
    if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    if (!read_residual(d, order, lp->entropy_coding_method.data.partitioned_rice.order, ch,
                       d->residual[ch], lp->entropy_coding_method.type == FLAC__ENTROPY_CODING_METHOD_PARTITIONED_RICE2))
        return 0;
    if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    memcpy(d->output[ch], lp->warmup, sizeof(int32_t) * order);
    unsigned n = d->frame.header.blocksize - order;
    int32_t *out = d->output[ch] + order;
    if (bps + lp->qlp_coeff_precision + ilog2u(order) <= 32) {
        if (bps <= 16 && lp->qlp_coeff_precision <= 16 && order >= 4)
            lpc_restore_16_mmx(d->residual[ch], n, lp->qlp_coeff, order, lp->quantization_level, out);
        else
            lpc_restore_32(d->residual[ch], n, lp->qlp_coeff, order, lp->quantization_level, out);
    } else {
        lpc_restore_64(d->residual[ch], n, lp->qlp_coeff, order, lp->quantization_level, out);
    }
    return 1;
}

/* read_subframe_ @0x10012480.  bps > 32 (side channel of a 32-bit STREAMINFO stream)
 * and wasted >= bps+1 are undefined in libFLAC (raw reads > 32 bits); this oracle, like
 * the GPU path, reports them as UNPARSEABLE_STREAM. */
static int read_subframe(oracle_decoder *d, int ch, unsigned bps) {
    uint32_t x;
    if (!br_u32(d, &x, 8)) return 0;
    unsigned wasted = x & 1u;
    x &= 0xFEu;
    FLAC__Subframe *sf = &d->frame.subframes[ch];
    if (wasted) {
        uint32_t u;
        if (!br_unary(d, &u)) return 0; /* @0x100124d4 */
        sf->wasted_bits = u + 1;
        if (sf->wasted_bits > bps) {
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
        bps -= sf->wasted_bits;
    } else {
        sf->wasted_bits = 0;
    }
    if (x & 0x80) { /* @0x10012537 */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    if (bps > 32) {
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    if (x == 0) {
        if (!read_subframe_constant(d, ch, bps)) return 0;
    } else if (x == 2) {
        if (!read_subframe_verbatim(d, ch, bps)) return 0;
    } else if (x < 16) { /* @0x10012590 */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    } else if (x <= 24) {
        if (!read_subframe_fixed(d, ch, bps, (x >> 1) & 7u)) return 0;
        if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    } else if (x < 64) { /* @0x100125f0 */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    } else {
        if (!read_subframe_lpc(d, ch, bps, ((x >> 1) & 31u) + 1)) return 0;
        if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    }
    if (wasted) { /* @0x10012660-0x1001267c */
        for (unsigned i = 0; i < d->frame.header.blocksize; i++)
            d->output[ch][i] = (int32_t)((uint32_t)d->output[ch][i] << sf->wasted_bits);
    }
    return 1;
}

/* read_frame_header_ @0x10011d70 */
static int read_frame_header(oracle_decoder *d) {
    uint32_t x;
    uint64_t xx;
    unsigned blocksize_hint = 0, sample_rate_hint = 0;
    uint8_t raw[16];
    unsigned rawlen = 2;
    int unparseable = 0;
    FLAC__FrameHeader *h = &d->frame.header;
    raw[0] = d->header_warmup[0];
    raw[1] = d->header_warmup[1];
    if (raw[1] & 0x02) unparseable = 1;
    for (int i = 0; i < 2; i++) {
        if (!br_u32(d, &x, 8)) return 0;
        if (x == 0xff) { /* sync code inside the header: @0x10011e18 */
            d->lookahead = 0xff;
            d->cached = 1;
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
        raw[rawlen++] = (uint8_t)x;
    }
    switch (x = raw[2] >> 4) {
    case 0: unparseable = 1; break;
    case 1: h->blocksize = 192; break;
    case 2: case 3: case 4: case 5: h->blocksize = 576u << (x - 2); break;
    case 6: case 7: blocksize_hint = x; break;
    default: h->blocksize = 256u << (x - 8); break;
    }
    switch (x = raw[2] & 0x0f) {
    case 0:
        if (d->has_stream_info) h->sample_rate = d->stream_info.data.stream_info.sample_rate;
        else unparseable = 1;
        break;
    case 1: h->sample_rate = 88200; break;
    case 2: h->sample_rate = 176400; break;
    case 3: h->sample_rate = 192000; break;
    case 4: h->sample_rate = 8000; break;
    case 5: h->sample_rate = 16000; break;
    case 6: h->sample_rate = 22050; break;
    case 7: h->sample_rate = 24000; break;
    case 8: h->sample_rate = 32000; break;
    case 9: h->sample_rate = 44100; break;
    case 10: h->sample_rate = 48000; break;
    case 11: h->sample_rate = 96000; break;
    case 12: case 13: case 14: sample_rate_hint = x; break;
    default:
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    x = (unsigned)(raw[3] >> 4);
    if (x & 8) {
        h->channels = 2;
        switch (x & 7) {
        case 0: h->channel_assignment = FLAC__CHANNEL_ASSIGNMENT_LEFT_SIDE; break;
        case 1: h->channel_assignment = FLAC__CHANNEL_ASSIGNMENT_RIGHT_SIDE; break;
        case 2: h->channel_assignment = FLAC__CHANNEL_ASSIGNMENT_MID_SIDE; break;
        default: unparseable = 1; break;
        }
    } else {
        h->channels = x + 1;
        h->channel_assignment = FLAC__CHANNEL_ASSIGNMENT_INDEPENDENT;
    }
    switch (x = (unsigned)(raw[3] & 0x0e) >> 1) {
    case 0:
        if (d->has_stream_info) h->bits_per_sample = d->stream_info.data.stream_info.bits_per_sample;
        else unparseable = 1;
        break;
    case 1: h->bits_per_sample = 8; break;
    case 2: h->bits_per_sample = 12; break;
    case 4: h->bits_per_sample = 16; break;
    case 5: h->bits_per_sample = 20; break;
    case 6: h->bits_per_sample = 24; break;
    default: unparseable = 1; break;
    }
    if (raw[3] & 0x01) unparseable = 1;
    if ((raw[1] & 0x01) ||
        (d->has_stream_info && d->stream_info.data.stream_info.min_blocksize != d->stream_info.data.stream_info.max_blocksize)) {
        if (!br_utf8_u64(d, &xx, raw, &rawlen)) return 0;
        if (xx == 0xffffffffffffffffull) {
            d->lookahead = raw[rawlen - 1];
            d->cached = 1;
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
        h->number_type = FLAC__FRAME_NUMBER_TYPE_SAMPLE_NUMBER;
        h->number.sample_number = xx;
    } else {
        if (!br_utf8_u32(d, &x, raw, &rawlen)) return 0;
        if (x == 0xffffffffu) {
            d->lookahead = raw[rawlen - 1];
            d->cached = 1;
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
        h->number_type = FLAC__FRAME_NUMBER_TYPE_FRAME_NUMBER;
        h->number.sample_number = 0;
        h->number.frame_number = x;
    }
    if (blocksize_hint) {
        if (!br_u32(d, &x, 8)) return 0;
        raw[rawlen++] = (uint8_t)x;
        if (blocksize_hint == 7) {
            uint32_t y;
            if (!br_u32(d, &y, 8)) return 0;
            raw[rawlen++] = (uint8_t)y;
            x = (x << 8) | y;
        }
        h->blocksize = x + 1;
    }
    if (sample_rate_hint) {
        if (!br_u32(d, &x, 8)) return 0;
        raw[rawlen++] = (uint8_t)x;
        if (sample_rate_hint != 12) {
            uint32_t y;
            if (!br_u32(d, &y, 8)) return 0;
            raw[rawlen++] = (uint8_t)y;
            x = (x << 8) | y;
        }
        if (sample_rate_hint == 12) h->sample_rate = x * 1000;
        else if (sample_rate_hint == 13) h->sample_rate = x;
        else h->sample_rate = x * 10;
    }
    if (!br_u32(d, &x, 8)) return 0;
    h->crc = (uint8_t)x;
    if (oracle_crc8(raw, rawlen) != (uint8_t)x) { /* @0x10012314 */
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_BAD_HEADER);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    d->raw_number_type = h->number_type;
    d->raw_number = (h->number_type == FLAC__FRAME_NUMBER_TYPE_FRAME_NUMBER) ? h->number.frame_number : h->number.sample_number;
    /* frame number -> sample number @0x1001231f-0x100123ca */
    d->next_fixed_block_size = 0;
    if (h->number_type == FLAC__FRAME_NUMBER_TYPE_FRAME_NUMBER) {
        uint32_t fn = h->number.frame_number;
        h->number_type = FLAC__FRAME_NUMBER_TYPE_SAMPLE_NUMBER;
        if (d->fixed_block_size) {
            h->number.sample_number = (uint64_t)d->fixed_block_size * fn;
        } else if (d->has_stream_info) {
            if (d->stream_info.data.stream_info.min_blocksize == d->stream_info.data.stream_info.max_blocksize) {
                h->number.sample_number = (uint64_t)d->stream_info.data.stream_info.min_blocksize * fn;
                d->next_fixed_block_size = d->stream_info.data.stream_info.max_blocksize;
            } else {
                unparseable = 1;
            }
        } else if (fn == 0) {
            h->number.sample_number = 0;
            d->next_fixed_block_size = h->blocksize;
        } else {
            h->number.sample_number = (uint64_t)h->blocksize * fn;
        }
    }
    if (unparseable) {
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return 1;
    }
    return 1;
}

/* read_frame_ @0x100118c0.  got_frame set when a frame reached the write stage. */
static int read_frame(oracle_decoder *d, int *got_frame, int *crc_ok_out) {
    *got_frame = 0;
    uint8_t hw[2] = {d->header_warmup[0], d->header_warmup[1]};
    d->crc_seed = crc16_update(0, hw, 2);
    d->crc_from = (size_t)(d->bitpos >> 3);
    if (!read_frame_header(d)) return 0;
    if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    if (!allocate_output(d, d->frame.header.blocksize, d->frame.header.channels)) return 0;
    for (unsigned ch = 0; ch < d->frame.header.channels; ch++) {
        unsigned bps = d->frame.header.bits_per_sample;
        switch (d->frame.header.channel_assignment) {
        case FLAC__CHANNEL_ASSIGNMENT_LEFT_SIDE: if (ch == 1) bps++; break;
        case FLAC__CHANNEL_ASSIGNMENT_RIGHT_SIDE: if (ch == 0) bps++; break;
        case FLAC__CHANNEL_ASSIGNMENT_MID_SIDE: if (ch == 1) bps++; break;
        default: break;
        }
        if (!read_subframe(d, (int)ch, bps)) return 0;
        if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    }
    /* read_zero_padding_ @0x10012fe0 */
    if (!br_aligned(d)) {
        uint32_t z;
        if (!br_u32(d, &z, 8u - (unsigned)(d->bitpos & 7u))) return 0;
        if (z != 0) {
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return 1;
        }
    }
    uint16_t crc = crc16_update(d->crc_seed, d->buf + d->crc_from, (size_t)(d->bitpos >> 3) - d->crc_from);
    uint32_t x;
    if (!br_u32(d, &x, 16)) return 0;
    d->frame.footer.crc = (uint16_t)x;
    const unsigned bs = d->frame.header.blocksize;
    int32_t **o = d->output;
    if (crc == x) { /* @0x10011a01; decorrelation @0x10011a37-0x10011adb */
        if (crc_ok_out) *crc_ok_out = 1;
        switch (d->frame.header.channel_assignment) {
        case FLAC__CHANNEL_ASSIGNMENT_LEFT_SIDE:
            for (unsigned i = 0; i < bs; i++) o[1][i] = (int32_t)((uint32_t)o[0][i] - (uint32_t)o[1][i]);
            break;
        case FLAC__CHANNEL_ASSIGNMENT_RIGHT_SIDE:
            for (unsigned i = 0; i < bs; i++) o[0][i] = (int32_t)((uint32_t)o[0][i] + (uint32_t)o[1][i]);
            break;
        case FLAC__CHANNEL_ASSIGNMENT_MID_SIDE:
            for (unsigned i = 0; i < bs; i++) {
                uint32_t mid = (uint32_t)o[0][i], side = (uint32_t)o[1][i];
                mid <<= 1;
                mid |= (side & 1u);
                o[0][i] = (int32_t)(mid + side) >> 1;
                o[1][i] = (int32_t)(mid - side) >> 1;
            }
            break;
        default: break;
        }
    } else { /* @0x10011af5-0x10011b30: error, then zero the output */
        if (crc_ok_out) *crc_ok_out = 0;
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_FRAME_CRC_MISMATCH);
        for (unsigned ch = 0; ch < d->frame.header.channels; ch++) memset(o[ch], 0, sizeof(int32_t) * bs);
    }
    *got_frame = 1;
    if (d->next_fixed_block_size) d->fixed_block_size = d->next_fixed_block_size;
    d->channels = d->frame.header.channels;
    d->channel_assignment = d->frame.header.channel_assignment;
    d->bits_per_sample = d->frame.header.bits_per_sample;
    d->sample_rate = d->frame.header.sample_rate;
    d->blocksize = d->frame.header.blocksize;
    d->samples_decoded = d->frame.header.number.sample_number + d->frame.header.blocksize;
    /* write_audio_frame_to_client_ @0x100131e0; a non-CONTINUE return makes read_frame_
     * return false WITHOUT touching the state (@0x10011bd3-0x10011be4).  While seeking,
     * only the frame holding the target sample reaches the client, with the samples before
     * the target shifted out (blocksize and sample number adjusted); it ends seek mode. */
    FLAC__StreamDecoderWriteStatus ws = FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
    if (d->is_seeking) {
        const uint64_t sn = d->frame.header.number.sample_number, next = sn + d->frame.header.blocksize;
        if (sn <= d->target_sample && d->target_sample < next) {
            const unsigned delta = (unsigned)(d->target_sample - sn);
            d->is_seeking = 0;
            FLAC__Frame last = d->frame;
            const int32_t *nb[FLAC__MAX_CHANNELS];
            for (unsigned ch = 0; ch < FLAC__MAX_CHANNELS; ch++)
                nb[ch] = ch < d->frame.header.channels ? d->output[ch] + delta : NULL;
            last.header.blocksize -= delta;
            last.header.number.sample_number += delta;
            ws = d->write_cb((const FLAC__StreamDecoder *)d, &last, nb, d->client);
        }
    } else {
        ws = d->write_cb((const FLAC__StreamDecoder *)d, &d->frame, (const int32_t *const *)d->output, d->client);
    }
    if (ws != FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE) return 0;
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    return 1;
}

/* frame_sync_ @0x10011760 */
static int frame_sync(oracle_decoder *d) {
    uint32_t x;
    int first = 1;
    uint64_t total = d->has_stream_info ? d->stream_info.data.stream_info.total_samples : 0;
    if (total > 0 && d->samples_decoded >= total) { /* @0x100117a7 */
        d->state = FLAC__STREAM_DECODER_END_OF_STREAM;
        return 1;
    }
    if (!br_aligned(d)) {
        if (!br_u32(d, &x, 8u - (unsigned)(d->bitpos & 7u))) return 0;
    }
    for (;;) {
        if (d->cached) {
            x = d->lookahead;
            d->cached = 0;
        } else {
            if (!br_u32(d, &x, 8)) return 0;
        }
        if (x == 0xff) {
            d->header_warmup[0] = (uint8_t)x;
            if (!br_u32(d, &x, 8)) return 0;
            if (x == 0xff) {
                d->lookahead = (uint8_t)x;
                d->cached = 1;
            } else if (x >> 2 == 0x3e) { /* @0x1001187c */
                d->header_warmup[1] = (uint8_t)x;
                d->state = FLAC__STREAM_DECODER_READ_FRAME;
                return 1;
            }
        }
        if (first) { /* @0x1001188f */
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            first = 0;
        }
    }
}

/* ------------------------------------------------------------------------ metadata */
static int skip_id3v2(oracle_decoder *d) {
    uint32_t x, skip = 0;
    if (!br_u32(d, &x, 24)) return 0;
    for (int i = 0; i < 4; i++) {
        if (!br_u32(d, &x, 8)) return 0;
        skip <<= 7;
        skip |= (x & 0x7f);
    }
    return br_skip_bytes(d, skip);
}

static int find_metadata(oracle_decoder *d) {
    static const uint8_t sync[4] = {'f', 'L', 'a', 'C'};
    static const uint8_t id3[3] = {'I', 'D', '3'};
    uint32_t x;
    unsigned i = 0, id = 0;
    int first = 1;
    while (i < 4) {
        if (d->cached) {
            x = d->lookahead;
            d->cached = 0;
        } else if (!br_u32(d, &x, 8)) {
            return 0;
        }
        if (x == sync[i]) {
            first = 1;
            i++;
            id = 0;
            continue;
        }
        if (x == id3[id]) {
            id++;
            i = 0;
            if (id == 3) {
                if (!skip_id3v2(d)) return 0;
            }
            continue;
        }
        id = 0;
        if (x == 0xff) {
            d->header_warmup[0] = (uint8_t)x;
            if (!br_u32(d, &x, 8)) return 0;
            if (x == 0xff) {
                d->lookahead = (uint8_t)x;
                d->cached = 1;
            } else if (x >> 2 == 0x3e) {
                d->header_warmup[1] = (uint8_t)x;
                d->state = FLAC__STREAM_DECODER_READ_FRAME;
                return 1;
            }
        }
        i = 0;
        if (first) {
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            first = 0;
        }
    }
    d->state = FLAC__STREAM_DECODER_READ_METADATA;
    return 1;
}

static int read_metadata(oracle_decoder *d) {
    uint32_t last, type, length;
    if (!br_u32(d, &last, 1) || !br_u32(d, &type, 7) || !br_u32(d, &length, 24)) return 0;
    if (type == FLAC__METADATA_TYPE_STREAMINFO) {
        FLAC__StreamMetadata *m = &d->stream_info;
        FLAC__StreamMetadata_StreamInfo *si = &m->data.stream_info;
        uint32_t v;
        memset(m, 0, sizeof *m);
        m->type = FLAC__METADATA_TYPE_STREAMINFO;
        m->is_last = last ? 1 : 0;
        m->length = length;
        if (!br_u32(d, &v, 16)) return 0;
        si->min_blocksize = v;
        if (!br_u32(d, &v, 16)) return 0;
        si->max_blocksize = v;
        if (!br_u32(d, &v, 24)) return 0;
        si->min_framesize = v;
        if (!br_u32(d, &v, 24)) return 0;
        si->max_framesize = v;
        if (!br_u32(d, &v, 20)) return 0;
        si->sample_rate = v;
        if (!br_u32(d, &v, 3)) return 0;
        si->channels = v + 1;
        if (!br_u32(d, &v, 5)) return 0;
        si->bits_per_sample = v + 1;
        if (!br_u64(d, &si->total_samples, 36)) return 0;
        if (!br_read_bytes(d, si->md5sum, 16)) return 0;
        if (!br_skip_bytes(d, length - 34u)) return 0; /* unsigned, as libFLAC */
        d->has_stream_info = 1;
        if (d->metadata_cb && !d->is_seeking) d->metadata_cb((const FLAC__StreamDecoder *)d, m, d->client);
    } else {
        /* SEEKTABLE is parsed by libFLAC for seeking only; other blocks are filtered out
         * by the default metadata_respond set (only STREAMINFO is reported). */
        if (!br_skip_bytes(d, length)) return 0;
    }
    if (last) {
        d->first_frame_offset = (uint64_t)(d->bitpos >> 3);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    }
    return 1;
}

/* ---------------------------------------------------------------------- public API */
oracle_decoder *oracle_new(void) {
    oracle_decoder *d = (oracle_decoder *)calloc(1, sizeof(oracle_decoder));
    d->state = FLAC__STREAM_DECODER_UNINITIALIZED;
    return d;
}

static void reset_state(oracle_decoder *d) {
    d->len = 0;
    d->bitpos = 0;
    d->cached = 0;
    d->has_stream_info = 0;
    d->samples_decoded = 0;
    d->fixed_block_size = d->next_fixed_block_size = 0;
    d->is_seeking = 0;
    d->first_frame_offset = 0;
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_METADATA;
}

int oracle_init_stream(oracle_decoder *d, FLAC__StreamDecoderReadCallback read,
                       FLAC__StreamDecoderSeekCallback seek, FLAC__StreamDecoderTellCallback tell,
                       FLAC__StreamDecoderLengthCallback length, FLAC__StreamDecoderEofCallback eof,
                       FLAC__StreamDecoderWriteCallback write,
                       FLAC__StreamDecoderMetadataCallback metadata,
                       FLAC__StreamDecoderErrorCallback error, void *client) {
    if (d->state != FLAC__STREAM_DECODER_UNINITIALIZED) return FLAC__STREAM_DECODER_INIT_STATUS_ALREADY_INITIALIZED;
    if (!read || !write || !error || (seek && (!tell || !length || !eof)))
        return FLAC__STREAM_DECODER_INIT_STATUS_INVALID_CALLBACKS;
    d->read_cb = read; d->seek_cb = seek; d->tell_cb = tell; d->length_cb = length; d->eof_cb = eof;
    d->write_cb = write; d->metadata_cb = metadata; d->error_cb = error; d->client = client;
    reset_state(d);
    return FLAC__STREAM_DECODER_INIT_STATUS_OK;
}

FLAC__bool oracle_finish(oracle_decoder *d) {
    if (d->state == FLAC__STREAM_DECODER_UNINITIALIZED) return 1;
    for (unsigned i = 0; i < FLAC__MAX_CHANNELS; i++) {
        free(d->output[i] ? d->output[i] - 4 : NULL);
        free(d->residual[i]);
        d->output[i] = d->residual[i] = NULL;
    }
    d->output_capacity = d->output_channels = 0;
    d->state = FLAC__STREAM_DECODER_UNINITIALIZED;
    return 1; /* MD5 checking is off by default and BirdNest never enables it */
}

void oracle_delete(oracle_decoder *d) {
    if (!d) return;
    oracle_finish(d);
    free(d->buf);
    free(d);
}

/* FLAC__stream_decoder_process_single @0x10010130 (jump table @0x100101a0) */
FLAC__bool oracle_process_single(oracle_decoder *d) {
    int got;
    for (;;) {
        switch (d->state) {
        case FLAC__STREAM_DECODER_SEARCH_FOR_METADATA:
            if (!find_metadata(d)) return 0;
            break;
        case FLAC__STREAM_DECODER_READ_METADATA:
            return read_metadata(d) ? 1 : 0;
        case FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC:
            if (!frame_sync(d)) return 1;
            break;
        case FLAC__STREAM_DECODER_READ_FRAME:
            if (!read_frame(d, &got, NULL)) return 0;
            if (got) return 1;
            break;
        case FLAC__STREAM_DECODER_END_OF_STREAM:
        case FLAC__STREAM_DECODER_ABORTED:
            return 1;
        default:
            return 0;
        }
    }
}

FLAC__bool oracle_process_until_end_of_metadata(oracle_decoder *d) {
    for (;;) {
        switch (d->state) {
        case FLAC__STREAM_DECODER_SEARCH_FOR_METADATA:
            if (!find_metadata(d)) return 0;
            break;
        case FLAC__STREAM_DECODER_READ_METADATA:
            if (!read_metadata(d)) return 0;
            break;
        case FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC:
        case FLAC__STREAM_DECODER_READ_FRAME:
        case FLAC__STREAM_DECODER_END_OF_STREAM:
        case FLAC__STREAM_DECODER_ABORTED:
            return 1;
        default:
            return 0;
        }
    }
}

FLAC__bool oracle_process_until_end_of_stream(oracle_decoder *d) {
    int got;
    for (;;) {
        switch (d->state) {
        case FLAC__STREAM_DECODER_SEARCH_FOR_METADATA:
            if (!find_metadata(d)) return 0;
            break;
        case FLAC__STREAM_DECODER_READ_METADATA:
            if (!read_metadata(d)) return 0;
            break;
        case FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC:
            if (!frame_sync(d)) return 1;
            break;
        case FLAC__STREAM_DECODER_READ_FRAME:
            if (!read_frame(d, &got, NULL)) return 0;
            break;
        case FLAC__STREAM_DECODER_END_OF_STREAM:
        case FLAC__STREAM_DECODER_ABORTED:
            return 1;
        default:
            return 0;
        }
    }
}

/* FLAC__stream_decoder_seek_absolute (libFLAC 1.2.1 stream_decoder.c): states 0-4 only,
 * needs the seek callback, target below STREAMINFO's total; is_seeking and MD5-off are set
 * BEFORE the metadata pass (so a seek issued before it suppresses the STREAMINFO callback),
 * the length callback must answer.  seek_to_absolute_sample_ then repositions the client
 * and decodes (errors suppressed, nothing delivered) until the frame holding the target,
 * which write_audio_frame_to_client_ delivers trimmed (read_frame above).  The oracle keeps
 * every byte it has read, so its repositioning is a restart of the bit reader at the first
 * frame (the observable callbacks are libFLAC's: only the trimmed target frame); a failed
 * search leaves SEEK_ERROR. */
FLAC__bool oracle_seek_absolute(oracle_decoder *d, FLAC__uint64 sample) {
    if (d->state > FLAC__STREAM_DECODER_END_OF_STREAM) return 0;
    if (!d->seek_cb) return 0;
    if (oracle_get_total_samples(d) > 0 && sample >= oracle_get_total_samples(d)) return 0;
    d->is_seeking = 1;
    FLAC__uint64 length = 0;
    if (d->length_cb((const FLAC__StreamDecoder *)d, &length, d->client) != FLAC__STREAM_DECODER_LENGTH_STATUS_OK) {
        d->is_seeking = 0;
        return 0;
    }
    if (d->state <= FLAC__STREAM_DECODER_READ_METADATA) {
        if (!oracle_process_until_end_of_metadata(d)) {
            d->is_seeking = 0;
            return 0;
        }
        if (oracle_get_total_samples(d) > 0 && sample >= oracle_get_total_samples(d)) {
            d->is_seeking = 0;
            return 0;
        }
    }
    /* FLAC__stream_decoder_flush + reposition at the first frame */
    d->target_sample = sample;
    d->bitpos = (uint64_t)d->first_frame_offset * 8u;
    d->cached = 0;
    d->samples_decoded = 0;
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    for (uint64_t guard = 0; guard < 100000000u && d->is_seeking; guard++) {
        int got;
        if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) {
            if (!frame_sync(d)) break;
        } else if (d->state == FLAC__STREAM_DECODER_READ_FRAME) {
            if (!read_frame(d, &got, NULL)) break; /* incl. ABORT from the target frame's write */
        } else {
            break;
        }
    }
    if (!d->is_seeking && d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) return 1;
    d->is_seeking = 0;
    d->state = FLAC__STREAM_DECODER_SEEK_ERROR;
    return 0;
}

FLAC__StreamDecoderState oracle_get_state(const oracle_decoder *d) { return d->state; }
FLAC__uint64 oracle_get_total_samples(const oracle_decoder *d) {
    return d->has_stream_info ? d->stream_info.data.stream_info.total_samples : 0;
}
unsigned oracle_get_channels(const oracle_decoder *d) { return d->channels; }
unsigned oracle_get_bits_per_sample(const oracle_decoder *d) { return d->bits_per_sample; }
unsigned oracle_get_sample_rate(const oracle_decoder *d) { return d->sample_rate; }

/* ------------------------------------------------------------------ test drivers */
typedef struct {
    const uint8_t *data;
    size_t len, pos;
    int chunk;
    int hit_eof;
    /* event capture */
    oracle_event *ev;
    int ev_cap, n_ev;
    int32_t *pcm;
    size_t pcm_cap, n_pcm;
    int frames, abort_at;
    oracle_decoder *dec;
} mem_client;

/* FLACDecoder.ReadCallback (FLACDecoder.cs:325-363) over an in-memory stream */
static FLAC__StreamDecoderReadStatus mem_read(const FLAC__StreamDecoder *dec, FLAC__byte *buffer,
                                              size_t *bytes, void *cd) {
    (void)dec;
    mem_client *c = (mem_client *)cd;
    size_t want = *bytes;
    if (want == 0) {
        c->hit_eof = 1;
        return FLAC__STREAM_DECODER_READ_STATUS_ABORT;
    }
    size_t length = want < (size_t)c->chunk ? want : (size_t)c->chunk;
    size_t avail = c->len - c->pos;
    size_t count = length < avail ? length : avail;
    memcpy(buffer, c->data + c->pos, count);
    c->pos += count;
    if (count < length) {
        c->hit_eof = 1;
        *bytes = count;
        return FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM;
    }
    *bytes = count;
    return FLAC__STREAM_DECODER_READ_STATUS_CONTINUE;
}

static FLAC__bool mem_eof(const FLAC__StreamDecoder *dec, void *cd) {
    (void)dec;
    return ((mem_client *)cd)->hit_eof;
}

static void push_event(mem_client *c, int kind, int status) {
    if (c->n_ev >= c->ev_cap) return;
    oracle_event *e = &c->ev[c->n_ev++];
    memset(e, 0, sizeof *e);
    e->kind = kind;
    e->status = status;
    e->state = c->dec ? (int)c->dec->state : 0;
}

static FLAC__StreamDecoderWriteStatus ev_write(const FLAC__StreamDecoder *dec, const FLAC__Frame *f,
                                               const FLAC__int32 *const buf[], void *cd) {
    (void)dec;
    mem_client *c = (mem_client *)cd;
    if (c->n_ev < c->ev_cap) {
        oracle_event *e = &c->ev[c->n_ev++];
        memset(e, 0, sizeof *e);
        e->kind = ORACLE_EV_WRITE;
        e->state = (int)c->dec->state;
        e->blocksize = f->header.blocksize;
        e->sample_rate = f->header.sample_rate;
        e->channels = f->header.channels;
        e->assignment = (uint32_t)f->header.channel_assignment;
        e->bps = f->header.bits_per_sample;
        e->crc8 = f->header.crc;
        e->sample_number = f->header.number.sample_number;
        e->pcm_offset = c->n_pcm;
    }
    for (unsigned ch = 0; ch < f->header.channels; ch++) {
        for (unsigned i = 0; i < f->header.blocksize; i++) {
            if (c->n_pcm < c->pcm_cap) c->pcm[c->n_pcm] = buf[ch][i];
            c->n_pcm++;
        }
    }
    int idx = c->frames++;
    return (idx == c->abort_at) ? FLAC__STREAM_DECODER_WRITE_STATUS_ABORT : FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
}

static void ev_meta(const FLAC__StreamDecoder *dec, const FLAC__StreamMetadata *m, void *cd) {
    (void)dec;
    mem_client *c = (mem_client *)cd;
    push_event(c, ORACLE_EV_METADATA, (int)m->type);
    if (c->n_ev > 0 && c->ev[c->n_ev - 1].kind == ORACLE_EV_METADATA && m->type == FLAC__METADATA_TYPE_STREAMINFO) {
        oracle_event *e = &c->ev[c->n_ev - 1];
        e->blocksize = m->data.stream_info.max_blocksize;
        e->sample_rate = m->data.stream_info.sample_rate;
        e->channels = m->data.stream_info.channels;
        e->bps = m->data.stream_info.bits_per_sample;
        e->sample_number = m->data.stream_info.total_samples;
    }
}

static void ev_error(const FLAC__StreamDecoder *dec, FLAC__StreamDecoderErrorStatus st, void *cd) {
    (void)dec;
    push_event((mem_client *)cd, ORACLE_EV_ERROR, (int)st);
}

int oracle_run(const uint8_t *data, size_t len, int driver, int read_chunk, int write_abort_at,
               oracle_event *ev, int ev_cap, int *n_ev, int32_t *pcm, size_t pcm_cap,
               size_t *n_pcm) {
    mem_client c;
    memset(&c, 0, sizeof c);
    c.data = data; c.len = len; c.chunk = read_chunk > 0 ? read_chunk : 16384;
    c.ev = ev; c.ev_cap = ev_cap; c.pcm = pcm; c.pcm_cap = pcm_cap; c.abort_at = write_abort_at;
    oracle_decoder *d = oracle_new();
    c.dec = d;
    int rc = oracle_init_stream(d, mem_read, NULL, NULL, NULL, mem_eof, ev_write, ev_meta, ev_error, &c);
    if (rc != 0) { oracle_delete(d); return -rc; }
    if (driver == 0) {
        int ok = oracle_process_until_end_of_metadata(d);
        push_event(&c, ORACLE_EV_RETURN, ok);
        if (ok) {
            for (int guard = 0; guard < 50000000; guard++) {
                if (d->state >= FLAC__STREAM_DECODER_END_OF_STREAM) break;
                ok = oracle_process_single(d);
                push_event(&c, ORACLE_EV_RETURN, ok);
                if (!ok) break;
            }
        }
    } else {
        int ok = oracle_process_until_end_of_stream(d);
        push_event(&c, ORACLE_EV_RETURN, ok);
    }
    *n_ev = c.n_ev;
    *n_pcm = c.n_pcm;
    oracle_delete(d);
    return 0;
}

/* FLACFileReader's seek pattern (FLACFileReader.cs:125-136, 267-301): Position set ->
 * the NEXT write callback copies its frame, then calls seek_absolute from inside itself;
 * the trimmed target frame arrives through a nested write callback.  seeks[2i] is the write
 * index (0-based) after which seek i is issued (-1: right after the metadata pass, before
 * any frame; -2: right after init, before the metadata pass), seeks[2i+1] the target sample.  Events as oracle_run; every seek_absolute
 * return is an ORACLE_EV_SEEK event.  Memory client with seek/tell/length callbacks. */
typedef struct {
    mem_client mc;
    const int64_t *seeks;
    int nseeks, next;
} seek_client;

static FLAC__StreamDecoderSeekStatus mem_seek(const FLAC__StreamDecoder *dec, FLAC__uint64 off, void *cd) {
    (void)dec;
    mem_client *c = (mem_client *)cd;
    if (off > c->len) return FLAC__STREAM_DECODER_SEEK_STATUS_ERROR;
    c->pos = (size_t)off;
    c->hit_eof = 0;
    return FLAC__STREAM_DECODER_SEEK_STATUS_OK;
}
static FLAC__StreamDecoderTellStatus mem_tell(const FLAC__StreamDecoder *dec, FLAC__uint64 *off, void *cd) {
    (void)dec;
    *off = ((mem_client *)cd)->pos;
    return FLAC__STREAM_DECODER_TELL_STATUS_OK;
}
static FLAC__StreamDecoderLengthStatus mem_length(const FLAC__StreamDecoder *dec, FLAC__uint64 *len, void *cd) {
    (void)dec;
    *len = ((mem_client *)cd)->len;
    return FLAC__STREAM_DECODER_LENGTH_STATUS_OK;
}

static void do_seek(seek_client *sc, oracle_decoder *d) {
    const int64_t target = sc->seeks[2 * sc->next + 1];
    sc->next++;
    FLAC__bool r = oracle_seek_absolute(d, (FLAC__uint64)target);
    push_event(&sc->mc, ORACLE_EV_SEEK, r);
}

static FLAC__StreamDecoderWriteStatus sk_write(const FLAC__StreamDecoder *dec, const FLAC__Frame *f,
                                               const FLAC__int32 *const buf[], void *cd) {
    seek_client *sc = (seek_client *)cd;
    const int idx = sc->mc.frames;
    (void)ev_write(dec, f, buf, &sc->mc); /* copies the frame (counts it) */
    if (sc->next < sc->nseeks && sc->seeks[2 * sc->next] == idx) do_seek(sc, sc->mc.dec);
    return FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
}

int oracle_run_seek(const uint8_t *data, size_t len, int read_chunk, const int64_t *seeks, int nseeks,
                    oracle_event *ev, int ev_cap, int *n_ev, int32_t *pcm, size_t pcm_cap, size_t *n_pcm) {
    seek_client sc;
    memset(&sc, 0, sizeof sc);
    mem_client *c = &sc.mc;
    c->data = data; c->len = len; c->chunk = read_chunk > 0 ? read_chunk : 16384;
    c->ev = ev; c->ev_cap = ev_cap; c->pcm = pcm; c->pcm_cap = pcm_cap; c->abort_at = -1;
    sc.seeks = seeks; sc.nseeks = nseeks;
    oracle_decoder *d = oracle_new();
    c->dec = d;
    int rc = oracle_init_stream(d, mem_read, mem_seek, mem_tell, mem_length, mem_eof, sk_write, ev_meta, ev_error, &sc);
    if (rc != 0) { oracle_delete(d); return -rc; }
    while (sc.next < sc.nseeks && sc.seeks[2 * sc.next] == -2) do_seek(&sc, d); /* before the metadata pass */
    int ok = oracle_process_until_end_of_metadata(d);
    push_event(c, ORACLE_EV_RETURN, ok);
    while (ok && sc.next < sc.nseeks && sc.seeks[2 * sc.next] < 0) do_seek(&sc, d);
    if (ok) {
        for (int guard = 0; guard < 50000000; guard++) {
            if (d->state >= FLAC__STREAM_DECODER_END_OF_STREAM) break;
            ok = oracle_process_single(d);
            push_event(c, ORACLE_EV_RETURN, ok);
            if (!ok) break;
        }
    }
    *n_ev = c->n_ev;
    *n_pcm = c->n_pcm;
    oracle_delete(d);
    return 0;
}

/* Frame-level decode for batch parity: memory client with no EOF surprises. */
typedef struct {
    const uint8_t *data;
    size_t len, pos;
    int32_t *planar;
    size_t cap;
    int err;
} frame_client;

static FLAC__StreamDecoderReadStatus fc_read(const FLAC__StreamDecoder *dec, FLAC__byte *buffer,
                                             size_t *bytes, void *cd) {
    (void)dec;
    frame_client *c = (frame_client *)cd;
    size_t avail = c->len - c->pos;
    size_t n = *bytes < avail ? *bytes : avail;
    memcpy(buffer, c->data + c->pos, n);
    c->pos += n;
    *bytes = n;
    return n ? FLAC__STREAM_DECODER_READ_STATUS_CONTINUE : FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM;
}

static FLAC__StreamDecoderWriteStatus fc_write(const FLAC__StreamDecoder *dec, const FLAC__Frame *f,
                                               const FLAC__int32 *const buf[], void *cd) {
    (void)dec;
    frame_client *c = (frame_client *)cd;
    size_t k = 0;
    for (unsigned ch = 0; ch < f->header.channels; ch++)
        for (unsigned i = 0; i < f->header.blocksize; i++, k++)
            if (k < c->cap) c->planar[k] = buf[ch][i];
    return FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
}

static void fc_error(const FLAC__StreamDecoder *dec, FLAC__StreamDecoderErrorStatus st, void *cd) {
    (void)dec;
    frame_client *c = (frame_client *)cd;
    if (c->err < 0 || c->err == FLAC__STREAM_DECODER_ERROR_STATUS_FRAME_CRC_MISMATCH) c->err = (int)st;
}

int oracle_decode_frame_at(const uint8_t *data, size_t len, size_t off,
                           const oracle_stream_params *sp, int32_t *planar, size_t planar_cap,
                           oracle_frame_result *res) {
    frame_client c;
    memset(&c, 0, sizeof c);
    memset(res, 0, sizeof *res);
    c.data = data + off;
    c.len = len - off;
    c.planar = planar;
    c.cap = planar_cap;
    c.err = -1;
    oracle_decoder *d = oracle_new();
    oracle_init_stream(d, fc_read, NULL, NULL, NULL, NULL, fc_write, NULL, fc_error, &c);
    if (sp && sp->has_stream_info) {
        FLAC__StreamMetadata_StreamInfo *si = &d->stream_info.data.stream_info;
        d->has_stream_info = 1;
        si->min_blocksize = sp->min_blocksize;
        si->max_blocksize = sp->max_blocksize;
        si->sample_rate = sp->sample_rate;
        si->channels = sp->channels;
        si->bits_per_sample = sp->bps;
        si->total_samples = sp->total_samples;
    }
    res->cached = -1;
    if (len - off < 2 || data[off] != 0xff || (data[off + 1] >> 2) != 0x3e) {
        res->error = FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC;
        oracle_delete(d);
        return 1 + FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC;
    }
    if (!br_need(d, 16)) { oracle_delete(d); res->error = 0; return 1; }
    d->header_warmup[0] = data[off];
    d->header_warmup[1] = data[off + 1];
    d->bitpos = 16;
    d->state = FLAC__STREAM_DECODER_READ_FRAME;
    int got = 0, crc_ok = 0;
    int ok = read_frame(d, &got, &crc_ok);
    FLAC__FrameHeader *h = &d->frame.header;
    res->blocksize = h->blocksize;
    res->sample_rate = h->sample_rate;
    res->channels = h->channels;
    res->assignment = (uint32_t)h->channel_assignment;
    res->bps = h->bits_per_sample;
    res->number_type = d->raw_number_type;
    res->number = d->raw_number;
    res->end_off = off + (size_t)((d->bitpos + 7) >> 3);
    res->cached = d->cached ? (int)d->lookahead : -1;
    res->crc_ok = got ? crc_ok : 0;
    int rv;
    if (!ok && !got) {
        res->error = FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM; /* truncated */
        rv = 100;
    } else if (got) {
        res->error = crc_ok ? -1 : FLAC__STREAM_DECODER_ERROR_STATUS_FRAME_CRC_MISMATCH;
        rv = 0;
    } else {
        res->error = c.err;
        rv = 1 + c.err;
    }
    oracle_delete(d);
    return rv;
}

/* ------------------------------------------------------------------ C# replays */
typedef struct {
    /* FLACDecoder fields */
    mem_client mc;
    uint8_t **packets;   /* FLACPacketQueue (FIFO) */
    size_t *plen, *poff;
    size_t qhead, qtail, qcap;
    int bits, channels, rate;
    int64_t total;
    int aborted_by_writer;
    jmp_buf jb;
    char *msg;
    int msg_cap;
} csd_client;

static const char *state_name(int s) {
    static const char *n[] = {"SearchForMetadata", "ReadMetadata", "SearchForFrameSync", "ReadFrame",
                              "EndOfStream", "OggError", "SeekError", "Aborted",
                              "MemoryAllocationError", "Uninitialized"};
    return (s >= 0 && s <= 9) ? n[s] : "?";
}

static const char *error_name(int s) {
    static const char *n[] = {"LostSync", "BadHeader", "FrameCrcMismatch", "UnparsableStream"};
    return (s >= 0 && s <= 3) ? n[s] : "?";
}

static void q_push(csd_client *c, uint8_t *p, size_t n) {
    if (c->qtail == c->qcap) {
        c->qcap = c->qcap ? c->qcap * 2 : 64;
        c->packets = (uint8_t **)realloc(c->packets, c->qcap * sizeof(uint8_t *));
        c->plen = (size_t *)realloc(c->plen, c->qcap * sizeof(size_t));
        c->poff = (size_t *)realloc(c->poff, c->qcap * sizeof(size_t));
    }
    c->packets[c->qtail] = p;
    c->plen[c->qtail] = n;
    c->poff[c->qtail] = 0;
    c->qtail++;
}

/* FLACDecoder.WriteCallback, FLACDecoder.cs:520-580 */
static FLAC__StreamDecoderWriteStatus csd_write(const FLAC__StreamDecoder *dec, const FLAC__Frame *f,
                                                const FLAC__int32 *const buf[], void *cd) {
    (void)dec;
    csd_client *c = (csd_client *)cd;
    if (f->header.bits_per_sample != 16) return FLAC__STREAM_DECODER_WRITE_STATUS_ABORT; /* :526-530 */
    unsigned bs = f->header.blocksize;
    uint8_t *p;
    size_t n;
    if (f->header.channels == 2) { /* :543-562 */
        n = 4u * bs;
        p = (uint8_t *)malloc(n ? n : 1);
        for (unsigned i = 0; i < bs; i++) {
            int32_t l = buf[0][i], r = buf[1][i];
            p[4 * i + 0] = (uint8_t)(l >> 0);
            p[4 * i + 1] = (uint8_t)(l >> 8);
            p[4 * i + 2] = (uint8_t)(r >> 0);
            p[4 * i + 3] = (uint8_t)(r >> 8);
        }
    } else { /* :564-577: channel 0 only */
        n = 2u * bs;
        p = (uint8_t *)malloc(n ? n : 1);
        for (unsigned i = 0; i < bs; i++) {
            int32_t l = buf[0][i];
            p[2 * i + 0] = (uint8_t)(l >> 0);
            p[2 * i + 1] = (uint8_t)(l >> 8);
        }
    }
    q_push(c, p, n);
    return FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
}

/* FLACDecoder.MetadataCallback, FLACDecoder.cs:431-473 (A18 layout trick included) */
static void csd_meta(const FLAC__StreamDecoder *dec, const FLAC__StreamMetadata *m, void *cd) {
    (void)dec;
    csd_client *c = (csd_client *)cd;
    if (m->type != FLAC__METADATA_TYPE_STREAMINFO) return;
    const uint8_t *raw = (const uint8_t *)m;
    int32_t hi, lo;
    memcpy(&hi, raw + 44, 4); /* "TotalSamplesHi" FieldOffset(32) = alignment padding */
    memcpy(&lo, raw + 48, 4); /* "TotalSamplesLo" FieldOffset(36) = low word */
    c->bits = (int)m->data.stream_info.bits_per_sample;
    c->channels = (int)m->data.stream_info.channels;
    c->rate = (int)m->data.stream_info.sample_rate;
    c->total = (int64_t)hi + (int64_t)lo; /* (long)(Hi << 32): C# masks the int shift to 0 */
}

static void csd_error(const FLAC__StreamDecoder *dec, FLAC__StreamDecoderErrorStatus st, void *cd) {
    csd_client *c = (csd_client *)cd;
    snprintf(c->msg, (size_t)c->msg_cap, "FLAC: Could not decode frame: %s - %s!", error_name((int)st),
             state_name((int)oracle_get_state((const oracle_decoder *)dec)));
    longjmp(c->jb, 1); /* FLACDecoder.cs:590-594 throws through the native frames */
}

int oracle_flacdecoder_copyto(const uint8_t *data, size_t len, int copy_chunk, uint8_t *out,
                              size_t cap, size_t *out_len, int32_t *fmt4, char *msg, int msg_cap) {
    csd_client *c = (csd_client *)calloc(1, sizeof(csd_client));
    c->mc.data = data; c->mc.len = len; c->mc.chunk = 16384; /* DEFAULT_MAX_BUFFER_SIZE :21 */
    c->msg = msg; c->msg_cap = msg_cap;
    msg[0] = 0;
    *out_len = 0;
    oracle_decoder *d = oracle_new();
    volatile int rc = 0;
    uint8_t *chunk = (uint8_t *)malloc((size_t)copy_chunk);
    if (setjmp(c->jb) == 0) {
        /* ctor :72-88 -- the read/eof callbacks see the mem_client at the head of csd_client */
        if (oracle_init_stream(d, mem_read, NULL, NULL, NULL, mem_eof, csd_write, csd_meta, csd_error, c) != 0) {
            snprintf(msg, (size_t)msg_cap, "FLAC: Could not open stream for reading!");
            rc = 1;
            goto done;
        }
        if (!oracle_process_until_end_of_metadata(d)) { /* FLACCheck :98-105 */
            snprintf(msg, (size_t)msg_cap, "FLAC: Could not Could not process until end of metadata - %s!",
                     state_name((int)d->state));
            rc = 1;
            goto done;
        }
        if (fmt4) { fmt4[0] = c->channels; fmt4[1] = c->rate; fmt4[2] = c->bits; fmt4[3] = (int32_t)c->total; }
        /* Stream.CopyTo: Read(chunk, 0, copy_chunk) until it returns 0 */
        for (;;) {
            int local = 0, space = copy_chunk, got = 0;
            while (space > 0) { /* Read :124-205 */
                if (c->qhead == c->qtail) { /* RequestAnotherFLACPacket :207-224 */
                    int st = (int)d->state;
                    if (st < FLAC__STREAM_DECODER_END_OF_STREAM) {
                        if (!oracle_process_single(d)) {
                            snprintf(msg, (size_t)msg_cap, "FLAC: Could not process single - %s!",
                                     state_name((int)d->state));
                            rc = 1;
                            goto done;
                        }
                    } else if (st >= FLAC__STREAM_DECODER_OGG_ERROR) {
                        snprintf(msg, (size_t)msg_cap, "FLAC: Decoding returned with critical state: %s",
                                 state_name(st));
                        rc = 1;
                        goto done;
                    }
                }
                if (c->qhead == c->qtail) break;
                size_t left = c->plen[c->qhead] - c->poff[c->qhead];
                if (left > (size_t)space) {
                    memcpy(chunk + local, c->packets[c->qhead] + c->poff[c->qhead], (size_t)space);
                    c->poff[c->qhead] += (size_t)space;
                    got += space;
                    space = 0;
                } else if (left > 0) {
                    memcpy(chunk + local, c->packets[c->qhead] + c->poff[c->qhead], left);
                    local += (int)left;
                    space -= (int)left;
                    got += (int)left;
                    free(c->packets[c->qhead]);
                    c->qhead++;
                }
            }
            if (got == 0) break;
            if (*out_len + (size_t)got <= cap) memcpy(out + *out_len, chunk, (size_t)got);
            *out_len += (size_t)got;
        }
    } else {
        rc = 1; /* exception from a callback */
    }
done:
    while (c->qhead < c->qtail) free(c->packets[c->qhead++]);
    free(c->packets); free(c->plen); free(c->poff); free(chunk);
    oracle_delete(d);
    free(c);
    return rc;
}

/* FLACFileReader replay */
typedef struct {
    mem_client mc;
    int si_channels, si_bits;
    int64_t total;
    int32_t *flac_samples; /* m_flacSamples */
    int spc;               /* m_samplesPerChannel */
    int idx;               /* m_flacSampleIndex */
    uint8_t *nbuf;         /* m_NAudioSampleBuffer */
    int nlen, noff;        /* Length, m_playbackBufferOffset */
    jmp_buf jb;
    char *msg;
    int msg_cap;
} cfr_client;

/* FLACFileReader.FLAC_WriteCallback :267-301.  Declared void in C# (LibFLACSharp.cs:205-206);
 * the replacement treats it as CONTINUE (SURVEY 8b hazard 2). */
static FLAC__StreamDecoderWriteStatus cfr_write(const FLAC__StreamDecoder *dec, const FLAC__Frame *f,
                                                const FLAC__int32 *const buf[], void *cd) {
    (void)dec;
    cfr_client *c = (cfr_client *)cd;
    if (!c->flac_samples) {
        c->spc = (int)f->header.blocksize;
        c->flac_samples = (int32_t *)calloc((size_t)c->spc * (size_t)(c->si_channels > 0 ? c->si_channels : 1), 4);
        c->idx = 0;
    }
    /* copies spc samples from each libFLAC channel buffer: stale tail on a short frame,
     * truncation on a longer one */
    for (int ch = 0; ch < c->si_channels; ch++)
        memcpy(c->flac_samples + (size_t)ch * (size_t)c->spc, buf[ch], (size_t)c->spc * 4u);
    return FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE;
}

static void cfr_meta(const FLAC__StreamDecoder *dec, const FLAC__StreamMetadata *m, void *cd) {
    (void)dec;
    cfr_client *c = (cfr_client *)cd;
    if (m->type != FLAC__METADATA_TYPE_STREAMINFO) return;
    const uint8_t *raw = (const uint8_t *)m;
    int32_t hi, lo;
    memcpy(&hi, raw + 44, 4);
    memcpy(&lo, raw + 48, 4);
    c->si_channels = (int)m->data.stream_info.channels;
    c->si_bits = (int)m->data.stream_info.bits_per_sample;
    c->total = (int64_t)hi + (int64_t)lo;
}

static void cfr_error(const FLAC__StreamDecoder *dec, FLAC__StreamDecoderErrorStatus st, void *cd) {
    cfr_client *c = (cfr_client *)cd;
    snprintf(c->msg, (size_t)c->msg_cap, "FLAC: Could not decode frame: %s - %s!", error_name((int)st),
             state_name((int)oracle_get_state((const oracle_decoder *)dec)));
    longjmp(c->jb, 1);
}

/* CopyFlacBufferToNAudioBuffer :208-254; returns -1 on IndexOutOfRange / NotSupported */
static int cfr_copy(cfr_client *c) {
    int start = c->noff;
    int full = c->noff >= c->nlen;
    for (; c->idx < c->spc && !full; c->idx++) {
        for (int ch = 0; ch < c->si_channels && !full; ch++) {
            int32_t s = c->flac_samples[c->idx + ch * c->spc];
            if (c->si_bits == 16) {
                if (c->noff + 2 > c->nlen) return -1;
                c->nbuf[c->noff++] = (uint8_t)s;
                c->nbuf[c->noff++] = (uint8_t)(s >> 8);
            } else if (c->si_bits == 24) {
                if (c->noff + 3 > c->nlen) return -1;
                c->nbuf[c->noff++] = (uint8_t)((s >> 0) & 0xFF);
                c->nbuf[c->noff++] = (uint8_t)((s >> 8) & 0xFF);
                c->nbuf[c->noff++] = (uint8_t)((s >> 16) & 0xFF);
            } else {
                return -2;
            }
            full = c->noff >= c->nlen;
        }
    }
    if (c->idx >= c->spc) c->idx = 0;
    return c->noff - start;
}

int oracle_filereader_readall(const uint8_t *data, size_t len, int buf_len, uint8_t *out,
                              size_t cap, size_t *out_len, char *msg, int msg_cap) {
    return oracle_filereader_readall_n(data, len, buf_len, buf_len, out, cap, out_len, msg, msg_cap);
}

/* The same with Read(buf, 0, num_bytes) on a buffer of buf_len bytes: the copy loop runs to
 * buf.Length, so a call may return more than num_bytes (FLACFileReader.cs:162-171, 211). */
int oracle_filereader_readall_n(const uint8_t *data, size_t len, int buf_len, int num_bytes, uint8_t *out,
                                size_t cap, size_t *out_len, char *msg, int msg_cap) {
    cfr_client *c = (cfr_client *)calloc(1, sizeof(cfr_client));
    c->mc.data = data; c->mc.len = len; c->mc.chunk = 1 << 30; /* init_file reads with fread */
    c->msg = msg; c->msg_cap = msg_cap;
    msg[0] = 0;
    *out_len = 0;
    c->nbuf = (uint8_t *)malloc((size_t)buf_len);
    c->nlen = buf_len;
    oracle_decoder *d = oracle_new();
    volatile int rc = 0;
    if (setjmp(c->jb) == 0) {
        if (oracle_init_stream(d, mem_read, NULL, NULL, NULL, mem_eof, cfr_write, cfr_meta, cfr_error, c) != 0) {
            snprintf(msg, (size_t)msg_cap, "FLAC: Could not open stream for reading!");
            rc = 1;
            goto done;
        }
        if (!oracle_process_until_end_of_metadata(d)) {
            snprintf(msg, (size_t)msg_cap, "FLAC: Could not Could not process until end of metadata - %s!",
                     state_name((int)d->state));
            rc = 1;
            goto done;
        }
        for (int calls = 0; calls < 100000000; calls++) { /* Read(buf, 0, buf.Length) :145-174 */
            int copied = 0;
            c->noff = 0;
            if (c->idx > 0) {
                int r = cfr_copy(c);
                if (r < 0) goto bad_copy;
                copied = r;
            }
            int spins = 0;
            while (copied < num_bytes) {
                if (++spins > 10000000) { /* the C# loop never ends (e.g. state Aborted) */
                    snprintf(msg, (size_t)msg_cap, "hang: Read() never returns (state %s)",
                             state_name((int)d->state));
                    rc = 2;
                    goto done;
                }
                oracle_process_single(d); /* result ignored :177-181 */
                if (d->state == FLAC__STREAM_DECODER_END_OF_STREAM) break;
                if (!c->flac_samples) { copied += 0; continue; }
                int r = cfr_copy(c);
                if (r < 0) goto bad_copy;
                copied += r;
            }
            if (copied == 0) break;
            if (*out_len + (size_t)copied <= cap) memcpy(out + *out_len, c->nbuf, (size_t)copied);
            *out_len += (size_t)copied;
        }
        goto done;
    bad_copy:
        snprintf(msg, (size_t)msg_cap, "%s",
                 c->si_bits == 16 || c->si_bits == 24 ? "Index was outside the bounds of the array."
                                                      : "Input FLAC bit depth is not supported!");
        rc = 1;
    } else {
        rc = 1;
    }
done:
    free(c->flac_samples);
    free(c->nbuf);
    oracle_delete(d);
    free(c);
    return rc;
}
