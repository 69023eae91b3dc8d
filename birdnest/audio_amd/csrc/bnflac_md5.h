/*
 * bnflac_md5.h -- MD5 (RFC 1321) for the STREAMINFO md5sum check, host side.
 *
 * libFLAC 1.2.1 hashes decoded PCM with FLAC__MD5Accumulate (LibFlac.dll@0x10007920):
 * samples interleaved by channel, each written as (bps + 7) / 8 little-endian bytes.
 * md5_accumulate() below takes libFLAC's planar write buffers in that convention.
 * SURVEY.md 8a A13, 8f-3.
 */
#ifndef BNFLAC_MD5_H
#define BNFLAC_MD5_H

#include <stdint.h>
#include <string.h>

struct Md5 {
    uint32_t h[4];
    uint64_t bytes;
    uint8_t blk[64];
    uint32_t fill;
};

static inline uint32_t md5_rol(uint32_t x, uint32_t c) { return (x << c) | (x >> (32u - c)); }

static inline void md5_init(Md5 &m) {
    m.h[0] = 0x67452301u;
    m.h[1] = 0xefcdab89u;
    m.h[2] = 0x98badcfeu;
    m.h[3] = 0x10325476u;
    m.bytes = 0;
    m.fill = 0;
}

static inline void md5_block(Md5 &m, const uint8_t *p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const uint32_t S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
               ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = m.h[0], b = m.h[1], c = m.h[2], d = m.h[3];
    for (uint32_t i = 0; i < 64; i++) {
        uint32_t f, g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + md5_rol(a + f + K[i] + w[g], S[(i >> 4) * 4 + (i & 3)]);
        a = t;
    }
    m.h[0] += a;
    m.h[1] += b;
    m.h[2] += c;
    m.h[3] += d;
}

static inline void md5_update(Md5 &m, const uint8_t *p, size_t n) {
    m.bytes += n;
    while (n) {
        const uint32_t take = (uint32_t)(n < 64u - m.fill ? n : 64u - m.fill);
        memcpy(m.blk + m.fill, p, take);
        m.fill += take;
        p += take;
        n -= take;
        if (m.fill == 64) {
            md5_block(m, m.blk);
            m.fill = 0;
        }
    }
}

static inline void md5_final(Md5 &m, uint8_t out[16]) {
    const uint64_t bits = m.bytes * 8u;
    const uint8_t pad = 0x80, zero = 0;
    md5_update(m, &pad, 1);
    while (m.fill != 56) md5_update(m, &zero, 1);
    uint8_t len[8];
    for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (8 * i));
    md5_update(m, len, 8);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(m.h[i] >> (8 * j));
}

/* FLAC__MD5Accumulate: per-channel int32 buffers -> interleaved (bps + 7) / 8-byte LE samples.
 * Sample i of channel c is chan[c][i * step]. */
static inline void md5_accumulate(Md5 &m, const int32_t *const *chan, uint32_t channels, uint64_t nsamples,
                                  uint64_t step, uint32_t bytes_per_sample) {
    uint8_t tmp[4096];
    uint32_t n = 0;
    for (uint64_t i = 0; i < nsamples; i++) {
        for (uint32_t c = 0; c < channels; c++) {
            const uint32_t v = (uint32_t)chan[c][i * step];
            for (uint32_t b = 0; b < bytes_per_sample; b++) tmp[n++] = (uint8_t)(v >> (8 * b));
            if (n > sizeof tmp - 32) {
                md5_update(m, tmp, n);
                n = 0;
            }
        }
    }
    if (n) md5_update(m, tmp, n);
}

#endif /* BNFLAC_MD5_H */
