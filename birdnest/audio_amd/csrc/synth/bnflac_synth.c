/*
 * bnflac_synth.c -- deterministic synthetic FLAC encoder (workload generator).
 *
 * Signal model (BASELINE.md section 3 / SURVEY.md 8d): per channel, a shared and a
 * private damped-resonator AR process (so stereo channels correlate), scaled to the
 * target level, plus white noise of the requested std that sets the residual size.
 * Every frame is coded with the requested subframe type/order; LPC coefficients come
 * from Levinson-Durbin on a windowed autocorrelation and are quantised to the
 * requested precision.  Residuals are computed with the arithmetic the libFLAC 1.2.1
 * decoder restores with (32-bit wrap or 64-bit per its dispatch rule), so decoding
 * must reproduce the source PCM bit for bit.
 */
#include "bnflac_synth.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ----------------------------------------------------------------------- RNG */
typedef struct { uint64_t s; } rng_t;
static uint64_t rng_next(rng_t *r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double rng_unit(rng_t *r) { return ((rng_next(r) >> 11) + 0.5) * (1.0 / 9007199254740992.0); }
static uint32_t rng_below(rng_t *r, uint32_t n) { return n ? (uint32_t)(rng_next(r) % n) : 0; }
static double rng_gauss(rng_t *r) {
    double u = rng_unit(r), v = rng_unit(r);
    return sqrt(-2.0 * log(u)) * cos(6.283185307179586 * v);
}

/* ----------------------------------------------------------------------- CRC */
static uint8_t crc8_tab[256];
static uint16_t crc16_tab[256];
static void crc_init(void) {
    static int ready;
    if (ready) return;
    for (int i = 0; i < 256; i++) {
        uint8_t c = (uint8_t)i;
        for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
        crc8_tab[i] = c;
        uint16_t w = (uint16_t)(i << 8);
        for (int b = 0; b < 8; b++) w = (uint16_t)((w & 0x8000) ? (w << 1) ^ 0x8005 : (w << 1));
        crc16_tab[i] = w;
    }
    ready = 1;
}
static uint8_t crc8(const uint8_t *p, size_t n) {
    uint8_t c = 0;
    for (size_t i = 0; i < n; i++) c = crc8_tab[c ^ p[i]];
    return c;
}
static uint16_t crc16(const uint8_t *p, size_t n) {
    uint16_t c = 0;
    for (size_t i = 0; i < n; i++) c = (uint16_t)((c << 8) ^ crc16_tab[(c >> 8) ^ p[i]]);
    return c;
}

/* ----------------------------------------------------------------------- MD5 */
typedef struct { uint32_t a, b, c, d; uint64_t len; uint8_t buf[64]; size_t n; } md5_t;
static const uint32_t md5_k[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t md5_r[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                  5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                  4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                  6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
static void md5_block(md5_t *m, const uint8_t *p) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = m->a, b = m->b, c = m->c, d = m->d;
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        uint32_t x = a + f + md5_k[i] + w[g];
        b = b + ((x << md5_r[i]) | (x >> (32 - md5_r[i])));
        a = t;
    }
    m->a += a; m->b += b; m->c += c; m->d += d;
}
static void md5_init(md5_t *m) { m->a = 0x67452301; m->b = 0xefcdab89; m->c = 0x98badcfe; m->d = 0x10325476; m->len = 0; m->n = 0; }
static void md5_update(md5_t *m, const uint8_t *p, size_t n) {
    m->len += n;
    while (n) {
        size_t t = 64 - m->n;
        if (t > n) t = n;
        memcpy(m->buf + m->n, p, t);
        m->n += t; p += t; n -= t;
        if (m->n == 64) { md5_block(m, m->buf); m->n = 0; }
    }
}
static void md5_final(md5_t *m, uint8_t out[16]) {
    uint64_t bits = m->len * 8;
    uint8_t pad = 0x80, z = 0;
    md5_update(m, &pad, 1);
    while (m->n != 56) md5_update(m, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (8 * i));
    md5_update(m, lb, 8);
    uint32_t v[4] = {m->a, m->b, m->c, m->d};
    for (int i = 0; i < 16; i++) out[i] = (uint8_t)(v[i / 4] >> (8 * (i % 4)));
}
void bnsyn_md5(const uint8_t *buf, size_t n, uint8_t out[16]) {
    md5_t m;
    md5_init(&m);
    md5_update(&m, buf, n);
    md5_final(&m, out);
}

/* ---------------------------------------------------------------- bit writer */
typedef struct { uint8_t *p; size_t cap, n; uint64_t acc; int nacc; int overflow; } bw_t;
static void bw_put(bw_t *w, uint32_t v, int bits) { /* bits <= 32 */
    if (bits <= 0) return;
    uint64_t mask = (bits == 32) ? 0xffffffffull : ((1ull << bits) - 1);
    w->acc = (w->acc << bits) | ((uint64_t)v & mask);
    w->nacc += bits;
    while (w->nacc >= 8) {
        w->nacc -= 8;
        if (w->n < w->cap) w->p[w->n] = (uint8_t)(w->acc >> w->nacc);
        else w->overflow = 1;
        w->n++;
    }
}
static void bw_put_signed(bw_t *w, int32_t v, int bits) { bw_put(w, (uint32_t)v, bits); }
static void bw_zeros(bw_t *w, uint64_t n) {
    while (n >= 32) { bw_put(w, 0, 32); n -= 32; }
    bw_put(w, 0, (int)n);
}
static void bw_align(bw_t *w) { if (w->nacc) bw_put(w, 0, 8 - w->nacc); }
static void bw_utf8(bw_t *w, uint64_t v) {
    if (v < 0x80) { bw_put(w, (uint32_t)v, 8); return; }
    int n;
    if (v < 0x800) n = 2;
    else if (v < 0x10000) n = 3;
    else if (v < 0x200000) n = 4;
    else if (v < 0x4000000) n = 5;
    else if (v < 0x80000000ull) n = 6;
    else n = 7;
    uint32_t lead = (uint32_t)((0xFF00u >> n) & 0xFF);
    bw_put(w, lead | (uint32_t)(v >> (6 * (n - 1))), 8);
    for (int i = n - 2; i >= 0; i--) bw_put(w, 0x80u | (uint32_t)((v >> (6 * i)) & 0x3F), 8);
}

/* ------------------------------------------------------------ prediction math */
static unsigned ilog2u(unsigned v) { unsigned l = 0; while (v >>= 1) l++; return l; }

/* libFLAC 1.2.1 restore arithmetic (mirrors the decoder dispatch). */
static int32_t lpc_pred(const int32_t *hist_end, const int32_t *q, unsigned order, int shift, int wide) {
    if (wide) {
        int64_t s = 0;
        for (unsigned j = 0; j < order; j++) s += (int64_t)q[j] * hist_end[-1 - (int)j];
        return (int32_t)(s >> shift);
    }
    uint32_t s = 0;
    for (unsigned j = 0; j < order; j++) s += (uint32_t)q[j] * (uint32_t)hist_end[-1 - (int)j];
    return (int32_t)s >> shift;
}

static int32_t fixed_pred(const int32_t *h, unsigned order) {
    uint32_t a = (uint32_t)h[-1], b = order > 1 ? (uint32_t)h[-2] : 0, c = order > 2 ? (uint32_t)h[-3] : 0,
             d = order > 3 ? (uint32_t)h[-4] : 0;
    switch (order) {
    case 0: return 0;
    case 1: return (int32_t)a;
    case 2: return (int32_t)((a << 1) - b);
    case 3: return (int32_t)(((a - b) << 1) + (a - b) + c);
    default: return (int32_t)(((a + c) << 2) - ((b << 2) + (b << 1)) - d);
    }
}

/* Levinson-Durbin on a Welch-windowed autocorrelation; returns lp[0..order-1] with
 * prediction x[n] ~= sum lp[j] x[n-1-j]. */
static void lpc_coefs(const int32_t *x, unsigned n, unsigned order, double *lp) {
    double *wx = (double *)malloc(sizeof(double) * (n ? n : 1));
    for (unsigned i = 0; i < n; i++) {
        double t = n > 1 ? (2.0 * i / (n - 1) - 1.0) : 0.0;
        wx[i] = x[i] * (1.0 - t * t);
    }
    double r[33];
    for (unsigned k = 0; k <= order; k++) {
        double s = 0;
        for (unsigned i = k; i < n; i++) s += wx[i] * wx[i - k];
        r[k] = s;
    }
    free(wx);
    r[0] *= 1.0 + 1e-9;
    if (r[0] <= 0) { for (unsigned j = 0; j < order; j++) lp[j] = 0; return; }
    double a[33] = {0}, tmp[33];
    double err = r[0];
    for (unsigned i = 1; i <= order; i++) {
        double acc = r[i];
        for (unsigned j = 1; j < i; j++) acc -= a[j] * r[i - j];
        double k = err > 0 ? acc / err : 0.0;
        memcpy(tmp, a, sizeof a);
        a[i] = k;
        for (unsigned j = 1; j < i; j++) a[j] = tmp[j] - k * tmp[i - j];
        err *= (1.0 - k * k);
        if (err <= 0) err = 1e-12;
    }
    for (unsigned j = 0; j < order; j++) lp[j] = a[j + 1];
}

/* quantise to `prec`-bit signed coefficients with the largest shift in [0,15] that fits */
static void quantize(const double *lp, unsigned order, unsigned prec, int32_t *q, int *shift) {
    int32_t qmax = (1 << (prec - 1)) - 1, qmin = -(1 << (prec - 1));
    double cmax = 0;
    for (unsigned j = 0; j < order; j++) if (fabs(lp[j]) > cmax) cmax = fabs(lp[j]);
    int sh = 15;
    if (cmax > 0) {
        while (sh > 0 && cmax * (double)(1 << sh) > qmax) sh--;
    }
    double e = 0;
    for (unsigned j = 0; j < order; j++) {
        e += lp[j] * (double)(1 << sh);
        long v = lround(e);
        if (v > qmax) v = qmax;
        if (v < qmin) v = qmin;
        e -= (double)v;
        q[j] = (int32_t)v;
    }
    *shift = sh;
}

/* --------------------------------------------------------------- residual coding */
static uint32_t zigzag(int32_t r) { return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31); }

static unsigned bits_signed(int32_t v) { /* bits to hold v as two's complement */
    unsigned b = 1;
    while (b < 32) {
        int32_t lo = -(int32_t)(1u << (b - 1)), hi = (int32_t)((1u << (b - 1)) - 1);
        if (v >= lo && v <= hi) return b;
        b++;
    }
    return 32;
}

typedef struct { int porder; uint32_t k[1 << 8]; uint32_t esc_bits[1 << 8]; uint64_t bits; } rice_plan;

static uint64_t plan_partition(const int32_t *r, unsigned n, int rice2, int allow_escape, uint32_t *k_out, uint32_t *esc_out) {
    unsigned kmax = rice2 ? 30 : 14;
    uint64_t best = UINT64_MAX;
    uint32_t bestk = 0;
    for (unsigned k = 0; k <= kmax; k++) {
        uint64_t c = 0;
        for (unsigned i = 0; i < n; i++) c += (uint64_t)(zigzag(r[i]) >> k) + 1 + k;
        if (c < best) { best = c; bestk = k; }
    }
    *esc_out = 0xFFFFFFFFu;
    unsigned nb = 0;
    for (unsigned i = 0; i < n; i++) { unsigned b = bits_signed(r[i]); if (b > nb) nb = b; }
    int all_zero = 1;
    for (unsigned i = 0; i < n; i++) if (r[i]) { all_zero = 0; break; }
    if (all_zero) nb = 0;
    if (nb <= 31) {
        uint64_t c = 5 + (uint64_t)nb * n;
        if (allow_escape || c < best) {
            if (allow_escape || c < best) { best = c; *esc_out = nb; }
        }
    }
    *k_out = bestk;
    return best + (rice2 ? 5 : 4);
}

static void plan_rice(const int32_t *res, unsigned bs, unsigned order, int porder_req, int rice2,
                      rng_t *rng, int escape_permille, rice_plan *pl) {
    int maxp = 8;
    int lo = 0, hi = maxp;
    if (porder_req >= 0) { lo = hi = porder_req > maxp ? maxp : porder_req; }
    pl->bits = UINT64_MAX;
    for (int p = hi; p >= lo; p--) {
        int pp = p;
        while (pp > 0 && ((bs & ((1u << pp) - 1)) || (bs >> pp) < order || (bs >> pp) == 0)) pp--;
        if (pp != p && porder_req < 0) continue;
        unsigned parts = 1u << pp;
        unsigned psz = pp ? bs >> pp : bs - order;
        rice_plan cand;
        cand.porder = pp;
        cand.bits = 6;
        const int32_t *r = res;
        for (unsigned i = 0; i < parts; i++) {
            unsigned cnt = (pp == 0) ? psz : (i == 0 ? psz - order : psz);
            int esc = escape_permille > 0 && (int)rng_below(rng, 1000) < escape_permille;
            cand.bits += plan_partition(r, cnt, rice2, esc, &cand.k[i], &cand.esc_bits[i]);
            r += cnt;
        }
        if (cand.bits < pl->bits) *pl = cand;
        if (porder_req >= 0) break;
    }
}

static void write_residual(bw_t *w, const int32_t *res, unsigned bs, unsigned order, const rice_plan *pl, int rice2) {
    bw_put(w, rice2 ? 1u : 0u, 2);
    bw_put(w, (uint32_t)pl->porder, 4);
    unsigned parts = 1u << pl->porder;
    unsigned psz = pl->porder ? bs >> pl->porder : bs - order;
    const int32_t *r = res;
    int plen = rice2 ? 5 : 4;
    for (unsigned i = 0; i < parts; i++) {
        unsigned cnt = (pl->porder == 0) ? psz : (i == 0 ? psz - order : psz);
        if (pl->esc_bits[i] != 0xFFFFFFFFu) {
            bw_put(w, rice2 ? 31u : 15u, plen);
            bw_put(w, pl->esc_bits[i], 5);
            for (unsigned j = 0; j < cnt; j++) bw_put_signed(w, r[j], (int)pl->esc_bits[i]);
        } else {
            uint32_t k = pl->k[i];
            bw_put(w, k, plen);
            for (unsigned j = 0; j < cnt; j++) {
                uint32_t u = zigzag(r[j]);
                bw_zeros(w, u >> k);
                bw_put(w, 1, 1);
                if (k) bw_put(w, u & ((1u << k) - 1), (int)k);
            }
        }
        r += cnt;
    }
}

/* --------------------------------------------------------------- subframes */
typedef struct {
    int type;     /* 0 const, 1 verbatim, 2 fixed, 3 lpc */
    unsigned order, prec;
} sf_choice;

static void encode_subframe(bw_t *w, const int32_t *x, unsigned bs, unsigned bps, sf_choice ch,
                            const bnsyn_params *p, rng_t *rng, int32_t *res_scratch) {
    /* wasted bits */
    uint32_t orv = 0;
    for (unsigned i = 0; i < bs; i++) orv |= (uint32_t)x[i];
    unsigned wb = 0;
    if (orv) { while (!((orv >> wb) & 1u)) wb++; }
    if (wb >= bps) wb = bps - 1;
    int all_same = 1;
    for (unsigned i = 1; i < bs; i++) if (x[i] != x[0]) { all_same = 0; break; }
    if (ch.type == 0 && !all_same) ch.type = 1;
    if (ch.type == 0) wb = 0;
    unsigned sbps = bps - wb;
    int32_t *v = res_scratch + bs; /* shifted samples */
    for (unsigned i = 0; i < bs; i++) v[i] = x[i] >> wb;
    if ((ch.type == 2 || ch.type == 3) && ch.order >= bs) ch.type = 1;
    unsigned hdr_type = 0;
    if (ch.type == 0) hdr_type = 0;
    else if (ch.type == 1) hdr_type = 1;
    else if (ch.type == 2) hdr_type = 8 + ch.order;
    else hdr_type = 32 + (ch.order - 1);
    bw_put(w, 0, 1);
    bw_put(w, hdr_type, 6);
    if (wb) {
        bw_put(w, 1, 1);
        bw_zeros(w, wb - 1);
        bw_put(w, 1, 1);
    } else {
        bw_put(w, 0, 1);
    }
    if (ch.type == 0) { bw_put_signed(w, v[0], (int)sbps); return; }
    if (ch.type == 1) { for (unsigned i = 0; i < bs; i++) bw_put_signed(w, v[i], (int)sbps); return; }
    int rice2 = p->rice2;
    rice_plan pl;
    if (ch.type == 2) {
        for (unsigned i = 0; i < ch.order; i++) bw_put_signed(w, v[i], (int)sbps);
        for (unsigned i = ch.order; i < bs; i++) res_scratch[i - ch.order] = (int32_t)((uint32_t)v[i] - (uint32_t)fixed_pred(v + i, ch.order));
        plan_rice(res_scratch, bs, ch.order, p->partition_order, rice2, rng, p->escape_permille, &pl);
        write_residual(w, res_scratch, bs, ch.order, &pl, rice2);
        return;
    }
    /* LPC */
    double lp[32];
    int32_t q[32];
    int shift;
    lpc_coefs(v, bs, ch.order, lp);
    /* libFLAC 1.2.1's encoder keeps <= 17-bit subframes on the 32-bit restore path:
     * qlp_coeff_precision = min(precision, 32 - subframe_bps - ilog2(order)) */
    if (p->prec_clamp && sbps <= 17) {
        const int lim = 32 - (int)sbps - (int)ilog2u(ch.order);
        if (lim >= 1 && (int)ch.prec > lim) ch.prec = (unsigned)lim;
    }
    quantize(lp, ch.order, ch.prec, q, &shift);
    int wide = (sbps + ch.prec + ilog2u(ch.order)) > 32;
    for (unsigned i = 0; i < ch.order; i++) bw_put_signed(w, v[i], (int)sbps);
    bw_put(w, ch.prec - 1, 4);
    bw_put_signed(w, shift, 5);
    for (unsigned j = 0; j < ch.order; j++) bw_put_signed(w, q[j], (int)ch.prec);
    for (unsigned i = ch.order; i < bs; i++)
        res_scratch[i - ch.order] = (int32_t)((uint32_t)v[i] - (uint32_t)lpc_pred(v + i, q, ch.order, shift, wide));
    plan_rice(res_scratch, bs, ch.order, p->partition_order, rice2, rng, p->escape_permille, &pl);
    write_residual(w, res_scratch, bs, ch.order, &pl, rice2);
}

/* ----------------------------------------------------------------- headers */
static const uint32_t kRates[12] = {0, 88200, 176400, 192000, 8000, 16000, 22050, 24000, 32000, 44100, 48000, 96000};

static void bs_code(uint32_t bs, int odd, uint32_t *code, int *extra_bits) {
    *extra_bits = 0;
    if (!odd) {
        if (bs == 192) { *code = 1; return; }
        for (uint32_t c = 2; c <= 5; c++) if (bs == (576u << (c - 2))) { *code = c; return; }
        for (uint32_t c = 8; c <= 15; c++) if (bs == (256u << (c - 8))) { *code = c; return; }
    }
    if (bs <= 256) { *code = 6; *extra_bits = 8; }
    else { *code = 7; *extra_bits = 16; }
}

static void sr_code(uint32_t sr, int odd, int force, uint32_t *code, int *extra_bits, uint32_t *extra) {
    *extra_bits = 0;
    *extra = 0;
    if (force >= 0) { *code = (uint32_t)force; }
    else {
        *code = 0;
        if (!odd) {
            for (uint32_t c = 1; c < 12; c++) if (kRates[c] == sr) { *code = c; return; }
        }
        if (sr % 1000 == 0 && sr / 1000 <= 255) *code = 12;
        else if (sr <= 65535) *code = 13;
        else if (sr % 10 == 0 && sr / 10 <= 65535) *code = 14;
        else { *code = 0; return; }
    }
    if (*code == 12) { *extra_bits = 8; *extra = sr / 1000; }
    else if (*code == 13) { *extra_bits = 16; *extra = sr; }
    else if (*code == 14) { *extra_bits = 16; *extra = sr / 10; }
}

static uint32_t bps_code(uint32_t bps) {
    switch (bps) {
    case 8: return 1;
    case 12: return 2;
    case 16: return 4;
    case 20: return 5;
    case 24: return 6;
    default: return 0;
    }
}

void bnsyn_default_params(bnsyn_params *p) {
    memset(p, 0, sizeof *p);
    p->sample_rate = 44100;
    p->channels = 2;
    p->bps = 16;
    p->blocksize = 4096;
    p->nframes = 16;
    p->subframe_mode = BNSYN_SUB_LPC;
    p->order = 8;
    p->qlp_precision = 0;
    p->partition_order = 4;
    p->stereo_mode = BNSYN_STEREO_INDEPENDENT;
    p->level = 0.5;
    p->noise = 0.006;
    p->impulse_permille = 0;
    p->seed = 1;
    p->write_header = 1;
    p->force_sr_code = -1;
    p->bs_min = 192;
    p->bs_max = 16384;
}

static const uint32_t kLegalBs[] = {192, 576, 1152, 2304, 4608, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768};

static uint32_t pick_bs(const bnsyn_params *p, rng_t *rng, uint32_t frame) {
    if (!p->variable_blocksize) {
        if (frame + 1 == p->nframes && p->last_blocksize) return p->last_blocksize;
        return p->blocksize;
    }
    uint32_t cand[16];
    int n = 0;
    for (unsigned i = 0; i < sizeof kLegalBs / sizeof kLegalBs[0]; i++)
        if (kLegalBs[i] >= p->bs_min && kLegalBs[i] <= p->bs_max) cand[n++] = kLegalBs[i];
    if (n == 0) return p->bs_min;
    return cand[rng_below(rng, (uint32_t)n)];
}

size_t bnsyn_max_bytes(const bnsyn_params *p) {
    uint64_t bs = p->variable_blocksize ? (p->bs_max ? p->bs_max : 65535) : p->blocksize;
    if (p->last_blocksize > bs) bs = p->last_blocksize;
    /* worst case: escaped partitions of FIXED-4 residuals (up to 16x the signal, +1 side bit:
     * bps + 5 bits each) or verbatim, + headers; bps + 8 bits per sample covers both */
    uint64_t per = (uint64_t)p->channels * (bs * (uint64_t)(p->bps + 8) / 8 + 64 + 4 * 32 + 16) + 64;
    return (size_t)(per * (uint64_t)p->nframes + 4096);
}

/* One resonator bank per channel plus a shared one. */
typedef struct { double a1, a2, y1, y2; } reson_t;
static double reson_step(reson_t *r, double x) {
    double y = x + r->a1 * r->y1 + r->a2 * r->y2;
    r->y2 = r->y1;
    r->y1 = y;
    return y;
}

int bnsyn_encode(const bnsyn_params *p, uint8_t *out, size_t cap, size_t *out_len, int32_t *pcm,
                 size_t pcm_cap, size_t *pcm_len, uint64_t *frame_offsets, size_t offsets_cap,
                 uint32_t *nframes_out) {
    crc_init();
    if (p->channels < 1 || p->channels > 8 || p->bps < 4 || p->bps > 32 || p->nframes == 0) return -2;
    if (!p->variable_blocksize && (p->blocksize < 1 || p->blocksize > 65535)) return -2;
    rng_t rng = {p->seed * 0x2545F4914F6CDD1Dull + 0x1234567ull};
    const unsigned C = p->channels;
    /* frame sizes first (deterministic) */
    uint32_t *bsz = (uint32_t *)malloc(sizeof(uint32_t) * p->nframes);
    uint64_t total = 0;
    uint32_t maxbs = 0, minbs = 0xFFFFFFFFu;
    for (uint32_t f = 0; f < p->nframes; f++) {
        bsz[f] = pick_bs(p, &rng, f);
        total += bsz[f];
        if (bsz[f] > maxbs) maxbs = bsz[f];
        if (bsz[f] < minbs) minbs = bsz[f];
    }
    /* source signal */
    const double fs = ldexp(1.0, (int)p->bps - 1);
    const int64_t smax = (int64_t)fs - 1, smin = -(int64_t)fs;
    int32_t *sig = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total * C + 1));
    {
        reson_t shared[2], own[8][2];
        for (int k = 0; k < 2; k++) {
            double rad = 0.995 - 0.01 * k, th = 0.02 + 0.07 * k + 0.01 * (double)(p->seed % 7);
            shared[k].a1 = 2 * rad * cos(th); shared[k].a2 = -rad * rad; shared[k].y1 = shared[k].y2 = 0;
        }
        for (unsigned c = 0; c < C; c++)
            for (int k = 0; k < 2; k++) {
                double rad = 0.99 - 0.02 * k, th = 0.05 + 0.11 * k + 0.013 * c;
                own[c][k].a1 = 2 * rad * cos(th); own[c][k].a2 = -rad * rad; own[c][k].y1 = own[c][k].y2 = 0;
            }
        double *raw = (double *)malloc(sizeof(double) * (size_t)(total * C + 1));
        double rms = 0;
        for (uint64_t n = 0; n < total; n++) {
            double e = rng_gauss(&rng);
            double s = reson_step(&shared[1], reson_step(&shared[0], e));
            for (unsigned c = 0; c < C; c++) {
                double o = reson_step(&own[c][1], reson_step(&own[c][0], rng_gauss(&rng)));
                double v = 0.8 * s + 0.45 * o;
                raw[n * C + c] = v;
                rms += v * v;
            }
        }
        rms = sqrt(rms / (double)(total * C + 1)) + 1e-30;
        double scale = (p->level * fs / 3.0) / rms;
        double nstd = p->noise * fs;
        for (uint64_t i = 0; i < total * C; i++) {
            double v = raw[i] * scale + nstd * rng_gauss(&rng);
            if (p->impulse_permille > 0 && (int)rng_below(&rng, 1000) < p->impulse_permille)
                v += (rng_below(&rng, 2) ? 0.4 : -0.4) * fs;
            int64_t q = (int64_t)llround(v);
            if (q > smax) q = smax;
            if (q < smin) q = smin;
            sig[i] = (int32_t)q;
        }
        free(raw);
    }
    /* per-frame shaping: wasted bits, constant frames (mixed mode) */
    {
        uint64_t base = 0;
        for (uint32_t f = 0; f < p->nframes; f++) {
            uint32_t bs = bsz[f];
            unsigned w = p->wasted_bits_max ? rng_below(&rng, p->wasted_bits_max + 1) : 0;
            int constant = (p->subframe_mode == BNSYN_SUB_CONSTANT) ||
                           (p->subframe_mode == BNSYN_SUB_MIXED && rng_below(&rng, 16) == 0);
            int32_t cval = (int32_t)(rng_below(&rng, 2001)) - 1000;
            for (uint32_t i = 0; i < bs; i++)
                for (unsigned c = 0; c < C; c++) {
                    int32_t *s = &sig[(base + i) * C + c];
                    if (constant) *s = cval + (int32_t)c * 7;
                    if (w) *s = (int32_t)((uint32_t)(*s >> w) << w);
                }
            base += bs;
        }
    }
    if (pcm) {
        size_t n = (size_t)(total * C);
        if (n > pcm_cap) { free(sig); free(bsz); return -1; }
        memcpy(pcm, sig, n * sizeof(int32_t));
    }
    if (pcm_len) *pcm_len = (size_t)(total * C);

    bw_t w = {out, cap, 0, 0, 0, 0};
    size_t si_pos = 0;
    if (p->write_header) {
        bw_put(&w, 0x664C6143u, 32);
        si_pos = w.n;
        bw_put(&w, 1, 1); /* last metadata block */
        bw_put(&w, 0, 7);
        bw_put(&w, 34, 24);
        bw_zeros(&w, 34 * 8); /* patched below */
    }
    int32_t *chx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxbs + 1) * (C > 2 ? C : 2));
    int32_t *scratch = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxbs + 1) * 2);
    uint32_t minfs = 0xFFFFFFFFu, maxfs = 0;
    uint64_t base = 0;
    for (uint32_t f = 0; f < p->nframes; f++) {
        uint32_t bs = bsz[f];
        size_t fstart = w.n;
        if (frame_offsets && f < offsets_cap) frame_offsets[f] = fstart;
        /* channel assignment */
        unsigned assign = 0;
        if (C == 2) {
            int m = p->stereo_mode;
            if (m == BNSYN_STEREO_CYCLE) m = (int)(f % 4);
            assign = (unsigned)m;
        }
        unsigned sub_bps[8];
        for (unsigned c = 0; c < C; c++) {
            sub_bps[c] = p->bps;
            for (uint32_t i = 0; i < bs; i++) chx[c * bs + i] = sig[(base + i) * C + c];
        }
        if (C == 2 && assign) {
            int32_t *L = chx, *R = chx + bs;
            for (uint32_t i = 0; i < bs; i++) {
                int32_t l = L[i], r = R[i];
                int32_t side = (int32_t)((uint32_t)l - (uint32_t)r);
                if (assign == 1) { R[i] = side; }
                else if (assign == 2) { L[i] = side; }
                else { L[i] = (int32_t)(((int64_t)l + (int64_t)r) >> 1); R[i] = side; }
            }
            if (assign == 1 || assign == 3) sub_bps[1]++;
            else sub_bps[0]++;
        }
        /* header */
        uint32_t bcode, scode, sextra;
        int bextra, sextra_bits;
        bs_code(bs, p->odd_headers && (f & 1), &bcode, &bextra);
        sr_code(p->sample_rate, p->odd_headers && (f & 2), p->force_sr_code, &scode, &sextra_bits, &sextra);
        uint32_t ccode = (C == 2 && assign) ? (7u + assign) : (C - 1);
        size_t hstart = w.n;
        bw_put(&w, 0xFFF8u | (p->variable_blocksize ? 1u : 0u), 16);
        bw_put(&w, bcode, 4);
        bw_put(&w, scode, 4);
        bw_put(&w, ccode, 4);
        bw_put(&w, bps_code(p->bps), 3);
        bw_put(&w, 0, 1);
        if (p->variable_blocksize) bw_utf8(&w, base);
        else bw_utf8(&w, f);
        if (bextra) bw_put(&w, bs - 1, bextra);
        if (sextra_bits) bw_put(&w, sextra, sextra_bits);
        if (w.n <= cap) bw_put(&w, crc8(out + hstart, w.n - hstart), 8);
        else bw_put(&w, 0, 8);
        /* subframes */
        for (unsigned c = 0; c < C; c++) {
            sf_choice sc;
            sc.prec = p->qlp_precision ? p->qlp_precision : 12 + rng_below(&rng, 4);
            switch (p->subframe_mode) {
            case BNSYN_SUB_FIXED: sc.type = 2; sc.order = p->order > 4 ? 4 : p->order; break;
            case BNSYN_SUB_VERBATIM: sc.type = 1; sc.order = 0; break;
            case BNSYN_SUB_CONSTANT: sc.type = 0; sc.order = 0; break;
            case BNSYN_SUB_MIXED: {
                uint32_t t = rng_below(&rng, 8);
                if (t == 0) { sc.type = 0; sc.order = 0; }
                else if (t == 1) { sc.type = 1; sc.order = 0; }
                else if (t <= 3) { sc.type = 2; sc.order = rng_below(&rng, 5); }
                else { sc.type = 3; sc.order = 1 + rng_below(&rng, 32); sc.prec = 5 + rng_below(&rng, 11); }
                break;
            }
            default: sc.type = 3; sc.order = p->order ? p->order : 8; break;
            }
            if (sc.type == 3 && sc.order > 32) sc.order = 32;
            encode_subframe(&w, chx + c * bs, bs, sub_bps[c], sc, p, &rng, scratch);
        }
        bw_align(&w);
        if (w.n <= cap) {
            uint16_t c16 = crc16(out + fstart, w.n - fstart);
            bw_put(&w, c16, 16);
        } else {
            bw_put(&w, 0, 16);
        }
        uint32_t fsz = (uint32_t)(w.n - fstart);
        if (fsz < minfs) minfs = fsz;
        if (fsz > maxfs) maxfs = fsz;
        base += bs;
    }
    free(chx);
    free(scratch);
    if (w.overflow || w.n > cap) { free(sig); free(bsz); return -1; }
    if (p->write_header) {
        bw_t h = {out + si_pos + 4, 34, 0, 0, 0, 0};
        uint32_t mnb = p->variable_blocksize ? minbs : p->blocksize;
        uint32_t mxb = p->variable_blocksize ? maxbs : p->blocksize;
        bw_put(&h, mnb, 16);
        bw_put(&h, mxb, 16);
        bw_put(&h, minfs, 24);
        bw_put(&h, maxfs, 24);
        bw_put(&h, p->sample_rate, 20);
        bw_put(&h, C - 1, 3);
        bw_put(&h, p->bps - 1, 5);
        bw_put(&h, (uint32_t)(total >> 32) & 0xF, 4);
        bw_put(&h, (uint32_t)total, 32);
        /* MD5 of interleaved little-endian samples, ceil(bps/8) bytes each */
        md5_t m;
        md5_init(&m);
        unsigned bytes = (p->bps + 7) / 8;
        uint8_t tmp[4096];
        size_t tn = 0;
        for (uint64_t i = 0; i < total * C; i++) {
            uint32_t v = (uint32_t)sig[i];
            for (unsigned b = 0; b < bytes; b++) tmp[tn++] = (uint8_t)(v >> (8 * b));
            if (tn > sizeof tmp - 8) { md5_update(&m, tmp, tn); tn = 0; }
        }
        md5_update(&m, tmp, tn);
        uint8_t dig[16];
        md5_final(&m, dig);
        for (int i = 0; i < 16; i++) bw_put(&h, dig[i], 8);
    }
    *out_len = w.n;
    if (nframes_out) *nframes_out = p->nframes;
    free(sig);
    free(bsz);
    return 0;
}
