/*
 * bnflac_sys.hip -- k_decode_sys: FLAC frame decode with the LPC recurrence restored by a
 * systolic lane quad per subframe (north_star's "blocked parallel-IIR for the LPC recurrence").
 *
 * Replaces, for every subframe type, libFLAC 1.2.1's read_subframe_* + restore kernels
 * (LibFlac.dll@0x10012480 .. @0x10012da0, FIXED @0x10003810, LPC 32-bit @0x1001be10 /
 * MMX16 @0x1001c000, LPC 64-bit @0x10006120) and the read_frame_ tail (@0x100118c0: zero
 * padding, CRC-16 @0x10011a01, zero fill @0x10011af5), with BirdNest.Audio's PCM packing
 * (FLACDecoder.cs:543-577, FLACFileReader.cs:220-237) -- SURVEY.md 8a rows A4-A12, A15, A17.
 *
 * Why.  libFLAC's restore s[n] = r[n] + ((sum_j c[j] s[n-1-j]) >> shift) floors at every
 * sample, so no exact prefix scan exists; the lane kernels (k_decode<W>, k_decode_st) run one
 * subframe per lane and are bound by that lane's serial chain (C5: 3,752 subframes of one file
 * are 59 waves on 1,024 SIMDs).  The sum itself is linear, though: every term c[d] s[m] can be
 * added as soon as s[m] exists.  So the pending samples' partial sums are kept in an
 * accumulator array spread over the lanes of a quad, and the serial remainder per sample is one
 * MAC, one shift and one add:
 *   - lane j of the quad owns samples n = j (mod 4); slot a of the lane holds the partial sum of
 *     the pending sample with (n / 4) mod A == a (P = 4A >= the order pending samples);
 *   - step n: the lane owning n finalises it (the shift of its slot, plus the residual), resets
 *     the slot (it now holds sample n + P), and broadcasts s[n] to the quad (one DPP quad_perm);
 *   - every lane then adds c[d] * s[n] to each slot, d = the slot sample's distance - 1; the
 *     coefficients are rotated per lane once per subframe (rc[u] = c[(j + u) mod P]), so every
 *     register index is a compile-time constant of the 32-step unrolled chunk.
 * Each sum is the exact 64-bit sum of the same products libFLAC adds (v_mad_i64_i32), so the
 * 64-bit path keeps (int32)(S >> shift) and the 32-bit paths (ia32, MMX16, FIXED) the low word
 * of S, shifted -- the wrapped int32 sum.  MMX16 reads saturated / truncated int16 history,
 * which is the identity while every sample fits int16; a subframe that leaves int16 hands its
 * frame back (below).
 *
 * Work split (one workgroup = 64 subframe slots, k_decode's frame-slot layout):
 *   wave 0 (the producer): one lane per subframe -- header, warm-ups, partitioned Rice / escape /
 *     VERBATIM residuals (k_decode's reader: LDS-DMA ring, rice_fused) into a [sample][slot] row
 *     buffer, 32 samples per chunk;
 *   waves 1..4 (restore): 16 subframes each, a lane quad per subframe, restore the previous
 *     chunk in place, then decorrelate and write the requested layout for their frames.
 * Two row buffers, one s_barrier per chunk: the producer decodes chunk k while the restore waves
 * finish chunk k - 1.  After the last chunk the producer reads the zero padding and the CRC-16
 * footer; the restore waves check each frame's CRC-16 with coalesced 1 KB loads (wave_crc_range,
 * the whole frame plus footer: zero iff it matches) and zero-fill a mismatch, as libFLAC does.
 *
 * Hand-back: a frame whose decode hits anything off the common path -- an error, truncation, a
 * 64-bit-path shift of 32 or more, an MMX16 subframe leaving int16 -- is flagged
 * BNF_FL_WAVE_REDO and appended to a device list; k_decode_list (the exact lane kernel
 * k_decode<32>, BNF_MODE_LIST) then decodes exactly those frames from scratch, so records and
 * bytes equal the lane path's for every frame.
 */
#define BNF_TU 8
#include "bnflac_kernels.hip"

#define SYS_CHK 32                   /* samples per chunk: one s_barrier per chunk */
#define SYS_RP 80                    /* row stride (dwords), [sample][slot]: 80 = 16 mod 64 banks */
#define SYS_CW 4                     /* restore waves per workgroup (16 subframe slots each) */
#define SYS_THREADS (64 * (1 + SYS_CW))
#define SYS_RD 8                     /* producer ring: 16-byte blocks per lane */
#define SYS_CS 33                    /* coefficient table stride per slot (bank spread) */

static_assert(SYS_CHK == 32, "the restore chunk is written for 32 samples (8 per quad lane)");
static_assert(64 * SYS_CS * 4 <= SYS_CHK * SYS_RP * 4, "the coefficient table overlays row buffer 1");
static_assert((8 * 256 + 512) * 2 <= SYS_CHK * SYS_RP * 4, "the CRC tables overlay row buffer 0");

enum { PM_NARROW = 0, PM_WIDE = 1, PM_MIXED = 2 };
#define SF_ACTIVE 1u
#define SF_WIDE 2u
#define SF_MMX 4u

/* frame states (per frame slot of the workgroup) */
enum { FS_NONE = 0, FS_DEC = 1, FS_TAIL = 2 };

struct SysShared {
    uint32_t ring[SYS_RD * RING_LANE_DW];  /* producer bit rings: LDS-DMA images, 1 KiB aligned (first) */
    int32_t rows[2][SYS_CHK * SYS_RP];     /* residuals in, samples out; [1] holds the coefficients at setup */
    uint32_t p_order[64], p_sh[64], p_flags[64], p_wasted[64], p_bs[64];
    uint32_t f_idx[64], f_bs[64], f_ch[64], f_as[64], f_state[64], f_end[64], f_crc[64], f_bad[64];
    uint64_t f_os[64], f_off[64], f_resume[64];
    uint32_t nchunks;
};

DEV void sys_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

/* 2-deep producer refill, every 16 samples: the blocks issued by the previous refill may stay in
 * flight; everything issued before it has landed (vmcnt retires in issue order and the producer
 * issues no other vector-memory ops).  Then the blocks up to SYS_RD past the cursor's block. */
struct SysQ {
    uint32_t d_last; /* DMA instructions of the previous refill (wave-uniform) */
    uint32_t e1;     /* the lane's iend when the previous refill started */
};
DEV void sys_refill(BR &b, bool want, SysQ &q) {
    wait_vm_n(q.d_last);
    b.vendw = max(b.vendw, q.e1 * 4u);
    q.e1 = b.iend;
    const uint32_t cb = b.wi >> 2;
    const uint32_t lo = max(b.iend, cb), hi = cb + b.rdepth;
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < SYS_RD; k++) {
        const uint32_t j = lo + (((uint32_t)k - lo) & (b.rdepth - 1u));
        const bool go = want && j < hi;
        if (__any(go)) {
            d++;
            if (go) dma_block(b, j, (uint32_t)k);
        }
    }
    if (want) b.iend = max(b.iend, hi);
    q.d_last = d;
}

/* ------------------------------------------------------------------ the restore quad */
/* c * x + acc exactly, one v_mad_i64_i32 (k_decode_sw's sw_mad: written out so the compiler
 * cannot widen the loop-invariant coefficient into a 64x64-bit multiply; the destination is
 * early-clobber, V_MAD_I64_I32 must not overlap a 32-bit source) */
DEV int64_t sys_mad(int32_t c, int32_t x, int64_t acc) {
    int64_t d;
    uint64_t co;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=&v"(d), "=&s"(co) : "v"(c), "v"(x), "v"(acc));
    return d;
}
/* lane j's broadcast of lane JJ of its quad (DPP quad_perm) */
template <int JJ> DEV int32_t quad_bcast(int32_t x) { return __builtin_amdgcn_mov_dpp(x, JJ * 0x55, 0xF, 0xF, false); }

/* 32 samples of a chunk.  v[q]: on entry the residual (or warm-up) of sample n0 + j + 4q, on exit
 * the sample.  FIRST: chunk 0, where samples below the order are raw warm-ups. */
template <int A, int PM, bool FIRST>
DEV void sys_steps(int64_t (&acc)[8], const int32_t (&rc)[32], int32_t (&v)[8], uint32_t j, uint32_t sh, bool wide,
                   uint32_t order) {
    constexpr int P = 4 * A;
#pragma unroll
    for (int t = 0; t < 32; t++) {
        const int jj = t & 3, q = t >> 2, a = q % A;
        if (j == (uint32_t)jj) { /* finalise sample n0 + t in the lane that owns it */
            const uint32_t lo = (uint32_t)acc[a], hi = (uint32_t)((uint64_t)acc[a] >> 32);
            int32_t pred;
            if (PM == PM_WIDE) pred = (int32_t)__builtin_amdgcn_alignbit(hi, lo, sh);
            else if (PM == PM_NARROW) pred = (int32_t)lo >> sh;
            else pred = (int32_t)__builtin_amdgcn_alignbit(wide ? hi : (uint32_t)((int32_t)lo >> 31), lo, sh);
            if (FIRST && (uint32_t)t < order) pred = 0;
            v[q] = (int32_t)((uint32_t)v[q] + (uint32_t)pred);
            acc[a] = 0;
        }
        int32_t bc;
        switch (jj) {
        case 0: bc = quad_bcast<0>(v[q]); break;
        case 1: bc = quad_bcast<1>(v[q]); break;
        case 2: bc = quad_bcast<2>(v[q]); break;
        default: bc = quad_bcast<3>(v[q]); break;
        }
#pragma unroll
        for (int a2 = 0; a2 < A; a2++) {
            const int u = ((4 * a2 - t - 1) % P + P) % P;
            acc[a2] = sys_mad(rc[u], bc, acc[a2]);
        }
    }
}

/* ------------------------------------------------------------------ pack */
/* The restore wave's frames of one chunk (final samples, wasted bits applied, in `row`) into the
 * caller's layout.  Generic per-value stores (any layout, any alignment, partial chunks). */
DEV void sys_pack(const SysShared &S, const int32_t *row, uint32_t w, uint32_t lane, uint32_t lg, uint32_t n0, int fmt,
                  const bnf_stream_params &sp, uint8_t *__restrict__ out) {
    const uint32_t cl = 1u << lg, nfw = 16u >> lg, fl0 = (16u * w) >> lg;
    for (uint32_t i = 0; i < nfw; i++) {
        const uint32_t fl = fl0 + i;
        if (S.f_state[fl] != FS_DEC) continue; /* wave-uniform */
        const uint32_t bs = S.f_bs[fl];
        if (n0 >= bs) continue;
        const uint32_t C = S.f_ch[fl], as = S.f_as[fl], nv = min((uint32_t)SYS_CHK, bs - n0);
        const uint64_t os = S.f_os[fl];
        const uint32_t s0 = fl * cl;
        const uint32_t fb = sp.bps == 24 ? 3u : 2u;
        for (uint32_t v = lane; v < nv * C; v += 64u) {
            const uint32_t n = v / C, c = v - n * C;
            int32_t x0 = row[n * SYS_RP + s0], x1 = C >= 2u ? row[n * SYS_RP + s0 + 1u] : 0;
            if (C == 2u) decorrelate(as, x0, x1);
            const int32_t x = c == 0u ? x0 : (c == 1u ? x1 : row[n * SYS_RP + s0 + c]);
            const uint64_t sn = os + n0 + n;
            switch (fmt) {
            case BNF_OUT_PLANAR32: ((int32_t *)out)[os * sp.channels + (uint64_t)c * bs + n0 + n] = x; break;
            case BNF_OUT_INTERLEAVED32: ((int32_t *)out)[sn * sp.channels + c] = x; break;
            case BNF_OUT_FLACDECODER: /* FLACDecoder.cs:543-577 */
                if (c == 0u) {
                    if (C == 2u) ((uint32_t *)out)[sn] = ((uint32_t)x0 & 0xffffu) | ((uint32_t)x1 << 16);
                    else ((uint16_t *)out)[sn] = (uint16_t)(uint32_t)x0;
                }
                break;
            default: { /* FLACFileReader.cs:220-237 */
                uint8_t *p = out + sn * sp.channels * fb + c * fb;
                p[0] = (uint8_t)x;
                p[1] = (uint8_t)(x >> 8);
                if (fb == 3u) p[2] = (uint8_t)(x >> 16);
            }
            }
        }
    }
}

/* ------------------------------------------------------------------ restore waves */
template <int A, int PM>
DEV void sys_restore(SysShared &S, uint32_t w, uint32_t lane, uint32_t lg, uint32_t nchunks, int fmt,
                     const bnf_stream_params &sp, uint8_t *__restrict__ out) {
    constexpr int P = 4 * A;
    const uint32_t g = lane >> 2, j = lane & 3u, pl = 16u * w + g;
    const uint32_t order = S.p_order[pl], flags = S.p_flags[pl], wasted = S.p_wasted[pl], bs = S.p_bs[pl];
    const uint32_t sh = S.p_sh[pl];
    const bool active = (flags & SF_ACTIVE) != 0u, wide = (flags & SF_WIDE) != 0u, mmx = (flags & SF_MMX) != 0u;
    int32_t rc[32];
    const int32_t *cf = S.rows[1] + pl * SYS_CS;
#pragma unroll
    for (int u = 0; u < 32; u++) rc[u] = u < P ? cf[(j + (uint32_t)u) & (uint32_t)(P - 1)] : 0;
    int64_t acc[8];
#pragma unroll
    for (int a = 0; a < 8; a++) acc[a] = 0;
    bool range_bad = false;
    sys_bar(); /* end of iteration 0: the producer's chunk 0 is in rows[0]; rows[1] may be overwritten */
    for (uint32_t k = 1; k <= nchunks; k++) {
        const uint32_t n0 = (k - 1u) * SYS_CHK;
        int32_t *row = S.rows[(k - 1u) & 1u];
        int32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = row[(j + 4u * q) * SYS_RP + pl];
        if (k == 1u) sys_steps<A, PM, true>(acc, rc, v, j, sh, wide, order);
        else sys_steps<A, PM, false>(acc, rc, v, j, sh, wide, order);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t n = n0 + j + 4u * q;
            if (active && n < bs) {
                row[(j + 4u * q) * SYS_RP + pl] = (int32_t)((uint32_t)v[q] << wasted);
                if (mmx && v[q] != (int32_t)(int16_t)v[q]) range_bad = true;
            }
        }
        lds_sync();
        sys_pack(S, row, w, lane, lg, n0, fmt, sp, out);
        sys_bar();
    }
    if (range_bad) S.f_bad[pl >> lg] = 1u;
}

template <int A>
DEV void sys_restore_pm(SysShared &S, uint32_t w, uint32_t lane, uint32_t lg, uint32_t nchunks, int fmt,
                        const bnf_stream_params &sp, uint8_t *out, int pm) {
    if (pm == PM_WIDE) sys_restore<A, PM_WIDE>(S, w, lane, lg, nchunks, fmt, sp, out);
    else if (pm == PM_NARROW) sys_restore<A, PM_NARROW>(S, w, lane, lg, nchunks, fmt, sp, out);
    else sys_restore<A, PM_MIXED>(S, w, lane, lg, nchunks, fmt, sp, out);
}

/* ------------------------------------------------------------------ the kernel */
__global__ void __launch_bounds__(SYS_THREADS) k_decode_sys(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                            uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes,
                                                            int fmt, uint8_t *__restrict__ out, uint64_t out_bytes,
                                                            bnf_frame_info *__restrict__ info,
                                                            const uint32_t *__restrict__ perm, uint32_t *__restrict__ redo,
                                                            uint32_t ablate) {
    __shared__ LDS_DMA_ALIGN SysShared S;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t lg = __builtin_ctz(chn_lanes), fpb = 64u >> lg;
    const uint64_t limit = nbytes * 8u;

    if (wave == 0) {
        /* ================================================= producer: setup */
        const uint32_t fl = lane >> lg, ch = lane & (chn_lanes - 1u);
        const uint32_t slot = blockIdx.x * fpb + fl;
        const uint32_t f = (fl < fpb && slot < nframes) ? (perm ? perm[slot] : slot) : 0u;
        const bool have = fl < fpb && slot < nframes;
        bnf_frame_info fi;
        if (have) fi = info[f];
        const bool frame_ok = have && fi.status == BNF_ST_OK;
        if (ch == 0) { S.f_state[fl] = FS_NONE; S.f_bad[fl] = 0; }
        bool ok = false;
        if (frame_ok && ch == 0) { /* decode_block's checks, with its records (SKIPPED) */
            ok = true;
            uint32_t unsupported = 0;
            if (fmt == BNF_OUT_FLACDECODER && fi.bps != 16) unsupported = 1;          /* WriteCallback abort :526-530 */
            if (fmt >= BNF_OUT_FLACDECODER && fi.channels > sp.channels) unsupported = 1;
            if (fmt == BNF_OUT_FILEREADER && sp.bps != 16 && sp.bps != 24) unsupported = 1; /* NotSupportedException :239-240 */
            if (unsupported) {
                ok = false;
                fi.status = BNF_ST_SKIPPED;
                fi.flags |= 4u;
                info[f] = fi;
            } else {
                uint64_t stride;
                switch (fmt) {
                case BNF_OUT_PLANAR32: case BNF_OUT_INTERLEAVED32: stride = 4ull * sp.channels; break;
                case BNF_OUT_FLACDECODER: stride = fi.channels == 2 ? 4u : 2u; break;
                default: stride = (uint64_t)sp.channels * (sp.bps == 24 ? 3u : 2u); break;
                }
                if ((fi.out_sample + fi.blocksize) * stride > out_bytes) {
                    ok = false;
                    fi.status = BNF_ST_SKIPPED;
                    fi.flags |= 2u;
                    info[f] = fi;
                } else if (fi.channels > chn_lanes) {
                    ok = false;
                    fi.status = BNF_ST_SKIPPED;
                    info[f] = fi;
                }
            }
            S.f_idx[fl] = f;
            S.f_bs[fl] = fi.blocksize;
            S.f_ch[fl] = fi.channels;
            S.f_as[fl] = fi.assignment;
            S.f_os[fl] = fi.out_sample;
            S.f_off[fl] = fi.frame_off;
            if (ok) S.f_state[fl] = FS_DEC;
        }
        lds_sync();
        const bool fok = frame_ok && S.f_state[fl] == FS_DEC;
        bool active = fok && ch < fi.channels;
        /* ---- subframe header: warm-ups into rows[0], coefficients into the table (rows[1]) */
        BR b;
        br_init(b, words, nbytes, (lds_u32 *)S.ring, lane, SYS_RD);
        RS rs;
        rs.verb = 0; rs.k = 0; rs.esc = 0; rs.left = 0; rs.pidx = 0; rs.nparts = 0; rs.psamples = 0;
        rs.order = 0; rs.plen = 4; rs.pesc = 15; rs.porder = 0;
        uint32_t st = BNF_ST_OK, trunc = 0, bs = 0, order = 0;
        int32_t err = -1;
        bool bad = false;
        int32_t *row0 = S.rows[0] + lane;
        int32_t *cf = S.rows[1] + lane * SYS_CS;
        uint32_t pflags = 0, psh = 0, pwasted = 0;
        if (active) {
            bs = fi.blocksize;
            br_seek(b, fi.frame_off * 8u + info[f].sub_start[ch]);
            SubHdr h;
            h.type = T_CONST; h.order = 0; h.wasted = 0; h.bps = 0; h.shift = 0; h.path = P_IA32; h.cval = 0;
            h.porder = 0; h.rice2 = 0;
            int32_t coef[32];
            st = parse_subframe_head<true, 32, SYS_RP>(b, sub_bps(fi, ch), bs, limit, h, row0, coef, err);
            if (st != BNF_ST_OK) {
                bad = true;
            } else {
                int32_t c[32];
#pragma unroll
                for (int t = 0; t < 32; t++) c[t] = (h.type == T_LPC && (uint32_t)t < h.order) ? coef[t] : 0;
                order = h.order;
                if (h.type == T_LPC) {
                    if (h.path == P_WIDE) {
                        if ((uint32_t)h.shift >= 32u) bad = true; /* libFLAC's _allshr by >= 32: the lane kernels' */
                        pflags |= SF_WIDE;
                        psh = (uint32_t)h.shift & 31u;
                    } else if (h.path == P_MMX16) {
                        pflags |= SF_MMX;
                        psh = ((uint32_t)h.shift >= 32u) ? 31u : (uint32_t)h.shift; /* psrad >= 32 -> 31 */
                    } else {
                        psh = (uint32_t)h.shift & 31u; /* sar & 31 */
                    }
                } else if (h.type == T_FIXED) { /* FIXED order o as LPC, shift 0, 32-bit wrap (@0x10003810) */
                    const uint32_t o = h.order;
                    c[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
                    c[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
                    c[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
                    c[3] = o == 4 ? -1 : 0;
                } else if (h.type == T_CONST) { /* order 1, coefficient 1, warm-up cval, zero residuals */
                    c[0] = 1;
                    order = 1;
                    row0[0] = h.cval;
                }
#pragma unroll
                for (int t = 0; t < 32; t++) cf[t] = c[t];
                pwasted = h.wasted;
                const bool rice = h.type == T_FIXED || h.type == T_LPC;
                rs.verb = rice ? 0u : 1u;
                rs.esc = rice ? 0u : 1u;
                rs.k = h.type == T_VERB ? h.bps : 0u;
                rs.left = rice ? 0u : 0x7fffffffu;
                rs.order = h.order;
                rs.porder = h.porder;
                rs.nparts = rice ? 1u << h.porder : 0u;
                rs.psamples = h.porder ? bs >> h.porder : bs - h.order;
                rs.plen = h.rice2 ? 5u : 4u;
                rs.pesc = h.rice2 ? 31u : 15u;
            }
        }
        if (bad) S.f_bad[fl] = 1u;
        active = active && !bad;
        S.p_order[lane] = active ? order : 0u;
        S.p_flags[lane] = (active ? SF_ACTIVE : 0u) | pflags;
        S.p_sh[lane] = psh;
        S.p_wasted[lane] = pwasted;
        S.p_bs[lane] = active ? bs : 0u;
        uint32_t mybs = active ? bs : 0u;
        for (int o = 32; o > 0; o >>= 1) mybs = max(mybs, (uint32_t)__shfl_xor(mybs, o));
        const uint32_t nchunks = (mybs + SYS_CHK - 1u) / SYS_CHK;
        if (lane == 0) S.nchunks = nchunks;
        wait_vm(); /* setup loads and seeks done: the refill counts start from zero */
        SysQ q;
        q.d_last = 0;
        q.e1 = b.iend;
        sys_bar(); /* B0: tables ready */
        /* ================================================= producer: chunks */
        for (uint32_t k = 0; k <= nchunks; k++) {
            if (k < nchunks) {
                const uint32_t n0 = k * SYS_CHK;
                int32_t *row = S.rows[k & 1u] + lane;
#pragma unroll
                for (uint32_t hh = 0; hh < 2u; hh++) {
                    const uint32_t h0 = n0 + 16u * hh;
                    sys_refill(b, active && h0 < bs, q);
                    const uint32_t lo = max(h0, order), hi = active ? min(h0 + 16u, bs) : 0u;
                    if (ablate & 8u) {
                        for (uint32_t n = lo; n < hi; n++) row[(n - n0) * SYS_RP] = 0;
                    } else {
                        for (uint32_t n = lo; n < hi; n++) row[(n - n0) * SYS_RP] = rice_fused(b, rs, limit, trunc, nullptr);
                    }
                }
            }
            sys_bar();
        }
        /* ================================================= producer: tail (read_frame_ @0x100118c0) */
        const bool last = active && ch + 1u == fi.channels;
        if (active) {
            finish_partitions(b, rs);
            if (br_pos(b) > limit || trunc) S.f_bad[fl] = 1u;
        }
        lds_sync();
        if (last && !S.f_bad[fl]) {
            bool tb = false;
            const uint32_t padbits = (uint32_t)((8u - (br_pos(b) & 7u)) & 7u); /* read_zero_padding_ @0x10012fe0 */
            const uint32_t z = br_read(b, padbits);
            if (br_pos(b) > limit || z != 0u) {
                tb = true;
            } else {
                const uint64_t end_byte = br_pos(b) >> 3;
                const uint32_t crc_read = br_read(b, 16);
                if (br_pos(b) > limit) {
                    tb = true;
                } else {
                    S.f_end[fl] = (uint32_t)(end_byte - fi.frame_off);
                    S.f_crc[fl] = crc_read;
                    S.f_resume[fl] = br_pos(b);
                    S.f_state[fl] = FS_TAIL;
                }
            }
            if (tb) S.f_bad[fl] = 1u;
        }
        wait_vm(); /* no ring DMA may land after the producer is done with the ring */
        /* the CRC-16 tables into rows[0] (free: the last chunk has been packed) */
        lds_u16 *T = (lds_u16 *)(lds_u32 *)S.rows[0], *TK = T + 8 * 256;
        for (uint32_t i = lane; i < 8u * 256u; i += 64u) T[i] = (&g_crc16_tab[0][0])[i];
        crc_tk_fill(TK, lane);
        sys_bar(); /* tail done */
        return;
    }

    /* ===================================================== restore waves */
    const uint32_t w = wave - 1u;
    sys_bar(); /* B0 */
    const uint32_t nchunks = S.nchunks;
    {
        const uint32_t pl = 16u * w + (lane >> 2);
        const uint32_t fl = S.p_flags[pl];
        const bool act = (fl & SF_ACTIVE) != 0u;
        uint32_t ord = act ? S.p_order[pl] : 0u;
        for (int o = 32; o > 0; o >>= 1) ord = max(ord, (uint32_t)__shfl_xor(ord, o));
        const bool any_w = any_lane(act && (fl & SF_WIDE)), any_n = any_lane(act && !(fl & SF_WIDE));
        const int pm = (ablate & 0x40000u) ? PM_MIXED : any_w ? (any_n ? PM_MIXED : PM_WIDE) : PM_NARROW;
        if (ord <= 4u) sys_restore_pm<1>(S, w, lane, lg, nchunks, fmt, sp, out, pm);
        else if (ord <= 8u) sys_restore_pm<2>(S, w, lane, lg, nchunks, fmt, sp, out, pm);
        else if (ord <= 16u) sys_restore_pm<4>(S, w, lane, lg, nchunks, fmt, sp, out, pm);
        else sys_restore_pm<8>(S, w, lane, lg, nchunks, fmt, sp, out, pm);
    }
    sys_bar(); /* tail done: frame table complete, CRC tables in rows[0] */
    /* ---- CRC-16 check, records, zero fill, hand-back (this wave's frames) */
    const lds_u16 *T = (const lds_u16 *)(const lds_u32 *)S.rows[0], *TK = T + 8 * 256;
    uint32_t lanec = 0;
    bool have_lanec = false;
    const uint32_t nfw = 16u >> lg, fl0 = (16u * w) >> lg;
    for (uint32_t i = 0; i < nfw; i++) {
        const uint32_t fl = fl0 + i;
        const uint32_t state = S.f_state[fl];
        if (state == FS_NONE) continue; /* wave-uniform */
        const uint32_t f = S.f_idx[fl];
        if (S.f_bad[fl] || state != FS_TAIL) { /* hand back to the exact lane kernel */
            if (lane == 0) {
                info[f].flags = info[f].flags | BNF_FL_WAVE_REDO;
                const uint32_t at = atomicAdd(&redo[0], 1u);
                redo[4u + at] = f;
            }
            continue;
        }
        const uint64_t f_off = S.f_off[fl], end_byte = f_off + S.f_end[fl];
        const uint32_t crc_read = S.f_crc[fl];
        bool pre = false;
        {
            const uint32_t cn = info[f].crc_next;
            pre = (cn & BNF_CN_VALID) && (cn & BNF_CN_ZERO) && f_off + (cn & BNF_CN_LEN) == end_byte + 2u;
        }
        uint32_t acc = 0;
        if (!pre && !(ablate & 1u)) {
            if (!have_lanec) {
                lanec = crc16_shift(1u, 16u * (63u - lane));
                have_lanec = true;
            }
            acc = wave_crc_range((const uint8_t *)words, f_off, end_byte + 2u, T, TK, lanec, lane);
        }
        const bool crc_ok = acc == 0u;
        uint32_t calc = crc_read;
        if (!crc_ok && lane == 0) calc = crc16_range((const uint8_t *)words, f_off, end_byte, T);
        if (lane == 0) {
            info[f].resume_bit = S.f_resume[fl];
            info[f].crc16_read = crc_read;
            info[f].crc16_calc = calc;
            info[f].crc_ok = crc_ok ? 1u : 0u;
        }
        if (!crc_ok) { /* libFLAC zero-fills a CRC-failed frame (@0x10011af5) */
            const uint32_t C = S.f_ch[fl], bsz = S.f_bs[fl];
            const uint64_t os = S.f_os[fl];
            uint64_t start, nb;
            switch (fmt) {
            case BNF_OUT_PLANAR32: start = os * sp.channels * 4u; nb = (uint64_t)C * bsz * 4u; break;
            case BNF_OUT_INTERLEAVED32: start = os * sp.channels * 4u; nb = (uint64_t)sp.channels * bsz * 4u; break;
            case BNF_OUT_FLACDECODER: start = os * (C == 2 ? 4u : 2u); nb = (uint64_t)bsz * (C == 2 ? 4u : 2u); break;
            default: {
                const uint32_t fb = sp.bps == 24 ? 3u : 2u;
                start = os * sp.channels * fb;
                nb = (uint64_t)bsz * sp.channels * fb;
            }
            }
            for (uint64_t x = lane; x < nb; x += 64u) out[start + x] = 0;
        }
    }
}

/* ------------------------------------------------------------------ host launcher */
extern "C" {
hipError_t bnf_upload_tables_tu8(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    return upload_tables(crc8, crc16x8, xpow);
}
void bnf_set_ablate_tu8(uint32_t v) { g_ablate = v; }
/* redo: [0] hand-back count (zeroed by the caller), [4..] the frames handed back */
hipError_t bnf_launch_decode_sys_tu8(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                     uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                     const uint32_t *perm, uint32_t *redo, uint32_t mode, hipStream_t s) {
    const uint32_t fpb = 64u / chn_lanes;
    const uint32_t nb = (nframes + fpb - 1u) / fpb;
    hipLaunchKernelGGL(k_decode_sys, dim3(nb), dim3(SYS_THREADS), 0, s, words, nbytes, nframes, sp, chn_lanes, fmt, out,
                       out_bytes, info, perm, redo, ablate_flags() | mode);
    return hipGetLastError();
}
} /* extern "C" */
