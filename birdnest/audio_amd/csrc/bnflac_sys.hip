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
#define SYS_RD 16                    /* producer ring: 16-byte blocks per lane (256 B ahead of the cursor) */
#define SYS_HALF 16                  /* producer step: residuals per refill and per fast run */
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
/* debug phase timers (ablate 0x100, bench.py --stats): s_memtime, wave-uniform points only.
 * Compiled in only with -DBNFLAC_PHASE_TIMERS (a variant build, tools/sys_stats.sh): a scalar-
 * memory op anywhere in the producer loop makes hipcc's LDS waits lgkmcnt(0) (the ring lookahead
 * reads then wait at every step instead of 1.5 steps later). */
DEV uint64_t sys_now(bool on) { return tnow(on); }

/* Producer refill, pipelined RQ deep: at refill r the DMAs of refills r - 1 .. r - RQ may stay
 * in flight (vmcnt retires in issue order and the producer issues no other vector-memory ops),
 * everything issued before them has landed.  Then the blocks up to SYS_RD past the cursor's
 * block, one exec-masked DMA per ring slot (each slot's LDS base is wave-uniform; lane l's block
 * j lands in slot j mod SYS_RD).  d[i]: DMA instructions of refill r - 1 - i (wave-uniform),
 * e[i]: the lane's iend after refill r - 1 - i (shift registers: compile-time indices).
 * Called every SYS_HALF residuals with RQ = 3, or once per chunk with RQ = 1 (ablate 0x1000000:
 * half the DMA instructions per residual, one chunk of latency cover). */
#define SYS_RQMAX 3
struct SysQ {
    uint32_t d[SYS_RQMAX];
    uint32_t e[SYS_RQMAX + 1];
    uint64_t tw, dw; /* stats mode: wait cycles, DMA instructions waited past (flushed once per wave) */
};
__device__ unsigned long long g_sys_dbg[4]; /* debug: refill wait cycles, DMA instructions (stats mode) */
template <int RQ>
DEV void sys_refill(BR &b, bool want, SysQ &q, bool tm = false) {
    static_assert(RQ >= 1 && RQ <= SYS_RQMAX, "refill depth");
    const uint64_t tw = tnow(tm);
    uint32_t fly = 0;
#pragma unroll
    for (int i = 0; i < RQ; i++) fly += q.d[i];
    wait_vm_n(fly);
#ifdef BNFLAC_PHASE_TIMERS
    if (tm) { /* no global atomics here: their vmcnt wait would drain the DMAs in flight */
        q.tw += tnow(tm) - tw;
        q.dw += fly;
    }
#else
    (void)tw;
#endif
    b.vendw = max(b.vendw, q.e[RQ] * 4u); /* issued by refill r - 1 - RQ or earlier: landed */
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
#pragma unroll
    for (int i = SYS_RQMAX - 1; i > 0; i--) q.d[i] = q.d[i - 1];
    q.d[0] = d;
#pragma unroll
    for (int i = SYS_RQMAX; i > 0; i--) q.e[i] = q.e[i - 1];
    q.e[0] = b.iend;
}

/* ------------------------------------------------------------------ producer fast path */
/* Ring byte address of word wi (bits 2-3 word in block, 4-9 lane, 10 and up slot), moved on one
 * word by ((ra | 0x3F3) + c) & SYS_RAM | lane bits (k_decode_st's incremental form): the ones in
 * bits 0-1 turn +c into +4, the ones in bits 4-9 carry a block wrap into the slot */
static_assert((SYS_RD & (SYS_RD - 1)) == 0 && SYS_RD <= 32, "ring slots: a power of two");
#define SYS_RAM (0xCu | ((SYS_RD - 1u) << 10))
DEV uint32_t sys_ra(uint32_t wi, uint32_t lane) { return ((wi & 3u) << 2) | (lane << 4) | (((wi >> 2) & (SYS_RD - 1u)) << 10); }
DEV void sys_adv(BR &b, uint32_t n, uint32_t laneb) { /* n <= 32, no landing check */
    uint32_t t;
    const bool c = __builtin_usub_overflow(b.s, n, &t);
    b.s = t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += (uint32_t)c;
    b.ra = (((b.ra | 0x3F3u) + (uint32_t)c) & SYS_RAM) | laneb;
}
DEV void sys_next_word(BR &b) { b.nx = *(const lds_u32 *)((const __attribute__((address_space(3))) uint8_t *)b.ring + b.ra); }
DEV void sys_resync(BR &b, uint32_t lane) { b.ra = sys_ra(b.wi, lane); b.vlim = b.vendw - 1u; }
DEV int32_t sys_zz(uint32_t u) { return (int32_t)((u >> 1) ^ (0u - (u & 1u))); }
/* SYS_HALF Rice codewords of one partition (parameter k; km = 31 - k, k1 = k + 1, k32 = 32 - k) as
 * one straight line.  PAIR: two codewords per 32-bit window (small k: C2's ~10-bit codewords) with
 * one advance.  A step moves the window by at most one word, so the word entering it at step
 * T + 2 is the one after the window's at step T + 1 or the one after that: the ring read of the
 * latter is issued at the end of step T and selected at step T + 2 (nw = c ? z : nw), a step and
 * a half after its issue -- the LDS latency is off the cursor chain.  No branch inside, so the
 * compiler counts the reads in flight (lgkmcnt(1..3)) instead of draining them at every merge.
 * The caller has made sure every word the run can reach has landed (wi + 2 + SYS_HALF words);
 * each residual goes to the lane's row as it is decoded, and a lane whose codeword (pair) does
 * not fit the window freezes its cursor there.  Returns the codewords decoded (SYS_HALF unless
 * frozen); the caller finishes a frozen lane's run with the generic reader. */
template <bool PAIR>
DEV uint32_t sys_rice_line(BR &b, bool on, uint32_t k, uint32_t km, uint32_t k1, uint32_t k32, int32_t *row,
                           uint32_t lane) {
    const uint32_t laneb = lane << 4;
    sys_resync(b, lane);
    uint32_t nw = b.nx, cprev = 0, z2 = 0, z1, cnt = 0;
    bool frozen = !on;
    {
        const uint32_t ra1 = (((b.ra | 0x3F3u) + 1u) & SYS_RAM) | laneb;
        z1 = *(const lds_u32 *)((const __attribute__((address_space(3))) uint8_t *)b.ring + ra1);
    }
#pragma unroll
    for (int T = 0; T < SYS_HALF; T += PAIR ? 2 : 1) {
        nw = cprev ? z2 : nw;
        const uint32_t w = br_peek(b);
        uint32_t u0, u1 = 0, n;
        bool sl;
        if (PAIR) {
            const uint32_t qa = min(ffbh(w), 32u);
            const uint32_t la = qa + k1;
            const uint32_t w2 = w << (la & 31u);
            const uint32_t qb = min(ffbh(w2), 32u);
            u0 = (qa << k) | __builtin_amdgcn_ubfe(w, km - qa, k);
            u1 = (qb << k) | __builtin_amdgcn_ubfe(w2, km - qb, k);
            n = la + qb + k1;
            sl = n > 32u;
        } else {
            const uint32_t q = ffbh(w); /* ~0u for an empty window: slow */
            u0 = (q << k) | __builtin_amdgcn_ubfe(w, km - q, k);
            n = q + k1;
            sl = q >= k32;
        }
        frozen = frozen || sl;
        uint32_t t;
        const bool c = __builtin_usub_overflow(b.s, frozen ? 0u : n, &t);
        b.s = t & 31u;
        b.hi = c ? b.lo : b.hi;
        b.lo = c ? __builtin_bswap32(nw) : b.lo;
        b.wi += (uint32_t)c;
        b.ra = (((b.ra | 0x3F3u) + (uint32_t)c) & SYS_RAM) | laneb;
        const uint32_t ra1 = (((b.ra | 0x3F3u) + 1u) & SYS_RAM) | laneb;
        const uint32_t zn = *(const lds_u32 *)((const __attribute__((address_space(3))) uint8_t *)b.ring + ra1);
        z2 = z1;
        z1 = zn;
        cprev = c;
        row[T * SYS_RP] = sys_zz(u0); /* a frozen lane's are rewritten by the caller */
        if (PAIR) row[(T + 1) * SYS_RP] = sys_zz(u1);
        cnt += frozen ? 0u : (PAIR ? 2u : 1u);
    }
    b.nx = cprev ? z2 : nw; /* the generic reader's ring[wi] */
    return cnt;
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
/* acc[(a + R) % A] += c[(a + R) % A] * bc for a < A, exactly (v_mad_i64_i32), as ONE asm
 * statement (the compiler puts a wait state after every inline asm statement it cannot see
 * into), in the order a = 0, 1, ...: slot R -- the one the next step finalises -- first */
template <int A, int R> DEV void sys_macs(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc);
template <int R> struct SysMacs1 {
    static DEV void run(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc) {
        uint64_t co;
        asm("v_mad_i64_i32 %0, %1, %3, %2, %0"
            : "+v"(acc[(0 + R) % 1]), "=&s"(co)
            : "v"(bc), "v"(c[(0 + R) % 1]));
    }
};
template <int R> struct SysMacs2 {
    static DEV void run(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc) {
        uint64_t co;
        asm("v_mad_i64_i32 %0, %2, %4, %3, %0\n\t"
        "v_mad_i64_i32 %1, %2, %5, %3, %1"
            : "+v"(acc[(0 + R) % 2]), "+v"(acc[(1 + R) % 2]), "=&s"(co)
            : "v"(bc), "v"(c[(0 + R) % 2]), "v"(c[(1 + R) % 2]));
    }
};
template <int R> struct SysMacs4 {
    static DEV void run(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc) {
        uint64_t co;
        asm("v_mad_i64_i32 %0, %4, %6, %5, %0\n\t"
        "v_mad_i64_i32 %1, %4, %7, %5, %1\n\t"
        "v_mad_i64_i32 %2, %4, %8, %5, %2\n\t"
        "v_mad_i64_i32 %3, %4, %9, %5, %3"
            : "+v"(acc[(0 + R) % 4]), "+v"(acc[(1 + R) % 4]), "+v"(acc[(2 + R) % 4]), "+v"(acc[(3 + R) % 4]), "=&s"(co)
            : "v"(bc), "v"(c[(0 + R) % 4]), "v"(c[(1 + R) % 4]), "v"(c[(2 + R) % 4]), "v"(c[(3 + R) % 4]));
    }
};
template <int R> struct SysMacs8 {
    static DEV void run(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc) {
        uint64_t co;
        asm("v_mad_i64_i32 %0, %8, %10, %9, %0\n\t"
        "v_mad_i64_i32 %1, %8, %11, %9, %1\n\t"
        "v_mad_i64_i32 %2, %8, %12, %9, %2\n\t"
        "v_mad_i64_i32 %3, %8, %13, %9, %3\n\t"
        "v_mad_i64_i32 %4, %8, %14, %9, %4\n\t"
        "v_mad_i64_i32 %5, %8, %15, %9, %5\n\t"
        "v_mad_i64_i32 %6, %8, %16, %9, %6\n\t"
        "v_mad_i64_i32 %7, %8, %17, %9, %7"
            : "+v"(acc[(0 + R) % 8]), "+v"(acc[(1 + R) % 8]), "+v"(acc[(2 + R) % 8]), "+v"(acc[(3 + R) % 8]), "+v"(acc[(4 + R) % 8]), "+v"(acc[(5 + R) % 8]), "+v"(acc[(6 + R) % 8]), "+v"(acc[(7 + R) % 8]), "=&s"(co)
            : "v"(bc), "v"(c[(0 + R) % 8]), "v"(c[(1 + R) % 8]), "v"(c[(2 + R) % 8]), "v"(c[(3 + R) % 8]), "v"(c[(4 + R) % 8]), "v"(c[(5 + R) % 8]), "v"(c[(6 + R) % 8]), "v"(c[(7 + R) % 8]));
    }
};
template <int A, int R> DEV void sys_macs(int64_t (&acc)[8], const int32_t (&c)[8], int32_t bc) {
    if constexpr (A == 1) SysMacs1<R>::run(acc, c, bc);
    else if constexpr (A == 2) SysMacs2<R>::run(acc, c, bc);
    else if constexpr (A == 4) SysMacs4<R>::run(acc, c, bc);
    else SysMacs8<R>::run(acc, c, bc);
}

/* lane j's broadcast of lane JJ of its quad (DPP quad_perm) */
template <int JJ> DEV int32_t quad_bcast(int32_t x) { return __builtin_amdgcn_mov_dpp(x, JJ * 0x55, 0xF, 0xF, false); }

/* 32 samples of a chunk.  v[q]: on entry the residual (or warm-up) of sample n0 + j + 4q, on exit
 * the sample.  FIRST: chunk 0, where samples below the order are raw warm-ups. */
template <int A, int PM, bool FIRST, int T>
DEV void sys_step(int64_t (&acc)[8], const int32_t (&rc)[32], int32_t (&v)[8], uint32_t j, uint32_t sh, bool wide,
                  uint32_t order) {
    constexpr int P = 4 * A, jj = T & 3, q = T >> 2, a = q % A, an = ((T + 1) >> 2) % A;
    /* finalise sample n0 + T: computed on every lane, kept by the lane that owns it (selects,
     * not an exec-masked branch: no SALU, no branch per step) */
    const bool own = j == (uint32_t)jj;
    const uint32_t lo = (uint32_t)acc[a], hi = (uint32_t)((uint64_t)acc[a] >> 32);
    int32_t pred;
    if (PM == PM_WIDE) pred = (int32_t)__builtin_amdgcn_alignbit(hi, lo, sh);
    else if (PM == PM_NARROW) pred = (int32_t)lo >> sh;
    else pred = (int32_t)__builtin_amdgcn_alignbit(wide ? hi : (uint32_t)((int32_t)lo >> 31), lo, sh);
    if (FIRST) {
        uint32_t ord = order;
        asm volatile("" : "+v"(ord)); /* compare per step: 32 hoisted lane masks spill */
        pred = (uint32_t)T < ord ? 0 : pred;
    }
    const int32_t nv = (int32_t)((uint32_t)v[q] + (uint32_t)pred);
    v[q] = own ? nv : v[q];
    acc[a] = own ? 0 : acc[a]; /* the slot now holds sample n0 + T + P */
    const int32_t bc = quad_bcast<jj>(v[q]);
    int32_t cs[8];
#pragma unroll
    for (int a2 = 0; a2 < 8; a2++) cs[a2] = a2 < A ? rc[((4 * a2 - T - 1) % P + P) % P] : 0;
    sys_macs<A, an>(acc, cs, bc);
}
template <int A, int PM, bool FIRST, int T>
DEV void sys_steps_from(int64_t (&acc)[8], const int32_t (&rc)[32], int32_t (&v)[8], uint32_t j, uint32_t sh, bool wide,
                        uint32_t order) {
    if constexpr (T < 32) {
        sys_step<A, PM, FIRST, T>(acc, rc, v, j, sh, wide, order);
        sys_steps_from<A, PM, FIRST, T + 1>(acc, rc, v, j, sh, wide, order);
    }
}
/* 32 samples of a chunk.  v[q]: on entry the residual (or warm-up) of sample n0 + j + 4q, on exit
 * the sample.  FIRST: chunk 0, where samples below the order are raw warm-ups. */
template <int A, int PM, bool FIRST>
DEV void sys_steps(int64_t (&acc)[8], const int32_t (&rc)[32], int32_t (&v)[8], uint32_t j, uint32_t sh, bool wide,
                   uint32_t order) {
    sys_steps_from<A, PM, FIRST, 0>(acc, rc, v, j, sh, wide, order);
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

/* Fast pack: every decoding frame of the wave has a power-of-two channel count and a 16-byte
 * aligned run; each lane writes whole 16-byte pieces of the wave's runs (one store instruction
 * covers the runs of several frames, coalesced).  Pieces per frame np: FLACDecoder stereo 8
 * (4 samples, L | R << 16), FLACDecoder other 4 (8 samples of channel 0, 16-bit), interleaved
 * int32 8C (4 values), FLACFileReader 2C fb (16 bytes of fb-byte values), planar int32 8C (4
 * samples of one channel).  The piece of each lane (at most two per lane: np <= 64 per frame,
 * 16 subframe slots per wave) and its frame's fields are set up once (sys_pack_prep); a chunk
 * then costs the value reads, the packing and one store per piece.  A chunk in which some frame
 * ends part-way takes the generic pack. */
DEV int32_t sys_val(const int32_t *row, uint32_t n, uint32_t s0, uint32_t c, uint32_t C, uint32_t as) {
    if (C == 2u) {
        const int2 x = *(const int2 *)(row + n * SYS_RP + s0);
        int32_t l = x.x, r = x.y;
        decorrelate(as, l, r);
        return c ? r : l;
    }
    return row[n * SYS_RP + s0 + c];
}
struct SysPk {
    bool ok;                 /* the wave qualifies (wave-uniform) */
    uint32_t C, lc, fb, cbytes;
    bool pv[2];              /* this lane's piece r exists and its frame decodes */
    uint32_t s0[2], as[2], p[2], bs[2];
    uint64_t at[2];          /* output byte of the piece in chunk 0 */
};
DEV void sys_pack_prep(SysPk &k, const SysShared &S, uint32_t w, uint32_t lane, uint32_t lg, int fmt,
                       const bnf_stream_params &sp) {
    const uint32_t cl = 1u << lg, nfw = 16u >> lg, fl0 = (16u * w) >> lg;
    k.fb = sp.bps == 24 ? 3u : 2u;
    uint32_t C = 0;
    bool ok = true;
    for (uint32_t i = 0; i < nfw; i++) {
        const uint32_t fl = fl0 + i;
        if (S.f_state[fl] != FS_DEC) continue;
        const uint32_t c = S.f_ch[fl], bs = S.f_bs[fl];
        const uint64_t os = S.f_os[fl];
        if (C == 0u) C = c;
        ok = ok && c == C && (c & (c - 1u)) == 0u;
        uint64_t base;
        switch (fmt) {
        case BNF_OUT_FLACDECODER: base = os * (c == 2u ? 4u : 2u); break;
        case BNF_OUT_INTERLEAVED32: ok = ok && c == sp.channels; base = os * sp.channels * 4u; break;
        case BNF_OUT_PLANAR32: ok = ok && (bs & 3u) == 0u; base = os * sp.channels * 4u; break;
        default: ok = ok && c == sp.channels; base = os * sp.channels * k.fb; break;
        }
        ok = ok && (base & 15u) == 0u;
    }
    k.ok = ok && C != 0u;
    k.pv[0] = k.pv[1] = false;
    if (!k.ok) return;
    k.C = C;
    k.lc = __builtin_ctz(C);
    uint32_t np, m3 = 0; /* np = pieces per frame; m3: np = 3 << e */
    switch (fmt) {
    case BNF_OUT_FLACDECODER: np = C == 2u ? 8u : 4u; k.cbytes = SYS_CHK * (C == 2u ? 4u : 2u); break;
    case BNF_OUT_INTERLEAVED32: np = 8u * C; k.cbytes = SYS_CHK * 4u * sp.channels; break;
    case BNF_OUT_PLANAR32: np = 8u * C; k.cbytes = SYS_CHK * 4u; break;
    default: np = 2u * C * k.fb; m3 = k.fb == 3u; k.cbytes = SYS_CHK * sp.channels * k.fb; break;
    }
    const uint32_t e = m3 ? __builtin_ctz(np / 3u) : __builtin_ctz(np);
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t P = lane + 64u * r;
        const uint32_t x = P >> e;
        const uint32_t i = m3 ? (__umulhi(x, 0xAAAAAAABu) >> 1) : x; /* P / np */
        const uint32_t pp = P - i * np;
        const uint32_t fl = fl0 + min(i, nfw - 1u);
        k.pv[r] = i < nfw && S.f_state[fl] == FS_DEC;
        k.s0[r] = fl * cl;
        k.as[r] = S.f_as[fl];
        k.bs[r] = S.f_bs[fl];
        k.p[r] = pp;
        const uint64_t os = S.f_os[fl];
        switch (fmt) {
        case BNF_OUT_FLACDECODER: k.at[r] = os * (C == 2u ? 4u : 2u) + 16u * pp; break;
        case BNF_OUT_INTERLEAVED32: k.at[r] = os * sp.channels * 4u + 16u * pp; break;
        case BNF_OUT_PLANAR32: k.at[r] = (os * sp.channels + (uint64_t)(pp >> 3) * k.bs[r]) * 4u + 16u * (pp & 7u); break;
        default: k.at[r] = os * sp.channels * k.fb + 16u * pp; break;
        }
    }
}
/* one chunk; false: the generic pack must run (a frame ends part-way through this chunk) */
DEV bool sys_pack_fast(const SysPk &k, const int32_t *row, uint32_t n0, int fmt, uint8_t *__restrict__ out) {
    if (!k.ok) return false;
    if (any_lane((k.pv[0] && n0 < k.bs[0] && n0 + SYS_CHK > k.bs[0]) || (k.pv[1] && n0 < k.bs[1] && n0 + SYS_CHK > k.bs[1])))
        return false;
    const uint32_t C = k.C, lc = k.lc;
    const uint64_t cofs = (uint64_t)(n0 / SYS_CHK) * k.cbytes;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        if (!any_lane(k.pv[r] && n0 < k.bs[r])) continue; /* piece 0's frame may be out while piece 1's decodes */
        if (!k.pv[r] || n0 >= k.bs[r]) continue;
        uint32_t s0 = k.s0[r], p = k.p[r];
        const uint32_t as = k.as[r];
        asm volatile("" : "+v"(s0), "+v"(p)); /* addresses per chunk: hoisted out of the chunk loop they take ~90 VGPRs */
        u32x4 v;
        switch (fmt) {
        case BNF_OUT_FLACDECODER:
            if (C == 2u) { /* FLACDecoder.cs:549-562: L | R << 16 */
                uint32_t d[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int2 xx = *(const int2 *)(row + (4u * p + q) * SYS_RP + s0);
                    int32_t l = xx.x, rr = xx.y;
                    decorrelate(as, l, rr);
                    d[q] = ((uint32_t)l & 0xffffu) | ((uint32_t)rr << 16);
                }
                v = u32x4{d[0], d[1], d[2], d[3]};
            } else { /* :564-577: channel 0 only, 16-bit */
                uint32_t d[4];
#pragma unroll
                for (int q = 0; q < 4; q++)
                    d[q] = ((uint32_t)row[(8u * p + 2u * q) * SYS_RP + s0] & 0xffffu) |
                           ((uint32_t)row[(8u * p + 2u * q + 1u) * SYS_RP + s0] << 16);
                v = u32x4{d[0], d[1], d[2], d[3]};
            }
            break;
        case BNF_OUT_INTERLEAVED32: {
            uint32_t d[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t vv = 4u * p + q;
                d[q] = (uint32_t)sys_val(row, vv >> lc, s0, vv & (C - 1u), C, as);
            }
            v = u32x4{d[0], d[1], d[2], d[3]};
            break;
        }
        case BNF_OUT_PLANAR32: {
            const uint32_t c = p >> 3, pp = p & 7u;
            uint32_t d[4];
#pragma unroll
            for (int q = 0; q < 4; q++) d[q] = (uint32_t)sys_val(row, 4u * pp + q, s0, c, C, as);
            v = u32x4{d[0], d[1], d[2], d[3]};
            break;
        }
        default: /* FLACFileReader.cs:220-237: fb bytes per value, little-endian, sample-major */
            if (k.fb == 3u) {
                const uint32_t b0 = 16u * p, vlo = __umulhi(b0, 0xAAAAAAABu) >> 1, off = b0 - 3u * vlo;
                int32_t xv[6];
#pragma unroll
                for (int q = 0; q < 6; q++) {
                    const uint32_t vv = min(vlo + q, SYS_CHK * C - 1u);
                    xv[q] = sys_val(row, vv >> lc, s0, vv & (C - 1u), C, as);
                }
                const uint32_t d0 = ((uint32_t)xv[0] & 0xFFFFFFu) | ((uint32_t)xv[1] << 24);
                const uint32_t d1 = (((uint32_t)xv[1] >> 8) & 0xFFFFu) | ((uint32_t)xv[2] << 16);
                const uint32_t d2 = (((uint32_t)xv[2] >> 16) & 0xFFu) | ((uint32_t)xv[3] << 8);
                const uint32_t d3 = ((uint32_t)xv[4] & 0xFFFFFFu) | ((uint32_t)xv[5] << 24);
                const uint32_t d4 = ((uint32_t)xv[5] >> 8) & 0xFFFFu;
                v = u32x4{__builtin_amdgcn_alignbyte(d1, d0, off), __builtin_amdgcn_alignbyte(d2, d1, off),
                          __builtin_amdgcn_alignbyte(d3, d2, off), __builtin_amdgcn_alignbyte(d4, d3, off)};
            } else {
                uint32_t d[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t v0 = 8u * p + 2u * q, v1 = v0 + 1u;
                    d[q] = ((uint32_t)sys_val(row, v0 >> lc, s0, v0 & (C - 1u), C, as) & 0xffffu) |
                           ((uint32_t)sys_val(row, v1 >> lc, s0, v1 & (C - 1u), C, as) << 16);
                }
                v = u32x4{d[0], d[1], d[2], d[3]};
            }
            break;
        }
        gst128((uint64_t)(uintptr_t)out + k.at[r] + cofs, v);
    }
    return true;
}

/* ------------------------------------------------------------------ restore waves */
template <int A, int PM>
DEV void sys_restore(SysShared &S, uint32_t w, uint32_t lane, uint32_t lg, uint32_t nchunks, int fmt,
                     const bnf_stream_params &sp, uint8_t *__restrict__ out, uint32_t ablate, const uint32_t *words,
                     uint32_t nblk) {
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
    SysPk pk;
    sys_pack_prep(pk, S, w, lane, lg, fmt, sp);
    const bool tm = (ablate & 0x100u) != 0;
    uint64_t t_st = 0, t_pk = 0, t_bw = 0;
    sys_bar(); /* end of iteration 0: the producer's chunk 0 is in rows[0]; rows[1] may be overwritten */
    for (uint32_t k = 1; k <= nchunks; k++) {
        const uint64_t t0 = sys_now(tm);
        const uint32_t n0 = (k - 1u) * SYS_CHK;
        int32_t *row = S.rows[(k - 1u) & 1u];
        int32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; q++) v[q] = row[(j + 4u * q) * SYS_RP + pl];
        if (ablate & 4u) { /* timing ablation: no restore */
        } else if (k == 1u) sys_steps<A, PM, true>(acc, rc, v, j, sh, wide, order);
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
        const uint64_t t1 = sys_now(tm);
        if (!(ablate & 2u)) {
            if ((ablate & 0x400000u) || !sys_pack_fast(pk, row, n0, fmt, out)) sys_pack(S, row, w, lane, lg, n0, fmt, sp, out);
        }
        const uint64_t t2 = sys_now(tm);
        sys_bar();
        const uint64_t t3 = sys_now(tm);
        t_st += t1 - t0;
        t_pk += t2 - t1;
        t_bw += t3 - t2;
    }
    if (tm && lane == 0) {
        atomicAdd(&g_stats[11], (unsigned long long)t_st);
        atomicAdd(&g_stats[12], (unsigned long long)t_pk);
        atomicAdd(&g_stats[13], (unsigned long long)t_bw);
    }
    if (range_bad) S.f_bad[pl >> lg] = 1u;
}

template <int A>
DEV void sys_restore_pm(SysShared &S, uint32_t w, uint32_t lane, uint32_t lg, uint32_t nchunks, int fmt,
                        const bnf_stream_params &sp, uint8_t *out, int pm, uint32_t ablate, const uint32_t *words,
                        uint32_t nblk) {
    if (pm == PM_WIDE) sys_restore<A, PM_WIDE>(S, w, lane, lg, nchunks, fmt, sp, out, ablate, words, nblk);
    else if (pm == PM_NARROW) sys_restore<A, PM_NARROW>(S, w, lane, lg, nchunks, fmt, sp, out, ablate, words, nblk);
    else sys_restore<A, PM_MIXED>(S, w, lane, lg, nchunks, fmt, sp, out, ablate, words, nblk);
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
        /* the record's fields one by one (a whole-record copy goes to scratch or, promoted, to LDS) */
        struct { uint32_t status, flags, bps, channels, blocksize, assignment; uint64_t out_sample, frame_off; } fi;
        fi.status = have ? info[f].status : (uint32_t)BNF_ST_SKIPPED;
        fi.flags = fi.bps = fi.channels = fi.blocksize = fi.assignment = 0;
        fi.out_sample = fi.frame_off = 0;
        if (have) {
            fi.flags = info[f].flags;
            fi.bps = info[f].bps;
            fi.channels = info[f].channels;
            fi.blocksize = info[f].blocksize;
            fi.assignment = info[f].assignment;
            fi.out_sample = info[f].out_sample;
            fi.frame_off = info[f].frame_off;
        }
        const bool frame_ok = have && fi.status == BNF_ST_OK;
        if (ch == 0) { S.f_state[fl] = FS_NONE; S.f_bad[fl] = 0; }
        bool ok = false;
        if (frame_ok && ch == 0) { /* decode_block's checks, with its records (SKIPPED: status and flags) */
            ok = true;
            uint32_t unsupported = 0;
            if (fmt == BNF_OUT_FLACDECODER && fi.bps != 16) unsupported = 1;          /* WriteCallback abort :526-530 */
            if (fmt >= BNF_OUT_FLACDECODER && fi.channels > sp.channels) unsupported = 1;
            if (fmt == BNF_OUT_FILEREADER && sp.bps != 16 && sp.bps != 24) unsupported = 1; /* NotSupportedException :239-240 */
            /* decode_block's outcome bits, each tested on its own (bit 2: the layout cannot
             * carry the frame, bit 1: it ends past out_bytes; both may be set) */
            uint64_t stride;
            switch (fmt) {
            case BNF_OUT_PLANAR32: case BNF_OUT_INTERLEAVED32: stride = 4ull * sp.channels; break;
            case BNF_OUT_FLACDECODER: stride = fi.channels == 2 ? 4u : 2u; break;
            default: stride = (uint64_t)sp.channels * (sp.bps == 24 ? 3u : 2u); break;
            }
            const bool past = (fi.out_sample + fi.blocksize) * stride > out_bytes;
            if (unsupported || past) {
                ok = false;
                info[f].status = BNF_ST_SKIPPED;
                info[f].flags = fi.flags | (unsupported ? 4u : 0u) | (past ? 2u : 0u);
            } else {
                if (fi.channels > chn_lanes) {
                    ok = false;
                    info[f].status = BNF_ST_SKIPPED;
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
        b.stats = (ablate & 0x100u) != 0; /* debug event counters (bench.py --stats) */
        STAT(b.stats, 5);
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
            /* subframe bps: +1 for the side channel (read_frame_ @0x100118c0, sub_bps) */
            const uint32_t sbps = fi.bps + (((fi.assignment == 1u || fi.assignment == 3u) && ch == 1u) || (fi.assignment == 2u && ch == 0u) ? 1u : 0u);
            st = parse_subframe_head<true, 32, SYS_RP>(b, sbps, bs, limit, h, row0, coef, err);
            if (st != BNF_ST_OK) {
                bad = true;
            } else {
                /* the coefficient table straight from the parse (a second 32-entry register copy
                 * made this setup the kernel's VGPR peak) */
#pragma unroll
                for (int t = 0; t < 32; t++) cf[t] = (h.type == T_LPC && (uint32_t)t < h.order) ? coef[t] : 0;
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
                    cf[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
                    cf[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
                    cf[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
                    cf[3] = o == 4 ? -1 : 0;
                } else if (h.type == T_CONST) { /* order 1, coefficient 1, warm-up cval, zero residuals */
                    cf[0] = 1;
                    order = 1;
                    row0[0] = h.cval;
                }
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
#pragma unroll
        for (int i = 0; i < SYS_RQMAX; i++) q.d[i] = 0;
#pragma unroll
        for (int i = 0; i <= SYS_RQMAX; i++) q.e[i] = b.iend;
        q.tw = q.dw = 0;
        const bool rf_chunk = !(ablate & 0x1000000u); /* refill once per chunk, 2 deep (ablate: every half, 4 deep) */
        sys_bar(); /* B0: tables ready */
        /* ================================================= producer: chunks */
        const bool tm = b.stats;
        uint64_t t_ref = 0, t_dec = 0, t_bar = 0;
        /* the wave's largest Rice parameter (selects the PAIR run), reduced again only after a
         * partition header: an upper bound for the lanes of a run, which only costs the pairing */
        uint32_t kmax = 0;
        bool kdirty = true;
        for (uint32_t k = 0; k <= nchunks; k++) {
            if (k < nchunks) {
                const uint32_t n0 = k * SYS_CHK;
                int32_t *row = S.rows[k & 1u] + lane;
#pragma unroll
                for (uint32_t hh = 0; hh < SYS_CHK / SYS_HALF; hh++) {
                    const uint32_t h0 = n0 + SYS_HALF * hh;
                    STAT(b.stats && active && h0 < bs, 4);
                    const uint64_t t0 = sys_now(tm);
                    if (ablate & 0x80000u) { /* ablation: landings only */
                    } else if (rf_chunk) {
                        if (hh == 0) sys_refill<1>(b, active && h0 < bs, q, tm);
                    } else {
                        sys_refill<3>(b, active && h0 < bs, q, tm);
                    }
                    const uint64_t t1 = sys_now(tm);
                    /* a run of SYS_HALF codewords of one Rice partition on every lane still decoding
                     * (partitions of 16 or more samples start on a run: their sizes are powers of
                     * two, partition 0 ends at one); else residual by residual */
                    const bool run = active && h0 + SYS_HALF <= bs && h0 >= order;
                    if (any_lane(run && rs.left == 0u && rs.pidx < rs.nparts)) {
                        if (run && rs.left == 0u && rs.pidx < rs.nparts) read_partition(b, rs);
                        kdirty = true;
                    }
                    const bool fast = !(ablate & 0x200000u) && !any_lane(active && h0 < bs && !(run && !rs.esc && rs.left >= SYS_HALF));
                    if (fast && any_lane(run) && kdirty) {
                        kmax = active ? rs.k : 0u;
                        for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor(kmax, o));
                        kdirty = false;
                    }
                    if (fast && any_lane(run)) {
                        const uint32_t kk = run ? rs.k : 0u;
                        /* every word the run can reach has landed */
                        if (__builtin_expect(any_lane(run && b.wi + 2u + SYS_HALF >= b.vendw), 0)) {
                            br_land(b, 2u + SYS_HALF);
                            b.nx = ring_word(b, b.wi);
                        }
                        int32_t *rrow = row + (h0 - n0) * SYS_RP;
                        const uint32_t got = kmax <= 9u ? sys_rice_line<true>(b, run, kk, 31u - kk, kk + 1u, 32u - kk, rrow, lane)
                                                        : sys_rice_line<false>(b, run, kk, 31u - kk, kk + 1u, 32u - kk, rrow, lane);
                        if (__builtin_expect(any_lane(run && got < SYS_HALF), 0)) { /* frozen lanes: the generic reader */
                            STAT(b.stats, 3);
                            if (run)
                                for (uint32_t i = got; i < SYS_HALF; i++) rrow[i * SYS_RP] = rice_one<true>(b, kk, limit, trunc);
                        }
                        if (run) rs.left -= SYS_HALF;
                    } else {
                        kdirty = true; /* rice_fused may read partition headers */
                        const uint32_t lo = max(h0, order), hi = active ? min(h0 + SYS_HALF, bs) : 0u;
                        if (ablate & 8u) {
                            for (uint32_t n = lo; n < hi; n++) row[(n - n0) * SYS_RP] = 0;
                        } else {
                            for (uint32_t n = lo; n < hi; n++) row[(n - n0) * SYS_RP] = rice_fused(b, rs, limit, trunc, nullptr);
                        }
                    }
                    const uint64_t t2 = sys_now(tm);
                    t_ref += t1 - t0;
                    t_dec += t2 - t1;
                }
            }
            const uint64_t t3 = sys_now(tm);
            sys_bar();
            t_bar += sys_now(tm) - t3;
        }
        if (tm && lane == 0) {
            atomicAdd(&g_stats[8], (unsigned long long)t_ref);
            atomicAdd(&g_stats[9], (unsigned long long)t_dec);
            atomicAdd(&g_stats[10], (unsigned long long)t_bar);
            atomicAdd(&g_sys_dbg[0], (unsigned long long)q.tw);
            atomicAdd(&g_sys_dbg[1], (unsigned long long)q.dw);
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
    const uint32_t nblk = (uint32_t)((nbytes + 15u) >> 4);
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
        if (ord <= 4u) sys_restore_pm<1>(S, w, lane, lg, nchunks, fmt, sp, out, pm, ablate, words, nblk);
        else if (ord <= 8u) sys_restore_pm<2>(S, w, lane, lg, nchunks, fmt, sp, out, pm, ablate, words, nblk);
        else if (ord <= 16u) sys_restore_pm<4>(S, w, lane, lg, nchunks, fmt, sp, out, pm, ablate, words, nblk);
        else sys_restore_pm<8>(S, w, lane, lg, nchunks, fmt, sp, out, pm, ablate, words, nblk);
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
        uint32_t acc = 0;
        if (!(ablate & 1u)) {
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
void bnf_set_ablate_tu8(uint32_t v) { g_ablate.store(v, std::memory_order_relaxed); }
hipError_t bnf_stats_tu8(uint64_t *out16, int reset) {
    uint64_t v[16];
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stats), sizeof v);
    if (e == hipSuccess) { /* slots 14, 15: refill wait cycles, DMA instructions waited past */
        uint64_t d[4];
        e = hipMemcpyFromSymbol(d, HIP_SYMBOL(g_sys_dbg), sizeof d);
        v[14] += d[0];
        v[15] += d[1];
        if (e == hipSuccess && reset) {
            static const uint64_t z4[4] = {0};
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_sys_dbg), z4, sizeof z4);
        }
    }
    if (e != hipSuccess) return e;
    for (int i = 0; i < 16; i++) out16[i] += v[i];
    if (reset) {
        static const uint64_t z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z);
    }
    return e;
}
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
