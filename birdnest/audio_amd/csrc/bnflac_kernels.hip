/*
 * bnflac_kernels.hip -- MI355X (gfx950) FLAC frame decode.
 *
 * Replaces the arithmetic of libFLAC 1.2.1's read_frame_ (LibFlac.dll@0x100118c0) and
 * everything under it, plus the PCM packing of
 * BirdNest.Audio's write callbacks (A15/A17), with these kernels:
 *
 *   k_sync_scan  -- candidate frame syncs: byte p with b[p]==0xFF, b[p+1]>>2==0x3e
 *                   (frame_sync_ @0x10011760's test), ordered compaction.
 *   k_parse      -- one lane per candidate: frame header (read_frame_header_
 *                   @0x10011d70, CRC-8), then walks subframes 0..C-2 to find where
 *                   each subframe starts (the Rice bit cursor is serial per frame).
 *   k_decode<W>  -- one lane per (frame, channel) subframe, 64-lane workgroups:
 *                   partitioned-Rice residuals (A9) fused with the FIXED/LPC restore
 *                   (libFLAC's exact 16-bit-MMX / ia32 / 64-bit dispatch, A7, A8) and
 *                   wasted bits (A5); then the workgroup decorrelates (A12) and writes
 *                   the requested PCM layout with coalesced stores; the channel lanes
 *                   of a frame check zero padding and the frame CRC-16 (A4, A11).
 *                   W = 8 serves frames whose LPC orders are all <= 8 (register ring
 *                   of 8, low VGPR count); W = 32 the rest.
 *
 * Bit reader.  Every lane owns an 8-slot ring of 16-byte blocks of its own bitstream in
 * LDS, filled by exec-masked LDS-DMA (global_load_lds_dwordx4) once per 32-sample
 * chunk; a chunk decodes from blocks that landed during the previous chunk, so HBM
 * latency is hidden behind a whole chunk of work and the per-codeword cursor advance
 * is branch-free (one ds_read_b32).  Words outside the landed range are read from
 * global memory directly (rare: jumps, very high bit rates).
 *
 * Integer-only, HBM/issue bound; no MFMA.  Bit-exactness is defined
 * by oracle/flac_oracle.c, which restates the same DLL behaviour on the CPU.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <atomic>
#include <mutex>
#include <type_traits>

#include "bnflac_device.h"

#define DEV __device__ __forceinline__

/* ------------------------------------------- CRC tables (CRC-8; slice-by-8 CRC-16 for k_decode<W>, k_decode_sys) */
/* Tables are filled by the host at module load (bnflac_runtime.cpp) into these: */
__constant__ uint8_t g_crc8_tab[256];
__constant__ uint16_t g_crc16_tab[8][256]; /* slice-by-8 */
__constant__ uint16_t g_crc16_xpow[40];    /* x^(8*2^j) mod P for j < 40 */
/* Debug event counters (wave-level events, enabled by ablate bit 0x100; timing runs
 * leave them off).  0 fused chunks, 1 generic chunks, 2 DMA landing waits, 3 slow Rice
 * codewords, 4 refills, 5 waves. */
__device__ unsigned long long g_stats[16]; /* 8.. : s_memtime cycles per phase, summed over waves */
/* Phase timers (s_memtime) for the debug counters; compiled in only with
 * -DBNFLAC_PHASE_TIMERS, because a scalar-memory op anywhere in the loop makes hipcc's
 * LDS waits conservative (lgkmcnt(0)). */
DEV uint64_t tnow(bool on) { /* call at wave-uniform points only */
#ifndef BNFLAC_PHASE_TIMERS
    (void)on;
    return 0ull;
#endif
    if (!on) return 0ull;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return t;
}
#define STAT(on, i) do { if (on) { if (__builtin_amdgcn_read_exec() && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) atomicAdd(&g_stats[i], 1ull); } } while (0)

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
/* LDS accesses to buffers that are never LDS-DMA targets, as inline asm: hipcc cannot tell
 * them from the DMA'd ring and would drain every vector-memory op (vmcnt(0)) first.
 * Completion is waited for explicitly (lds_sync / lgkmcnt). */
DEV void lds_st128(const void *a, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"((uint32_t)(uintptr_t)a), "v"(v) : "memory");
}
DEV u32x4 lds_ld128(const void *a) { /* result valid after s_waitcnt lgkmcnt(0) */
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)a) : "memory");
    return v;
}
DEV void lds_st128(const lds_u32x4 *a, u32x4 v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"((uint32_t)(uintptr_t)a), "v"(v) : "memory");
}
DEV u32x4 lds_ld128(const lds_u32x4 *a) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)a) : "memory");
    return v;
}
DEV void lds_st64(const void *a, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"((uint32_t)(uintptr_t)a), "v"(v) : "memory");
}
DEV uint64_t lds_ld64(const void *a) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)a) : "memory");
    return v;
}
typedef __attribute__((address_space(1))) const void gvoid;
/* 16-byte global store through an integer address: the address-space cast keeps it a
 * global_store (a generic pointer would make it a flat store, which also counts in
 * lgkmcnt -- every later LDS wait would then wait for the HBM write) */
DEV void gst128(uint64_t addr, u32x4 v) { *(__attribute__((address_space(1))) u32x4 *)addr = v; }

/* Mode bits carried in the kernels' `ablate` word (set by the launchers, never a timing
 * ablation).  Mode bit: the lane kernel decodes only the frames k_decode_sys handed back (BNF_FL_WAVE_REDO). */
#define BNF_MODE_WREDO 0x4000u
/* Mode bit: k_decode_sw ran before the other lane kernels (they take its SW frames only when
 * it handed them back).  Host ablation bit BNF_ABLATE_NO_SW: do not launch it. */
#define BNF_MODE_SW 0x8000u
#define BNF_ABLATE_NO_SW 0x10000u
/* Mode bit: k_decode_list -- the frames of a device list (k_decode_sys's hand-backs), every
 * class, decoded by this instance (no class split, stereo fast-path frames included). */
#define BNF_MODE_LIST 0x20000u
/* Mode bit: k_decode_seg -- the W = 32 instance also takes the W16 class's blocks. */
#define BNF_MODE_SEG 0x80000000u
/* Mode bits of the W = 8 instance when its two jobs run as two launches (bnf_launch_decode):
 * NOST -- the narrow non-stereo frames only (the decode order's class 1; beside k_decode_st,
 * so it never reads a stereo frame's hand-back bit); STREDO -- only the stereo frames
 * k_decode_st handed back (class 0; after it). */
#define BNF_MODE_NOST 0x40000u
#define BNF_MODE_STREDO 0x80000u
#define BNF_ABLATE_NO_W8SPLIT 0x100000u /* host A/B bit: the W = 8 instance as one launch */

/* ----------------------------------------------------------------- bit reader */
#define RING_MAX 16       /* 16-byte slots per lane (k_parse and k_decode_st use 8) */
#define RING_LANE_DW 256  /* dwords per slot row (64 lanes x 4) */

/* MSB-first bit stream.  Window hi:lo (big-endian words); the cursor is 32-s bits into
 * hi (s in [0,31]; s == 0 means the cursor sits at the start of lo), so the next 32 bits
 * are alignbit(hi, lo, s) for every cursor position.  nx = raw (little-endian) word wi,
 * the next to enter the window; it is re-read from the ring on every advance. */
struct BR {
    const uint32_t *__restrict__ w; /* stream words (16-byte aligned base) */
    uint32_t nw;                    /* words readable (allocation covers nblk*4) */
    uint32_t nblk;                  /* 16-byte blocks readable */
    lds_u32 *ring;                  /* slot 0 of lane 0 (wave-uniform) */
    lds_u32 *lring;                 /* this lane's word-0 entry */
    uint32_t rdepth, wmask;         /* ring slots (power of 2 <= RING_MAX); ring word mask */
    uint32_t wi, s, hi, lo, nx;
    uint32_t vendw, iend;           /* words < vendw landed in the ring; blocks < iend issued */
    uint32_t iend_old;              /* k_decode's 2-deep DMA pipeline: issued two refills ago */
    uint32_t ra, vlim;              /* k_decode_st: ring byte address of word wi (with the lane's bits), vendw - 1 */
    bool stats;
};

DEV void br_init(BR &b, const uint32_t *words, uint64_t nbytes, lds_u32 *ring, uint32_t lane, uint32_t rdepth) {
    b.rdepth = rdepth;
    b.wmask = 4u * rdepth - 1u;
    b.w = words;
    b.nblk = (uint32_t)((nbytes + 15u) >> 4);
    b.nw = b.nblk * 4u;
    b.ring = ring;
    b.lring = ring + lane * 4u;
    b.wi = 2;
    b.s = b.hi = b.lo = b.nx = 0;
    b.vendw = b.iend = 0;
    b.iend_old = 0;
    b.stats = false;
}

DEV void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
/* vmcnt retires in issue order (loads, stores and LDS-DMA together): waiting until at most
 * N are outstanding completes everything older than the youngest N */
template <int N> DEV void wait_vm_but() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
/* the same with a wave-uniform run-time count (vmcnt is an immediate: jump table) */
DEV void wait_vm_n(uint32_t n) {
    switch (__builtin_amdgcn_readfirstlane(min(n, 63u))) {
#define WVN(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define WVN8(k) WVN(k) WVN(k + 1) WVN(k + 2) WVN(k + 3) WVN(k + 4) WVN(k + 5) WVN(k + 6) WVN(k + 7)
        WVN8(0) WVN8(8) WVN8(16) WVN8(24) WVN8(32) WVN8(40) WVN8(48) WVN8(56)
#undef WVN8
#undef WVN
    default: break;
    }
}
/* single-wave workgroups: LDS exchange between lanes needs only the LDS queue drained
 * (and the compiler kept from reordering); no s_barrier, no vmcnt drain of stores/DMA */
DEV void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

DEV uint32_t gword(const BR &b, uint32_t w) { return (w < b.nw) ? b.w[w] : 0u; }
/* ring layout [slot][lane][4 words] (16 bytes per lane per slot, the LDS-DMA dwordx4
 * image); block j lives in slot j % rdepth */
DEV uint32_t ring_off(const BR &b, uint32_t w) { /* dword offset of word w from lring */
    return ((w & (b.wmask & ~3u)) << 6) + (w & 3u);
}
DEV uint32_t ring_word(const BR &b, uint32_t w) { return b.lring[ring_off(b, w)]; }
/* LDS-DMA destination invariant.  A global_load_lds_dwordx4 writes lane l's 16 bytes at
 * (destination base + 16 l); round 2 found that a base that is not 1 KiB aligned writes the
 * wrong LDS bytes with no fault (wrong PCM).  Every ring slot row is one
 * whole 1 KiB image, so the invariant is: ring bases 1 KiB aligned (LDS_DMA_ALIGN on every
 * __shared__ ring) and slot offsets multiples of 1 KiB (the static_asserts below).  Debug
 * builds (-DBNFLAC_DEBUG_ASSERTS) also check every base at run time. */
#define LDS_DMA_ALIGN __attribute__((aligned(1024)))
static_assert(RING_LANE_DW * 4 == 1024, "a ring slot row must be exactly one 1 KiB LDS-DMA image");
DEV void dma_check_base(const lds_u32 *base) {
#ifdef BNFLAC_DEBUG_ASSERTS
    if (((uint32_t)(uintptr_t)base & 1023u) != 0u) __builtin_trap();
#else
    (void)base;
#endif
}
/* One LDS-DMA: 16 bytes per lane to dst + 16 lane.  (Issued as inline asm instead, hidden from
 * the waitcnt pass, it measured 1-2% slower on k_decode_st in round 4.) */
DEV void lds_dma16(const void *g, lds_u32 *dst) {
    dma_check_base(dst);
    __builtin_amdgcn_global_load_lds((gvoid *)g, (lds_void *)dst, 16, 0, 0);
}
DEV void dma_block(const BR &b, uint32_t j, uint32_t slot) { /* one 16-byte block per lane */
    lds_dma16(b.w + (uint64_t)min(j, b.nblk - 1u) * 4u, b.ring + slot * RING_LANE_DW);
}
/* The same with the instruction's immediate offset (one address for consecutive blocks).  The
 * offset moves the LDS destination as well as the global address (measured on gfx950,
 * tools/dbg_glds_off.hip), so the LDS base passed is the slot row minus the offset: the
 * row still receives lane l's 16 bytes at +16 l. */
template <int OFF>
DEV void lds_dma16_off(const void *g, lds_u32 *row) {
    dma_check_base(row); /* the row the data lands in (the base passed is row - OFF / 4) */
    __builtin_amdgcn_global_load_lds((gvoid *)g, (lds_void *)(row - OFF / 4), 16, OFF, 0);
}

/* Issue the blocks this lane will need next (exec-masked LDS-DMA per ring slot).  Blocks
 * issued earlier have landed once the wait returns.  The block of word wi is kept: br_adv
 * re-reads it. */
template <int KEEP = 0> /* KEEP: younger vector-memory ops (PCM stores) that may stay in flight */
DEV void br_refill(BR &b) {
    wait_vm_but<KEEP>();
    b.vendw = b.iend * 4u;
    /* whole 64-byte lines: [iend, first line of the cursor + rdepth); a 4-slot ring (one
     * line) refills from the cursor's block instead */
    const uint32_t need = b.rdepth >= 8u ? ((b.wi >> 2) & ~3u) : (b.wi >> 2);
    const uint32_t lo = max(b.iend, need), hi = need + b.rdepth;
#pragma unroll 1 /* rare path (seeks, landings), inlined at every cursor advance: keep it small */
    for (int s = 0; s < RING_MAX; s++) {
        if ((uint32_t)s >= b.rdepth) break; /* wave-uniform */
        const uint32_t j = lo + (((uint32_t)s - lo) & (b.rdepth - 1u));
        if (j < hi) dma_block(b, j, (uint32_t)s);
    }
    b.iend = max(b.iend, hi);
}

/* Rare path: word wi is not in the landed part of the ring (a jump, or a lane that
 * consumed more than the ring held): wait for what is in flight, refill if still short. */
DEV void br_drained(BR &b) { /* every vector-memory op of this wave has completed (per lane) */
    b.vendw = b.iend * 4u;
    b.iend_old = b.iend;
}
DEV void br_land(BR &b, uint32_t margin = 0) { /* afterwards words wi .. wi + margin have landed */
    STAT(b.stats, 2);
    wait_vm();
    br_drained(b);
    if (b.wi + margin >= b.vendw) {
        br_refill(b);
        wait_vm();
        br_drained(b);
    }
}

/* Blocking seek (subframe starts, skips). */
DEV void br_seek(BR &b, uint64_t bit) {
    b.s = (uint32_t)(0u - bit) & 31u;
    const uint32_t hw = (uint32_t)((bit + b.s) >> 5) - 1u; /* word holding the cursor (-1 at bit 0) */
    b.hi = __builtin_bswap32(gword(b, hw));
    b.lo = __builtin_bswap32(gword(b, hw + 1u));
    b.wi = hw + 2u;
    b.iend = (b.wi >> 2) & ~3u;
    br_refill(b);
    wait_vm();
    br_drained(b);
    b.nx = ring_word(b, b.wi);
}

/* k_decode's refill: a 2-deep pipeline.  Waits only for the DMAs issued two refills ago
 * (vmcnt counts loads, stores and LDS-DMA together and retires them in issue order, so
 * letting the younger q.s_last + q.d_last + q.s_prev ops stay outstanding is exact), marks
 * those blocks landed, and issues the next blocks.  Blocks issued now become readable two
 * chunks later; the ring keeps ~6 blocks ahead of the cursor.  Called by the whole wave
 * (the counts must be wave-uniform); `want` masks the lanes that refill.  A full drain in
 * between (br_land, seek) only completes more, so the counts stay safe without reset. */
struct VmQ {
    uint32_t d_last, s_last, s_prev; /* DMAs of the last refill; stores since it; before it */
};
DEV void br_refill2(BR &b, bool want, VmQ &q, bool nowait = false) {
    if (!nowait) wait_vm_n(q.s_last + q.d_last + q.s_prev); /* nowait: timing ablation 0x200 only */
    if (want) b.vendw = b.iend_old * 4u;
    /* the ring holds rdepth/4 whole lines; a lane whose cursor (word wi) is in the newest
     * line fetches the next line into the oldest line's slots: 4 x 16-byte DMAs hitting
     * one cache line */
    const uint32_t curl = (b.wi >> 2) & ~3u;
    const bool go = want && b.iend <= curl + 4u;
    const uint32_t slot0 = b.iend & (b.rdepth - 1u); /* multiple of 4 */
    uint32_t d = 0;
#pragma unroll
    for (int h = 0; h < RING_MAX / 4; h++) {
        if ((uint32_t)(h * 4) >= b.rdepth) break; /* wave-uniform */
        const bool gh = go && slot0 == (uint32_t)(h * 4);
        if (__any(gh)) { /* wave-uniform: the 4 DMAs below are issued exactly when this holds */
            d += 4;
            if (gh) {
#pragma unroll
                for (int k = 0; k < 4; k++) dma_block(b, b.iend + k, (uint32_t)(h * 4 + k));
            }
        }
    }
    if (want) {
        b.iend_old = b.iend;
        if (go) b.iend += 4u;
    }
    q.s_prev = q.s_last;
    q.s_last = 0;
    q.d_last = d;
}

/* k_decode's refill (1-deep): br_issue, after a chunk's entropy phase, fetches the 16-byte
 * blocks up to rdepth past the block of the cursor word (never that block's slot, which
 * br_adv re-reads), so at least (rdepth - 1) * 16 bytes lie ahead of the cursor; br_wait1,
 * before the next entropy phase, waits for them -- only the PCM stores packed since (at
 * least q.s_last of them, all younger) may stay in flight -- and marks them landed.  The
 * restore and the pack run in between.  A lane that needs more within one chunk lands
 * (br_land). */
DEV void br_wait1(BR &b, VmQ &q) {
    wait_vm_n(q.s_last);
    b.vendw = b.iend * 4u;
    q.s_last = 0;
}
DEV void br_issue(BR &b, bool want) {
    const uint32_t cb = b.wi >> 2;
    const uint32_t lo = max(b.iend, cb), hi = cb + b.rdepth;
#pragma unroll
    for (int k = 0; k < RING_MAX; k++) {
        if ((uint32_t)k >= b.rdepth) break; /* wave-uniform */
        const uint32_t j = lo + (((uint32_t)k - lo) & (b.rdepth - 1u)); /* the block for slot k */
        const bool go = want && j < hi;
        if (__any(go)) {
            if (go) dma_block(b, j, (uint32_t)k);
        }
    }
    if (want) b.iend = max(b.iend, hi);
}

DEV uint64_t br_pos(const BR &b) { return ((uint64_t)(b.wi - 1u) << 5) - b.s; }
DEV uint32_t br_peek(const BR &b) { return __builtin_amdgcn_alignbit(b.hi, b.lo, b.s); }
/* Pending LDS store carried into the next cursor advance (fused decode): issuing it after
 * the window update and before the next ring read keeps every LDS op covered by the next
 * lgkmcnt wait a whole codeword old. */
struct PendW {
    int32_t *at;
    int32_t v;
    bool on;
};
DEV bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; } /* wave-uniform */
/* leading zeros, ~0u for 0 (v_ffbh_u32; asm so the compiler assumes no range).  An asm
 * statement makes hipcc's waitcnt pass wait lgkmcnt(0) before it; the builtin form
 * (x ? clz(x) : ~0u, also one v_ffbh_u32) keeps counted waits but measured 1-2% slower on
 * k_decode_st (round 4) and no different on k_decode_sys. */
DEV uint32_t ffbh(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}


template <bool CHECK = true>
DEV void br_adv(BR &b, uint32_t n, PendW *pw = nullptr) { /* n <= 32; branch-free except the rare landing check */
    const int32_t t = (int32_t)b.s - (int32_t)n;
    const bool c = t < 0;
    b.s = (uint32_t)t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += c ? 1u : 0u;
    if (CHECK && __builtin_expect(any_lane(b.wi >= b.vendw), 0)) br_land(b);
    if (pw && pw->on) *pw->at = pw->v;
    /* issue the ring read after the window update (an artificial data dependency of the
     * address on the new lo), so the wait for the previous word (one codeword old) is not
     * merged with a wait for this one; other instructions stay free to move */
    uint32_t off = ring_off(b, b.wi);
    asm volatile("" : "+v"(off) : "v"(b.lo));
    b.nx = b.lring[off];
}
template <bool CHECK = true>
DEV uint32_t br_read(BR &b, uint32_t n) { /* 0..32 bits */
    uint32_t v = n ? (br_peek(b) >> ((32u - n) & 31u)) : 0u;
    br_adv<CHECK>(b, n);
    return v;
}
template <bool CHECK = true>
DEV int32_t br_read_s(BR &b, uint32_t n) {
    uint32_t v = br_read<CHECK>(b, n);
    uint32_t s = (32u - n) & 31u;
    return (int32_t)(v << s) >> s;
}
DEV void br_skip(BR &b, uint64_t n) {
    if (n <= 32) br_adv(b, (uint32_t)n);
    else br_seek(b, br_pos(b) + n);
}
/* count zeros up to and including the terminating 1 (read_unary_unsigned @0x10001960) */
DEV bool br_unary(BR &b, uint32_t &q, uint64_t limit) {
    uint32_t acc = 0;
    for (;;) {
        uint32_t p = br_peek(b);
        if (p) {
            uint32_t z = (uint32_t)__builtin_clz(p);
            acc += z;
            br_adv(b, z + 1u);
            q = acc;
            return true;
        }
        acc += 32u;
        br_adv(b, 32u);
        if (br_pos(b) > limit) {
            q = acc;
            return false;
        }
    }
}

DEV uint8_t crc8_bytes(const uint8_t *p, uint32_t n) {
    uint8_t c = 0;
    for (uint32_t i = 0; i < n; i++) c = g_crc8_tab[c ^ p[i]];
    return c;
}

/* ------------------------------------------------------ wave-uniform bit reader */
/* The reader of the wave-per-frame kernels (k_parse_wave): one cursor for the whole wave
 * (every lane holds the same value), over a ring of WR_SLOTS windows of 256 stream words in
 * LDS.  Window j holds words [w0 + 256 j, w0 + 256 j + 256) and sits in slot j % WR_SLOTS; one
 * global_load_lds_dwordx4 fills it (64 lanes x 16 B, coalesced).  Windows are fetched ahead
 * of the cursor (up to WR_SLOTS - 1) and waited for with an exact vmcnt: the wave issues no
 * other vector-memory ops while it reads.  Header fields are read at the uniform cursor
 * (two broadcast LDS reads per field); the Rice scan (wave_rice_skip) reads each lane's own
 * segment words from the same ring. */
#define WR_SLOTS 8 /* a 16-word-per-lane scan pass spans 5 windows */
#define WR_WIN 256u /* words per window (1 KiB) */
struct WR {
    const uint32_t *__restrict__ w;
    uint32_t nblk;   /* 16-byte blocks readable */
    lds_u32 *ring;   /* WR_SLOTS KiB, 1 KiB aligned */
    uint32_t w0;     /* stream word of window 0 (multiple of WR_WIN) */
    uint32_t issued; /* windows issued (0 .. issued-1) */
    uint32_t landed; /* windows known to have landed */
    uint64_t pos;    /* bit cursor (absolute, MSB-first) */
    uint64_t st[8];  /* debug counters (g_pw_stats layout), flushed once per wave */
};
DEV uint32_t wr_u(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEV void wr_issue(WR &r) { /* window r.issued into its slot */
    const uint32_t j = r.issued++;
    const uint32_t blk = (r.w0 >> 2) + j * (WR_WIN / 4u) + (threadIdx.x & 63u);
    lds_dma16(r.w + (uint64_t)min(blk, r.nblk - 1u) * 4u, r.ring + (j % WR_SLOTS) * WR_WIN);
}
DEV void wr_reset(WR &r, uint32_t wa) {
    wait_vm();
    r.w0 = wa & ~(WR_WIN - 1u);
    r.issued = r.landed = 0;
}
DEV void wr_init(WR &r, const uint32_t *words, uint64_t nbytes, lds_u32 *ring, uint64_t bit) {
    r.w = words;
    r.nblk = (uint32_t)((nbytes + 15u) >> 4);
    r.ring = ring;
    r.pos = bit;
    r.w0 = wr_u((uint32_t)(bit >> 5)) & ~(WR_WIN - 1u);
    r.issued = r.landed = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r.st[i] = 0;
}
/* words [wa, wb] readable (wb - wa < WR_SLOTS - 2 windows); fetches ahead */
DEV void wr_need(WR &r, uint32_t wa, uint32_t wb) {
    wa = wr_u(wa);
    wb = wr_u(wb);
    if (wa < r.w0 || ((wa - r.w0) / WR_WIN) > r.issued + 2u) wr_reset(r, wa);
    const uint32_t lo = (wa - r.w0) / WR_WIN, hi = (wb - r.w0) / WR_WIN;
    while (r.issued < lo + WR_SLOTS) wr_issue(r);
    if (hi >= r.landed) { /* at most WR_SLOTS - 1 younger windows may stay in flight */
        switch (wr_u(r.issued - 1u - hi)) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        }
        r.landed = hi + 1u;
    }
}
static_assert(WR_SLOTS == 8, "wr_need's vmcnt switch covers WR_SLOTS - 1 windows in flight");
DEV uint32_t wr_word(const WR &r, uint32_t w) { return __builtin_bswap32(r.ring[(w - r.w0) & (WR_SLOTS * WR_WIN - 1u)]); }
DEV uint32_t wr_peek(WR &r) { /* the 32 bits at the cursor */
    const uint32_t wi = (uint32_t)(r.pos >> 5);
    wr_need(r, wi, wi + 1u);
    const uint32_t hi = wr_u(wr_word(r, wi)), lo = wr_u(wr_word(r, wi + 1u));
    const uint32_t s = (uint32_t)r.pos & 31u;
    return s ? __builtin_amdgcn_alignbit(hi, lo, 32u - s) : hi;
}
DEV uint64_t br_pos(const WR &r) { return r.pos; }
DEV uint32_t br_peek(WR &r) { return wr_peek(r); }
DEV void br_seek(WR &r, uint64_t bit) { r.pos = bit; }
DEV void br_skip(WR &r, uint64_t n) { r.pos += n; }
DEV uint32_t br_read(WR &r, uint32_t n) { /* 0..32 bits */
    const uint32_t v = n ? (wr_peek(r) >> ((32u - n) & 31u)) : 0u;
    r.pos += n;
    return v;
}
DEV int32_t br_read_s(WR &r, uint32_t n) {
    const uint32_t v = br_read(r, n), s = (32u - n) & 31u;
    return (int32_t)(v << s) >> s;
}
DEV bool br_unary(WR &r, uint32_t &q, uint64_t limit) { /* read_unary_unsigned @0x10001960 */
    uint32_t acc = 0;
    for (;;) {
        const uint32_t p = wr_peek(r);
        if (p) {
            const uint32_t z = (uint32_t)__builtin_clz(p);
            r.pos += z + 1u;
            q = acc + z;
            return true;
        }
        acc += 32u;
        r.pos += 32u;
        if (r.pos > limit) {
            q = acc;
            return false;
        }
    }
}

/* ------------------------------------------------------------ frame header */
enum { E_LOST_SYNC = 0, E_BAD_HEADER = 1, E_CRC = 2, E_UNPARSEABLE = 3 };

/* read_frame_header_ @0x10011d70: fills fi; returns BNF_ST_* (OK also when the header
 * is flagged unparseable -- the caller reports that after the number conversion). */
template <class R> /* R: BR (lane cursor) or WR (wave-uniform cursor) */
DEV uint32_t parse_header(R &b, uint64_t fbit, uint64_t limit, const bnf_stream_params &sp,
                          bnf_frame_info &fi) {
    /* the header's CRC-8 is folded in as each byte is read (no byte buffer: a per-lane array
     * indexed at run time would live in scratch memory) */
    uint32_t crc = 0, last = 0, b2 = 0, b3 = 0;
    auto take = [&](uint32_t v) { crc = g_crc8_tab[crc ^ v]; last = v; };
    uint32_t unparseable = 0, bs_hint = 0, sr_hint = 0, x;
    br_seek(b, fbit);
    take(br_read(b, 8));
    const uint32_t b1 = br_read(b, 8);
    take(b1);
    fi.cached = -1;
    if (b1 & 0x02) unparseable = 1;
    for (int i = 0; i < 2; i++) {
        x = br_read(b, 8);
        if (x == 0xff) {
            fi.cached = 0xff;
            fi.err = E_BAD_HEADER;
            fi.resume_bit = br_pos(b);
            return BNF_ST_ERROR;
        }
        take(x);
        if (i == 0) b2 = x;
        else b3 = x;
    }
    x = b2 >> 4;
    if (x == 0) unparseable = 1;
    else if (x == 1) fi.blocksize = 192;
    else if (x <= 5) fi.blocksize = 576u << (x - 2);
    else if (x <= 7) bs_hint = x;
    else fi.blocksize = 256u << (x - 8);
    x = b2 & 0x0f;
    switch (x) {
    case 0:
        if (sp.has_stream_info) fi.sample_rate = sp.sample_rate;
        else unparseable = 1;
        break;
    case 1: fi.sample_rate = 88200; break;
    case 2: fi.sample_rate = 176400; break;
    case 3: fi.sample_rate = 192000; break;
    case 4: fi.sample_rate = 8000; break;
    case 5: fi.sample_rate = 16000; break;
    case 6: fi.sample_rate = 22050; break;
    case 7: fi.sample_rate = 24000; break;
    case 8: fi.sample_rate = 32000; break;
    case 9: fi.sample_rate = 44100; break;
    case 10: fi.sample_rate = 48000; break;
    case 11: fi.sample_rate = 96000; break;
    case 15:
        fi.err = E_BAD_HEADER;
        fi.resume_bit = br_pos(b);
        return BNF_ST_ERROR;
    default: sr_hint = x; break;
    }
    x = b3 >> 4;
    if (x & 8) {
        fi.channels = 2;
        if ((x & 7) <= 2) fi.assignment = (x & 7) + 1;
        else unparseable = 1;
    } else {
        fi.channels = x + 1;
        fi.assignment = 0;
    }
    x = (b3 & 0x0e) >> 1;
    switch (x) {
    case 0:
        if (sp.has_stream_info) fi.bps = sp.bps;
        else unparseable = 1;
        break;
    case 1: fi.bps = 8; break;
    case 2: fi.bps = 12; break;
    case 4: fi.bps = 16; break;
    case 5: fi.bps = 20; break;
    case 6: fi.bps = 24; break;
    default: unparseable = 1; break;
    }
    if (b3 & 0x01) unparseable = 1;
    /* UTF-8 frame/sample number (@0x10001e20 / @0x10001f60), with libFLAC's truthiness tests */
    const bool is64 = (b1 & 0x01) || (sp.has_stream_info && sp.min_blocksize != sp.max_blocksize);
    {
        uint64_t v = 0;
        uint32_t n;
        bool bad = false;
        x = br_read(b, 8);
        take(x);
        if (!(x & 0x80)) { v = x; n = 0; }
        else if ((x & 0xC0) && !(x & 0x20)) { v = x & 0x1F; n = 1; }
        else if ((x & 0xE0) && !(x & 0x10)) { v = x & 0x0F; n = 2; }
        else if ((x & 0xF0) && !(x & 0x08)) { v = x & 0x07; n = 3; }
        else if ((x & 0xF8) && !(x & 0x04)) { v = x & 0x03; n = 4; }
        else if ((x & 0xFC) && !(x & 0x02)) { v = x & 0x01; n = 5; }
        else if (is64 && (x & 0xFE) && !(x & 0x01)) { v = 0; n = 6; }
        else { bad = true; n = 0; }
        for (; !bad && n; n--) {
            x = br_read(b, 8);
            take(x);
            if (!(x & 0x80) || (x & 0x40)) bad = true;
            else v = (v << 6) | (x & 0x3F);
        }
        if (!is64 && !bad) v &= 0xffffffffull; /* 32-bit accumulation (6 bytes max => 31 bits) */
        if (bad) {
            fi.cached = (int32_t)last;
            fi.err = E_BAD_HEADER;
            fi.resume_bit = br_pos(b);
            return BNF_ST_ERROR;
        }
        fi.number_type = is64 ? 1u : 0u;
        fi.number = v;
    }
    if (bs_hint) {
        x = br_read(b, 8);
        take(x);
        if (bs_hint == 7) {
            uint32_t y = br_read(b, 8);
            take(y);
            x = (x << 8) | y;
        }
        fi.blocksize = x + 1;
    }
    if (sr_hint) {
        x = br_read(b, 8);
        take(x);
        if (sr_hint != 12) {
            uint32_t y = br_read(b, 8);
            take(y);
            x = (x << 8) | y;
        }
        fi.sample_rate = (sr_hint == 12) ? x * 1000u : (sr_hint == 13 ? x : x * 10u);
    }
    x = br_read(b, 8);
    fi.crc8 = x;
    if (br_pos(b) > limit) return BNF_ST_TRUNC;
    if (crc != (x & 0xffu)) {
        fi.err = E_BAD_HEADER;
        fi.resume_bit = br_pos(b);
        return BNF_ST_ERROR;
    }
    /* the frame->sample number conversion can also flag UNPARSEABLE (@0x10012372):
     * fixed-number header, no fixed block size yet, STREAMINFO min != max.  That
     * combination is impossible (min != max forces 64-bit numbers), so only the
     * header-field flag remains; the host replays the conversion itself. */
    fi.unparseable = unparseable;
    if (unparseable) {
        fi.err = E_UNPARSEABLE;
        fi.resume_bit = br_pos(b);
        return BNF_ST_ERROR;
    }
    return BNF_ST_OK;
}

DEV uint32_t sub_bps(const bnf_frame_info &fi, uint32_t ch) {
    uint32_t bps = fi.bps;
    if ((fi.assignment == 1 && ch == 1) || (fi.assignment == 2 && ch == 0) || (fi.assignment == 3 && ch == 1)) bps++;
    return bps;
}

/* ------------------------------------------------------------ subframe parse */
enum { T_CONST = 0, T_VERB = 1, T_FIXED = 2, T_LPC = 3 };
enum { P_MMX16 = 0, P_IA32 = 1, P_WIDE = 2 };

struct SubHdr {
    uint32_t type, order, wasted, bps; /* bps after removing wasted bits */
    uint32_t prec;
    int32_t shift;
    uint32_t porder, rice2;
    int32_t cval;
    uint32_t path;
};

/* read_subframe_ @0x10012480 up to (and including) the residual coding header.
 * STORE: warm-ups go to warm[u * WS] and coefficients to coef[u] for u < NW, in loops
 * unrolled to NW (compile-time indices: register arrays stay in registers).  Returns
 * BNF_ST_*; on ERROR sets err and the reader position is where libFLAC stops. */
template <bool STORE, int NW = 32, int WS = 1, class R = BR>
DEV uint32_t parse_subframe_head(R &b, uint32_t bps, uint32_t bs, uint64_t limit, SubHdr &h,
                                 int32_t *warm, int32_t *coef, int32_t &err) {
    uint32_t x = br_read(b, 8);
    uint32_t wflag = x & 1u;
    x &= 0xFEu;
    h.wasted = 0;
    if (wflag) {
        uint32_t u;
        if (!br_unary(b, u, limit)) return BNF_ST_TRUNC;
        h.wasted = u + 1u;
        if (h.wasted > bps) { err = E_UNPARSEABLE; return BNF_ST_ERROR; }
        bps -= h.wasted;
    }
    if (x & 0x80) { err = E_LOST_SYNC; return BNF_ST_ERROR; }
    if (bps > 32) { err = E_UNPARSEABLE; return BNF_ST_ERROR; }
    h.bps = bps;
    h.order = 0;
    h.porder = 0;
    h.rice2 = 0;
    h.path = P_IA32;
    if (x == 0) {
        h.type = T_CONST;
        h.cval = br_read_s(b, bps);
        return BNF_ST_OK;
    }
    if (x == 2) { h.type = T_VERB; return BNF_ST_OK; }
    if (x < 16) { err = E_UNPARSEABLE; return BNF_ST_ERROR; }
    if (x <= 24) {
        h.type = T_FIXED;
        h.order = (x >> 1) & 7u;
    } else if (x < 64) {
        err = E_UNPARSEABLE;
        return BNF_ST_ERROR;
    } else {
        h.type = T_LPC;
        h.order = ((x >> 1) & 31u) + 1u;
    }
    if (STORE) {
#pragma unroll
        for (int u = 0; u < NW; u++)
            if ((uint32_t)u < h.order) warm[u * WS] = br_read_s(b, bps);
        for (uint32_t u = NW; u < h.order; u++) br_read_s(b, bps);
    } else {
        for (uint32_t u = 0; u < h.order; u++) br_read_s(b, bps);
    }
    if (h.type == T_LPC) {
        uint32_t p = br_read(b, 4);
        if (p == 15) { err = E_LOST_SYNC; return BNF_ST_ERROR; }
        h.prec = p + 1;
        h.shift = br_read_s(b, 5);
        if (STORE) {
#pragma unroll
            for (int u = 0; u < NW; u++)
                if ((uint32_t)u < h.order) coef[u] = br_read_s(b, h.prec);
            for (uint32_t u = NW; u < h.order; u++) br_read_s(b, h.prec);
        } else {
            for (uint32_t u = 0; u < h.order; u++) br_read_s(b, h.prec);
        }
        uint32_t ilog = 31u - (uint32_t)__builtin_clz(h.order);
        if (bps + h.prec + ilog <= 32) h.path = (bps <= 16 && h.prec <= 16 && h.order >= 4) ? P_MMX16 : P_IA32;
        else h.path = P_WIDE;
    }
    uint32_t m = br_read(b, 2);
    if (m > 1) { err = E_UNPARSEABLE; return BNF_ST_ERROR; }
    h.rice2 = m;
    h.porder = br_read(b, 4);
    /* read_residual_partitioned_rice_ sanity checks (@0x10012e1e, @0x10012e41) */
    if (h.porder == 0) {
        if (bs < h.order) { err = E_LOST_SYNC; return BNF_ST_ERROR; }
    } else {
        if ((bs >> h.porder) < h.order) { err = E_LOST_SYNC; return BNF_ST_ERROR; }
        if (bs & ((1u << h.porder) - 1u)) { err = E_UNPARSEABLE; return BNF_ST_ERROR; } /* see oracle */
    }
    return br_pos(b) > limit ? BNF_ST_TRUNC : BNF_ST_OK;
}

DEV uint32_t st_hmask(uint32_t h, uint32_t o) { /* little-endian dword at line offset o: bytes below h cleared */
    return h <= o ? ~0u : (h >= o + 4u ? 0u : (~0u << (8u * (h - o))));
}
/* ------------------------------------------------- CRC-16 remainder arithmetic
 * (the table-free zero test, st_crc16_ok below, and k_parse's prefix of it) */
struct CrcZ {
    uint32_t r0, r1, px; /* remainder mod T^4; XOR of every word (parity) */
};
DEV void crcz_w(CrcZ &c, uint32_t le) { /* one little-endian stream word */
    const uint32_t W = __builtin_bswap32(le);
    const uint32_t H = __builtin_amdgcn_alignbit(c.r1, c.r0, 28);
    const uint32_t n0 = W ^ H ^ (H << 4);
    c.r1 = c.r0 ^ (H >> 28);
    c.r0 = n0;
}
DEV void crcz_blk(CrcZ &c, uint4 v) {
    c.px ^= v.x ^ v.y ^ v.z ^ v.w;
    crcz_w(c, v.x);
    crcz_w(c, v.y);
    crcz_w(c, v.z);
    crcz_w(c, v.w);
}
/* k_parse's part of a 2-channel frame's CRC-16 (round 6).  The decode kernels' tail re-reads
 * the whole frame for the CRC-16, and every wave of a CU reaches its tail together, so those
 * bytes go at the HBM rate with nothing beside them.  k_parse walks subframe 0 anyway: its ring
 * holds those bytes, so it folds every whole 64-byte line before subframe 1's line into the
 * same T^4 remainder (from the ring while the line is one of its two, else one reload, L2-warm),
 * one 16-byte block at a time (three live state words: k_parse's occupancy is LDS-bound at 5
 * waves per SIMD, ~100 VGPRs), and the decode tail continues from there, re-reading only the
 * rest of the frame. */
/* The prefix state: the remainder mod Q(y) = y^15 + y + 1, y = x^32, in 15 words.  Q(y) =
 * T(x^32) = T(x)^32 is a multiple of T, so it keeps M mod T; with whole words as the
 * coefficients a 64-byte line is 18 word XORs at once (S y^16 + sum W[i] y^(15-i): y^15 = y + 1,
 * y^16 = y^2 + y; checked against bit-serial division mod T in Python while writing this)
 * against 96 VALU through the T^4 form, and the words are taken as loaded (little-endian): a
 * byte swap permutes the bits of every word alike, so it is applied to the 15 state words
 * once, at the hand-off (crcp_z).  k_parse<1> 128 VGPRs, 4 waves per SIMD: C2 k_parse 2.52 ->
 * 2.16 ms against the T^4 form (1.95 without a prefix), C3 the same as with it (10.43 vs
 * 10.47 ms per step; a build at 146 VGPRs, 3 waves, had cost C3's plain walk 0.5 ms). */
struct CrcP {
    uint32_t s[15]; /* s[k]: the coefficient of y^k (little-endian words) */
    uint32_t px;    /* XOR of every word (parity) */
    uint32_t wc;    /* next line to fold (absolute 64-byte line index); ~0: no prefix for this frame */
};
DEV void crcp_init(CrcP &c) {
#pragma unroll
    for (int k = 0; k < 15; k++) c.s[k] = 0u;
    c.px = 0u;
    c.wc = ~0u;
}
DEV void crcp_fold(CrcP &c, const u32x4 (&v)[4]) {
    const uint32_t W[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                            v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
    c.px ^= W[0] ^ W[1] ^ W[2] ^ W[3] ^ W[4] ^ W[5] ^ W[6] ^ W[7] ^ W[8] ^ W[9] ^ W[10] ^ W[11] ^ W[12] ^ W[13] ^
            W[14] ^ W[15];
    const uint32_t r0 = c.s[13] ^ c.s[14] ^ W[15] ^ W[0], r1 = c.s[0] ^ c.s[13] ^ W[14] ^ W[0],
                   r2 = c.s[0] ^ c.s[1] ^ c.s[14] ^ W[13];
#pragma unroll
    for (int d = 14; d >= 3; d--) c.s[d] = c.s[d - 2] ^ c.s[d - 1] ^ W[15 - d]; /* descending: old s[d-2], s[d-1] */
    c.s[2] = r2;
    c.s[1] = r1;
    c.s[0] = r0;
    c.wc++;
}
/* the remainder in the decode tails' T^4 form (st_crc16_ok continues it) */
DEV CrcZ crcp_z(const CrcP &c) {
    CrcZ z{0u, 0u, 0u};
#pragma unroll
    for (int k = 14; k >= 0; k--) crcz_w(z, c.s[k]);
    z.px = c.px;
    return z;
}
/* fold the lines before line cl (whole wave).  The ring holds the two lines [iend / 4 - 2,
 * iend / 4), and the refill keeps the line of word wi (the reader's next word) and the one
 * after it: so before a refill, cl = wi / 16 -- every line the reader has loaded, which the
 * refill may overwrite -- folds from the ring (a line behind a landing refill reads again
 * from global memory, L2-warm; bounding by the cursor's bit position instead left 22% of C2's
 * lines to that path: the word lookahead crosses a line first).  The frame's first line is
 * folded before the walk (parse_frame), so these are whole lines. */
template <bool ALL = false, class C> /* ALL: every line before cl (the walk's end); else at most one (a refill point) */
DEV void crcp_hook(C &c, const BR &b, uint32_t lane, uint32_t cl) {
    for (uint32_t it = 0; any_lane(c.wc < cl) && (ALL || it == 0u); it++) {
        if (c.wc < cl) {
            const uint32_t L = c.wc;
            u32x4 v[4];
            if (L + 2u >= (b.iend >> 2)) {
#pragma unroll
                for (uint32_t i = 0; i < 4; i++)
                    v[i] = lds_ld128((const lds_u32x4 *)(b.ring + (((L & 1u) * 4u + i) * RING_LANE_DW) + lane * 4u));
                lds_sync();
                crcp_fold(c, v);
            } else { /* overwritten by a refill: read it again (each path folds: no merge of v) */
                const u32x4 *g = (const u32x4 *)((const uint8_t *)b.w + (uint64_t)L * 64u);
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) v[i] = g[i];
                crcp_fold(c, v);
            }
        }
    }
}

#define CRC_LINES 4 /* 64-byte lines in flight per lane: each lane walks its own frame */

/* Zero test of the CRC-16 remainder of [b0, b1), the frame with its footer (read_frame_'s
 * check @0x10011a01: the footer equals the CRC of the frame bytes iff the CRC of frame + footer
 * is zero), by arithmetic, with no tables (round 6).  P = x^16 + x^15 + x^2 + 1 = (x + 1) T with
 * T = x^15 + x + 1, so M = 0 mod P iff M has even parity and M = 0 mod T.  The remainder mod
 * T^4 = x^60 + x^4 + 1 (a multiple of T) costs five VALU per 32-bit word: with the state
 * r = r1:r0 (60 bits; r1's top four bits are stale copies of bits alignbit already took),
 * r x^32 + W = (r0 mod x^28) x^32 + W + H (x^4 + 1), H = r >> 28.  Leading zero bytes leave M
 * unchanged and trailing ones multiply it by a power of x (invertible mod T), so whole 16-byte
 * blocks with the bytes outside [b0, b1) cleared give the same verdict.  The 11-bit LDS tables
 * this replaces cost 0.75 bank-conflicted lookups per byte on the CU's one LDS pipe. */
DEV uint32_t byte_keep(int32_t lo, int32_t hi, int32_t w) { /* bytes 4w..4w+3 kept iff in [lo, hi) */
    const int32_t a = min(max(lo - 4 * w, 0), 4), b = min(max(hi - 4 * w, 0), 4);
    const uint32_t mlo = a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
    const uint32_t mhi = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
    return mlo & mhi;
}
DEV bool crcz_zero(const CrcZ &c) {
    if (__builtin_popcount(c.px) & 1) return false;
    uint64_t v = ((uint64_t)(c.r1 & 0x0FFFFFFFu) << 32) | c.r0;
#pragma unroll
    for (int i = 0; i < 4; i++) { /* x^15 = x + 1: degree 59 -> 45 -> 31 -> 17 -> 14 */
        const uint64_t h = v >> 15;
        v = (v & 0x7FFFu) ^ h ^ (h << 1);
    }
    return v == 0;
}
/* the 64-byte line at q into the remainder, its bytes below h cleared (h = 0: whole line) */
DEV void crcz_line(CrcZ &c, uint4 (&v)[4], uint32_t h) {
    if (h) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            v[u].x &= st_hmask(h, 16u * u);
            v[u].y &= st_hmask(h, 16u * u + 4u);
            v[u].z &= st_hmask(h, 16u * u + 8u);
            v[u].w &= st_hmask(h, 16u * u + 12u);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) crcz_blk(c, v[u]);
}
/* CRC-16 verdict of [b0, b1) with NL 64-byte lines in flight per lane, continuing c, which
 * already holds the lines [b0 & ~63, from) (from: a line boundary) */
template <int NL = CRC_LINES>
DEV bool st_crc16_ok(const uint8_t *__restrict__ bytes, uint64_t b0, uint64_t b1, CrcZ c = CrcZ{0u, 0u, 0u},
                     uint64_t from = 0) {
    const uint64_t p0 = max(b0 & ~(uint64_t)63u, from);
    const uint32_t h = p0 < b0 ? (uint32_t)(b0 & 63u) : 0u;
    const uint32_t nl = b1 > p0 ? (uint32_t)((b1 - p0) >> 6) : 0u;
    uint64_t p = p0;
    if (nl) {
        const uint4 *q = (const uint4 *)(bytes + p0);
        uint4 buf[NL][4];
#pragma unroll
        for (int d = 0; d < NL; d++)
#pragma unroll
            for (int u = 0; u < 4; u++) buf[d][u] = q[4u * min((uint32_t)d, nl - 1u) + u];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            buf[0][u].x &= st_hmask(h, 16u * u);
            buf[0][u].y &= st_hmask(h, 16u * u + 4u);
            buf[0][u].z &= st_hmask(h, 16u * u + 8u);
            buf[0][u].w &= st_hmask(h, 16u * u + 12u);
        }
        for (uint32_t i = 0; i < nl; i += NL) {
#pragma unroll
            for (int d = 0; d < NL; d++) {
                if (i + d < nl) {
#pragma unroll
                    for (int u = 0; u < 4; u++) crcz_blk(c, buf[d][u]);
                    const uint32_t j = min(i + d + NL, nl - 1u);
#pragma unroll
                    for (int u = 0; u < 4; u++) buf[d][u] = q[4u * j + u];
                }
            }
        }
        p = p0 + (uint64_t)nl * 64u;
    }
    /* the rest, [p, b1): up to four 16-byte blocks (each starts below b1, so it lies inside the
     * 16-byte-rounded allocation), bytes below b0 (a frame inside one line) or from b1 on cleared */
    const uint32_t nr = (uint32_t)((b1 - p + 15u) >> 4);
    uint4 t[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) t[i] = i < nr ? *(const uint4 *)(bytes + p + 16u * i) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        if (i < nr) {
            const int64_t lo = (int64_t)b0 - (int64_t)(p + 16u * i), hi = (int64_t)b1 - (int64_t)(p + 16u * i);
            const int32_t l32 = (int32_t)max(min(lo, (int64_t)16), (int64_t)0);
            const int32_t h32 = (int32_t)max(min(hi, (int64_t)16), (int64_t)0);
            uint4 v = t[i];
            v.x &= byte_keep(l32, h32, 0);
            v.y &= byte_keep(l32, h32, 1);
            v.z &= byte_keep(l32, h32, 2);
            v.w &= byte_keep(l32, h32, 3);
            crcz_blk(c, v);
        }
    }
    return crcz_zero(c);
}
/* The CRC-16 hand-off to the decode tails, 8 words per frame (crcp[8f..8f+7]): r0, r1 |
 * parity << 31 of a prefix, the lines it holds + 1 (0: none), frame_off's low word (a check);
 * the span to the next frame's offset (0: none), the verdict over that span, frame_off's low
 * word.  Written by k_parse (crc_mode 1: the prefix; 2: both). */
#define CRCP_WORDS 8u
/* the decode tails' CRC-16 verdict of the frame [b0, b1): the hand-off's verdict when the
 * frame ends where the next one starts, else its prefix continued, else the whole frame */
DEV bool st_crc16_frame(const uint8_t *__restrict__ bytes, const uint32_t *__restrict__ crcp, uint32_t f, uint64_t b0,
                        uint64_t b1) {
    if (crcp) {
        const u32x4 v = *(const u32x4 *)(crcp + CRCP_WORDS * (uint64_t)f + 4u);
        if (v.x && v.z == (uint32_t)b0 && b0 + v.x == b1) return v.y != 0u;
        const u32x4 q = *(const u32x4 *)(crcp + CRCP_WORDS * (uint64_t)f);
        const uint64_t from = ((b0 >> 6) + q.z - 1u) * 64u;
        if (q.z && q.w == (uint32_t)b0 && from <= b1)
            return st_crc16_ok(bytes, b0, b1, CrcZ{q.x, q.y & 0x0FFFFFFFu, q.y >> 31}, from);
    }
    return st_crc16_ok(bytes, b0, b1);
}

/* One step of k_parse's residual walk: up to two Rice codewords of the current partition
 * (parameter k; km = 31 - k, k1 = k + 1).  Two codewords per 32-bit window when both fit:
 * the second's prefix is counted in the window shifted past the first (zeros shifted in
 * can only make it not fit).  Predicated: a lane with rem == 0 advances 0 bits.  Branch-free
 * but for the rare long prefix: the conditions are combined with & (the && chain compiled to
 * an exec-masked region per step), and the leading-zero counts use the builtin form (the
 * asm one costs a wait state after each), ~30 VALU per step instead of ~55 (round 4). */
DEV uint32_t ffbh_b(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : ~0u; }

/* Skip the residual of a FIXED/LPC subframe (k_parse's cursor walk).  One loop over the
 * subframe's codewords: a lane whose partition is done reads the next partition header
 * (and skips escaped partitions) on a rare path inside the same loop, so lanes whose
 * partitions have different lengths (mixed partition orders in one wave) keep stepping
 * together instead of waiting for the longest partition of every partition index.  The
 * body is predicated (a lane with nothing left advances 0 bits), and the refill counter is
 * read as a scalar (the wave's lanes step together; it only paces refills every 32
 * codewords).  Returns BNF_ST_TRUNC when the walk runs past the buffer.
 * Round 5: the steps move the cursor the way k_decode_st's fused pairs do -- the ring byte
 * address ra carried along (one carry into the slot bits instead of ring_off per read), the
 * landing check once per two steps (a step moves wi by at most one word), and the second
 * codeword's prefix counted in (w << len1) | 1, so no clamp is needed: a window without its
 * stop bit reads as 31 zeros and the pair does not fit. */
DEV uint32_t pk_ra(uint32_t wi, uint32_t lane) { return ((wi & 3u) << 2) | (lane << 4) | (((wi >> 2) & 7u) << 10); }
DEV void pk_resync(BR &b, uint32_t lane) {
    b.ra = pk_ra(b.wi, lane);
    b.vlim = b.vendw - 1u;
}
DEV void pk_next_word(BR &b) { b.nx = *(const lds_u32 *)((const __attribute__((address_space(3))) uint8_t *)b.ring + b.ra); }
DEV void pk_step(BR &b, uint32_t &rem, uint32_t k1, bool &stall, uint32_t laneb) {
    const bool live = rem != 0u;
    const uint32_t w = br_peek(b);
    const uint32_t q1 = min(ffbh_b(w), 32u); /* 32 for an empty window: no fit */
    const uint32_t len1 = q1 + k1;
    const uint32_t q2 = ffbh_b((w << (len1 & 31u)) | 1u);
    const uint32_t len2 = len1 + q2 + k1; /* both codewords: fits iff <= 32 (and the first fits) */
    const bool fit1 = live & (len1 <= 32u);
    const bool fit2 = fit1 & (rem >= 2u) & (len2 <= 32u);
    stall = stall | (live & !fit1);
    const uint32_t n = fit2 ? len2 : (fit1 ? len1 : 0u);
    rem -= fit2 ? 2u : (fit1 ? 1u : 0u);
    uint32_t t;
    const bool c = __builtin_usub_overflow(b.s, n, &t); /* the window moves on a word */
    b.s = t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += (uint32_t)c;
    b.ra = (((b.ra | 0x3F3u) + (uint32_t)c) & 0x1C0Cu) | laneb;
}
/* The bulk step: two codewords of a lane that has plenty left in its partition, nothing but
 * the fit test (nf counts the steps whose pair did not fit: the lane did not move, and it
 * stays put for the iteration's remaining steps, as they see the same window).  (w | 1) keeps
 * the count finite; an empty window reads as 31 zeros, which cannot fit. */
DEV void pkb_step(BR &b, uint32_t k1, uint32_t &nf, uint32_t laneb) {
    const uint32_t w = br_peek(b);
    const uint32_t len1 = (uint32_t)__builtin_clz(w | 1u) + k1;
    const uint32_t n = len1 + (uint32_t)__builtin_clz((w << (len1 & 31u)) | 1u) + k1;
    const bool fit = n <= 32u;
    nf += fit ? 0u : 1u;
    uint32_t t;
    const bool c = __builtin_usub_overflow(b.s, fit ? n : 0u, &t);
    b.s = t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += (uint32_t)c;
    b.ra = (((b.ra | 0x3F3u) + (uint32_t)c) & 0x1C0Cu) | laneb;
}
/* BULK: with the bulk iterations (a separate instance: the plain loop keeps its registers);
 * CP: fold the CRC-16 prefix (crcp_hook) before each refill */
template <bool BULK, bool CP, class C>
DEV uint32_t skip_residual_t(BR &b, const SubHdr &h, uint32_t bs, uint64_t limit, uint32_t ablate, C &cp) {
    const uint32_t parts = 1u << h.porder;
    const uint32_t psamples = h.porder ? bs >> h.porder : bs - h.order;
    const uint32_t plen = h.rice2 ? 5u : 4u, pesc = h.rice2 ? 31u : 15u;
    const uint32_t lane = threadIdx.x & 63u, laneb = lane << 4;
    uint32_t since = BULK ? 16u : 0u, p = 0, rem = 0, k = 0, k1 = 1;
    bool tr = false;
    pk_resync(b, lane);
    while (any_lane(rem != 0u || p < parts)) {
        if (BULK) {
            if (__builtin_amdgcn_readfirstlane(since) >= 12u && !(ablate & 32u)) { /* every 12-14 steps */
                if (CP) crcp_hook(cp, b, lane, b.wi >> 4); /* the lines loaded, before the refill overwrites them */
                br_refill(b);
                pk_resync(b, lane);
                since = 0;
            }
            since += 2u;
        } else if ((__builtin_amdgcn_readfirstlane(since++) & 7u) == 0u && !(ablate & 32u)) { /* every 16 steps */
            if (CP) crcp_hook(cp, b, lane, b.wi >> 4);
            br_refill(b);
            pk_resync(b, lane);
        }
        const bool sw = rem == 0u && p < parts;
        if (__builtin_expect(any_lane(sw), 0)) { /* partition headers (read_residual_partitioned_rice_ @0x10012da0) */
            if (sw) {
                do {
                    if (br_pos(b) > limit) { /* the previous partition ended past the buffer */
                        tr = true;
                        p = parts;
                        break;
                    }
                    const uint32_t kk = br_read(b, plen);
                    const uint32_t cnt = (h.porder == 0 || p > 0) ? psamples : psamples - h.order;
                    p++;
                    if (kk >= pesc) { /* escaped: cnt raw values of nb bits */
                        const uint32_t nb = br_read(b, 5);
                        br_skip(b, (uint64_t)nb * cnt);
                    } else {
                        k = kk;
                        k1 = kk + 1u;
                        rem = cnt; /* 0: the empty first partition (order == partition size) */
                    }
                } while (rem == 0u && p < parts);
            }
            pk_resync(b, lane);
        }
        /* bulk iterations: every lane has 8+ codewords left in its partition and a Rice
         * parameter whose pairs mostly fit one window (C2: all but the partition ends) --
         * four pair steps with the landing check after the first and third; at most three
         * per outer iteration, so one refill paces both (at most 14 steps apart). */
#pragma unroll 1
        for (uint32_t it = 0; BULK && it < 3u && !any_lane(rem < 8u || k1 > 10u); it++) {
            uint32_t nf = 0;
            pkb_step(b, k1, nf, laneb);
            bool ld = b.wi >= b.vlim;
            pk_next_word(b);
            if (__builtin_expect(any_lane(ld), 0)) {
                br_land(b, 1u);
                pk_resync(b, lane);
                pk_next_word(b);
            }
            pkb_step(b, k1, nf, laneb);
            pk_next_word(b);
            pkb_step(b, k1, nf, laneb);
            ld = b.wi >= b.vlim;
            pk_next_word(b);
            if (__builtin_expect(any_lane(ld), 0)) {
                br_land(b, 1u);
                pk_resync(b, lane);
                pk_next_word(b);
            }
            pkb_step(b, k1, nf, laneb);
            pk_next_word(b);
            rem -= 8u - 2u * nf;
            since += 4u;
            if (__builtin_expect(any_lane(nf != 0u), 0)) {
                if (nf) { /* a pair that did not fit: its first codeword alone, generic reader */
                    uint32_t qq;
                    if (br_unary(b, qq, limit)) {
                        br_adv(b, k);
                        rem--;
                    } else {
                        tr = true;
                        rem = 0;
                        p = parts;
                    }
                }
                pk_resync(b, lane);
            }
        }
        if (BULK && !any_lane(rem != 0u || p < parts)) break;
        /* two steps per switch test (a lane that finishes its partition in the first one
         * idles in the second), per landing check and per slow-path test */
        bool stall = false;
        pk_step(b, rem, k1, stall, laneb);
        const bool ld = b.wi >= b.vlim; /* word wi + 1 (the next step's read) not known to have landed */
        pk_next_word(b);
        if (__builtin_expect(any_lane(ld), 0)) {
            br_land(b, 1u);
            pk_resync(b, lane);
            pk_next_word(b);
        }
        pk_step(b, rem, k1, stall, laneb);
        pk_next_word(b);
        if (__builtin_expect(any_lane(stall), 0)) {
            if (stall) { /* a unary prefix too long for the window */
                uint32_t qq;
                if (br_unary(b, qq, limit)) {
                    br_adv(b, k);
                    rem--;
                } else { /* truncated: this lane stops walking */
                    tr = true;
                    rem = 0;
                    p = parts;
                }
            }
            pk_resync(b, lane);
        }
    }
    return (tr || br_pos(b) > limit) ? BNF_ST_TRUNC : BNF_ST_OK;
}
/* The bulk instance when every lane's first partition has a small Rice parameter (k <= 9:
 * pairs of codewords fit a window; C2's k = 8), peeked at the cursor, which sits on that
 * parameter; the plain loop otherwise (C3 / C4: larger parameters, short partitions). */
template <bool CP, class C>
DEV uint32_t skip_residual(BR &b, const SubHdr &h, uint32_t bs, uint64_t limit, uint32_t ablate, C &cp) {
    const uint32_t k0 = br_peek(b) >> (h.rice2 ? 27u : 28u);
    if (!any_lane(k0 > 9u)) return skip_residual_t<true, CP>(b, h, bs, limit, ablate, cp);
    return skip_residual_t<false, CP>(b, h, bs, limit, ablate, cp);
}

/* ------------------------------------------- wave-cooperative Rice boundary scan */
/* Skip `cnt` Rice codewords of parameter k (k + 1 = k1) from the wave-uniform cursor r.pos,
 * with the whole wave on one partition (option ii; north_star's
 * "wavefront prefix-scan for the Rice bit-cursor").  One pass covers 64 stream words: lane i
 * owns the 32 bits of word ws + i (ws = the cursor's word) and can see the next two words.
 *  1. Speculation: every lane decodes codeword lengths from the start of its word (lane 0
 *     from the true cursor), recording the codeword starts it visits in a 32-bit mask and the
 *     first start at or past the word's end (`exit`, relative to the word: 32..94).
 *  2. Splice: lane i's true entry is lane i-1's exit - 32.  A lane whose entry was not its
 *     speculative one re-decodes from it until it lands on a start in its mask (Rice decoding
 *     from a given position is deterministic, so from there the paths coincide) or leaves the
 *     word (its exit changed: the next lane re-checks).  Repeated until no exit changes;
 *     lane 0 is always right, so the loop ends within 64 rounds (in practice 1-3).
 *  3. Count: an inclusive wave scan of the per-lane counts gives the codeword index at every
 *     word; if the partition ends inside the pass, the lane holding its last codeword finds the
 *     end (the next codeword start), otherwise the cursor moves to lane 63's exit.
 * A window of 32 zero bits (a unary prefix >= 32, rare: escapes exist for such values) sends
 * the rest of the partition to a uniform serial walk (wave_rice_skip_serial).  Returns false
 * when that walk runs past `limit` (libFLAC's reader would block: TRUNC). */
DEV bool wave_rice_skip_serial(WR &r, uint32_t cnt, uint32_t k, uint64_t limit) {
    for (; cnt; cnt--) {
        uint32_t q;
        if (!br_unary(r, q, limit)) return false;
        r.pos += k;
    }
    return true;
}
/* DPP lane moves (wave_shr:1 and the row_shr / row_bcast steps of an inclusive wave scan):
 * VALU-latency exchanges instead of ds_bpermute round trips through the LDS queue */
DEV uint32_t dpp_prev(uint32_t x) { /* lane i gets lane i-1's x; lane 0 gets 0 */
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, true);
}
DEV uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true); /* row_shr:1 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true); /* row_shr:2 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true); /* row_shr:4 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true); /* row_shr:8 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); /* row_bcast:15 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); /* row_bcast:31 */
    return x;
}
/* debug counters of the wave scan (k_parse_wave's `stats` argument; BNFLAC_PW_STATS=1):
 * 0 passes, 1 splice rounds, 2 serial fallbacks, 3 partitions, 4 frames, 5 wave-cycles (s_memtime) in scans,
 * 6 of them in window waits, 7 in splices */
__device__ unsigned long long g_pw_stats[8];
DEV void pw_stat(WR &r, bool on, int i, unsigned long long v = 1ull) {
    if (on) r.st[i] += v;
}
DEV void pw_flush(const WR &r, bool on) {
    if (on && (threadIdx.x & 63u) == 0u) {
#pragma unroll
        for (int i = 0; i < 8; i++) atomicAdd(&g_pw_stats[i], (unsigned long long)r.st[i]);
    }
}
/* One lane's segment walk: SW stream words (w[0..SW-1]; w[SW] holds the following word, for
 * prefixes that cross the segment's end).  From bit `pos` (relative to w[0]'s first bit) it
 * measures codeword lengths (q + 1 + k; the k low bits are not read) and sets the start bit of
 * every codeword that starts inside the segment in nm[].  STOP: stop at a start already in om[]
 * (the rest of that path is known).  Unrolled per word so every register index is static.
 * Returns the first start at or past the segment's end (32 SW .. 32 SW + 62), or the stop point. */
template <int SW, bool STOP>
DEV uint32_t seg_walk(const uint32_t (&w)[SW + 1], uint32_t pos, uint32_t k1, uint32_t nsteps, const uint32_t (&om)[SW],
                      uint32_t (&nm)[SW], bool &slow, bool &merged) {
    /* Straight-line, predicated steps (no divergent loop): at most nsteps = floor(31 / k1) + 1
     * codewords start in one word (wave-uniform), so word j runs nsteps steps and a lane whose
     * cursor has left the word (or stopped) advances 0.  A word is skipped when no lane is
     * still inside it. */
#pragma unroll
    for (int j = 0; j < SW; j++) nm[j] = 0u;
    slow = merged = false;
#pragma unroll
    for (int j = 0; j < SW; j++) {
        const uint32_t lo = 32u * (uint32_t)j, hi = lo + 32u;
        if (!any_lane(!merged && !slow && pos < hi)) continue;
        const uint64_t pair = ((uint64_t)w[j] << 32) | w[j + 1];
        for (uint32_t t = 0; t < nsteps; t++) { /* uniform trip count */
            const uint32_t rb = pos - lo; /* in [0, 32) while the cursor is in this word */
            const bool in = !merged && !slow && pos < hi;
            const bool stop = STOP && in && ((om[j] >> (rb & 31u)) & 1u);
            const uint32_t q = ffbh((uint32_t)((pair << (rb & 31u)) >> 32));
            const bool sl = q >= 32u;
            const bool act = in && !stop && !sl;
            nm[j] |= act ? (1u << (rb & 31u)) : 0u;
            pos += act ? q + k1 : 0u;
            merged = merged || stop;
            slow = slow || (in && !stop && sl);
        }
    }
    return pos;
}
/* DEC: also decode the codewords (a wave-cooperative residual decode; round 3's k_decode_wave
 * used it, nothing does now): the values of the partition's codewords go
 * to dst[0 .. cnt) (zig-zag decoded, libFLAC's 32-bit unsigned (q << k) | lsb) -- each lane
 * decodes the codewords whose starts its walk recorded, their lengths known from the next
 * start, the k low bits read from the ring. */
DEV int32_t rice_zigzag(uint32_t u) { return (int32_t)((u >> 1) ^ (0u - (u & 1u))); }
DEV bool wave_rice_serial_dec(WR &r, uint32_t cnt, uint32_t k, uint64_t limit, int32_t *dst) {
    for (uint32_t i = 0; i < cnt; i++) {
        uint32_t q;
        if (!br_unary(r, q, limit)) return false;
        const uint32_t u = (q << k) | br_read(r, k);
        if ((threadIdx.x & 63u) == 0u) dst[i] = rice_zigzag(u);
    }
    return true;
}
template <int SW, bool DEC = false>
DEV bool wave_rice_skip(WR &r, uint32_t cnt, uint32_t k, uint64_t limit, bool stats = false, int32_t *dst = nullptr) {
    constexpr uint32_t SB = 32u * SW; /* bits per lane per pass */
    const uint32_t lane = threadIdx.x & 63u, k1 = k + 1u;
    pw_stat(r, stats, 3);
    while (cnt) {
        pw_stat(r, stats, 0);
        const uint64_t p = r.pos;
        if (p > limit) return true; /* the caller reports TRUNC from the position */
        const uint32_t ws = wr_u((uint32_t)(p >> 5)), e0 = (uint32_t)p & 31u;
        const uint64_t tw0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        wr_need(r, ws, ws + 64u * SW + (DEC ? 1u : 0u)); /* DEC: a last codeword's low bits may reach one word further */
        if (stats) pw_stat(r, true, 6, __builtin_amdgcn_s_memtime() - tw0);
        uint32_t w[SW + 2]; /* w[SW + 1]: only DEC reads it (a last codeword's low bits) */
#pragma unroll
        for (int j = 0; j <= SW + (DEC ? 1 : 0); j++) w[j] = wr_word(r, ws + SW * lane + (uint32_t)j);
        /* 1. speculative walk of this lane's segment from its first bit (lane 0: the cursor).
         * `slow` only matters if the lane turns out to lie inside the partition. */
        uint32_t ent = lane ? 0u : e0;
        uint32_t m[SW];
        bool slow, merged;
        const uint32_t nsteps = 31u / k1 + 1u; /* codeword starts per word, at most */
        uint32_t none[SW];
#pragma unroll
        for (int j = 0; j < SW; j++) none[j] = 0u;
        uint32_t exit = seg_walk<SW, false>((const uint32_t(&)[SW + 1])w, ent, k1, nsteps, none, m, slow, merged);
        if (slow) exit = SB;
        /* 2. splice: a lane whose true entry (the previous lane's exit - SB) differs re-walks
         * from it until it meets a start of its own walk (the paths coincide from there) or
         * leaves the segment (its exit changed: the next lane re-checks) */
        const uint64_t ts0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
        for (;;) {
            const uint32_t pe = dpp_prev(exit); /* all lanes active: a DPP read of a lane outside exec yields 0 */
            const uint32_t te = lane ? pe - SB : e0;
            const bool redo = te != ent;
            if (!any_lane(redo)) break;
            pw_stat(r, stats, 1);
            if (redo) {
                if (te >= SB) { /* the previous lane's last codeword covers this segment */
#pragma unroll
                    for (int j = 0; j < SW; j++) m[j] = 0u;
                    exit = te;
                    slow = false;
                } else {
                    uint32_t nm[SW];
                    bool s2, mg;
                    const uint32_t pos = seg_walk<SW, true>((const uint32_t(&)[SW + 1])w, te, k1, nsteps, m, nm, s2, mg);
                    if (mg) { /* merged at pos: the old starts from pos on, its exit and slow flag hold */
#pragma unroll
                        for (int j = 0; j < SW; j++) {
                            const uint32_t lo = 32u * (uint32_t)j;
                            const uint32_t keep = pos <= lo ? ~0u : (pos >= lo + 32u ? 0u : (~0u << (pos - lo)));
                            m[j] = nm[j] | (m[j] & keep);
                        }
                    } else {
#pragma unroll
                        for (int j = 0; j < SW; j++) m[j] = nm[j];
                        exit = s2 ? SB : pos;
                        slow = s2;
                    }
                }
                ent = te;
            }
        }
        if (stats) pw_stat(r, true, 7, __builtin_amdgcn_s_memtime() - ts0);
        /* 3. count */
        uint32_t n = 0;
#pragma unroll
        for (int j = 0; j < SW; j++) n += (uint32_t)__builtin_popcount(m[j]);
        const uint32_t incl = wave_incl_scan(n);
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t L = total >= cnt ? wr_u((uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(incl >= cnt))) : 63u;
        /* a slow lane at or before the last lane that matters: measure this partition serially */
        if (__builtin_amdgcn_ballot_w64(slow && lane <= L)) {
            pw_stat(r, stats, 2);
            return DEC ? wave_rice_serial_dec(r, cnt, k, limit, dst) : wave_rice_skip_serial(r, cnt, k, limit);
        }
        if (DEC) { /* this lane's codewords with index < cnt, in stream order */
            uint32_t after[SW]; /* the first start in a later word of the segment, or the exit */
            uint32_t nf = exit;
#pragma unroll
            for (int j = SW - 1; j >= 0; j--) {
                after[j] = nf;
                if (m[j]) nf = 32u * (uint32_t)j + (uint32_t)__builtin_ctz(m[j]);
            }
            uint32_t i = incl - n;
#pragma unroll
            for (int j = 0; j < SW; j++) {
                /* a codeword starting in word j ends (its k low bits) within words j .. j + 2 */
                const uint64_t p01 = ((uint64_t)w[j] << 32) | w[j + 1], p12 = ((uint64_t)w[j + 1] << 32) | w[j + 2];
                uint32_t mm = m[j];
                while (mm && i < cnt) {
                    const uint32_t pos = (uint32_t)__builtin_ctz(mm);
                    mm &= mm - 1u;
                    const uint32_t next = mm ? (uint32_t)__builtin_ctz(mm) : after[j] - 32u * (uint32_t)j; /* from word j */
                    const uint32_t q = next - pos - k1, g = next - k; /* the k low bits end at the next start */
                    const uint64_t pp = g >= 32u ? p12 : p01;
                    const uint32_t bits = (uint32_t)((pp << (g & 31u)) >> 32);
                    const uint32_t lsb = k ? bits >> (32u - k) : 0u;
                    dst[i] = rice_zigzag((q << k) | lsb);
                    i++;
                }
            }
        }
        if (total < cnt) {
            cnt -= total;
            if (DEC) dst += total;
            r.pos = ((uint64_t)(ws + SW * 63u) << 5) + __builtin_amdgcn_readlane(exit, 63);
            continue;
        }
        /* the lane holding codeword #cnt; its end is the next codeword start */
        uint32_t endpos = exit;
        if (lane == L) {
            uint32_t j = cnt - (incl - n) + 1u; /* 1-based index of the start after the partition's last codeword */
            bool found = false;
#pragma unroll
            for (int t = 0; t < SW; t++) {
                const uint32_t c = (uint32_t)__builtin_popcount(m[t]);
                if (!found && j <= c) {
                    uint32_t mm = m[t];
                    for (uint32_t d = j; d > 1u; d--) mm &= mm - 1u;
                    endpos = 32u * (uint32_t)t + (uint32_t)__builtin_ctz(mm);
                    found = true;
                }
                if (!found) j -= c;
            }
        }
        r.pos = ((uint64_t)(ws + SW * L) << 5) + __builtin_amdgcn_readlane(endpos, L);
        cnt = 0;
    }
    return true;
}
/* skip_residual for the wave-uniform reader: partition headers read at the uniform cursor,
 * each partition's codewords skipped by the wave scan (same TRUNC/OK outcomes as the lane walk) */
/* Pass width for a partition: lane segments of SW words, so that one pass of 64 lanes (2048 SW
 * bits) covers about the whole partition -- a short partition (C2: ~2,600 bits) would waste a
 * wide pass, a long one (C5: ~60,000 bits) would pay per-pass overheads many times.  seg > 0
 * forces a width (BNFLAC_PW_SEG, experiments). */
DEV bool wave_rice_skip_any(WR &r, uint32_t cnt, uint32_t k, uint64_t limit, bool stats, int seg) {
    const uint32_t est = cnt * (k + 2u); /* bits, at about one unary zero per codeword */
    const int sw = seg > 0 ? seg : est > 6u * 2048u ? 16 : est > 3u * 2048u ? 8 : est > 3u * 1024u ? 4 : est > 1536u ? 2 : 1;
    switch (sw) {
    case 1: return wave_rice_skip<1>(r, cnt, k, limit, stats);
    case 2: return wave_rice_skip<2>(r, cnt, k, limit, stats);
    case 4: return wave_rice_skip<4>(r, cnt, k, limit, stats);
    case 8: return wave_rice_skip<8>(r, cnt, k, limit, stats);
    default: return wave_rice_skip<16>(r, cnt, k, limit, stats);
    }
}
/* a partition decode (DEC) at the pass width wave_rice_skip_any picks */
DEV bool wave_rice_dec_any(WR &r, uint32_t cnt, uint32_t k, uint64_t limit, int32_t *dst) {
    const uint32_t est = cnt * (k + 2u);
    const int sw = est > 6u * 2048u ? 16 : est > 3u * 2048u ? 8 : est > 3u * 1024u ? 4 : est > 1536u ? 2 : 1;
    switch (sw) {
    case 1: return wave_rice_skip<1, true>(r, cnt, k, limit, false, dst);
    case 2: return wave_rice_skip<2, true>(r, cnt, k, limit, false, dst);
    case 4: return wave_rice_skip<4, true>(r, cnt, k, limit, false, dst);
    case 8: return wave_rice_skip<8, true>(r, cnt, k, limit, false, dst);
    default: return wave_rice_skip<16, true>(r, cnt, k, limit, false, dst);
    }
}
/* cnt signed raw values of nb bits (an escaped partition, a VERBATIM subframe) into dst,
 * 64 at a time (one value per lane) */
DEV void wave_read_raw(WR &r, uint32_t cnt, uint32_t nb, int32_t *dst) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t base = r.pos;
    for (uint32_t i0 = 0; i0 < cnt; i0 += 64u) {
        const uint64_t b0 = base + (uint64_t)i0 * nb;
        const uint32_t wa = (uint32_t)(b0 >> 5), wb = (uint32_t)((b0 + 64ull * nb) >> 5) + 1u;
        wr_need(r, wa, wb);
        const uint32_t i = i0 + lane;
        const uint64_t bit = b0 + (uint64_t)lane * nb;
        const uint32_t w = (uint32_t)(bit >> 5), sh = (uint32_t)bit & 31u;
        const uint32_t hi = wr_word(r, w), lo = wr_word(r, w + 1u);
        const uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, 32u - sh) : hi;
        const uint32_t s = (32u - nb) & 31u;
        if (i < cnt) dst[i] = nb ? (int32_t)((v >> s) << s) >> s : 0;
    }
    r.pos = base + (uint64_t)cnt * nb;
}
/* Small partitions (round 5): a wave pass costs about the same whatever the partition size
 * (window loads, the speculative walk, ~4 splice rounds), so a subframe of 256 partitions of
 * 16 codewords paid 256 passes -- one C5 file whose encoder picked high partition orders took
 * 0.85 ms to parse against 0.32 ms for the others, and set the 8-file launch at 0.96 ms
 * (tools/c5_parse_ab.py).  Below PW_SCALAR_MAX samples per partition the whole residual is
 * walked by the scalar unit instead: 64 stream words sit one per lane in a VGPR, the cursor is
 * an SGPR, each codeword is two v_readlane, a 64-bit scalar shift, s_flbit and an add, and the
 * partition headers are read the same way.  Same positions, TRUNC and slow-prefix rules as the
 * pass (a window of 32 zero bits goes to br_unary). */
#define PW_SCALAR_MAX 64u
struct SWin { /* 64 stream words [base, base + 64) held one per lane */
    uint32_t base, v;
};
DEV void swin_load(WR &r, SWin &s, uint32_t wi) {
    s.base = wr_u(wi);
    wr_need(r, s.base, s.base + 64u);
    s.v = wr_word(r, s.base + (threadIdx.x & 63u));
}
/* the 32 bits at bit position pos (the window reloaded when pos leaves it) */
DEV uint32_t swin_peek(WR &r, SWin &s, uint64_t pos) {
    uint32_t wi = wr_u((uint32_t)(pos >> 5));
    if (wi < s.base || wi + 1u >= s.base + 64u) swin_load(r, s, wi);
    const uint32_t i = wi - s.base, sh = (uint32_t)pos & 31u;
    const uint32_t hi = __builtin_amdgcn_readlane(s.v, i), lo = __builtin_amdgcn_readlane(s.v, i + 1u);
    /* the shift-0 case apart: the 64-bit form compiled to a funnel shift that returned the
     * low word at a word-aligned cursor */
    return sh ? __builtin_amdgcn_alignbit(hi, lo, 32u - sh) : hi;
}
DEV uint32_t wave_skip_residual_scalar(WR &r, const SubHdr &h, uint32_t bs, uint64_t limit) {
    const uint32_t parts = 1u << h.porder;
    const uint32_t psamples = h.porder ? bs >> h.porder : bs - h.order;
    const uint32_t plen = h.rice2 ? 5u : 4u, pesc = h.rice2 ? 31u : 15u;
    SWin s;
    swin_load(r, s, wr_u((uint32_t)(r.pos >> 5)));
    uint64_t pos = r.pos;
    for (uint32_t p = 0; p < parts; p++) {
        if (pos > limit) break; /* the previous partition ended past the buffer */
        const uint32_t kk = swin_peek(r, s, pos) >> (32u - plen);
        pos += plen;
        uint32_t cnt = (h.porder == 0 || p > 0) ? psamples : psamples - h.order;
        if (kk >= pesc) {
            const uint32_t nb = swin_peek(r, s, pos) >> 27;
            pos += 5u + (uint64_t)nb * cnt;
            continue;
        }
        const uint32_t k1 = kk + 1u;
        while (cnt) {
            if (pos > limit) break;
            const uint32_t w = swin_peek(r, s, pos);
            if (w == 0u) { /* a unary prefix longer than the window: the generic reader */
                r.pos = pos;
                uint32_t q;
                if (!br_unary(r, q, limit)) return BNF_ST_TRUNC;
                pos = r.pos + kk;
                cnt--;
                swin_load(r, s, wr_u((uint32_t)(pos >> 5)));
                continue;
            }
            const uint32_t la = (uint32_t)__builtin_clz(w) + k1;
            /* a second codeword in the same window when both fit */
            const uint32_t w2 = la < 32u ? (w << la) : 0u;
            const uint32_t lb = w2 ? (uint32_t)__builtin_clz(w2) + k1 : 64u;
            if (cnt >= 2u && la + lb <= 32u) {
                pos += la + lb;
                cnt -= 2u;
            } else {
                pos += la;
                cnt--;
            }
        }
    }
    r.pos = pos;
    return pos > limit ? BNF_ST_TRUNC : BNF_ST_OK;
}
DEV uint32_t wave_skip_residual(WR &r, const SubHdr &h, uint32_t bs, uint64_t limit, bool stats, int seg) {
    const uint32_t parts = 1u << h.porder;
    const uint32_t psamples = h.porder ? bs >> h.porder : bs - h.order;
    const uint32_t plen = h.rice2 ? 5u : 4u, pesc = h.rice2 ? 31u : 15u;
    if (psamples <= PW_SCALAR_MAX && seg >= 0) return wave_skip_residual_scalar(r, h, bs, limit);
    for (uint32_t p = 0; p < parts; p++) {
        if (br_pos(r) > limit) return BNF_ST_TRUNC; /* the previous partition ended past the buffer */
        const uint32_t kk = wr_u(br_read(r, plen));
        const uint32_t cnt = (h.porder == 0 || p > 0) ? psamples : psamples - h.order;
        if (kk >= pesc) {
            const uint32_t nb = wr_u(br_read(r, 5));
            r.pos += (uint64_t)nb * cnt;
        } else if (cnt && !wave_rice_skip_any(r, cnt, kk, limit, stats, seg)) {
            return BNF_ST_TRUNC;
        }
    }
    return br_pos(r) > limit ? BNF_ST_TRUNC : BNF_ST_OK;
}

#if BNF_TU == 0
/* =============================================================== k_sync_scan */
#define SCAN_BYTES_PER_THREAD 16
#define SCAN_THREADS 256

DEV bool is_sync(const uint8_t *__restrict__ d, uint64_t n, uint64_t p) {
    return p + 1 < n && d[p] == 0xFF && (d[p + 1] >> 2) == 0x3E;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_sync_count(const uint8_t *__restrict__ d, uint64_t n,
                                                             uint32_t *__restrict__ block_counts) {
    __shared__ uint32_t red[SCAN_THREADS / 64];
    uint64_t base = ((uint64_t)blockIdx.x * SCAN_THREADS + threadIdx.x) * SCAN_BYTES_PER_THREAD;
    uint32_t c = 0;
    for (int i = 0; i < SCAN_BYTES_PER_THREAD; i++) c += is_sync(d, n, base + i) ? 1u : 0u;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int i = 0; i < SCAN_THREADS / 64; i++) s += red[i];
        block_counts[blockIdx.x] = s;
    }
}

/* single-workgroup exclusive scan (in place), total in *total */
__global__ void __launch_bounds__(1024) k_scan_u32(uint32_t *__restrict__ v, uint32_t n, uint32_t *__restrict__ total) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 1024) {
        uint32_t i = base + threadIdx.x;
        uint32_t x = i < n ? v[i] : 0u;
        uint32_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(incl, o);
            if ((threadIdx.x & 63) >= (unsigned)o) incl += y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        if (threadIdx.x < 16) {
            uint32_t s = wsum[threadIdx.x];
            for (int o = 1; o < 16; o <<= 1) {
                uint32_t y = __shfl_up(s, o, 16);
                if (threadIdx.x >= (unsigned)o) s += y;
            }
            wsum[threadIdx.x] = s;
        }
        __syncthreads();
        uint32_t wprefix = (threadIdx.x >= 64) ? wsum[(threadIdx.x >> 6) - 1] : 0u;
        if (i < n) v[i] = carry + wprefix + incl - x;
        __syncthreads();
        if (threadIdx.x == 1023) carry += wprefix + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_sync_write(const uint8_t *__restrict__ d, uint64_t n,
                                                             const uint32_t *__restrict__ block_offs,
                                                             uint64_t *__restrict__ out, uint32_t cap) {
    __shared__ uint32_t wtot[SCAN_THREADS / 64];
    uint64_t base = ((uint64_t)blockIdx.x * SCAN_THREADS + threadIdx.x) * SCAN_BYTES_PER_THREAD;
    uint32_t c = 0;
    for (int i = 0; i < SCAN_BYTES_PER_THREAD; i++) c += is_sync(d, n, base + i) ? 1u : 0u;
    uint32_t incl = c;
    const uint32_t lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o);
        if (lane >= (unsigned)o) incl += y;
    }
    if (lane == 63) wtot[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t wpre = 0;
    for (uint32_t wv = 0; wv < (threadIdx.x >> 6); wv++) wpre += wtot[wv];
    uint32_t pos = block_offs[blockIdx.x] + wpre + incl - c;
    for (int i = 0; i < SCAN_BYTES_PER_THREAD; i++) {
        if (is_sync(d, n, base + i)) {
            if (pos < cap) out[pos] = base + i;
            pos++;
        }
    }
}

/* ==================================================================== k_parse */
#define PARSE_RD 8 /* ring slots per lane (8 KB of LDS per wave, 5 waves per SIMD) */
static_assert(PARSE_RD == 8, "pk_ra and the walk's pair steps (slot masks 0x3F3 / 0x1C0C, slot bits 10-12) assume an 8-slot ring");
/* One lane per candidate frame: header + cursor walk over subframes 0..C-2.  Also
 * flags frames with an LPC order above 8 (they go to k_decode<32>). */
template <int CPM> /* the CRC-16 hand-off (crc_mode): 1 the prefix, 2 the prefix and the verdict */
DEV void parse_frame(const uint32_t *__restrict__ words, uint64_t nbytes, const uint64_t *__restrict__ frame_offs,
                     uint32_t nframes, const bnf_stream_params &sp, const uint64_t *__restrict__ out_sample_in,
                     uint64_t base_sample, bnf_frame_info *__restrict__ info, uint32_t ablate, lds_u32 *ring,
                     uint32_t f, uint32_t *__restrict__ crcp) {
    if (f >= nframes) return;
    bnf_frame_info fi;
    fi.status = BNF_ST_OK;
    fi.err = -1;
    fi.frame_off = frame_offs[f];
    fi.resume_bit = 0;
    fi.cached = -1;
    fi.blocksize = fi.sample_rate = fi.channels = fi.assignment = fi.bps = 0;
    fi.number_type = 0;
    fi.unparseable = 0;
    fi.number = 0;
    fi.out_sample = 0;
    fi.crc8 = fi.crc16_calc = fi.crc16_read = fi.crc_ok = 0;
    fi.flags = 0;
    fi.reserved = 0;
    /* sub_start is kept in registers and written by select chains: indexing fi.sub_start
     * with the runtime channel would put the whole record in scratch */
    uint32_t ss[8];
#pragma unroll
    for (int c = 0; c < 8; c++) ss[c] = 0;
    const uint64_t limit = nbytes * 8u;
    const uint64_t fbit = fi.frame_off * 8u;
    BR b;
    br_init(b, words, nbytes, ring, threadIdx.x, PARSE_RD);
    CrcP cp; /* the CRC-16 prefix of a 2-channel frame (crcp != nullptr: the batch decode's hand-off) */
    crcp_init(cp);
    uint32_t st = parse_header(b, fbit, limit, sp, fi);
    if (st == BNF_ST_ERROR && br_pos(b) > limit) st = BNF_ST_TRUNC;
    if (CPM && crcp != nullptr && st == BNF_ST_OK && fi.channels == 2u && !(ablate & 16u)) {
        /* the frame's first line, its bytes below frame_off cleared (L2-warm: the ring's
         * refill just read it) */
        const uint32_t h = (uint32_t)(fi.frame_off & 63u);
        const u32x4 *g = (const u32x4 *)((const uint8_t *)words + (fi.frame_off & ~(uint64_t)63u));
        u32x4 v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            v[i] = g[i];
            v[i].x &= st_hmask(h, 16u * i);
            v[i].y &= st_hmask(h, 16u * i + 4u);
            v[i].z &= st_hmask(h, 16u * i + 8u);
            v[i].w &= st_hmask(h, 16u * i + 12u);
        }
        cp.wc = (uint32_t)(fi.frame_off >> 6);
        crcp_fold(cp, v);
    }
    if (st == BNF_ST_OK) {
        /* position in the batch output */
        uint64_t sample;
        if (fi.number_type == 1) sample = fi.number;
        else if (sp.has_stream_info && sp.min_blocksize == sp.max_blocksize) sample = (uint64_t)sp.min_blocksize * fi.number;
        else sample = (uint64_t)fi.blocksize * fi.number;
        fi.out_sample = out_sample_in ? out_sample_in[f] : sample - base_sample;
        uint32_t maxorder = 0;
        bool raw = false; /* a CONSTANT or VERBATIM subframe: k_decode_st would hand the frame back */
        for (uint32_t ch = 0; ch < fi.channels; ch++) {
            const uint32_t here = (uint32_t)(br_pos(b) - fbit);
#pragma unroll
            for (int c = 0; c < 8; c++) ss[c] = (uint32_t)c == ch ? here : ss[c];
            if (ch + 1 == fi.channels) {
                /* the last subframe is walked by k_decode; only peek at its type byte */
                const uint32_t x = br_peek(b) >> 24;
                if (!(x & 0x80u) && (x & 0x7Eu) >= 0x40u) maxorder = max(maxorder, ((x >> 1) & 31u) + 1u);
                raw = raw || (x & 0x7Eu) < 4u;
                break;
            }
            if (ablate & 16u) {
#pragma unroll
                for (int c = 0; c < 8; c++) ss[c] = (uint32_t)c == ch + 1 ? here : ss[c];
                continue;
            }
            SubHdr h;
            int32_t err = -1;
            uint32_t bps = sub_bps(fi, ch);
            st = parse_subframe_head<false>(b, bps, fi.blocksize, limit, h, nullptr, nullptr, err);
            if (st == BNF_ST_OK) {
                if (h.type == T_LPC) maxorder = max(maxorder, h.order);
                raw = raw || h.type == T_CONST || h.type == T_VERB;
                /* the prefix only for the frames k_decode_st / k_decode_sw can take */
                if (!(h.type == T_FIXED || h.type == T_LPC) || h.order > (fi.bps > 16u ? 12u : 8u)) cp.wc = ~0u;
                if (h.type == T_VERB) br_skip(b, (uint64_t)h.bps * fi.blocksize);
                else if (h.type == T_FIXED || h.type == T_LPC) st = skip_residual<CPM != 0>(b, h, fi.blocksize, limit, ablate, cp);
                if (st == BNF_ST_OK && br_pos(b) > limit) st = BNF_ST_TRUNC;
            }
            if (st == BNF_ST_ERROR && br_pos(b) > limit) st = BNF_ST_TRUNC;
            if (st != BNF_ST_OK) {
                if (st == BNF_ST_ERROR) {
                    fi.err = err;
                    fi.resume_bit = br_pos(b);
                }
                break;
            }
        }
        /* decode instance: LPC orders above 16 -> k_decode<32>; 9..16, or LPC at more than 16
         * bits (libFLAC's 64-bit restore is then the usual path) -> k_decode<16>; 16-bit stereo
         * with FIXED/LPC subframes only -> k_decode_st; the rest -> k_decode<8> */
        if (maxorder > 16) fi.flags |= BNF_FL_W32;
        else if (maxorder > 8 || (maxorder > 0 && fi.bps > 16)) fi.flags |= BNF_FL_W16;
        else if (fi.channels == 2 && fi.bps <= 16 && !raw) fi.flags |= BNF_FL_ST;
        if (maxorder > 0 && maxorder <= 12 && fi.channels == 2 && fi.bps > 16 && fi.bps <= 24 && !raw) fi.flags |= BNF_FL_SW;
    }
    fi.status = st;
#pragma unroll
    for (int c = 0; c < 8; c++) fi.sub_start[c] = ss[c];
    info[f] = fi;
    if (CPM && crcp) { /* the hand-off (CRCP_WORDS) to the k_decode_st / k_decode_sw tails */
        u32x4 o = u32x4{0u, 0u, 0u, 0u}, o2 = u32x4{0u, 0u, 0u, 0u};
        const uint32_t l1 = (uint32_t)(br_pos(b) >> 9); /* subframe 1's line */
        if (cp.wc != ~0u && st == BNF_ST_OK) {
            crcp_hook<true>(cp, b, threadIdx.x & 63u, l1); /* every line before subframe 1's line (or more) */
            const CrcZ z = crcp_z(cp);
            o = u32x4{z.r0, (z.r1 & 0x0FFFFFFFu) | ((uint32_t)(__builtin_popcount(z.px) & 1) << 31),
                      cp.wc - (uint32_t)(fi.frame_off >> 6) + 1u, (uint32_t)fi.frame_off};
            /* the rest up to the next frame's offset: where a frame of a contiguous batch ends
             * (frame + footer), so its tail need not read the frame again */
            const uint64_t nx = CPM == 2 && f + 1u < nframes ? frame_offs[f + 1u] : 0u;
            if (CPM == 2 && nx >= (uint64_t)cp.wc * 64u && nx <= nbytes && nx - fi.frame_off < (1u << 24))
                o2 = u32x4{(uint32_t)(nx - fi.frame_off),
                           st_crc16_ok<2>((const uint8_t *)words, fi.frame_off, nx, z, (uint64_t)cp.wc * 64u) ? 1u : 0u,
                           (uint32_t)fi.frame_off, 0u};
        }
        *(u32x4 *)(crcp + CRCP_WORDS * (uint64_t)f) = o;
        *(u32x4 *)(crcp + CRCP_WORDS * (uint64_t)f + 4u) = o2;
    }
}

#endif /* BNF_TU == 0 */

/* ================================================================== k_decode */
#define DEC_LANES 64
#define RP 72 /* row-buffer stride (dwords) between samples: [sample][lane]; 4*RP = 32 mod 64 banks */

struct RS { /* residual reader state */
    uint32_t verb;   /* 1: VERBATIM raw values of `k` bits */
    uint32_t k, esc, left, pidx, nparts, psamples, order, plen, pesc, porder;
};

/* Rice partition header (read_residual_partitioned_rice_ @0x10012da0) */
template <bool CHECK = true>
DEV void read_partition(BR &b, RS &s) {
    const uint32_t kk = br_read<CHECK>(b, s.plen);
    s.left = (s.porder == 0 || s.pidx > 0) ? s.psamples : s.psamples - s.order;
    if (kk < s.pesc) {
        s.k = kk;
        s.esc = 0;
    } else {
        s.k = br_read<CHECK>(b, 5);
        s.esc = 1;
    }
    s.pidx++;
}

/* One Rice codeword (the block reader @0x10001b30/@0x1001aed0: u = (q << k) | lsb in
 * 32-bit unsigned, zig-zag). */
template <bool CHECK = true> /* false: the caller made sure the ring holds the word this reads */
DEV int32_t rice_one(BR &b, uint32_t k, uint64_t limit, uint32_t &trunc, PendW *pw = nullptr) {
    const uint32_t w = br_peek(b);
    /* v_ffbh gives ~0u for w == 0, which fails the unsigned test below like any prefix
     * too long for the window: the slow path then reads it */
    const uint32_t q0 = ffbh(w);
    const bool fast = q0 <= 31u - k;
    uint32_t u = (q0 << k) | __builtin_amdgcn_ubfe(w, 31u - k - q0, k);
    const bool slow = any_lane(!fast); /* wave-uniform, taken before the advance (stays in SGPRs) */
    br_adv<CHECK>(b, fast ? q0 + 1u + k : 0u, pw);
    if (__builtin_expect(slow, 0)) { /* the work is per lane */
        STAT(b.stats, 3);
        if (!fast) { /* long unary prefix: read_unary_unsigned, then the k low bits */
            uint32_t q;
            if (!br_unary(b, q, limit)) trunc = 1;
            u = (q << k) | br_read(b, k);
        }
    }
    return (int32_t)((u >> 1) ^ (0u - (u & 1u)));
}

/* next residual on the fused paths: a new partition's header and escaped (raw) partitions
 * inline behind wave-uniform tests, so a chunk need not lie inside one partition; Rice
 * codewords as rice_one.  An escaped lane issues its pending row write itself. */
DEV int32_t rice_fused(BR &b, RS &rs, uint64_t limit, uint32_t &trunc, PendW *pw) {
    /* one landing check per residual: with words wi .. wi+2 in the landed ring, the up to two
     * partition headers and one value below (<= 49 bits) advance unchecked; only a long
     * unary prefix (rice_one's slow path) reads on with checks */
    if (__builtin_expect(any_lane(b.wi + 2u >= b.vendw), 0)) {
        br_land(b, 2u);
        b.nx = ring_word(b, b.wi);
    }
    const bool np = rs.left == 0;
    if (__builtin_expect(any_lane(np), 0)) {
        if (np) {
            do { /* partition 0 holds no samples when the order equals the partition size */
                if (rs.pidx < rs.nparts) {
                    read_partition<false>(b, rs);
                } else { /* more samples than the partitions carry: a damaged frame */
                    trunc = 1;
                    rs.left = 0x7fffffffu;
                }
            } while (rs.left == 0);
        }
    }
    rs.left--;
    if (__builtin_expect(any_lane(rs.esc != 0u), 0)) {
        if (rs.esc) {
            if (pw && pw->on) *pw->at = pw->v;
            if (pw) pw->on = false;
            return br_read_s<false>(b, rs.k);
        }
    }
    return rice_one<false>(b, rs.k, limit, trunc, pw);
}

DEV void finish_partitions(BR &b, RS &s) {
    if (s.verb) return;
    while (s.pidx < s.nparts) {
        uint32_t kk = br_read(b, s.plen);
        if (kk >= s.pesc) br_read(b, 5);
        s.pidx++;
    }
}

/* saturate to int16 (packssdw) / the low 16 bits as int16 (MMX16 history words) */
DEV int32_t sat16(int32_t x) { return (int32_t)(int16_t)min(max(x, -32768), 32767); }
DEV int32_t tr16(int32_t x) { return (int32_t)(int16_t)(uint16_t)(uint32_t)x; }
/* ---------------------------------------------------------------- k_decode restore
 * Every subframe type is restored as one linear predictor over 32-bit samples, so a wave
 * whose lanes hold different types and libFLAC paths runs ONE instruction stream:
 *   - libFLAC's 32-bit paths (the ia32 routine @0x1001be10, the MMX16 one @0x1001c000)
 *     both compute the low 32 bits of sum c[t] * x[t] -- MMX16 on history that is saturated
 *     to int16 (taps 4..) or truncated to int16 (taps 0..3, the last pmaddwd pair), ia32 in
 *     int32 wrap -- and shift that (psrad: >= 32 -> 31; sar: & 31);
 *   - the 64-bit path (FLAC__lpc_restore_signal_wide @0x10006120) shifts the exact sum;
 *   - FIXED order o (FLAC__fixed_restore_signal @0x10003810, int32 wrap) is LPC with coefficients
 *     1 | 2,-1 | 3,-3,1 | 4,-6,4,-1 and shift 0; CONSTANT is order 1, coefficient 1,
 *     warm-up cval and zero residuals; VERBATIM is order 0 with the raw values as residuals.
 * Per sample: W exact 64-bit MACs (v_mad_i64_i32, tools/ubench_mad.hip) in two chains, the
 * history in a register ring with compile-time indices (W samples unrolled by recursion). */
struct Pred {
    int32_t sh;       /* effective shift of the lane's path */
    uint32_t order;   /* samples before it are warm-ups (raw in the rows) */
    uint32_t wasted;  /* output = sample << wasted */
    bool mmx, wide;
};

/* the prediction of the sample at ring position T from the W history values; only the
 * first NT taps (the wave's coefficients past NT are all zero: NT covers its largest order) */
template <int T, int W, int NT>
DEV int32_t pred_at(const int32_t (&c)[W], const int32_t (&x)[W], const int32_t (&xt)[4], const Pred &p) {
    int64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int t = 0; t < NT; t++) {
        const int32_t hv = (t < 4) ? xt[(T - 1 - t) & 3] : x[((T - 1 - t) % W + W) % W];
        if (t & 1) s1 += (int64_t)c[t] * (int64_t)hv;
        else s0 += (int64_t)c[t] * (int64_t)hv;
    }
    /* keep the two MAC chains apart (the compiler would re-associate them into one) */
    asm volatile("" : "+v"(s0), "+v"(s1));
    const int64_t S = s0 + s1;
    return p.wide ? (int32_t)(S >> p.sh) : ((int32_t)S >> p.sh);
}
template <int T, int W>
DEV void push_at(int32_t (&x)[W], int32_t (&xt)[4], const Pred &p, int32_t s) {
    x[T % W] = p.mmx ? sat16(s) : s;
    xt[T & 3] = p.mmx ? tr16(s) : s;
}

/* split path, samples T..W-1 of the W-sample group at row j (rows hold warm-ups /
 * residuals on entry, output samples on exit); n = subframe sample index of row j */
template <int T, int W, int NT>
DEV void restore_steps(int32_t *row, const int32_t (&c)[W], int32_t (&x)[W], int32_t (&xt)[4], const Pred &p,
                       uint32_t n, uint32_t nv, uint32_t j) {
    if constexpr (T < W) {
        const int32_t v = row[(j + T) * RP];
        const int32_t pr = pred_at<T, W, NT>(c, x, xt, p);
        const int32_t s = (n + (uint32_t)T < p.order) ? v : (int32_t)((uint32_t)v + (uint32_t)pr);
        push_at<T, W>(x, xt, p, s);
        if (j + (uint32_t)T < nv) row[(j + T) * RP] = (int32_t)((uint32_t)s << p.wasted);
        restore_steps<T + 1, W, NT>(row, c, x, xt, p, n, nv, j);
    }
}

/* fused path (a full chunk past the warm-up): each residual goes from the bit reader
 * straight into the predictor, so the bit-cursor chain and the MAC chains of neighbouring
 * samples overlap; each row write is issued in the next codeword's cursor advance */
template <int T, int W, int NT>
DEV void fused_steps(BR &b, RS &rs, int32_t *row, const int32_t (&c)[W], int32_t (&x)[W], int32_t (&xt)[4],
                     const Pred &p, uint64_t limit, uint32_t &trunc, PendW &pw, uint32_t j) {
    if constexpr (T < W) {
        const int32_t r = rice_fused(b, rs, limit, trunc, &pw);
        const int32_t s = (int32_t)((uint32_t)r + (uint32_t)pred_at<T, W, NT>(c, x, xt, p));
        push_at<T, W>(x, xt, p, s);
        pw.v = (int32_t)((uint32_t)s << p.wasted);
        pw.at = row + (j + T) * RP;
        pw.on = true;
        fused_steps<T + 1, W, NT>(b, rs, row, c, x, xt, p, limit, trunc, pw, j);
    }
}
template <int CH, int W, int NT>
DEV void fused_chunk(BR &b, RS &rs, int32_t *row, const int32_t (&c)[W], int32_t (&x)[W], int32_t (&xt)[4],
                     const Pred &p, uint64_t limit, uint32_t &trunc) {
    PendW pw;
    pw.at = row;
    pw.v = 0;
    pw.on = false;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)CH; j += W) fused_steps<0, W, NT>(b, rs, row, c, x, xt, p, limit, trunc, pw, j);
    *pw.at = pw.v;
}

/* restore one chunk of CH rows (nv of them valid), W-sample groups */
template <int CH, int W, int NT>
DEV void restore_chunk(int32_t *row, const int32_t (&c)[W], int32_t (&x)[W], int32_t (&xt)[4], const Pred &p,
                       uint32_t n0, uint32_t nv) {
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)CH; j += W) restore_steps<0, W, NT>(row, c, x, xt, p, n0 + j, nv, j);
}

/* CRC-16 (poly 0x8005) over bytes [b0, b1), slice-by-8 with the tables in LDS. */
DEV uint32_t crc16_step8(uint32_t crc, uint32_t w0, uint32_t w1, const lds_u16 *T) {
    const uint32_t a = w0 ^ (crc << 16);
    return T[7 * 256 + (a >> 24)] ^ T[6 * 256 + ((a >> 16) & 0xff)] ^ T[5 * 256 + ((a >> 8) & 0xff)] ^
           T[4 * 256 + (a & 0xff)] ^ T[3 * 256 + (w1 >> 24)] ^ T[2 * 256 + ((w1 >> 16) & 0xff)] ^
           T[1 * 256 + ((w1 >> 8) & 0xff)] ^ T[w1 & 0xff];
}
DEV uint32_t crc16_range(const uint8_t *__restrict__ bytes, uint64_t b0, uint64_t b1, const lds_u16 *T) {
    uint32_t crc = 0;
    uint64_t p = b0;
    while (p < b1 && (p & 15u)) { crc = ((crc << 8) ^ T[((crc >> 8) ^ bytes[p]) & 0xff]) & 0xffff; p++; }
    const uint4 *q = (const uint4 *)(bytes + p);
    const uint32_t nq = (uint32_t)((b1 - p) >> 4);
    uint32_t i = 0;
    for (; i + 4 <= nq; i += 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = q[i + u];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            crc = crc16_step8(crc, __builtin_bswap32(v[u].x), __builtin_bswap32(v[u].y), T);
            crc = crc16_step8(crc, __builtin_bswap32(v[u].z), __builtin_bswap32(v[u].w), T);
        }
    }
    for (; i < nq; i++) {
        const uint4 v = q[i];
        crc = crc16_step8(crc, __builtin_bswap32(v.x), __builtin_bswap32(v.y), T);
        crc = crc16_step8(crc, __builtin_bswap32(v.z), __builtin_bswap32(v.w), T);
    }
    p += (uint64_t)nq * 16u;
    while (p < b1) { crc = ((crc << 8) ^ T[((crc >> 8) ^ bytes[p]) & 0xff]) & 0xffff; p++; }
    return crc;
}

/* a * b mod P over GF(2) (16-bit polynomials) */
DEV uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 15; i >= 0; i--) {
        r = (r & 0x8000u) ? ((r << 1) ^ 0x8005u) & 0xffffu : (r << 1);
        if ((b >> i) & 1u) r ^= a;
    }
    return r;
}
/* crc * x^(8*nbytes) mod P: shift a CRC over nbytes appended bytes */
DEV uint32_t crc16_shift(uint32_t crc, uint64_t nbytes) {
    for (int j = 0; j < 40 && nbytes; j++, nbytes >>= 1)
        if (nbytes & 1u) crc = gf_mul(crc, g_crc16_xpow[j]);
    return crc;
}


/* Wave-cooperative CRC-16 of one byte range (the whole wave, coalesced 1 KB loads).
 * Layout: 16-byte pieces counted back from e = round_up(b1, 16); lane l takes pieces
 * 63 - l + 64 m, so every wave load is 64 consecutive pieces.  Each lane runs a CRC over
 * its own pieces with the 1008 bytes between them as zeros (x^(8*1008) by table TK), the
 * result is shifted to e by lanec = x^(8*16*(63 - l)), and the lanes are XOR-reduced.
 * Returns (wave-uniform) CRC([b0, b1)) * x^(8(e - b1)) mod P: zero iff the range's CRC is
 * zero (x is invertible mod P).  Bytes outside
 * [b0, b1) are masked to 0 (leading zeros leave a zero-initialised CRC at 0). */
DEV uint32_t crc_mulk(uint32_t a, const lds_u16 *TK) { return TK[a & 0xffu] ^ TK[256u + (a >> 8)]; }
DEV uint4 gld16(const uint8_t *p) { /* a global (not flat) 16-byte load */
    const u32x4 v = *(__attribute__((address_space(1))) const u32x4 *)(uintptr_t)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
DEV uint32_t wave_crc_range(const uint8_t *__restrict__ bytes, uint64_t b0, uint64_t b1, const lds_u16 *T,
                            const lds_u16 *TK, uint32_t lanec, uint32_t lane) {
    const uint64_t e = (b1 + 15u) & ~15ull, a0 = b0 & ~15ull;
    const uint32_t np = (uint32_t)((e - a0) >> 4), M = (np + 63u) >> 6;
    uint32_t acc = 0;
    for (uint32_t m0 = 0; m0 < M; m0 += 4u) {
        uint4 v[4];
        uint64_t pp[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t m = m0 + (uint32_t)u;
            const uint32_t r = 63u - lane + 64u * (M - 1u - min(m, M - 1u));
            pp[u] = e - 16ull * (r + 1u);
            v[u] = (m < M && r < np) ? gld16(bytes + pp[u]) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (m0 + (uint32_t)u >= M) break; /* wave-uniform */
            const int64_t lo = (int64_t)b0 - (int64_t)pp[u], hi = (int64_t)b1 - (int64_t)pp[u];
            const bool edge = lo > 0 || hi < 16;
            if (any_lane(edge)) {
                if (edge) {
                    const int32_t l32 = (int32_t)max(min(lo, (int64_t)16), (int64_t)0);
                    const int32_t h32 = (int32_t)max(min(hi, (int64_t)16), (int64_t)0);
                    v[u].x &= byte_keep(l32, h32, 0);
                    v[u].y &= byte_keep(l32, h32, 1);
                    v[u].z &= byte_keep(l32, h32, 2);
                    v[u].w &= byte_keep(l32, h32, 3);
                }
            }
            acc = crc_mulk(acc, TK);
            acc = crc16_step8(acc, __builtin_bswap32(v[u].x), __builtin_bswap32(v[u].y), T);
            acc = crc16_step8(acc, __builtin_bswap32(v[u].z), __builtin_bswap32(v[u].w), T);
        }
    }
    acc = gf_mul(acc, lanec);
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    return acc;
}
/* the TK table (x^(8*1008) by bytes) into LDS, by the whole wave */
DEV void crc_tk_fill(lds_u16 *TK, uint32_t lane) {
    const uint32_t K = crc16_shift(1u, 1008u);
    for (uint32_t i = lane; i < 256u; i += 64u) {
        TK[i] = (uint16_t)gf_mul(i, K);
        TK[256u + i] = (uint16_t)gf_mul(i << 8, K);
    }
}

#if BNF_TU == 0
/* ============================================================== k_parse
 * One lane per frame (parse_frame: the lane-serial subframe walk), 64 frames per single-wave
 * workgroup, in the parse order when there is one. */
template <int CPM>
__global__ void __launch_bounds__(64) k_parse(const uint32_t *__restrict__ words, uint64_t nbytes,
                                              const uint64_t *__restrict__ frame_offs, uint32_t nframes,
                                              bnf_stream_params sp, const uint64_t *__restrict__ out_sample_in,
                                              uint64_t base_sample, bnf_frame_info *__restrict__ info, uint32_t ablate,
                                              const uint32_t *__restrict__ perm, uint32_t *__restrict__ crcp) {
    __shared__ LDS_DMA_ALIGN uint32_t ring[PARSE_RD * RING_LANE_DW]; /* the bit ring */
    const uint32_t slot = blockIdx.x * 64u + threadIdx.x; /* parse order (launch_order<1>) */
    parse_frame<CPM>(words, nbytes, frame_offs, nframes, sp, out_sample_in, base_sample, info, ablate, (lds_u32 *)ring,
                (perm && slot < nframes) ? perm[slot] : slot, crcp);
}

/* =========================================================== k_parse_wave
 * One wave per frame: the same record as parse_frame (header, subframe starts, decode class),
 * with the header and subframe headers read at a wave-uniform cursor (WR) and each Rice
 * partition of subframes 0..C-2 crossed by the wave-cooperative scan (wave_rice_skip).
 * For launches with few frames (C5's files, one stream in the reader) the lane-per-frame walk
 * is one lane's serial chain over C-1 subframes with ~59 waves on 256 CUs; here every frame
 * has a wave of its own.  Identical records are a tested property (tests/test_gpu_parse_wave.py). */
__global__ void __launch_bounds__(64) k_parse_wave(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                   const uint64_t *__restrict__ frame_offs, uint32_t nframes,
                                                   bnf_stream_params sp, const uint64_t *__restrict__ out_sample_in,
                                                   uint64_t base_sample, bnf_frame_info *__restrict__ info,
                                                   uint32_t stats, int seg) {
    __shared__ LDS_DMA_ALIGN uint32_t ring[WR_SLOTS * WR_WIN];
    const uint32_t lane = threadIdx.x, f = blockIdx.x;
    if (f >= nframes) return;
    bnf_frame_info fi;
    fi.status = BNF_ST_OK;
    fi.err = -1;
    fi.frame_off = frame_offs[f];
    fi.resume_bit = 0;
    fi.cached = -1;
    fi.blocksize = fi.sample_rate = fi.channels = fi.assignment = fi.bps = 0;
    fi.number_type = 0;
    fi.unparseable = 0;
    fi.number = 0;
    fi.out_sample = 0;
    fi.crc8 = fi.crc16_calc = fi.crc16_read = fi.crc_ok = 0;
    fi.flags = 0;
    fi.reserved = 0;
    uint32_t ss[8];
#pragma unroll
    for (int c = 0; c < 8; c++) ss[c] = 0;
    const uint64_t limit = nbytes * 8u;
    const uint64_t fbit = fi.frame_off * 8u;
    WR r;
    wr_init(r, words, nbytes, (lds_u32 *)ring, fbit);
    pw_stat(r, stats != 0u, 4);
    uint32_t st = parse_header(r, fbit, limit, sp, fi);
    if (st == BNF_ST_ERROR && br_pos(r) > limit) st = BNF_ST_TRUNC;
    if (st == BNF_ST_OK) {
        uint64_t sample;
        if (fi.number_type == 1) sample = fi.number;
        else if (sp.has_stream_info && sp.min_blocksize == sp.max_blocksize) sample = (uint64_t)sp.min_blocksize * fi.number;
        else sample = (uint64_t)fi.blocksize * fi.number;
        fi.out_sample = out_sample_in ? out_sample_in[f] : sample - base_sample;
        uint32_t maxorder = 0;
        bool raw = false;
        const uint32_t nch = wr_u(fi.channels), bs = wr_u(fi.blocksize);
        for (uint32_t ch = 0; ch < nch; ch++) {
            const uint32_t here = (uint32_t)(br_pos(r) - fbit);
#pragma unroll
            for (int c = 0; c < 8; c++) ss[c] = (uint32_t)c == ch ? here : ss[c];
            if (ch + 1 == nch) {
                const uint32_t x = br_peek(r) >> 24;
                if (!(x & 0x80u) && (x & 0x7Eu) >= 0x40u) maxorder = max(maxorder, ((x >> 1) & 31u) + 1u);
                raw = raw || (x & 0x7Eu) < 4u;
                break;
            }
            SubHdr h;
            int32_t err = -1;
            st = parse_subframe_head<false>(r, sub_bps(fi, ch), bs, limit, h, nullptr, nullptr, err);
            if (st == BNF_ST_OK) {
                if (h.type == T_LPC) maxorder = max(maxorder, h.order);
                raw = raw || h.type == T_CONST || h.type == T_VERB;
                if (h.type == T_VERB) br_skip(r, (uint64_t)h.bps * bs);
                else if (h.type == T_FIXED || h.type == T_LPC) {
                    const uint64_t t0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
                    st = wave_skip_residual(r, h, bs, limit, stats != 0u, seg);
                    if (stats) pw_stat(r, true, 5, __builtin_amdgcn_s_memtime() - t0);
                }
                if (st == BNF_ST_OK && br_pos(r) > limit) st = BNF_ST_TRUNC;
            }
            if (st == BNF_ST_ERROR && br_pos(r) > limit) st = BNF_ST_TRUNC;
            if (st != BNF_ST_OK) {
                if (st == BNF_ST_ERROR) {
                    fi.err = err;
                    fi.resume_bit = br_pos(r);
                }
                break;
            }
        }
        if (maxorder > 16) fi.flags |= BNF_FL_W32;
        else if (maxorder > 8 || (maxorder > 0 && fi.bps > 16)) fi.flags |= BNF_FL_W16;
        else if (fi.channels == 2 && fi.bps <= 16 && !raw) fi.flags |= BNF_FL_ST;
        if (maxorder > 0 && maxorder <= 12 && fi.channels == 2 && fi.bps > 16 && fi.bps <= 24 && !raw) fi.flags |= BNF_FL_SW;
    }
    fi.status = st;
#pragma unroll
    for (int c = 0; c < 8; c++) fi.sub_start[c] = ss[c];
    wait_vm(); /* no DMA may land in the ring after the wave is gone */
    pw_flush(r, stats != 0u);
    /* the record, one dword per lane (32 lanes, one store) */
    const uint32_t *src = (const uint32_t *)&fi;
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) v = lane == (uint32_t)i ? src[i] : v;
    if (lane < 32u) ((uint32_t *)&info[f])[lane] = v;
}


/* The batch API's defined output for a frame whose status is not OK (bnflac_decode_parsed):
 * after every decode kernel, the output range of each ERROR / TRUNC frame whose header
 * parsed (sub_start[0] != 0: a CRC-8-checked header, so its position is the one the frame
 * would have been written to) is zero-filled, as a CRC-failed frame is; a frame whose header
 * did not parse has no range and is not written.  The lane kernels may have stored part of a
 * frame before finding its error; this pass overwrites that.  One lane per frame reads the
 * record; each bad frame is then filled by the whole wave (rare). */
__global__ void __launch_bounds__(64) k_fill_bad(const bnf_frame_info *__restrict__ info, uint32_t nframes,
                                                 bnf_stream_params sp, int fmt, uint8_t *__restrict__ out,
                                                 uint64_t out_bytes) {
    const uint32_t f = blockIdx.x * 64u + threadIdx.x;
    bool bad = false;
    uint64_t start = 0, n = 0;
    if (f < nframes) {
        const uint32_t st = info[f].status;
        if ((st == BNF_ST_ERROR || st == BNF_ST_TRUNC) && info[f].sub_start[0] != 0u) {
            const uint32_t C = info[f].channels, bsz = info[f].blocksize;
            const uint64_t os = info[f].out_sample;
            switch (fmt) {
            /* the frame's own slot only: a planar frame with more channels than sp.channels
             * would reach into the next frame's slot, so the fill stops at sp.channels */
            case BNF_OUT_PLANAR32: start = os * sp.channels * 4u; n = (uint64_t)min(C, sp.channels) * bsz * 4u; break;
            case BNF_OUT_INTERLEAVED32: start = os * sp.channels * 4u; n = (uint64_t)sp.channels * bsz * 4u; break;
            case BNF_OUT_FLACDECODER: start = os * (C == 2 ? 4u : 2u); n = (uint64_t)bsz * (C == 2 ? 4u : 2u); break;
            default: {
                const uint32_t fb = sp.bps == 24 ? 3u : 2u;
                start = os * sp.channels * fb;
                n = (uint64_t)bsz * sp.channels * fb;
            }
            }
            bad = n != 0 && start <= out_bytes && n <= out_bytes - start;
        }
    }
    uint64_t m = __ballot(bad);
    while (m) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        m &= m - 1u;
        const uint64_t s0 = __shfl(start, l), n0 = __shfl(n, l);
        for (uint64_t i = threadIdx.x; i < n0; i += 64u) out[s0 + i] = 0;
    }
}
#endif

/* Channel decorrelation (read_frame_ @0x10011a37-0x10011adb), 32-bit wrap. */
DEV void decorrelate(uint32_t as, int32_t &v0, int32_t &v1) {
    if (as == 1) v1 = (int32_t)((uint32_t)v0 - (uint32_t)v1);
    else if (as == 2) v0 = (int32_t)((uint32_t)v0 + (uint32_t)v1);
    else if (as == 3) {
        uint32_t mid = (uint32_t)v0, side = (uint32_t)v1;
        mid = (mid << 1) | (side & 1u);
        v0 = (int32_t)(mid + side) >> 1;
        v1 = (int32_t)(mid - side) >> 1;
    }
}

/* Pack one chunk: every lane writes a contiguous run of CH/chn_lanes samples of its own
 * frame (metadata in registers), reading the frame's channel rows from LDS.  Stereo
 * FLACDecoder / interleaved-int32 runs go out as 16-byte stores; FLACFileReader runs (2 or
 * 3 bytes per value, all channels) are packed into dwords in registers and go out as 16-,
 * 4- or 1-byte stores by alignment.  Returns how many store instructions this lane issued
 * (the caller takes the wave minimum over storing lanes: a lower bound on the wave's
 * stores keeps the refill's counted vmcnt wait exact or conservative). */
template <int FMT, int CH> constexpr uint32_t pack_fast_stores() { return FMT == BNF_OUT_INTERLEAVED32 ? CH / 4 : CH / 8; }

/* 4 values of fb bytes each (little-endian) -> fb dwords of the byte stream */
DEV void pack4(const int32_t (&v)[4], uint32_t fb, uint32_t (&d)[3]) {
    if (fb == 3) {
        d[0] = ((uint32_t)v[0] & 0xFFFFFFu) | ((uint32_t)v[1] << 24);
        d[1] = (((uint32_t)v[1] >> 8) & 0xFFFFu) | ((uint32_t)v[2] << 16);
        d[2] = (((uint32_t)v[2] >> 16) & 0xFFu) | ((uint32_t)v[3] << 8);
    } else {
        d[0] = ((uint32_t)v[0] & 0xFFFFu) | ((uint32_t)v[1] << 16);
        d[1] = ((uint32_t)v[2] & 0xFFFFu) | ((uint32_t)v[3] << 16);
        d[2] = 0;
    }
}

template <int FMT, int CH>
DEV uint32_t pack_lane(const int32_t *lds, uint32_t lane, uint32_t chn_lanes, uint32_t n0, bool fok, uint32_t bs,
                       uint32_t C, uint32_t as, uint64_t os, uint32_t stream_channels, uint32_t fr_bytes,
                       uint8_t *__restrict__ out) {
    const uint32_t lg = __builtin_ctz(chn_lanes); /* a power of 2 (lanes_for) */
    const uint32_t per = (uint32_t)CH >> lg;
    const uint32_t fl = lane >> lg, part = lane & (chn_lanes - 1u);
    const uint32_t i0 = part * per;
    if (!fok || n0 + i0 >= bs) return 0;
    const uint32_t cnt = min(per, bs - (n0 + i0));
    const int32_t *rows = lds + i0 * RP + fl * chn_lanes; /* channel c of sample q: rows[q * RP + c] */
    const uint32_t bpsmp = (FMT == BNF_OUT_INTERLEAVED32) ? 8u : 4u;
    /* vector path (stereo): the frame's two lanes take interleaved 4-sample groups
     * (lane h: samples 8g+4h .. 8g+4h+3), so each 16-byte store instruction writes 32
     * contiguous bytes per frame; dword alignment is enough for a global dwordx4 store, so
     * frames starting at any sample (variable blocksizes) take this path too */
    const uintptr_t base = (uintptr_t)out + (uintptr_t)(os + n0) * bpsmp;
    if ((FMT == BNF_OUT_FLACDECODER || FMT == BNF_OUT_INTERLEAVED32) && C == 2 && chn_lanes == 2 && n0 + CH <= bs &&
        (FMT == BNF_OUT_FLACDECODER || stream_channels == 2) && (base & 3u) == 0) {
        const int32_t *frows = lds + fl * 2u; /* (L, R) of sample i at frows[i * RP] */
#pragma unroll
        for (int g = 0; g < CH / 8; g++) {
            const uint32_t i = 8u * g + 4u * part;
            int32_t l[4], r[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int2 v = *(const int2 *)(frows + (i + q) * RP);
                l[q] = v.x;
                r[q] = v.y;
                decorrelate(as, l[q], r[q]);
            }
            if (FMT == BNF_OUT_FLACDECODER) { /* FLACDecoder.cs:543-562: L | R << 16 */
                gst128(base + i * 4u, u32x4{((uint32_t)l[0] & 0xffffu) | ((uint32_t)r[0] << 16),
                                            ((uint32_t)l[1] & 0xffffu) | ((uint32_t)r[1] << 16),
                                            ((uint32_t)l[2] & 0xffffu) | ((uint32_t)r[2] << 16),
                                            ((uint32_t)l[3] & 0xffffu) | ((uint32_t)r[3] << 16)});
            } else {
                gst128(base + i * 8u, u32x4{(uint32_t)l[0], (uint32_t)r[0], (uint32_t)l[1], (uint32_t)r[1]});
                gst128(base + i * 8u + 16u, u32x4{(uint32_t)l[2], (uint32_t)r[2], (uint32_t)l[3], (uint32_t)r[3]});
            }
        }
        return pack_fast_stores<FMT, CH>();
    }
    if (FMT == BNF_OUT_FILEREADER && C == stream_channels) { /* FLACFileReader.cs:220-237 */
        /* the run: cnt samples x C channels, values slot-ordered (sample-major), fb bytes each;
         * per is a multiple of 4, so full runs are whole groups of 4 values = fb dwords */
        const uint32_t fb = fr_bytes, slots = cnt * C;
        uint8_t *o = out + (os + n0 + i0) * (uint64_t)stream_channels * fb;
        const uintptr_t oa = (uintptr_t)o;
        const uint32_t ngrp = slots >> 2, rem = slots & 3u;
        const bool a16 = (oa & 15u) == 0 && (fb == 3 ? (ngrp & 3u) == 0 : (ngrp & 1u) == 0) && rem == 0;
        const bool a4 = (oa & 3u) == 0 && rem == 0;
        uint32_t nst = 0;
        if (a16 || a4) {
            /* the run's dwords in registers (compile-time indices: up to CH/4 groups of fb) */
            uint32_t dw[CH / 4 * 3];
            uint32_t q = 0, c = 0; /* sample and channel of value k = q * C + c (no division) */
#pragma unroll
            for (int g = 0; g < CH / 4; g++) {
                int32_t v[4] = {0, 0, 0, 0};
                if ((uint32_t)g < ngrp) {
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        v[u] = rows[q * RP + c];
                        if (++c == C) { c = 0; q++; }
                    }
                    if (C == 2) { /* stereo pairs are whole within a group of 4 */
                        decorrelate(as, v[0], v[1]);
                        decorrelate(as, v[2], v[3]);
                    }
                }
                uint32_t d[3];
                pack4(v, fb, d);
                if (fb == 3) {
                    dw[3 * g] = d[0];
                    dw[3 * g + 1] = d[1];
                    dw[3 * g + 2] = d[2];
                } else { /* 16-bit: 2 dwords per group, packed densely */
                    dw[2 * g] = d[0];
                    dw[2 * g + 1] = d[1];
                }
            }
            const uint32_t ndw = ngrp * fb;
            if (a16) {
#pragma unroll
                for (int u = 0; u < CH * 3 / 16; u++)
                    if ((uint32_t)(4 * u) < ndw) {
                        *(uint4 *)(o + 16u * u) = make_uint4(dw[4 * u], dw[4 * u + 1], dw[4 * u + 2], dw[4 * u + 3]);
                        nst++;
                    }
            } else {
#pragma unroll
                for (int u = 0; u < CH * 3 / 4; u++)
                    if ((uint32_t)u < ndw) {
                        *(uint32_t *)(o + 4u * u) = dw[u];
                        nst++;
                    }
            }
        } else { /* unaligned or ragged run: byte stores */
            for (uint32_t k = 0; k < slots; k++) {
                const uint32_t q = k / C, c = k - q * C;
                int32_t v0 = rows[q * RP + c];
                if (C == 2) { /* the pair of this sample */
                    int32_t l = rows[q * RP], r = rows[q * RP + 1];
                    decorrelate(as, l, r);
                    v0 = c ? r : l;
                }
                uint8_t *p = o + (uint64_t)k * fb;
                p[0] = (uint8_t)v0;
                p[1] = (uint8_t)(v0 >> 8);
                if (fb == 3) p[2] = (uint8_t)(v0 >> 16);
                nst += fb;
            }
        }
        return nst;
    }
    uint32_t nst = 0;
    for (uint32_t q = 0; q < cnt; q++) {
        const uint32_t n = n0 + i0 + q;
        int32_t v[8];
#pragma unroll
        for (int c = 0; c < 8; c++) v[c] = ((uint32_t)c < C) ? rows[q * RP + c] : 0;
        if (C == 2) decorrelate(as, v[0], v[1]);
        if (FMT == BNF_OUT_PLANAR32) {
            int32_t *o = (int32_t *)out + os * stream_channels;
            for (uint32_t c = 0; c < C; c++) o[(uint64_t)c * bs + n] = v[c];
            nst += C;
        } else if (FMT == BNF_OUT_INTERLEAVED32) {
            int32_t *o = (int32_t *)out + (os + n) * stream_channels;
            for (uint32_t c = 0; c < C; c++) o[c] = v[c];
            nst += C;
        } else if (FMT == BNF_OUT_FLACDECODER) { /* FLACDecoder.cs:543-577 */
            if (C == 2) {
                uint32_t *o = (uint32_t *)out;
                o[os + n] = ((uint32_t)v[0] & 0xffffu) | ((uint32_t)v[1] << 16);
            } else {
                uint16_t *o = (uint16_t *)out;
                o[os + n] = (uint16_t)(uint32_t)v[0];
            }
            nst += 1;
        } else { /* FLACFileReader.cs:220-237: 2 or 3 bytes per sample, all channels */
            uint8_t *o = out + (os + n) * (uint64_t)stream_channels * fr_bytes;
            for (uint32_t c = 0; c < C; c++) {
                o[c * fr_bytes + 0] = (uint8_t)v[c];
                o[c * fr_bytes + 1] = (uint8_t)(v[c] >> 8);
                if (fr_bytes == 3) o[c * fr_bytes + 2] = (uint8_t)(v[c] >> 16);
            }
            nst += C * fr_bytes;
        }
    }
    return nst;
}

/* FLACFileReader 24-bit runs (FLACFileReader.cs:220-237) flushed as wide runs: the chunk's
 * output is fpb frame runs of CH samples x C channels x 3 bytes (CH = 32: 6C 16-byte pieces
 * per frame); lane i writes pieces i, i + 64, ... in frame-major order, so the 64 lanes of one
 * store cover ~1 KB of a few frames' runs instead of 64 scattered 16-byte pieces.  Each piece
 * is 6 values (bytes 16p .. 16p+15 lie in values floor(16p/3) .. +5), read from the rows of
 * its frame (decorrelated when stereo) and byte-aligned with v_alignbyte.  The frame table
 * (output byte base, assignment, channels, ok) sits in the row buffer's spare columns
 * (64..71 of rows 0..15).  Requires every frame of the wave to have a full, 16-byte-aligned
 * chunk with C == the stream's channels (the caller checks).  Returns this lane's stores. */
DEV uint32_t *wide_tbl(int32_t *lds, uint32_t fr) { return (uint32_t *)lds + (fr >> 1) * RP + 64u + (fr & 1u) * 4u; }
template <int CH>
DEV uint32_t pack_wide24(int32_t *lds, uint32_t lane, uint32_t cl, uint32_t n0, uint32_t C, uint8_t *__restrict__ out) {
    static_assert(CH * 3 % 16 == 0 && DEC_LANES * 6 >= CH * 3 * 64 / 16, "6 pieces per lane cover a chunk");
    const uint32_t fpb = DEC_LANES / cl, ppf = (uint32_t)CH * C * 3u / 16u, np = fpb * ppf;
    uint32_t nst = 0;
#pragma unroll
    for (int u = 0; u < CH * 3 / 16; u++) {
        const uint32_t P = (uint32_t)u * 64u + lane;
        const uint32_t fr = P / ppf, pp = P - fr * ppf;
        const uint32_t *t = wide_tbl(lds, min(fr, fpb - 1u));
        const uint32_t meta = t[2];
        if (P >= np || !((meta >> 8) & 1u)) continue;
        const uint32_t b0 = 16u * pp, vlo = b0 / 3u, off = b0 - 3u * vlo;
        const int32_t *rows = lds + fr * cl;
        int32_t v[6];
        if (C == 2u) {
            const uint32_t q0 = vlo >> 1, odd = vlo & 1u, as = meta & 15u;
            int32_t L[4], R[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int2 x = *(const int2 *)(rows + min(q0 + (uint32_t)q, (uint32_t)CH - 1u) * RP);
                L[q] = x.x;
                R[q] = x.y;
                decorrelate(as, L[q], R[q]);
            }
            v[0] = odd ? R[0] : L[0];
            v[1] = odd ? L[1] : R[0];
            v[2] = odd ? R[1] : L[1];
            v[3] = odd ? L[2] : R[1];
            v[4] = odd ? R[2] : L[2];
            v[5] = odd ? L[3] : R[2];
        } else {
            uint32_t q = vlo / C, c = vlo - q * C;
#pragma unroll
            for (int i = 0; i < 6; i++) {
                v[i] = rows[q * RP + c];
                if (++c == C) { c = 0; q++; }
            }
        }
        const uint32_t d0 = ((uint32_t)v[0] & 0xFFFFFFu) | ((uint32_t)v[1] << 24);
        const uint32_t d1 = (((uint32_t)v[1] >> 8) & 0xFFFFu) | ((uint32_t)v[2] << 16);
        const uint32_t d2 = (((uint32_t)v[2] >> 16) & 0xFFu) | ((uint32_t)v[3] << 8);
        const uint32_t d3 = ((uint32_t)v[4] & 0xFFFFFFu) | ((uint32_t)v[5] << 24);
        const uint32_t d4 = ((uint32_t)v[5] >> 8) & 0xFFFFu;
        const uint64_t ob = (((uint64_t)t[1] << 32) | t[0]) + (uint64_t)n0 * C * 3u + b0;
        gst128((uint64_t)(uintptr_t)out + ob,
               u32x4{__builtin_amdgcn_alignbyte(d1, d0, off), __builtin_amdgcn_alignbyte(d2, d1, off),
                     __builtin_amdgcn_alignbyte(d3, d2, off), __builtin_amdgcn_alignbyte(d4, d3, off)});
        nst++;
    }
    return nst;
}

/* restore-path dispatch (per lane); the tap count is the instance's (orders below it run
 * with zero coefficients), so a wave takes at most one variant per libFLAC path */
#define LPC_DISPATCH(FN, ...)                                                                     \
    do {                                                                                           \
        if (h.path == P_MMX16) FN<CHK, MAXW, P_MMX16>(__VA_ARGS__);                                \
        else if (h.path == P_IA32) FN<CHK, MAXW, P_IA32>(__VA_ARGS__);                             \
        else FN<CHK, MAXW, P_WIDE>(__VA_ARGS__);                                                   \
    } while (0)

/* one block of fpb decode-order slots (the body of k_decode) */
template <int MAXW, int CHK, int RD>
DEV void decode_block(uint32_t blk, uint32_t *ring, int32_t *lds, const uint32_t *__restrict__ words, uint64_t nbytes,
                      uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes, int fmt, uint8_t *__restrict__ out,
                      uint64_t out_bytes, bnf_frame_info *__restrict__ info, const uint32_t *__restrict__ perm,
                      uint32_t ablate) {
    static_assert(MAXW <= CHK && CHK % 8 == 0 && RD <= RING_MAX, "chunk must hold the predictor ring");
    static_assert(CHK * RP >= 1024 + 512, "row buffer also holds the CRC tables and the tail's frame table");
    /* per-frame tables overlay the buffers while those are idle: the setup exchange uses
     * the ring before its first DMA, the tail uses the row buffer after the last pack */
    uint32_t *f_bs = ring, *f_ch = ring + 64, *f_as = ring + 128, *f_ok = ring + 192;
    uint64_t *f_out = (uint64_t *)(ring + 256);
    uint32_t *t_bs = (uint32_t *)lds + 1024, *t_ch = t_bs + 64, *t_ok = t_bs + 128, *t_endbit = t_bs + 192,
             *t_bad = t_bs + 256, *t_pre = t_bs + 448;
    uint64_t *t_out = (uint64_t *)(t_bs + 320);

    const uint32_t lane = threadIdx.x;
    const uint32_t lg = __builtin_ctz(chn_lanes); /* a power of 2 (lanes_for) */
    const uint32_t fpb = DEC_LANES >> lg;
    const uint32_t fl = lane >> lg, ch = lane & (chn_lanes - 1u);
    /* frame of this lane group: slot order, or the decode order k_order built (class, then
     * blocksize: similar frames share a wave) */
    const uint32_t slot = blk * fpb + fl;
    const uint32_t f = (perm && fl < fpb && slot < nframes) ? perm[slot] : slot;
    const uint64_t limit = nbytes * 8u;

    bnf_frame_info fi;
    bool have = (fl < fpb) && (slot < nframes);
    if (ablate & BNF_MODE_WREDO) have = have && (info[f].flags & BNF_FL_WAVE_REDO); /* after k_decode_sys: its hand-backs */
    /* k_decode_sw's frames (BNF_MODE_SW: it ran first) are this kernel's only once handed back */
    const bool sw_on = (ablate & BNF_MODE_SW) != 0;
    const bool lst = (ablate & BNF_MODE_LIST) != 0; /* k_decode_list: every frame of the list is this instance's */
    if (lst) {
        if (!__any(have)) return;
    } else if (MAXW != 8) { /* most blocks are not this instance's: leave on two words of the record */
        const uint32_t fl = have ? info[f].flags : 0u;
        const bool w = have && info[f].status == BNF_ST_OK && (fl & (BNF_FL_W16 | BNF_FL_W32)) && !(fl & BNF_FL_ST) &&
                       !(sw_on && (fl & BNF_FL_SW) && !(fl & BNF_FL_REDO));
        if (!__any(w)) return;
    } else { /* W = 8: narrow non-stereo frames, and stereo frames k_decode_st handed back */
        bool w = false;
        if (have && info[f].status == BNF_ST_OK) {
            const uint32_t fl = info[f].flags;
            if ((fl & BNF_FL_ST) && !(ablate & 0x400u)) w = !(ablate & BNF_MODE_NOST) && (fl & BNF_FL_REDO) != 0;
            else w = !(ablate & BNF_MODE_STREDO) && !(fl & (BNF_FL_W16 | BNF_FL_W32));
        }
        if (!__any(w)) return;
    }
    if (have) fi = info[f];
    /* Stereo frames (BNF_FL_ST) are k_decode_st's, unless it handed them back (BNF_FL_REDO):
     * those are decoded by the W = 8 instance, which runs after k_decode_st on its stream.
     * The W = 16 and 32 instances run beside them on a second stream and never look at
     * ST frames (the ST bit is k_parse's and does not change; REDO may be being set). */
    const bool st_frame = have && (fi.flags & BNF_FL_ST) && !(ablate & 0x400u) && !lst;
    if (st_frame && (MAXW != 8 || (ablate & BNF_MODE_NOST) || !(fi.flags & BNF_FL_REDO))) have = false;
    if (MAXW == 8 && (ablate & BNF_MODE_STREDO) && !st_frame) have = false;
    if (have && sw_on && (fi.flags & BNF_FL_SW) && !(fi.flags & BNF_FL_REDO)) have = false;
    bool frame_ok = have && fi.status == BNF_ST_OK;
    /* one wave per workgroup: the W = 8, 16 and 32 instances split the blocks between them
     * by the widest class among the block's non-ST frames (k_parse's flags); the W = 8
     * instance also takes the handed-back ST frames of the other instances' blocks */
    if (!lst) {
        const bool a32 = __any(frame_ok && !st_frame && (fi.flags & BNF_FL_W32)) != 0;
        const bool a16 = __any(frame_ok && !st_frame && (fi.flags & BNF_FL_W16)) != 0;
        const int cls = a32 ? 32 : (a16 ? 16 : 8);
        if (cls != MAXW && !(MAXW == 32 && cls == 16 && (ablate & BNF_MODE_SEG))) {
            if (MAXW != 8) return;
            have = have && st_frame; /* a W16/W32 block: only its handed-back ST frames */
            frame_ok = frame_ok && st_frame;
            if (!__any(have)) return;
        }
    }

    bool active = frame_ok && ch < fi.channels && fi.channels <= chn_lanes;
    if (lane < fpb) { f_ok[lane] = 0; f_bs[lane] = 0; }
    __syncthreads();
    if (have && ch == 0) {
        f_bs[fl] = frame_ok ? fi.blocksize : 0;
        f_ch[fl] = fi.channels;
        f_as[fl] = fi.assignment;
        f_out[fl] = fi.out_sample;
        uint32_t ok = frame_ok;
        uint32_t unsupported = 0;
        if (fmt == BNF_OUT_FLACDECODER && fi.bps != 16) unsupported = 1;          /* WriteCallback abort :526-530 */
        if (fmt >= BNF_OUT_FLACDECODER && fi.channels > sp.channels) unsupported = 1;
        if (fmt == BNF_OUT_FILEREADER && sp.bps != 16 && sp.bps != 24) unsupported = 1; /* NotSupportedException :239-240 */
        if (frame_ok && unsupported) {
            ok = 0;
            fi.status = BNF_ST_SKIPPED;
            fi.flags |= 4u;
            info[f] = fi;
        }
        {   /* never write outside the caller's buffer (bad frame numbers, short buffers) */
            uint64_t stride;
            switch (fmt) {
            case BNF_OUT_PLANAR32: case BNF_OUT_INTERLEAVED32: stride = 4ull * sp.channels; break;
            case BNF_OUT_FLACDECODER: stride = fi.channels == 2 ? 4u : 2u; break;
            default: stride = (uint64_t)sp.channels * (sp.bps == 24 ? 3u : 2u); break;
            }
            if (frame_ok && (fi.out_sample + fi.blocksize) * stride > out_bytes) {
                ok = 0;
                fi.status = BNF_ST_SKIPPED;
                fi.flags |= 2u;
                info[f] = fi;
            }
        }
        if (fi.channels > chn_lanes) {
            ok = 0;
            if (frame_ok) { fi.status = BNF_ST_SKIPPED; info[f] = fi; }
        }
        f_ok[fl] = ok;
    }

    __syncthreads();
    const bool fok = have && f_ok[fl];
    active = active && fok;
    const uint32_t fbs = fok ? f_bs[fl] : 0u, fch = have ? fi.channels : 0u, fas = fok ? f_as[fl] : 0u;
    const uint64_t fos = fok ? f_out[fl] : 0u;
    lds_sync(); /* the ring's first DMA may overwrite the tables only after these reads */
    const bool wide_fmt = fmt == BNF_OUT_FILEREADER && sp.bps == 24u && !(ablate & 0x2000u);
    if (wide_fmt && fl < fpb && ch == 0) { /* pack_wide24's frame table (row buffer spare columns) */
        uint32_t *t = wide_tbl(lds, fl);
        const uint64_t ob = fos * sp.channels * 3u;
        t[0] = (uint32_t)ob;
        t[1] = (uint32_t)(ob >> 32);
        t[2] = fas | (fch << 4) | ((fok ? 1u : 0u) << 8);
    }
    const uint64_t f_off = have ? fi.frame_off : 0u;

    /* ---- subframe setup */
    BR b;
    br_init(b, words, nbytes, (lds_u32 *)ring, lane, RD);
    b.stats = (ablate & 0x100u) != 0;
    STAT(b.stats, 5);
    const bool tmon = b.stats;
    const uint64_t t_start = tnow(tmon);
    uint64_t tm_dec = 0, tm_ref = 0, tm_pack = 0;
    SubHdr h;
    h.type = T_CONST; h.order = 0; h.wasted = 0; h.bps = 0; h.shift = 0; h.path = P_IA32; h.cval = 0;
    h.porder = 0; h.rice2 = 0;
    RS rs;
    rs.verb = 0; rs.k = 0; rs.esc = 0; rs.left = 0; rs.pidx = 0; rs.nparts = 0; rs.psamples = 0;
    rs.order = 0; rs.plen = 4; rs.pesc = 15; rs.porder = 0;
    int32_t c[MAXW], x[MAXW], xt[4]; /* coefficients; history ring (MMX16: int16 words) */
#pragma unroll
    for (int t = 0; t < MAXW; t++) { c[t] = 0; x[t] = 0; }
#pragma unroll
    for (int t = 0; t < 4; t++) xt[t] = 0;
    Pred pd;
    pd.sh = 0; pd.order = 0; pd.wasted = 0; pd.mmx = false; pd.wide = false;
    uint32_t trunc = 0, st = BNF_ST_OK;
    int32_t err = -1;
    uint32_t bs = 0;
    int32_t *row = lds + lane;
    if (active) {
        bs = fi.blocksize;
        /* read from HBM: indexing the local record by the runtime channel would spill it to scratch */
        br_seek(b, fi.frame_off * 8u + info[f].sub_start[ch]);
        int32_t coef[MAXW]; /* orders above MAXW are rejected below */
        /* warm-ups go straight to the rows of chunk 0: raw, they are output samples */
        st = parse_subframe_head<true, MAXW, RP>(b, sub_bps(fi, ch), bs, limit, h, row, coef, err);
        if (st == BNF_ST_OK && h.type == T_LPC && h.order > MAXW) {
            st = BNF_ST_ERROR; /* k_parse mis-flagged: cannot happen for the subframes it read */
            err = E_UNPARSEABLE;
        }
        if (st == BNF_ST_OK) {
            /* the subframe as a linear predictor (see Pred) */
            pd.order = h.order;
            pd.wasted = h.wasted;
            if (h.type == T_LPC) {
#pragma unroll
                for (int t = 0; t < MAXW; t++) c[t] = ((uint32_t)t < h.order) ? coef[t] : 0;
                pd.mmx = h.path == P_MMX16;
                pd.wide = h.path == P_WIDE;
                if (h.path == P_MMX16) pd.sh = ((uint32_t)h.shift >= 32u) ? 31 : h.shift;
                else if (h.path == P_IA32) pd.sh = h.shift & 31;
                else pd.sh = min((uint32_t)h.shift & 0xFFu, 63u);
            } else if (h.type == T_FIXED) {
                const uint32_t o = h.order;
                c[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
                c[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
                c[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
                c[3] = o == 4 ? -1 : 0;
            } else if (h.type == T_CONST) {
                c[0] = 1;
                pd.order = 1;
                row[0] = h.cval;
            }
            /* residual reader: FIXED / LPC partitioned Rice; VERBATIM as one endless escaped
             * partition of bps-bit raw values; CONSTANT the same with 0-bit values (no bits) */
            const bool rice = h.type == T_FIXED || h.type == T_LPC;
            rs.verb = rice ? 0u : 1u; /* no partition headers to finish */
            rs.esc = rice ? 0u : 1u;
            rs.k = h.type == T_VERB ? h.bps : 0u;
            rs.left = rice ? 0u : 0x7fffffffu;
            rs.order = h.order;
            rs.porder = h.porder;
            rs.nparts = rice ? 1u << h.porder : 0u;
            rs.psamples = h.porder ? bs >> h.porder : bs - h.order;
            rs.plen = h.rice2 ? 5u : 4u;
            rs.pesc = h.rice2 ? 31u : 15u;
        } else {
            active = false;
        }
    }

    /* block-wide number of chunks */
    uint32_t mybs = active ? bs : 0u;
    for (int o = 32; o > 0; o >>= 1) mybs = max(mybs, (uint32_t)__shfl_xor(mybs, o));
    const uint32_t nchunks = (mybs + CHK - 1) / CHK;
    /* W = 16 instance: a wave whose orders (taps with a nonzero coefficient: LPC and
     * FIXED order, CONSTANT 1, VERBATIM 0) all fit NTAP_LO runs the predictor with NTAP_LO
     * MACs per sample (C3's LPC-12 in k_decode<16>: 12 instead of 16) */
    constexpr int NTAP_LO = MAXW * 3 / 4;
    uint32_t mytaps = active ? pd.order : 0u;
    for (int o = 32; o > 0; o >>= 1) mytaps = max(mytaps, (uint32_t)__shfl_xor(mytaps, o));
    const bool ntap_lo = mytaps <= (uint32_t)NTAP_LO;

    const uint64_t t_loop = tnow(tmon);
    wait_vm(); /* setup loads done: the pipeline counts start from zero */
    VmQ vq;
    vq.d_last = vq.s_last = vq.s_prev = 0;
    for (uint32_t kc = 0; kc < nchunks; kc++) {
        const uint32_t n0 = kc * CHK;
        const uint32_t nvalid = (active && n0 < bs) ? min((uint32_t)CHK, bs - n0) : 0u;
        const uint64_t ta = tnow(tmon);
        br_wait1(b, vq); /* the lines fetched after the last entropy phase have landed */
        /* full chunks past the warm-up: fused decode + restore; the warm-up chunk and a
         * frame's last partial chunk: residuals into the rows, then the restore */
        const bool fused = nvalid == CHK && n0 >= pd.order && !(ablate & 0x80Cu);
        if (fused) {
            STAT(b.stats, 0);
            if (MAXW == 16 && ntap_lo) fused_chunk<CHK, MAXW, NTAP_LO>(b, rs, row, c, x, xt, pd, limit, trunc);
            else fused_chunk<CHK, MAXW, MAXW>(b, rs, row, c, x, xt, pd, limit, trunc);
        } else if (nvalid) {
            STAT(b.stats, 1);
            const uint32_t i0 = (n0 < pd.order) ? min(pd.order - n0, nvalid) : 0u;
            if (ablate & 8u) {
                for (uint32_t i = i0; i < nvalid; i++) row[i * RP] = (int32_t)i;
            } else {
                for (uint32_t i = i0; i < nvalid; i++) row[i * RP] = rice_fused(b, rs, limit, trunc, nullptr);
            }
        }
        const uint64_t tb = tnow(tmon);
        {   /* whole wave: fetch ahead while the restore and the pack run */
            const bool want = nvalid && h.type != T_CONST && n0 + CHK < bs;
            STAT(b.stats && want, 4);
            br_issue(b, want);
        }
        if (!fused && nvalid && !(ablate & 4u)) {
            if (MAXW == 16 && ntap_lo) restore_chunk<CHK, MAXW, NTAP_LO>(row, c, x, xt, pd, n0, nvalid);
            else restore_chunk<CHK, MAXW, MAXW>(row, c, x, xt, pd, n0, nvalid);
        }
        lds_sync();
        const uint64_t tc = tnow(tmon);
        tm_dec += tb - ta;
        tm_ref += tc - tb;
        uint32_t pk = 0;
        switch ((ablate & 2u) ? -1 : fmt) {
        case -1:
            break;
        case BNF_OUT_PLANAR32:
            pk = pack_lane<BNF_OUT_PLANAR32, CHK>(lds, lane, chn_lanes, n0, fok, fbs, fch, fas, fos, sp.channels, 0, out);
            break;
        case BNF_OUT_INTERLEAVED32:
            pk = pack_lane<BNF_OUT_INTERLEAVED32, CHK>(lds, lane, chn_lanes, n0, fok, fbs, fch, fas, fos, sp.channels, 0, out);
            break;
        case BNF_OUT_FLACDECODER:
            pk = pack_lane<BNF_OUT_FLACDECODER, CHK>(lds, lane, chn_lanes, n0, fok, fbs, fch, fas, fos, sp.channels, 0, out);
            break;
        default: {
            bool wide = false;
            if (CHK == 32 && wide_fmt) { /* every frame of the wave: a full aligned chunk of all the stream's channels */
                const bool bad = have && fok && !(fch == sp.channels && n0 + CHK <= fbs &&
                                                  (((fos + n0) * sp.channels * 3u) & 15u) == 0u);
                wide = !any_lane(bad);
            }
            if (wide) pk = pack_wide24<CHK>(lds, lane, chn_lanes, n0, sp.channels, out);
            else
                pk = pack_lane<BNF_OUT_FILEREADER, CHK>(lds, lane, chn_lanes, n0, fok, fbs, fch, fas, fos, sp.channels,
                                                        sp.bps == 24 ? 3u : 2u, out);
            break;
        }
        }
        /* account this chunk's stores for the next refill's counted vmcnt wait: every store
         * of a lane is a store instruction of the wave, so the wave issued at least the
         * largest per-lane count (a lower bound keeps the wait exact or conservative) */
        {
            uint32_t m = pk;
            for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
            vq.s_last += m;
        }
        lds_sync();
        tm_pack += tnow(tmon) - tc;
    }
    const uint64_t t_loopend = tnow(tmon);

    /* ---- last subframe end, zero padding, CRC-16 (read_frame_ @0x100118c0 tail).  The
     * frame record is re-read here (only scalars stay live across the chunk loop). */
    if (lane < fpb) { t_ok[lane] = 0; t_bad[lane] = 0; t_endbit[lane] = 0; }
    lds_sync();
    if (have && ch == 0) {
        t_ok[fl] = fok ? 1u : 0u;
        t_ch[fl] = fch;
        t_bs[fl] = fbs;
        t_out[fl] = fos;
    }
    lds_sync();
    const bool last = fok && frame_ok && ch + 1 == fch && fch <= chn_lanes;
    if (active) {
        finish_partitions(b, rs);
        if (br_pos(b) > limit) trunc = 1;
    }
    uint32_t t_status = BNF_ST_OK, t_crc_read = 0;
    int32_t t_err = -1;
    uint64_t t_resume = 0;
    bool t_resume_set = false;
    if (last) {
        if (st == BNF_ST_ERROR && br_pos(b) > limit) st = BNF_ST_TRUNC;
        if (st == BNF_ST_ERROR) {
            t_status = BNF_ST_ERROR;
            t_err = err;
            t_resume = br_pos(b);
            t_resume_set = true;
        } else if (st == BNF_ST_TRUNC || trunc) {
            t_status = BNF_ST_TRUNC;
        } else {
            /* read_zero_padding_ @0x10012fe0 */
            const uint32_t padbits = (uint32_t)((8u - (br_pos(b) & 7u)) & 7u);
            const uint32_t z = br_read(b, padbits);
            if (br_pos(b) > limit) {
                t_status = BNF_ST_TRUNC;
            } else if (z != 0) {
                t_status = BNF_ST_ERROR;
                t_err = E_LOST_SYNC;
                t_resume = br_pos(b);
                t_resume_set = true;
            } else {
                const uint64_t end_byte = br_pos(b) >> 3;
                const uint32_t crc_read = br_read(b, 16);
                if (br_pos(b) > limit) {
                    t_status = BNF_ST_TRUNC;
                } else {
                    t_endbit[fl] = (uint32_t)(end_byte - f_off);
                    t_crc_read = crc_read;
                    t_resume = br_pos(b);
                    t_resume_set = true;
                }
            }
        }
        if (t_status != BNF_ST_OK) t_bad[fl] = 1;
    }
    lds_sync();
    /* CRC-16 over [frame_off, end): split across
     * the frame's channel lanes, combined by polynomial shifts (CRC is linear:
     * crc(A|B) = crc(A)*x^(8|B|) + crc(B)). */
    uint32_t part = 0;
    const bool crc_lane = fok && frame_ok && ch < fch && !t_bad[fl];
    lds_u16 *T = (lds_u16 *)(lds_u32 *)lds;
    if (__any(crc_lane)) { /* the rows are free now: stage the slice-by-8 CRC tables there */
        __syncthreads();
        for (uint32_t i = lane; i < 8u * 256u; i += DEC_LANES) T[i] = (&g_crc16_tab[0][0])[i];
        __syncthreads();
    }
    if (crc_lane) {
        const uint64_t len = t_endbit[fl];
        const uint32_t nl = fch;
        const uint64_t per = (len + nl - 1) / nl;
        const uint64_t s0 = f_off + min(len, per * ch), s1 = f_off + min(len, per * (ch + 1));
        if (!(ablate & 1u)) {
            part = crc16_range((const uint8_t *)words, s0, s1, T);
            part = crc16_shift(part, f_off + len - s1);
        }
    }
    /* xor-reduce within each frame's lane group */
    uint32_t acc = part;
    for (uint32_t o = 1; o < chn_lanes; o <<= 1) acc ^= __shfl_xor(acc, o);
    if ((ablate & 1u) && last && t_status == BNF_ST_OK) acc = t_crc_read;
    if (last) {
        bnf_frame_info fo = info[f];
        fo.status = t_status;
        if (t_status == BNF_ST_ERROR) fo.err = t_err;
        if (t_resume_set) fo.resume_bit = t_resume;
        if (t_status == BNF_ST_OK) {
            fo.crc16_read = t_crc_read;
            fo.crc16_calc = acc;
            fo.crc_ok = (acc == t_crc_read) ? 1u : 0u;
            if (!fo.crc_ok) t_bad[fl] = 2; /* libFLAC zero-fills a CRC-failed frame (@0x10011af5) */
        }
        info[f] = fo;
    }
    __syncthreads();
    if (tmon && lane == 0) {
        const uint64_t t_end = tnow(tmon);
        atomicAdd(&g_stats[8], (unsigned long long)(t_loop - t_start));
        atomicAdd(&g_stats[9], (unsigned long long)tm_dec);
        atomicAdd(&g_stats[10], (unsigned long long)tm_ref);
        atomicAdd(&g_stats[11], (unsigned long long)tm_pack);
        atomicAdd(&g_stats[12], (unsigned long long)(t_end - t_loopend));
    }
    /* zero-fill CRC-failed frames' output */
    for (uint32_t fl2 = 0; fl2 < fpb; fl2++) {
        if (t_bad[fl2] != 2 || !t_ok[fl2]) continue;
        uint64_t nbytes_fr, start;
        const uint32_t C = t_ch[fl2], bsz = t_bs[fl2];
        switch (fmt) {
        case BNF_OUT_PLANAR32: start = t_out[fl2] * sp.channels * 4u; nbytes_fr = (uint64_t)C * bsz * 4u; break;
        case BNF_OUT_INTERLEAVED32: start = t_out[fl2] * sp.channels * 4u; nbytes_fr = (uint64_t)sp.channels * bsz * 4u; break;
        case BNF_OUT_FLACDECODER: start = t_out[fl2] * (C == 2 ? 4u : 2u); nbytes_fr = (uint64_t)bsz * (C == 2 ? 4u : 2u); break;
        default: {
            const uint32_t fb = sp.bps == 24 ? 3u : 2u;
            start = t_out[fl2] * sp.channels * fb;
            nbytes_fr = (uint64_t)bsz * sp.channels * fb;
        }
        }
        for (uint64_t i = lane; i < nbytes_fr; i += DEC_LANES) out[start + i] = 0;
    }
    wait_vm(); /* no ring DMA may land after the wave is gone */
}

/* The W instances, one block of decode-order slots per workgroup.  seg (W = 16 / 32, with
 * perm): the decode order's bucket ends (k_order_place leaves seg[k] = end of bucket k), so
 * a block outside the instance's class segment leaves on two scalar loads, before reading
 * any frame record (C2: all 32,768 blocks of each side launch).  A persistent grid over the
 * segment (workgroups claiming blocks from a counter) removed those waves altogether but
 * compiled the block body ~7% slower inside the loop (C3 13.1 -> 13.9 ms, C4 27.7 -> 29.6;
 * same with a full-size grid), for no C2 gain (12.33 -> 12.30 ms): DESIGN.md section 9. */
template <int MAXW, int CHK, int RD>
__global__ void __launch_bounds__(DEC_LANES, 2) k_decode(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                      uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes,
                                                      int fmt, uint8_t *__restrict__ out, uint64_t out_bytes,
                                                      bnf_frame_info *__restrict__ info,
                                                      const uint32_t *__restrict__ perm, uint32_t ablate,
                                                      const uint32_t *__restrict__ seg) {
    __shared__ LDS_DMA_ALIGN uint32_t ring[RD * RING_LANE_DW];
    __shared__ int32_t lds[CHK * RP]; /* [sample][lane] */
    if (seg) { /* W = 8: only as one of its two launches (BNF_MODE_NOST / BNF_MODE_STREDO) */
        const uint32_t fpb = DEC_LANES >> __builtin_ctz(chn_lanes);
        const uint32_t c = MAXW == 32 ? 3u : MAXW == 16 ? 2u : (ablate & BNF_MODE_NOST) ? 1u : 0u; /* order_key's class */
        const uint32_t lo = c ? seg[c * 64u - 1u] / fpb : 0u, end = (seg[c * 64u + 63u] + fpb - 1u) / fpb;
        if (blockIdx.x < lo || blockIdx.x >= end) return;
    }
    decode_block<MAXW, CHK, RD>(blockIdx.x, ring, lds, words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info,
                                perm, ablate);
}

/* k_decode_sys's hand-backs: the frames of a device list (list[0] = count, list[4..] = frame
 * indices), decoded from scratch by the exact lane kernel.  The count is only known on the
 * device, so a small grid strides over the list's blocks (an empty list costs one load per
 * workgroup). */
template <int MAXW, int CHK, int RD>
__global__ void __launch_bounds__(DEC_LANES, 2) k_decode_list(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                           bnf_stream_params sp, uint32_t chn_lanes, int fmt,
                                                           uint8_t *__restrict__ out, uint64_t out_bytes,
                                                           bnf_frame_info *__restrict__ info,
                                                           const uint32_t *__restrict__ list, uint32_t ablate) {
    __shared__ LDS_DMA_ALIGN uint32_t ring[RD * RING_LANE_DW];
    __shared__ int32_t lds[CHK * RP];
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(list[0]);
    const uint32_t fpb = DEC_LANES >> __builtin_ctz(chn_lanes);
    const uint32_t nb = (cnt + fpb - 1u) / fpb;
    for (uint32_t blk = blockIdx.x; blk < nb; blk += gridDim.x) {
        decode_block<MAXW, CHK, RD>(blk, ring, lds, words, nbytes, cnt, sp, chn_lanes, fmt, out, out_bytes, info, list + 4,
                                    ablate | BNF_MODE_LIST | BNF_MODE_WREDO);
        __syncthreads();
    }
}

/* The W16 and W32 classes of the decode order in one small grid striding over their blocks
 * (seg: k_order's bucket ends, classes 2 and 3 are adjacent), the usual class rules.  Launched
 * instead of the two full-size side grids when the previous batch had no such frames (C2):
 * an empty segment costs two loads per workgroup of a 512-workgroup launch, where the side
 * grids were 32,768 early-exiting waves each. */
template <int MAXW, int CHK, int RD>
__global__ void __launch_bounds__(DEC_LANES, 2) k_decode_seg(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                          uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes,
                                                          int fmt, uint8_t *__restrict__ out, uint64_t out_bytes,
                                                          bnf_frame_info *__restrict__ info,
                                                          const uint32_t *__restrict__ perm, uint32_t ablate,
                                                          const uint32_t *__restrict__ seg) {
    __shared__ LDS_DMA_ALIGN uint32_t ring[RD * RING_LANE_DW];
    __shared__ int32_t lds[CHK * RP];
    const uint32_t fpb = DEC_LANES >> __builtin_ctz(chn_lanes);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(seg[2u * 64u - 1u]) / fpb;
    const uint32_t end = (__builtin_amdgcn_readfirstlane(seg[3u * 64u + 63u]) + fpb - 1u) / fpb;
    for (uint32_t blk = lo + blockIdx.x; blk < end; blk += gridDim.x) {
        decode_block<MAXW, CHK, RD>(blk, ring, lds, words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info,
                                    perm, ablate);
        __syncthreads();
    }
}

#if BNF_TU == 0
/* ============================================================ frame chain (8f-1)
 * Which sync candidates are frames.  libFLAC finds the next frame where the previous one
 * ends (read_frame_ leaves the reader after the CRC-16 footer, frame_sync_ @0x10011760
 * looks for a sync code right there).  A frame's footer makes the CRC-16 of the whole
 * frame zero, so without decoding anything: candidate j follows valid candidate i iff
 * CRC-16(bytes[c_i, c_j)) == 0 and j itself has a valid header (CRC-8) and subframe walk;
 * the first such j is taken.
 * With P(y) = CRC-16(bytes[0, y)) and R(y) = P(y) * x^(8(N - y)) mod G (N = nbytes, x is
 * invertible mod G), CRC-16(bytes[a, b)) * x^(8(N - b)) = R(b) + R(a), so the test is the
 * equality of two per-candidate keys R(c).  R(c_j) is the XOR prefix over the gaps
 * g < j of CRC-16(gap g) * x^(8(N - end of g)).  The stream's frames are then the
 * successor chain from the first valid candidate at or after the first frame offset,
 * found by pointer doubling (log2 n rounds) and compacted in stream order. */
#define CHAIN_WIN (1u << 16) /* candidates looked at past a frame start for its successor */
#define KEY_OK 0x10000u      /* key bit 16: the candidate parsed as a valid frame start */

/* CRC-16 of the gap between consecutive candidates (the last one runs to nbytes), shifted
 * to the end of the buffer: one wave per gap, 16-byte-aligned slices per lane, lane CRCs
 * shifted to the buffer end and XOR-reduced. */
__global__ void __launch_bounds__(256) k_gap_crc(const uint8_t *__restrict__ bytes, uint64_t nbytes,
                                                 const uint64_t *__restrict__ cand, uint32_t ncand,
                                                 uint32_t *__restrict__ gap_w) {
    __shared__ uint16_t tab[8 * 256];
    for (uint32_t i = threadIdx.x; i < 8u * 256u; i += 256u) tab[i] = (&g_crc16_tab[0][0])[i];
    __syncthreads();
    const lds_u16 *T = (const lds_u16 *)(lds_u32 *)tab;
    const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (g >= ncand) return;
    const uint64_t b0 = cand[g];
    const uint64_t b1 = g + 1 < ncand ? cand[g + 1] : nbytes;
    const uint64_t slice = ((b1 - b0 + 63u) / 64u + 15u) & ~15ull;
    const uint64_t s0 = min(b1, b0 + slice * lane);
    const uint64_t s1 = min(b1, s0 + slice);
    uint32_t c = s0 < s1 ? crc16_shift(crc16_range(bytes, s0, s1, T), nbytes - s1) : 0u;
    for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o);
    if (lane == 0) gap_w[g] = c;
}

/* single-workgroup exclusive XOR scan of the gap words -> keys (in place), KEY_OK added */
__global__ void __launch_bounds__(1024) k_chain_keys(uint32_t *__restrict__ v, uint32_t n,
                                                     const bnf_frame_info *__restrict__ info) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t x = i < n ? v[i] : 0u;
        uint32_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if ((threadIdx.x & 63) >= (unsigned)o) incl ^= y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < 16; w++) wsum[w] ^= wsum[w - 1];
        __syncthreads();
        const uint32_t wprefix = (threadIdx.x >= 64) ? wsum[(threadIdx.x >> 6) - 1] : 0u;
        if (i < n) v[i] = (carry ^ wprefix ^ incl ^ x) | (info[i].status == BNF_ST_OK ? KEY_OK : 0u);
        __syncthreads();
        if (threadIdx.x == 1023) carry ^= wprefix ^ incl;
        __syncthreads();
    }
}

/* succ[i]: index of the candidate where frame i ends, -1 if none (or i is not valid);
 * head: the first valid candidate at or after first_off (atomicMin; preset to INT_MAX). */
__global__ void __launch_bounds__(256) k_chain_succ(const uint64_t *__restrict__ cand, uint32_t ncand,
                                                    const uint32_t *__restrict__ key, uint64_t first_off,
                                                    int32_t *__restrict__ succ, int32_t *__restrict__ head) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= ncand) return;
    int32_t s = -1;
    const uint32_t want = key[i];
    if (want & KEY_OK) {
        if (cand[i] >= first_off) atomicMin(head, (int32_t)i);
        const uint32_t jend = (uint32_t)min((uint64_t)ncand, (uint64_t)i + 1u + CHAIN_WIN);
        for (uint32_t j = i + 1; j < jend; j++)
            if (key[j] == want) {
                s = (int32_t)j;
                break;
            }
    }
    succ[i] = s;
}

/* pointer doubling: dst[i] = src[src[i]] */
__global__ void __launch_bounds__(256) k_chain_jump(const int32_t *__restrict__ src, int32_t *__restrict__ dst,
                                                    uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const int32_t a = src[i];
    dst[i] = a < 0 ? -1 : src[a];
}

/* mark[jump[i]] for every marked i.  Levels are applied from the longest jump down: the
 * marked set becomes {succ^t(head) : t < 2^levels}.  A mark set during the same launch
 * only adds further chain members, so the in-launch races are harmless. */
__global__ void __launch_bounds__(256) k_chain_mark(const int32_t *__restrict__ jump, uint32_t *__restrict__ mark,
                                                    uint32_t n, const int32_t *__restrict__ head, int first) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    if (first) {
        if ((int32_t)i == *head) mark[i] = 1u;
        return;
    }
    if (mark[i]) {
        const int32_t j = jump[i];
        if (j >= 0) mark[j] = 1u;
    }
}

/* write the chain in stream order: pos = exclusive scan of mark */
__global__ void __launch_bounds__(256) k_chain_compact(const uint64_t *__restrict__ cand, uint32_t ncand,
                                                       const bnf_frame_info *__restrict__ info,
                                                       const uint32_t *__restrict__ mark, const uint32_t *__restrict__ pos,
                                                       uint64_t *__restrict__ bs, uint32_t scratch_cap) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= ncand || !mark[i]) return;
    const uint32_t p = pos[i];
    if (p < scratch_cap) bs[p] = info[i].blocksize;
}

/* single-workgroup exclusive scan of v[0, *n) (64-bit), total in *total */
__global__ void __launch_bounds__(1024) k_scan_u64(uint64_t *__restrict__ v, const uint32_t *__restrict__ n_ptr,
                                                   uint32_t cap, uint64_t *__restrict__ total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    const uint32_t n = min(*n_ptr, cap);
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t x = i < n ? v[i] : 0ull;
        uint64_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(incl, o);
            if ((threadIdx.x & 63) >= (unsigned)o) incl += y;
        }
        if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < 16; w++) wsum[w] += wsum[w - 1];
        __syncthreads();
        const uint64_t wprefix = (threadIdx.x >= 64) ? wsum[(threadIdx.x >> 6) - 1] : 0ull;
        if (i < n) v[i] = carry + wprefix + incl - x;
        __syncthreads();
        if (threadIdx.x == 1023) carry += wprefix + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

/* outputs; frames starting at or past total_samples are dropped (frame_sync_'s EOS rule,
 * @0x100117a7): nframes = min(chain length, first such position) */
__global__ void __launch_bounds__(256) k_chain_emit(const uint64_t *__restrict__ cand, uint32_t ncand,
                                                    const bnf_frame_info *__restrict__ info,
                                                    const uint32_t *__restrict__ mark, const uint32_t *__restrict__ pos,
                                                    const uint64_t *__restrict__ out_sample, bnf_stream_params sp,
                                                    uint64_t *__restrict__ d_offs, uint64_t *__restrict__ d_os,
                                                    bnf_frame_info *__restrict__ d_info, uint32_t cap,
                                                    uint32_t *__restrict__ nframes) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= ncand || !mark[i]) return;
    const uint32_t p = pos[i];
    if (p >= cap) return;
    const uint64_t os = out_sample[p];
    if (sp.has_stream_info && sp.total_samples > 0 && os >= sp.total_samples) {
        atomicMin(nframes, p);
        return;
    }
    d_offs[p] = cand[i];
    if (d_os) d_os[p] = os;
    if (d_info) {
        bnf_frame_info fi = info[i];
        fi.out_sample = os;
        d_info[p] = fi;
    }
}
#endif /* BNF_TU == 0 */

#if BNF_TU == 3 || BNF_TU == 4 || BNF_TU == 7 /* TU 7: k_decode_sw, on the same helpers */
/* =============================================================== k_decode_st
 * Stereo fast path: one lane per 2-channel frame (both subframes, two independent bit
 * cursors), 64 frames per single-wave workgroup.  Same arithmetic as k_decode (read_frame_
 * @0x100118c0 and below) and the same PCM layouts (A15/A17), but:
 *   - the two channels' Rice + predictor chains interleave in one lane (ILP 2);
 *   - decorrelation (@0x10011a37-0x10011adb) and the PCM pack happen in registers, so
 *     there is no row buffer in LDS (LDS = the two bitstream rings, 16 KB per wave); a
 *     DPP transpose inside each lane quad turns each frame's chunk of PCM into one 64-byte
 *     store run (16 frames per store instruction);
 *   - FIXED (@0x10003810), LPC MMX-16 and LPC ia32 restores share one predictor: four
 *     v_dot2_i32_i16 over the history kept as packed 16-bit sample pairs (the pmaddwd
 *     shape).  That is exact while every sample fits 16 bits (coefficients always do:
 *     qlp precision <= 15): the products are exact and the sums wrap mod 2^32 like the
 *     MMX paddd, the ia32 imul/add and the FIXED int arithmetic.  Each channel tracks its
 *     sample range; a frame that leaves int16 is handed back.
 * Frames it declines (VERBATIM/CONSTANT/64-bit-path subframes, errors, truncation, CRC
 * mismatch, out-of-range samples, unsupported layouts) get BNF_FL_REDO and are decoded
 * again, exactly, by k_decode<8>, which runs after it on the same stream. */
#define ST_CHK 16 /* samples per chunk of k_decode_sw (one 64-byte FLACDecoder run per frame) */
#define ST2_CHK 32 /* samples per chunk of k_decode_st: one 128-byte FLACDecoder line per frame (round 5) */
#define ST_RD 8  /* 16-byte ring slots per lane and channel: two 64-byte groups */

struct StCh {
    BR b;
    uint32_t cp[4]; /* coefficient pairs (c[2k] | c[2k+1] << 16, 0 past the order) */
    uint32_t q[8];  /* history: q[m & 7] = s_m | s_(m-1) << 16 (16-bit halves) */
    int32_t sh;         /* effective shift of the libFLAC path */
    uint32_t k, km, k1, k32; /* Rice parameter, 31 - k, k + 1, 32 - k */
    uint32_t esc, left, pidx, nparts, psamples, plen, pesc, porder, order;
    uint32_t wasted;
    int32_t lim, mx, mn; /* operand range of the path, sample range seen */
};

/* lo | hi << 16 from the low halves */
DEV uint32_t st_pk(int32_t lo, int32_t hi) { return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u); }
typedef short st_s2 __attribute__((ext_vector_type(2)));
DEV int32_t st_d2(uint32_t a, uint32_t b, int32_t acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(st_s2, a), __builtin_bit_cast(st_s2, b), acc, false);
}
/* dot2 with a zero accumulator: the VOP3P form takes the inline 0 (the compiler picks
 * v_dot2c, whose accumulator is its destination, and copies a zero register into it first) */
DEV int32_t st_d2z(uint32_t a, uint32_t b) {
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

/* subframe header -> fast-path state; false: hand the frame back */
DEV bool st_setup(StCh &z, uint32_t bps, uint32_t bs, uint64_t limit) {
    SubHdr h;
    int32_t warm[8], coef[8], err = -1;
    const uint32_t st = parse_subframe_head<true, 8>(z.b, bps, bs, limit, h, warm, coef, err);
    if (st != BNF_ST_OK) return false;
    if (h.type != T_FIXED && h.type != T_LPC) return false;
    if (h.type == T_LPC && (h.order > 8 || h.path == P_WIDE)) return false;
    if (h.bps > 17) return false; /* samples cannot stay within int16 */
    int32_t c[8], w[8];
    bool in16 = true;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        c[t] = 0;
        w[t] = ((uint32_t)t < h.order) ? warm[t] : 0;
        in16 = in16 && w[t] >= -32768 && w[t] <= 32767;
    }
    if (!in16) return false;
    z.sh = 0;
    z.lim = 0x7FFF;
    if (h.type == T_LPC) {
#pragma unroll
        for (int t = 0; t < 8; t++) c[t] = ((uint32_t)t < h.order) ? coef[t] : 0;
        if (h.path == P_MMX16) z.sh = ((uint32_t)h.shift >= 32u) ? 31 : h.shift;
        else z.sh = h.shift & 31;
    } else { /* FIXED order o as LPC: 1 | 2,-1 | 3,-3,1 | 4,-6,4,-1 (32-bit wrap, shift 0) */
        const uint32_t o = h.order;
        c[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
        c[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
        c[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
        c[3] = o == 4 ? -1 : 0;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) z.cp[k] = st_pk(c[2 * k], c[2 * k + 1]);
#pragma unroll
    for (int t = 0; t < 8; t++) z.q[t] = st_pk(w[t], t ? w[t - 1] : 0);
    z.order = h.order;
    z.wasted = h.wasted;
    z.porder = h.porder;
    z.nparts = 1u << h.porder;
    z.psamples = h.porder ? bs >> h.porder : bs - h.order;
    z.plen = h.rice2 ? 5u : 4u;
    z.pesc = h.rice2 ? 31u : 15u;
    z.left = 0;
    z.pidx = 0;
    z.esc = 0;
    z.k = 0;
    z.km = 31;
    z.k1 = 1;
    z.k32 = 32;
    z.mx = 0;
    z.mn = 0;
    return true;
}

template <class Z>
DEV void st_partition(Z &z) { /* read_residual_partitioned_rice_ @0x10012da0 */
    const uint32_t kk = br_read(z.b, z.plen);
    z.left = (z.porder == 0 || z.pidx > 0) ? z.psamples : z.psamples - z.order;
    if (kk < z.pesc) {
        z.k = kk;
        z.esc = 0;
    } else {
        z.k = br_read(z.b, 5);
        z.esc = 1;
    }
    z.km = 31u - z.k;
    z.k1 = z.k + 1u;
    z.k32 = 32u - z.k;
    z.pidx++;
}

/* every DMA issued before the wave's `nst` youngest vector-memory ops has landed */
DEV void st_land(BR &b, uint32_t nst) {
    STAT(b.stats, 2);
    wait_vm_n(nst);
    b.vendw = b.iend * 4u;
    if (b.wi >= b.vendw) { /* outran the whole ring: blocking refill (rare) */
        br_refill(b);
        wait_vm();
        br_drained(b);
    }
}

/* branch-free advance by n <= 32 bits; the landing check waits only for the DMAs */
DEV void st_adv(BR &b, uint32_t n, uint32_t nst) {
    const int32_t t = (int32_t)b.s - (int32_t)n;
    const bool c = t < 0;
    b.s = (uint32_t)t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += c ? 1u : 0u;
    if (__builtin_expect(any_lane(b.wi >= b.vendw), 0)) st_land(b, nst);
    uint32_t off = ring_off(b, b.wi);
    asm volatile("" : "+v"(off) : "v"(b.lo));
    b.nx = b.lring[off];
}

/* one Rice codeword of a non-escaped partition (@0x10001b30 semantics, zig-zag) */
template <class Z>
DEV int32_t st_rice(Z &z, uint64_t limit, uint32_t &trunc, uint32_t nst) {
    const uint32_t w = br_peek(z.b);
    const uint32_t q = ffbh(w); /* ~0u for an empty window: slow */
    const bool slow = q >= z.k32; /* prefix + stop bit + k bits overrun the 32-bit window */
    uint32_t u = (q << z.k) | __builtin_amdgcn_ubfe(w, z.km - q, z.k);
    const bool anyslow = any_lane(slow);
    st_adv(z.b, slow ? 0u : q + z.k1, nst);
    if (__builtin_expect(anyslow, 0)) {
        STAT(z.b.stats, 3);
        if (slow) {
            uint32_t qq;
            if (!br_unary(z.b, qq, limit)) trunc = 1;
            u = (qq << z.k) | br_read(z.b, z.k);
        }
    }
    return (int32_t)((u >> 1) ^ (0u - (u & 1u)));
}

/* next residual, any partition state (warm-up excluded) */
template <class Z>
DEV int32_t st_next(Z &z, uint64_t limit, uint32_t &trunc, uint32_t nst) {
    while (z.left == 0) {
        if (z.pidx >= z.nparts) {
            trunc = 1;
            return 0;
        }
        st_partition(z);
    }
    z.left--;
    if (z.esc) return br_read_s(z.b, z.k);
    return st_rice(z, limit, trunc, nst);
}

/* pred(n) = sum_j c[j] * s_(n-1-j) for sample n = I (mod 8), both channels: four dot2 over
 * the pairs q[n-1], q[n-3], q[n-5], q[n-7] */
template <int I>
DEV void st_dot2(const StCh &a, const StCh &b, int32_t &pa, int32_t &pb) {
#define Q_(z, j) z.q[(I + 8 - (j)) & 7]
    pa = st_d2(a.cp[3], Q_(a, 7), st_d2(a.cp[2], Q_(a, 5), st_d2(a.cp[1], Q_(a, 3), st_d2z(a.cp[0], Q_(a, 1)))));
    pb = st_d2(b.cp[3], Q_(b, 7), st_d2(b.cp[2], Q_(b, 5), st_d2(b.cp[1], Q_(b, 3), st_d2z(b.cp[0], Q_(b, 1)))));
#undef Q_
}

/* The older taps of the NEXT sample's prediction (n = T + 1): pairs q[T-1], q[T-3], q[T-5],
 * all known at step T, so only the newest pair's dot2 remains between consecutive samples
 * (st_fin2). */
template <int T>
DEV void st_pre2(const StCh &a, const StCh &b, int32_t &pa, int32_t &pb) {
#define P_(z, j) z.q[(T + 8 - (j)) & 7]
    pa = st_d2(a.cp[3], P_(a, 6), st_d2(a.cp[2], P_(a, 4), st_d2z(a.cp[1], P_(a, 2))));
    pb = st_d2(b.cp[3], P_(b, 6), st_d2(b.cp[2], P_(b, 4), st_d2z(b.cp[1], P_(b, 2))));
#undef P_
}
/* pred = dot2(cp[0], q[n-1]) + pre for both channels (the critical-path pair) */
DEV void st_fin2(const StCh &a, const StCh &b, uint32_t qa, uint32_t qb, int32_t prea, int32_t preb, int32_t &pa,
                 int32_t &pb) {
    pa = st_d2(a.cp[0], qa, prea);
    pb = st_d2(b.cp[0], qb, preb);
}

DEV void st_range(StCh &z, int32_t s0, int32_t s1) {
    z.mx = max(z.mx, max(s0, s1));
    z.mn = min(z.mn, min(s0, s1));
}

/* Channel decorrelation of 4 sample pairs; wave-uniform assignment takes a scalar branch */
DEV void st_decor4(bool uni, uint32_t as_u, uint32_t as, int32_t (&L)[4], int32_t (&R)[4]) {
    const uint32_t a = uni ? as_u : as;
    if (a == 1) {
#pragma unroll
        for (int q = 0; q < 4; q++) R[q] = (int32_t)((uint32_t)L[q] - (uint32_t)R[q]);
    } else if (a == 2) {
#pragma unroll
        for (int q = 0; q < 4; q++) L[q] = (int32_t)((uint32_t)L[q] + (uint32_t)R[q]);
    } else if (a == 3) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t side = (uint32_t)R[q], mid = ((uint32_t)L[q] << 1) | (side & 1u);
            L[q] = (int32_t)(mid + side) >> 1;
            R[q] = (int32_t)(mid - side) >> 1;
        }
    }
}

/* The same with the wave's assignment known at compile time (AS >= 0; AS < 0: st_decor4).
 * Only for waves without wasted bits: the samples are then int16 (k_decode_st hands back a
 * frame that leaves int16), so M/S needs no 32-bit wrap and takes its 4-instruction form,
 * L = M + ((S + 1) >> 1), R = L - S: (2M + (S & 1) + S) >> 1 = M + ((S + (S & 1)) >> 1), and
 * S + (S & 1) and S + 1 halve to the same floor for both parities of S. */
template <int AS>
DEV void st_decor4t(bool uni, uint32_t as_u, uint32_t as, int32_t (&L)[4], int32_t (&R)[4]) {
    if (AS < 0) {
        st_decor4(uni, as_u, as, L, R);
    } else if (AS == 1) {
#pragma unroll
        for (int q = 0; q < 4; q++) R[q] = L[q] - R[q];
    } else if (AS == 2) {
#pragma unroll
        for (int q = 0; q < 4; q++) L[q] = L[q] + R[q];
    } else if (AS == 3) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int32_t l = L[q] + ((R[q] + 1) >> 1);
            R[q] = l - R[q];
            L[q] = l;
        }
    }
}

/* Decorrelation of two consecutive samples of both channels straight from the packed history
 * pairs (a: channel 0's, b: channel 1's; low half the later sample), in 16-bit lanes: the
 * FLACDecoder/FLACFileReader 16-bit layouts keep the low 16 bits of L and R, and every
 * operation here is exact mod 2^16 (M/S: ceil(S/2) = S - (S >> 1) stays within int16). */
typedef unsigned short st_u2 __attribute__((ext_vector_type(2)));
typedef short st_i2 __attribute__((ext_vector_type(2)));
template <int AS>
DEV void st_pair_lr(uint32_t a, uint32_t b, uint32_t &l, uint32_t &r) {
    const st_u2 x = __builtin_bit_cast(st_u2, a), y = __builtin_bit_cast(st_u2, b);
    st_u2 L = x, R = y;
    if (AS == 1) R = x - y;
    else if (AS == 2) L = x + y;
    else if (AS == 3) {
        const st_u2 h = y - __builtin_bit_cast(st_u2, __builtin_bit_cast(st_i2, b) >> (st_i2){1, 1});
        L = x + h;
        R = L - y;
    }
    l = __builtin_bit_cast(uint32_t, L);
    r = __builtin_bit_cast(uint32_t, R);
}
/* the four 16-bit L | R << 16 words of samples n-3..n from the pairs (n-3, n-2) and (n-1, n) */
template <int AS>
DEV u32x4 st_pack4(uint32_t a01, uint32_t b01, uint32_t a23, uint32_t b23) {
    uint32_t l01, r01, l23, r23;
    st_pair_lr<AS>(a01, b01, l01, r01);
    st_pair_lr<AS>(a23, b23, l23, r23);
    return u32x4{__builtin_amdgcn_perm(r01, l01, 0x07060302u), __builtin_amdgcn_perm(r01, l01, 0x05040100u),
                 __builtin_amdgcn_perm(r23, l23, 0x07060302u), __builtin_amdgcn_perm(r23, l23, 0x05040100u)};
}

/* Pack and store samples n..n+3 of this lane's frame (nv of them valid); returns whether
 * this lane issued a store.  dst: the frame's first byte in the layout (planar: channel 0). */
template <int FMT>
DEV bool st_emit4(uint8_t *dst, uint32_t n, uint32_t nv, bool al, uint32_t bs, const int32_t (&L)[4],
                  const int32_t (&R)[4]) {
    if (nv == 0) return false;
    if (FMT == BNF_OUT_FLACDECODER || FMT == BNF_OUT_FILEREADER) { /* 16-bit L | R << 16 */
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) w[q] = __builtin_amdgcn_perm((uint32_t)R[q], (uint32_t)L[q], 0x05040100u);
        uint32_t *o = (uint32_t *)(dst + (uint64_t)n * 4u);
        if (al && nv == 4) *(uint4 *)o = make_uint4(w[0], w[1], w[2], w[3]);
        else
            for (uint32_t q = 0; q < nv; q++) o[q] = w[q];
    } else if (FMT == BNF_OUT_INTERLEAVED32) {
        int32_t *o = (int32_t *)(dst + (uint64_t)n * 8u);
        if (al && nv == 4) {
            *(int4 *)o = make_int4(L[0], R[0], L[1], R[1]);
            *(int4 *)(o + 4) = make_int4(L[2], R[2], L[3], R[3]);
        } else {
            for (uint32_t q = 0; q < nv; q++) { o[2 * q] = L[q]; o[2 * q + 1] = R[q]; }
        }
    } else { /* PLANAR32: channel 0 then channel 1, bs samples each */
        int32_t *o0 = (int32_t *)dst + n, *o1 = (int32_t *)dst + bs + n;
        if (al && nv == 4) {
            *(int4 *)o0 = make_int4(L[0], L[1], L[2], L[3]);
            *(int4 *)o1 = make_int4(R[0], R[1], R[2], R[3]);
        } else {
            for (uint32_t q = 0; q < nv; q++) { o0[q] = L[q]; o1[q] = R[q]; }
        }
    }
    return true;
}

/* 1-deep ring pipeline in 64-byte groups: the ring holds the cursor's group and the next
 * one; once the cursor has entered the newer of the two, the older group's slots take the
 * group after it (four 16-byte LDS-DMAs into one half cache line).  Fetching whole groups
 * rather than every free block keeps a cursor's refills to one per 64 bytes consumed: a
 * cursor's line does not survive in L2 between chunks (64 x 2 cursors per wave), so each
 * refill costs a line fetch from the fabric.  A group fetched now lands before the next
 * refill's wait; the cursor needs it only after the ~64 bytes of the current group.
 * Whole wave: exec-masked, and only the slot groups some lane needs are issued. */
DEV uint32_t st_refill_issue(BR &b, bool want) { /* returns a lower bound of the DMA instructions issued */
    const uint32_t cg = (b.wi >> 2) & ~3u; /* first block of the cursor's group */
    const bool go = want && b.iend == cg + 4u;
    const uint32_t h = b.iend & 4u; /* the free group's slots: 0-3 or 4-7 */
    /* a group wholly inside the buffer: one address, the four blocks by immediate offset
     * (round 5: ~20 fewer VALU per refill and channel); the buffer's last blocks clamped */
    const bool whole = b.iend + 3u < b.nblk;
    const uint32_t *a = b.w + (uint64_t)b.iend * 4u;
    uint32_t nd = 0;
#pragma unroll
    for (int g = 0; g < 2; g++) {
        const bool gg = go && h == 4u * (uint32_t)g;
        if (__any(gg)) {
            nd += 4u;
            if (gg) {
                lds_u32 *row = b.ring + 4u * (uint32_t)g * RING_LANE_DW;
                if (__builtin_expect(whole, 1)) {
                    lds_dma16_off<0>(a, row);
                    lds_dma16_off<16>(a, row + RING_LANE_DW);
                    lds_dma16_off<32>(a, row + 2 * RING_LANE_DW);
                    lds_dma16_off<48>(a, row + 3 * RING_LANE_DW);
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) dma_block(b, b.iend + (uint32_t)k, 4u * (uint32_t)g + (uint32_t)k);
                }
            }
        }
    }
    if (go) b.iend += 4u;
    return nd;
}


/* Fused-path cursor (4-slot ring).  ra is the LDS byte offset of ring word wi inside the
 * channel's ring: bits 2-3 word in block, 4-9 lane, 10-11 slot.  Moving it one word on is
 * ((ra | 0x3F3) + c) & 0x1C0C | lane bits: the ones in bits 0-1 turn +c into +4, the ones in
 * bits 4-9 carry a block wrap into the slot. */
DEV uint32_t st_ra(uint32_t wi, uint32_t lane) { return ((wi & 3u) << 2) | (lane << 4) | (((wi >> 2) & 7u) << 10); }
/* Advance by n <= 32 bits without the landing check: s - n borrows exactly when the window
 * moves on a word, and that borrow steps wi and ra (v_sub_co / v_addc). */
DEV void st_adv_nc(BR &b, uint32_t n, uint32_t laneb) {
    uint32_t t;
    const bool c = __builtin_usub_overflow(b.s, n, &t);
    b.s = t & 31u;
    b.hi = c ? b.lo : b.hi;
    b.lo = c ? __builtin_bswap32(b.nx) : b.lo;
    b.wi += (uint32_t)c;
    b.ra = (((b.ra | 0x3F3u) + (uint32_t)c) & 0x1C0Cu) | laneb;
}
DEV void st_next_word(BR &b) { b.nx = *(const lds_u32 *)((const __attribute__((address_space(3))) uint8_t *)b.ring + b.ra); }
DEV void st_resync(BR &b, uint32_t lane) { /* after generic-reader moves: ra, vlim from wi, vendw */
    b.ra = st_ra(b.wi, lane);
    b.vlim = b.vendw - 1u;
}
/* rare cases of a fused step, per channel: the cursor entered ring words not known to have
 * landed (wait for the DMAs, read the word again), or a unary prefix too long for the window
 * (the lane did not advance: decode the codeword with the generic reader) */
template <class Z>
DEV void st_rare(Z &z, bool sl, bool ld, uint32_t &u, uint64_t limit, uint32_t &trunc, uint32_t nst,
                uint32_t lane) {
    if (any_lane(ld)) {
        st_land(z.b, nst); /* lands the next two words (the check runs every other step) */
        if (z.b.wi + 1u >= z.b.vendw) { /* the word after wi is beyond the ring: refill (rare) */
            wait_vm();
            br_refill(z.b);
            wait_vm();
            br_drained(z.b);
        }
        st_next_word(z.b);
    }
    if (any_lane(sl)) {
        STAT(z.b.stats, 3);
        if (sl) {
            uint32_t qq;
            if (!br_unary(z.b, qq, limit)) trunc = 1;
            u = (qq << z.k) | br_read(z.b, z.k);
        }
    }
    st_resync(z.b, lane);
}

/* 4x4 transpose of 16-byte units across the 4 lanes of each quad, in registers (DPP
 * quad_perm, no LDS): on entry v[e] is unit e of this lane's frame, on exit v[i] is unit
 * (lane & 3) of the frame of quad lane i.  Two exchange stages (lane bit 0 with unit bit 0,
 * then bit 1): unit e is replaced by the partner's unit e ^ b where (lane ^ e) & b. */
template <int CTRL>
DEV uint32_t st_qperm(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true); }
template <int CTRL, int B>
DEV void st_quad_stage(u32x4 (&v)[4], bool pbit) {
    u32x4 n[4];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const bool take = ((e & B) != 0) != pbit; /* (lane ^ e) & B */
        const u32x4 o = v[e ^ B];
        const u32x4 x = u32x4{st_qperm<CTRL>(o.x), st_qperm<CTRL>(o.y), st_qperm<CTRL>(o.z), st_qperm<CTRL>(o.w)};
        n[e] = take ? x : v[e];
    }
#pragma unroll
    for (int e = 0; e < 4; e++) v[e] = n[e];
}
DEV void st_quad_transpose(u32x4 (&v)[4], bool podd, bool phi) {
    st_quad_stage<0xB1, 1>(v, podd); /* quad_perm [1,0,3,2] */
    st_quad_stage<0x4E, 2>(v, phi);  /* quad_perm [2,3,0,1] */
}
/* quad lane i's 64-bit value (DPP quad_perm [i,i,i,i]) */
DEV uint64_t st_quad_bcast64(uint64_t x, uint32_t i) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    switch (i) {
    case 0: lo = st_qperm<0x00>(lo); hi = st_qperm<0x00>(hi); break;
    case 1: lo = st_qperm<0x55>(lo); hi = st_qperm<0x55>(hi); break;
    case 2: lo = st_qperm<0xAA>(lo); hi = st_qperm<0xAA>(hi); break;
    default: lo = st_qperm<0xFF>(lo); hi = st_qperm<0xFF>(hi); break;
    }
    return ((uint64_t)hi << 32) | lo;
}

/* The restore and output of sample T of both channels, given the folded Rice values u0 / u1
 * (zig-zag applied here). */
template <int T, int FMT, int AS, int PO, int NPK> /* PO: the group's first unit in pk */
DEV void st_lpc_out(StCh &z0, StCh &z1, uint32_t u0, uint32_t u1, int32_t (&L)[4], int32_t (&R)[4], bool as_uni,
                    uint32_t as_u, uint32_t as, uint8_t *dst, uint32_t nbase, bool al, uint32_t bs, bool store,
                    u32x4 (&pk)[NPK], int32_t &pre0, int32_t &pre1, bool anyw) {
    constexpr bool STG = (FMT == BNF_OUT_FLACDECODER || FMT == BNF_OUT_FILEREADER);
    int32_t p0, p1, n0, n1;
    st_fin2(z0, z1, z0.q[(T + 7) & 7], z1.q[(T + 7) & 7], pre0, pre1, p0, p1); /* this sample's prediction */
    st_pre2<T>(z0, z1, n0, n1);                                                /* the next one's older taps */
    pre0 = n0;
    pre1 = n1;
    const int32_t s0 = (int32_t)(((u0 >> 1) ^ (0u - (u0 & 1u))) + (uint32_t)(p0 >> z0.sh));
    const int32_t s1 = (int32_t)(((u1 >> 1) ^ (0u - (u1 & 1u))) + (uint32_t)(p1 >> z1.sh));
    if (T & 1) {
        st_range(z0, L[(T + 3) & 3], s0);
        st_range(z1, R[(T + 3) & 3], s1);
    }
    z0.q[T] = __builtin_amdgcn_perm(z0.q[(T + 7) & 7], (uint32_t)s0, 0x05040100u);
    z1.q[T] = __builtin_amdgcn_perm(z1.q[(T + 7) & 7], (uint32_t)s1, 0x05040100u);
    L[T & 3] = s0;
    R[T & 3] = s1;
    if ((T & 3) == 3) {
        if (AS < 0 && __builtin_expect(anyw, 0)) { /* wasted bits (wave-uniform test; AS >= 0: none) */
#pragma unroll
            for (int q = 0; q < 4; q++) {
                L[q] = (int32_t)((uint32_t)L[q] << z0.wasted);
                R[q] = (int32_t)((uint32_t)R[q] << z1.wasted);
            }
        }
        if (STG && AS >= 0) { /* no wasted bits: the history pairs hold the samples */
            pk[PO + (T >> 2)] = st_pack4<AS>(z0.q[(T + 6) & 7], z1.q[(T + 6) & 7], z0.q[T], z1.q[T]);
            return;
        }
        st_decor4t<AS>(as_uni, as_u, as, L, R);
        if (STG) {
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; q++) w[q] = __builtin_amdgcn_perm((uint32_t)R[q], (uint32_t)L[q], 0x05040100u);
            pk[PO + (T >> 2)] = u32x4{w[0], w[1], w[2], w[3]};
        } else if (store) {
            st_emit4<FMT>(dst, nbase + (uint32_t)T - 3u, 4u, al, bs, L, R);
        }
    }
}

/* Two Rice codewords of one channel from one 32-bit window (the pair fits when their lengths
 * sum to <= 32: always at C2's parameters, k = 8 and ~10-bit codewords).  The second's prefix
 * is counted in the window shifted past the first; the prefix counts are taken of (x | 1), so
 * a prefix that runs off the window reads as 31 zeros and the pair as not fitting (a fast
 * v_or instead of a clamp after the count, round 5).  Returns the bits
 * both take, or 0 with sl set (the lane then decodes the two with the generic reader). */
DEV uint32_t st_rice_pair(const StCh &z, uint32_t &ua, uint32_t &ub, bool &sl) {
    const uint32_t w = br_peek(z.b);
    const uint32_t qa = (uint32_t)__builtin_clz(w | 1u); /* 31 for an empty window: n > 32 below */
    const uint32_t la = qa + z.k1;
    const uint32_t w2 = w << (la & 31u); /* la >= 32: garbage, and n > 32 below */
    const uint32_t qb = (uint32_t)__builtin_clz(w2 | 1u);
    ua = (qa << z.k) | __builtin_amdgcn_ubfe(w, z.km - qa, z.k);
    ub = (qb << z.k) | __builtin_amdgcn_ubfe(w2, z.km - qb, z.k);
    const uint32_t n = la + qb + z.k1;
    sl = n > 32u;
    return sl ? 0u : n;
}
/* rare cases of a pair step, per channel: the ring words past the landed ones, or a pair that
 * does not fit the window (both codewords through the generic reader) */
DEV void st_rare_pair(StCh &z, bool sl, bool ld, uint32_t &ua, uint32_t &ub, uint64_t limit, uint32_t &trunc,
                      uint32_t nst, uint32_t lane) {
    if (any_lane(ld)) {
        st_land(z.b, nst);
        if (z.b.wi + 1u >= z.b.vendw) {
            wait_vm();
            br_refill(z.b);
            wait_vm();
            br_drained(z.b);
        }
        st_next_word(z.b);
    }
    if (any_lane(sl)) {
        STAT(z.b.stats, 3);
        if (sl) {
            uint32_t qq;
            if (!br_unary(z.b, qq, limit)) trunc = 1;
            ua = (qq << z.k) | br_read(z.b, z.k);
            if (!br_unary(z.b, qq, limit)) trunc = 1;
            ub = (qq << z.k) | br_read(z.b, z.k);
        }
    }
    st_resync(z.b, lane);
}
/* Samples T and T + 1 (T even) of both channels: one window peek, one cursor advance and one
 * ring read per channel for two codewords, then
 * the two restores in order. */
template <int T, int FMT, int AS, int PO, int NPK>
DEV void st_fused_pair(StCh &z0, StCh &z1, int32_t (&L)[4], int32_t (&R)[4], uint64_t limit, uint32_t &trunc,
                       uint32_t nq, bool as_uni, uint32_t as_u, uint32_t as, uint8_t *dst, uint32_t nbase, bool al,
                       uint32_t bs, bool store, u32x4 (&pk)[NPK], int32_t &pre0, int32_t &pre1,
                       uint32_t lane, bool anyw) {
    static_assert((T & 1) == 0, "pairs start on even samples");
    constexpr bool STG = (FMT == BNF_OUT_FLACDECODER || FMT == BNF_OUT_FILEREADER);
    constexpr uint32_t spg = (FMT == BNF_OUT_INTERLEAVED32 || FMT == BNF_OUT_PLANAR32) ? 2u : 1u;
    const uint32_t nqt = nq + ((!STG && T >= 4 && store) ? spg : 0u); /* + this group's direct store */
    uint32_t u0a, u0b, u1a, u1b;
    bool sl0, sl1;
    const uint32_t n0 = st_rice_pair(z0, u0a, u0b, sl0), n1 = st_rice_pair(z1, u1a, u1b, sl1);
    const uint32_t laneb = lane << 4;
    st_adv_nc(z0.b, n0, laneb);
    st_adv_nc(z1.b, n1, laneb);
    /* checked at every other pair (T = 0, 4): the word read now (read again after a landing)
     * and the one the next pair reads must have landed; that pair moves wi by at most one,
     * and the pair after it checks its own word again */
    constexpr bool CHK = (T & 2) == 0;
    const bool ld0 = CHK && z0.b.wi >= z0.b.vlim, ld1 = CHK && z1.b.wi >= z1.b.vlim;
    st_next_word(z0.b);
    st_next_word(z1.b);
    if (__builtin_expect(any_lane(sl0 || sl1 || ld0 || ld1), 0)) {
        st_rare_pair(z0, sl0, ld0, u0a, u0b, limit, trunc, nqt, lane);
        st_rare_pair(z1, sl1, ld1, u1a, u1b, limit, trunc, nqt, lane);
    }
    st_lpc_out<T, FMT, AS, PO, NPK>(z0, z1, u0a, u1a, L, R, as_uni, as_u, as, dst, nbase, al, bs, store, pk, pre0, pre1, anyw);
    st_lpc_out<T + 1, FMT, AS, PO, NPK>(z0, z1, u0b, u1b, L, R, as_uni, as_u, as, dst, nbase, al, bs, store, pk, pre0, pre1, anyw);
}

/* One sample of both channels on the general path: warm-up, partition headers anywhere,
 * escaped partitions, the frame's last partial chunk.  Returns whether a store was issued. */
template <int T, int FMT>
DEV bool st_gen_step(StCh &z0, StCh &z1, int32_t (&L)[4], int32_t (&R)[4], uint64_t limit, uint32_t &trunc,
                     uint32_t nst, bool as_uni, uint32_t as_u, uint32_t as, uint8_t *dst, uint32_t n, bool valid,
                     bool al, uint32_t bs, bool store) {
    const bool v = valid && n < bs;
    int32_t s0 = 0, s1 = 0;
    if (v) {
        int32_t p0, p1;
        st_dot2<T>(z0, z1, p0, p1);
        if (n < z0.order) s0 = (int32_t)(int16_t)z0.q[T];
        else s0 = (int32_t)((uint32_t)st_next(z0, limit, trunc, nst) + (uint32_t)(p0 >> z0.sh));
        if (n < z1.order) s1 = (int32_t)(int16_t)z1.q[T];
        else s1 = (int32_t)((uint32_t)st_next(z1, limit, trunc, nst) + (uint32_t)(p1 >> z1.sh));
        st_range(z0, s0, s0);
        st_range(z1, s1, s1);
        z0.q[T] = __builtin_amdgcn_perm(z0.q[(T + 7) & 7], (uint32_t)s0, 0x05040100u);
        z1.q[T] = __builtin_amdgcn_perm(z1.q[(T + 7) & 7], (uint32_t)s1, 0x05040100u);
    }
    L[T & 3] = (int32_t)((uint32_t)s0 << z0.wasted);
    R[T & 3] = (int32_t)((uint32_t)s1 << z1.wasted);
    bool stored = false;
    if ((T & 3) == 3) {
        const uint32_t nq = n - 3u;
        const uint32_t nv = (valid && nq < bs) ? min(4u, bs - nq) : 0u;
        st_decor4(as_uni, as_u, as, L, R);
        if (store) stored = st_emit4<FMT>(dst, nq, nv, al, bs, L, R);
    }
    return stored;
}

template <int FMT>
__global__ void __launch_bounds__(64, 2) k_decode_st(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                     uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes,
                                                     uint8_t *__restrict__ out, uint64_t out_bytes,
                                                     bnf_frame_info *__restrict__ info,
                                                     const uint32_t *__restrict__ perm, uint32_t ablate,
                                                     const uint32_t *__restrict__ crcp) {
    constexpr bool STG = (FMT == BNF_OUT_FLACDECODER || FMT == BNF_OUT_FILEREADER);
    constexpr uint32_t ST_SPG = (FMT == BNF_OUT_INTERLEAVED32 || FMT == BNF_OUT_PLANAR32) ? 2u : 1u; /* stores per 4 samples */
    /* 16 KB: both channels' bitstream rings; 4 KB: the flush tile (20 KB, 8 waves per CU) */
    __shared__ LDS_DMA_ALIGN uint32_t ring[2 * ST_RD * RING_LANE_DW + 1024]; /* the two rings, then the 4 KB flush tile */
    static_assert((ST_RD * RING_LANE_DW * 4) % 1024 == 0, "channel 1's ring base must stay 1 KiB aligned (LDS-DMA)");
    const uint32_t lane = threadIdx.x;
    const uint32_t slot = blockIdx.x * 64u + lane;
    const uint32_t f = (perm && slot < nframes) ? perm[slot] : slot; /* decode order (k_order) */
    const uint64_t limit = nbytes * 8u;
    bnf_frame_info fi;
    const bool have = f < nframes;
    if (have) fi = info[f];
    const bool mine = have && fi.status == BNF_ST_OK && (fi.flags & BNF_FL_ST) && !(fi.flags & BNF_FL_REDO) &&
                      (!(ablate & BNF_MODE_WREDO) || (fi.flags & BNF_FL_WAVE_REDO));
    if (!__any(mine)) return;

    /* layouts this kernel writes; anything else (and every skip rule of k_decode's setup)
     * goes back to k_decode<8> */
    uint64_t stride = 0;
    bool ok = mine && fi.channels == 2 && chn_lanes >= 2;
    if (FMT == BNF_OUT_FLACDECODER) { stride = 4; ok = ok && fi.bps == 16 && sp.channels >= 2; }
    else if (FMT == BNF_OUT_FILEREADER) { stride = 4; ok = ok && sp.channels == 2 && sp.bps == 16; }
    else if (FMT == BNF_OUT_INTERLEAVED32) { stride = 8; ok = ok && sp.channels == 2; }
    else { stride = 4ull * sp.channels; ok = ok && sp.channels == 2; }
    const uint32_t bs = ok ? fi.blocksize : 0u;
    const uint64_t os = ok ? fi.out_sample : 0u;
    ok = ok && (os + bs) * stride <= out_bytes;
    uint8_t *dst = out + os * stride; /* the frame's first byte (planar: channel 0's) */
    const bool al = (((uintptr_t)dst) & 15u) == 0 && (FMT != BNF_OUT_PLANAR32 || (bs & 3u) == 0);

    StCh z0, z1;
    lds_u32 *ring0 = (lds_u32 *)ring, *ring1 = (lds_u32 *)ring + ST_RD * RING_LANE_DW;
    br_init(z0.b, words, nbytes, ring0, lane, ST_RD);
    br_init(z1.b, words, nbytes, ring1, lane, ST_RD);
    z0.b.stats = z1.b.stats = (ablate & 0x100u) != 0;
    STAT(z0.b.stats, 5);
    const bool tmon = z0.b.stats;
    const uint64_t t_start = tnow(tmon);
    uint64_t tm_dec = 0, tm_ref = 0, tm_pack = 0;
    if (ok) {
        br_seek(z0.b, fi.frame_off * 8u + fi.sub_start[0]);
        ok = st_setup(z0, sub_bps(fi, 0), bs, limit);
    }
    if (ok) {
        br_seek(z1.b, fi.frame_off * 8u + fi.sub_start[1]);
        ok = st_setup(z1, sub_bps(fi, 1), bs, limit);
    }
    const uint32_t as = ok ? fi.assignment : 0u;
    const bool anyw = any_lane(ok && (z0.wasted | z1.wasted) != 0u);
    const uint32_t as_u = __builtin_amdgcn_readfirstlane(as);
    const bool as_uni = !any_lane(ok && as != as_u);
    /* the fused chunks' compile-time assignment: one per wave, no wasted bits */
    const int as_fix = (as_uni && !anyw && as_u <= 3u) ? (int)as_u : -1;
    /* the flush's staging: the 4 KB past the two rings, not
     * an LDS-DMA target */
    lds_u32x4 *stg = (lds_u32x4 *)((lds_u32 *)ring + 2u * ST_RD * RING_LANE_DW);
    static_assert(sizeof(ring) >= (2 * ST_RD * RING_LANE_DW + 1024) * 4, "the flush's 4 KB staging tile lies past the two rings");

    uint32_t mybs = ok ? bs : 0u;
    for (int o = 32; o > 0; o >>= 1) mybs = max(mybs, (uint32_t)__shfl_xor(mybs, o));
    const uint32_t nchunks = (mybs + ST2_CHK - 1) / ST2_CHK;
    uint32_t trunc = 0;
    wait_vm(); /* setup loads done: the store count starts from zero */
    uint32_t nst = 0; /* vector-memory ops (PCM stores) issued by this wave since the last refill's DMAs */
    const bool sto = !(ablate & 2u);
    /* refill: wait for the previous refill's DMAs (every store since stays in flight), then
     * issue the next blocks; stores issued after it are younger.  (Round 5: waiting for the
     * refill before last instead, with the landing check covering the newest group, measured
     * 32% slower on C2: a lane entering its newest group stalls the whole wave.) */
    auto refill = [&](bool want) {
        wait_vm_n(nst);
        z0.b.vendw = z0.b.iend * 4u;
        z1.b.vendw = z1.b.iend * 4u;
        st_refill_issue(z0.b, want);
        st_refill_issue(z1.b, want);
        nst = 0;
    };
    const uint64_t t_loop = tnow(tmon);
    for (uint32_t kc = 0; kc < nchunks; kc++) {
        const uint64_t ta = tnow(tmon);
        const uint32_t n0 = kc * ST2_CHK;
        const bool valid = ok && n0 < bs;
        bool fast = valid && n0 >= 8u && n0 + ST2_CHK <= bs && !(ablate & 12u);
        if (fast) { /* partition headers at the chunk boundary (aligned partitions) */
            if (z0.left == 0 && z0.pidx < z0.nparts) st_partition(z0);
            if (z1.left == 0 && z1.pidx < z1.nparts) st_partition(z1);
            fast = !z0.esc && !z1.esc && z0.left >= ST2_CHK && z1.left >= ST2_CHK;
        }
        const bool fused = !any_lane(valid && !fast);
        u32x4 pk[4], pk0[4]; /* STG: the chunk's eight 16-byte units of this lane's frame run (128 bytes): pk0 from the first half, pk from the second */
        if (fused) {
            if (valid) {
                STAT(z0.b.stats, 0);
                int32_t pre0, pre1;
                st_pre2<7>(z0, z1, pre0, pre1); /* older taps of the chunk's first sample */
                st_resync(z0.b, lane);
                st_resync(z1.b, lane);
                /* the chunk's 4 groups of 8 samples, a refill after the second; AS >= 0: the
                 * wave's one assignment, no wasted bits (st_decor4t), compiled per assignment */
                auto chunk = [&](auto as_c) {
                    constexpr int AS = decltype(as_c)::value;
                    auto group = [&](auto g_c, uint32_t nb) {
                        constexpr uint32_t G = decltype(g_c)::value;
                        int32_t L[4], R[4];
                        const uint32_t nq = nst + (STG ? 0u : G * 2u * ST_SPG); /* stores issued since the DMAs (at least) */
#define FPAIR(T) st_fused_pair<T, FMT, AS, 2 * G, 4>(z0, z1, L, R, limit, trunc, nq, as_uni, as_u, as, dst, nb, al, bs, sto, pk, pre0, pre1, lane, anyw)
                        FPAIR(0); FPAIR(2); FPAIR(4); FPAIR(6);
#undef FPAIR
                    };
#pragma unroll 1
                    for (uint32_t h = 0; h < 2; h++) { /* two halves of 16 samples, a refill between */
                        const uint32_t nb = n0 + 16u * h;
                        group(std::integral_constant<uint32_t, 0>(), nb);
                        group(std::integral_constant<uint32_t, 1>(), nb + 8u);
                        if (h == 0) {
                            if (STG) {
#pragma unroll
                                for (int u = 0; u < 4; u++) pk0[u] = pk[u];
                            } else if (sto) {
                                nst += 4u * ST_SPG;
                            }
                            refill(true); /* the chunk's first half is decoded: n0 + 16 < bs */
                            st_resync(z0.b, lane);
                            st_resync(z1.b, lane);
                        }
                    }
                };
                switch (as_fix) {
                case 0: chunk(std::integral_constant<int, 0>()); break;
                case 1: chunk(std::integral_constant<int, 1>()); break;
                case 2: chunk(std::integral_constant<int, 2>()); break;
                case 3: chunk(std::integral_constant<int, 3>()); break;
                default: chunk(std::integral_constant<int, -1>()); break;
                }
                z0.left -= ST2_CHK;
                z1.left -= ST2_CHK;
            } else {
                refill(false); /* the wave's mid-chunk refill, for this lane's wait */
            }
            if (!STG && sto && any_lane(valid)) nst += 4u * ST_SPG;
        } else {
            STAT(z0.b.stats, 1);
#pragma unroll 1
            for (uint32_t g = 0; g < ST2_CHK / 8; g++) {
                int32_t L[4], R[4];
                const uint32_t nb = n0 + g * 8u;
                bool st0, st1;
#define GSTEP(T) st_gen_step<T, FMT>(z0, z1, L, R, limit, trunc, nst, as_uni, as_u, as, dst, nb + T, valid, al, bs, sto)
                GSTEP(0); GSTEP(1); GSTEP(2);
                st0 = GSTEP(3);
                if (any_lane(st0)) nst += 1u; /* at least one store instruction */
                GSTEP(4); GSTEP(5); GSTEP(6);
                st1 = GSTEP(7);
                if (any_lane(st1)) nst += 1u;
#undef GSTEP
                if (g == 1) refill(valid && nb + 8u < bs);
            }
        }
        const uint64_t tb = tnow(tmon);
        tm_dec += tb - ta;
        refill(valid && n0 + ST2_CHK < bs);
        const uint64_t tc = tnow(tmon);
        tm_ref += tc - tb;
        if (STG && fused) {
            /* flush: every frame's 128-byte run of the chunk as one whole cache line.  Two
             * rounds of 32 frames through the 4 KB staging tile: the round's lanes write their
             * eight units (the slot of unit u of frame f is u ^ (f & 7): conflict-free
             * ds_write_b128), then lane l reads unit l & 7 of frame (l >> 3) + 8 i and stores
             * it: each store instruction writes 8 whole lines.  Every lane is active here
             * (a lane whose frame has ended stores nothing: its run address is 0). */
            uint64_t run = (valid && sto) ? (uint64_t)(uintptr_t)(dst + (uint64_t)n0 * 4u) : 0ull;
            /* timing ablation 0x10000000: the same stores into one 64 KB window per XCD (an
             * L2-resident footprint: the HBM write traffic without the instructions); wrong PCM */
            if ((ablate & 0x10000000u) && run && out_bytes >= (1u << 20)) /* the window needs 513 KB */
                run = (uint64_t)(uintptr_t)(out + (uint64_t)(blockIdx.x & 7u) * 65536u + lane * 1024u + ((n0 * 4u) & 1023u));
            const uint32_t rlo = (uint32_t)run, rhi = (uint32_t)(run >> 32);
            const uint32_t fr = lane & 31u, ul = lane & 7u;
#pragma unroll
            for (uint32_t r = 0; r < 2; r++) {
                if ((lane >> 5) == r) {
#pragma unroll
                    for (uint32_t u = 0; u < 8; u++) lds_st128(stg + fr * 8u + (u ^ (fr & 7u)), u < 4 ? pk0[u] : pk[u - 4]);
                }
                lds_sync();
                /* the round's four units and run addresses, one wait for all of them */
                u32x4 v[4];
                uint64_t a[4];
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    const uint32_t f = (lane >> 3) + 8u * i;      /* frame within the round */
                    v[i] = lds_ld128(stg + f * 8u + (ul ^ (f & 7u)));
                    const uint32_t src = (32u * r + f) * 4u;     /* its lane, for ds_bpermute */
                    a[i] = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)rhi) << 32) |
                           (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)rlo);
                }
                lds_sync();
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    if (a[i]) gst128(a[i] + 16u * ul, v[i]);
                    if (any_lane(a[i] != 0)) nst += 1u;
                }
            }
        }
        tm_pack += tnow(tmon) - tc;
    }
    const uint64_t t_loopend = tnow(tmon);

    /* ---- end of the last subframe, zero padding, CRC-16 (read_frame_ tail) */
    uint32_t crc_read = 0;
    uint64_t end_byte = 0, resume = 0;
    if (ok) {
        if (z0.mx > z0.lim || z0.mn < -z0.lim - 1 || z1.mx > z1.lim || z1.mn < -z1.lim - 1) ok = false;
        if (trunc) ok = false;
    }
    if (ok) {
        while (z1.pidx < z1.nparts) { /* finish_partitions */
            const uint32_t kk = br_read(z1.b, z1.plen);
            if (kk >= z1.pesc) br_read(z1.b, 5);
            z1.pidx++;
        }
        const uint32_t padbits = (uint32_t)((8u - (br_pos(z1.b) & 7u)) & 7u);
        const uint32_t zp = br_read(z1.b, padbits);
        if (br_pos(z1.b) > limit || zp != 0) ok = false;
        end_byte = br_pos(z1.b) >> 3;
        crc_read = br_read(z1.b, 16);
        if (br_pos(z1.b) > limit) ok = false;
        resume = br_pos(z1.b);
    }
    /* CRC-16 of the frame bytes (read_frame_'s footer check @0x10011a01), by the table-free
     * zero test over frame + footer (st_crc16_ok; round 6: 10.8 -> 10.5 ms on C2 against round
     * 5's 11-bit LDS tables, same box), continuing k_parse's prefix of the lines before channel
     * 1 when the batch has one (st_crc16_frame: 10.7 -> 9.6 ms).  The tail is bound by the
     * re-read: every wave of a CU reaches it together, so those bytes go at the HBM rate with no
     * decode beside them (no CRC at all: ~8.6 ms).  Keeping the remainder running inside the
     * chunk loop instead needs live VGPRs the loop does not have at 256: it spilled (11-89
     * VGPRs in two attempts) and ran 30% slower with the fold off. */
    uint32_t crc = crc_read;
    if (ok && !(ablate & 1u) && !st_crc16_frame((const uint8_t *)words, crcp, f, fi.frame_off, end_byte + 2u)) ok = false;
    if (ok && crc != crc_read) ok = false;
    if (ok) {
        info[f].resume_bit = resume;
        info[f].crc16_read = crc_read;
        info[f].crc16_calc = crc;
        info[f].crc_ok = 1u;
    } else if (mine) {
        info[f].flags = fi.flags | BNF_FL_REDO;
    }
    if (tmon && lane == 0) {
        const uint64_t t_end = tnow(tmon);
        atomicAdd(&g_stats[8], (unsigned long long)(t_loop - t_start));
        atomicAdd(&g_stats[9], (unsigned long long)tm_dec);
        atomicAdd(&g_stats[10], (unsigned long long)tm_ref);
        atomicAdd(&g_stats[11], (unsigned long long)tm_pack);
        atomicAdd(&g_stats[12], (unsigned long long)(t_end - t_loopend));
    }
}

#if BNF_TU == 7
/* ============================================================ k_decode_sw
 * One lane per stereo frame above 16 bits (C3: 96 kHz / 24-bit, M/S, wasted bits, LPC-12),
 * k_decode_st's design with libFLAC's wide restore (lpc_restore_signal_wide @0x10006120):
 * - two cursors per lane (one per subframe) on the same 8-slot LDS-DMA rings, refilled in
 *   64-byte groups once per 32-sample chunk (st_refill_issue), one Rice codeword per channel
 *   per step (C3's ~12.6-bit codewords: a pair overruns a 32-bit window on ~1% of lanes, which
 *   would send ~3 of 4 wave steps down the rare path);
 * - the exact predictor: Sum c[j] * x[n-1-j] in 64 bits (v_mad_i64_i32), the 11 older taps of
 *   the next sample summed while the current one is decoded (two chains), so one MAC sits
 *   between consecutive samples; libFLAC's 64-bit path keeps (int32)(S >> shift) (one
 *   v_alignbit for shift < 32), the 32-bit paths (ia32, FIXED) ((int32)S) >> shift;
 * - wasted bits, decorrelation and the output layout in registers: FLACFileReader's 3-byte
 *   LE pack (FLACFileReader.cs:230-237) as v_perm words, 48 bytes per 8 stereo samples in
 *   three 16-byte stores; interleaved / planar int32 in four;
 * - tail as k_decode_st: zero padding, CRC-16 footer, the frame's CRC-16 from the LDS field
 *   tables, zero-fill on mismatch (@0x10011af5).
 * Frames it declines (MMX16 path, orders above 12, CONSTANT / VERBATIM, a 64-bit shift of 32 or
 * more, errors, truncation) get BNF_FL_REDO and k_decode<16> decodes them from scratch. */
#define SW_TAPS 12
struct StW {
    BR b;
    int32_t c[SW_TAPS]; /* coefficients, 0 past the order (FIXED order o as LPC, shift 0) */
    int32_t x[16];      /* history ring: x[n & 15] = sample n of the subframe */
    int32_t sh;         /* shift of the libFLAC path (< 32) */
    uint32_t wide;      /* 1: 64-bit path */
    uint32_t k, km, k1, k32;
    uint32_t esc, left, pidx, nparts, psamples, plen, pesc, porder, order;
    uint32_t wasted;
};

DEV bool sw_setup(StW &z, uint32_t bps, uint32_t bs, uint64_t limit) {
    SubHdr h;
    int32_t warm[SW_TAPS], coef[SW_TAPS], err = -1;
    const uint32_t st = parse_subframe_head<true, SW_TAPS>(z.b, bps, bs, limit, h, warm, coef, err);
    if (st != BNF_ST_OK) return false;
    if (h.type != T_FIXED && h.type != T_LPC) return false;
    if (h.order > SW_TAPS) return false;
    if (h.type == T_LPC && h.path == P_MMX16) return false;
    if (h.type == T_LPC && h.path == P_WIDE && ((uint32_t)h.shift & 0xFFu) >= 32u) return false;
#pragma unroll
    for (int t = 0; t < SW_TAPS; t++) z.c[t] = (h.type == T_LPC && (uint32_t)t < h.order) ? coef[t] : 0;
    if (h.type == T_FIXED) { /* FIXED order o: 1 | 2,-1 | 3,-3,1 | 4,-6,4,-1 (@0x10003810, 32-bit wrap) */
        const uint32_t o = h.order;
        z.c[0] = o == 1 ? 1 : o == 2 ? 2 : o == 3 ? 3 : o == 4 ? 4 : 0;
        z.c[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
        z.c[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
        z.c[3] = o == 4 ? -1 : 0;
    }
#pragma unroll
    for (int t = 0; t < 16; t++) z.x[t] = (t < SW_TAPS && (uint32_t)t < h.order) ? warm[t < SW_TAPS ? t : 0] : 0;
    z.wide = (h.type == T_LPC && h.path == P_WIDE) ? 1u : 0u;
    z.sh = h.type == T_LPC ? (int32_t)((uint32_t)h.shift & (z.wide ? 0xFFu : 31u)) : 0;
    z.order = h.order;
    z.wasted = h.wasted;
    z.porder = h.porder;
    z.nparts = 1u << h.porder;
    z.psamples = h.porder ? bs >> h.porder : bs - h.order;
    z.plen = h.rice2 ? 5u : 4u;
    z.pesc = h.rice2 ? 31u : 15u;
    z.left = 0;
    z.pidx = 0;
    z.esc = 0;
    z.k = 0;
    z.km = 31;
    z.k1 = 1;
    z.k32 = 32;
    return true;
}

/* c * x + acc exactly: one v_mad_i64_i32, written out.  With the coefficients loop-invariant
 * the compiler hoisted their sign extension out of the chunk loop and then emitted full
 * 64x64-bit multiplies (mad_u64_u32 + 2 mul_lo + add3); keeping the extension beside each
 * multiply with an empty asm spilled (256 VGPRs). */
/* vdst early-clobber: the 64-bit result must not overlap a 32-bit source (LLVM's own
 * constraint on V_MAD_I64_I32; a build whose allocator overlapped them decoded garbage) */
DEV int64_t sw_mad(int32_t c, int32_t x, int64_t acc) {
    int64_t d;
    uint64_t co;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=&v"(d), "=&s"(co) : "v"(c), "v"(x), "v"(acc));
    return d;
}
/* the 11 older taps of sample n + 1 (n = T mod 16): Sum_{j=1..11} c[j] * x[n - j], two chains
 * (oldest taps first), as one asm block: the compiler puts a wait state after every inline
 * asm statement (it cannot see its hazards), so one statement per sum, not per MAC */
template <int T>
DEV int64_t sw_pre(const StW &z) {
    static_assert(SW_TAPS == 12, "sw_pre is written out for 12 taps");
#define XJ(j) z.x[(T - (j) + 32) & 15]
    int64_t a, b;
    uint64_t cc;
    asm("v_mad_i64_i32 %0, %2, %3, %4, 0\n\t"
        "v_mad_i64_i32 %1, %2, %5, %6, 0\n\t"
        "v_mad_i64_i32 %0, %2, %7, %8, %0\n\t"
        "v_mad_i64_i32 %1, %2, %9, %10, %1\n\t"
        "v_mad_i64_i32 %0, %2, %11, %12, %0\n\t"
        "v_mad_i64_i32 %1, %2, %13, %14, %1\n\t"
        "v_mad_i64_i32 %0, %2, %15, %16, %0\n\t"
        "v_mad_i64_i32 %1, %2, %17, %18, %1\n\t"
        "v_mad_i64_i32 %0, %2, %19, %20, %0\n\t"
        "v_mad_i64_i32 %1, %2, %21, %22, %1\n\t"
        "v_mad_i64_i32 %0, %2, %23, %24, %0\n\t"
        "v_lshl_add_u64 %0, %0, 0, %1"
        : "=&v"(a), "=&v"(b), "=&s"(cc)
        : "v"(z.c[11]), "v"(XJ(11)), "v"(z.c[10]), "v"(XJ(10)), "v"(z.c[9]), "v"(XJ(9)), "v"(z.c[8]), "v"(XJ(8)),
          "v"(z.c[7]), "v"(XJ(7)), "v"(z.c[6]), "v"(XJ(6)), "v"(z.c[5]), "v"(XJ(5)), "v"(z.c[4]), "v"(XJ(4)),
          "v"(z.c[3]), "v"(XJ(3)), "v"(z.c[2]), "v"(XJ(2)), "v"(z.c[1]), "v"(XJ(1)));
#undef XJ
    return a;
}
/* the path's prediction from the exact sum; PATH 0: every channel of the wave takes the
 * 64-bit path, 2: per channel */
template <int PATH>
DEV int32_t sw_shift(const StW &z, int64_t S) {
    const uint32_t lo = (uint32_t)S, hi = (uint32_t)((uint64_t)S >> 32);
    const int32_t w = (int32_t)__builtin_amdgcn_alignbit(hi, lo, (uint32_t)z.sh); /* (int32)(S >> sh), sh < 32 */
    if (PATH == 0) return w;
    return z.wide ? w : ((int32_t)lo >> z.sh);
}
/* the full prediction of sample n (T = n mod 16), general path */
template <int T, int PATH>
DEV int32_t sw_full(const StW &z) {
    return sw_shift<PATH>(z, sw_mad(z.c[0], z.x[(T + 15) & 15], sw_pre<(T + 15) & 15>(z)));
}

template <int AS>
DEV void sw_decor(uint32_t as, int32_t &l, int32_t &r) {
    if (AS < 0) decorrelate(as, l, r);
    else decorrelate((uint32_t)AS, l, r);
}

/* FLACFileReader's 24-bit LE pack of 8 stereo samples (FLACFileReader.cs:230-237): 48 bytes */
DEV void sw_pack24(const int32_t (&L)[8], const int32_t (&R)[8], uint32_t (&d)[12]) {
#pragma unroll
    for (int h = 0; h < 4; h++) {
        const uint32_t l0 = (uint32_t)L[2 * h], r0 = (uint32_t)R[2 * h], l1 = (uint32_t)L[2 * h + 1], r1 = (uint32_t)R[2 * h + 1];
        d[3 * h] = __builtin_amdgcn_perm(r0, l0, 0x04020100u);     /* l0.b0 l0.b1 l0.b2 r0.b0 */
        d[3 * h + 1] = __builtin_amdgcn_perm(l1, r0, 0x05040201u); /* r0.b1 r0.b2 l1.b0 l1.b1 */
        d[3 * h + 2] = __builtin_amdgcn_perm(r1, l1, 0x06050402u); /* l1.b2 r1.b0 r1.b1 r1.b2 */
    }
}

/* The FLACFileReader line flush (C3).  A 16-sample chunk is 96 bytes of a frame's run, so two
 * chunks are three 64-byte lines: an even chunk completes line 0 and leaves the first half of
 * line 1 (carry), an odd chunk completes lines 1 and 2.  Each lane puts a line's four 16-byte
 * units into its own 64-byte LDS slot; the flush then has every lane store one unit of the
 * line of frame (lane >> 2) + 16 i, i = 0..3: four stores of sixteen whole lines each, instead
 * of per-lane 16-byte stores scattered over 64 lines.  Cross-lane reads (the slots, the run
 * addresses by ds_bpermute) happen only at chunk end with every lane active: inside a chunk a
 * lane whose frame has ended is masked off, and a read of its registers would yield nothing. */
struct SwLn {
    u32x4 c0, c1;     /* even chunk: the carried first half of line 1 */
    u32x4 h0, h1, h2, h3; /* odd chunk: line 2 (a2 from the first group, b0..b2 from the second) */
};
DEV void sw_line_group(lds_u32x4 *stg, uint32_t lane, bool odd, bool carry, SwLn &q, const uint32_t (&d)[12],
                       int g, uint8_t *run) {
    const u32x4 u0 = u32x4{d[0], d[1], d[2], d[3]}, u1 = u32x4{d[4], d[5], d[6], d[7]}, u2 = u32x4{d[8], d[9], d[10], d[11]};
    lds_u32x4 *my = stg + lane * 4u;
    if (!odd) {
        if (g == 0) { my[0] = u0; my[1] = u1; my[2] = u2; }
        else { my[3] = u0; q.c0 = u1; q.c1 = u2; }
    } else if (g == 0) {
        if (carry) { my[0] = q.c0; my[1] = q.c1; my[2] = u0; my[3] = u1; }
        else { /* no carried half: the first half of line 1 was stored directly */
            gst128((uint64_t)(uintptr_t)run, u0);
            gst128((uint64_t)(uintptr_t)run + 16u, u1);
        }
        q.h0 = u2;
    } else {
        q.h1 = u0; q.h2 = u1; q.h3 = u2;
    }
}
/* The run base and blocksize of frame (lane >> 2) + 16 i (0 for a frame that is not
 * decoded), fetched once per wave by ds_bpermute with every lane active */
struct SwRuns {
    uint64_t a[4];
    uint32_t bs[4];
};
DEV void sw_runs(SwRuns &r, uint64_t run, uint32_t bs, uint32_t lane) {
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const int src = (int)(((lane >> 2) + 16u * i) << 2);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)run);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(run >> 32));
        r.a[i] = ((uint64_t)hi << 32) | lo;
        r.bs[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(run ? bs : 0u));
    }
}
/* every lane active: the slots' line at byte `off` of the chunk's frames (those whose run
 * reaches sample n0 + 16); returns the store instructions issued */
DEV uint32_t sw_line_flush(const lds_u32x4 *stg, const SwRuns &r, uint32_t n0, int32_t off, uint32_t lane) {
    uint32_t n = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const uint32_t src = (lane >> 2) + 16u * i;
        const bool on = n0 + ST_CHK <= r.bs[i];
        const u32x4 v = stg[src * 4u + (lane & 3u)];
        if (on) gst128(r.a[i] + (uint64_t)((int64_t)n0 * 6 + off) + 16u * (lane & 3u), v);
        if (any_lane(on)) n++;
    }
    return n;
}

/* 8 stereo samples n..n+7 of this lane's frame (nv valid) into the layout; al: 16-byte
 * aligned runs (then 3 or 4 16-byte stores).  Returns whether the aligned path stored. */
template <int FMT>
DEV bool sw_emit8(uint8_t *dst, uint32_t n, uint32_t nv, bool al, uint32_t bs, const int32_t (&L)[8], const int32_t (&R)[8]) {
    if (nv == 0) return false;
    if (FMT == BNF_OUT_FILEREADER) { /* 24-bit LE, L R L R ... */
        uint32_t d[12];
        sw_pack24(L, R, d);
        uint8_t *o = dst + (uint64_t)n * 6u;
        if (al && nv == 8) {
#pragma unroll
            for (int u = 0; u < 3; u++)
                gst128((uint64_t)(uintptr_t)(o + 16 * u), u32x4{d[4 * u], d[4 * u + 1], d[4 * u + 2], d[4 * u + 3]});
            return true;
        }
        const uint32_t nb = nv * 6u;
        if ((((uintptr_t)o) & 3u) == 0) {
            for (uint32_t i = 0; i < nb / 4u; i++) ((uint32_t *)o)[i] = d[i];
            if (nb & 3u) { /* nv odd: two bytes of the last word */
                const uint32_t v = d[nb / 4u];
                o[nb - 2] = (uint8_t)v;
                o[nb - 1] = (uint8_t)(v >> 8);
            }
        } else {
            for (uint32_t i = 0; i < nb; i++) o[i] = (uint8_t)(d[i >> 2] >> (8u * (i & 3u)));
        }
        return false;
    } else if (FMT == BNF_OUT_INTERLEAVED32) {
        int32_t *o = (int32_t *)(dst + (uint64_t)n * 8u);
        if (al && nv == 8) {
#pragma unroll
            for (int u = 0; u < 4; u++) *(int4 *)(o + 4 * u) = make_int4(L[2 * u], R[2 * u], L[2 * u + 1], R[2 * u + 1]);
            return true;
        }
        for (uint32_t q = 0; q < nv; q++) { o[2 * q] = L[q]; o[2 * q + 1] = R[q]; }
        return false;
    } else { /* PLANAR32 */
        int32_t *o0 = (int32_t *)dst + n, *o1 = (int32_t *)dst + bs + n;
        if (al && nv == 8) {
            *(int4 *)o0 = make_int4(L[0], L[1], L[2], L[3]);
            *(int4 *)(o0 + 4) = make_int4(L[4], L[5], L[6], L[7]);
            *(int4 *)o1 = make_int4(R[0], R[1], R[2], R[3]);
            *(int4 *)(o1 + 4) = make_int4(R[4], R[5], R[6], R[7]);
            return true;
        }
        for (uint32_t q = 0; q < nv; q++) { o0[q] = L[q]; o1[q] = R[q]; }
        return false;
    }
}
template <int FMT> constexpr uint32_t sw_stores8() { return FMT == BNF_OUT_FILEREADER ? 3u : 4u; }

/* One sample of both channels on the fused path (T = n mod 16): a Rice codeword per channel
 * (k_decode_st's single step), the prediction from the older-tap sum of the previous step
 * plus the newest tap, the next sample's older taps, the history, and at T = 7 / 15 the 8
 * samples' wasted bits, decorrelation and stores. */
template <int T, int FMT, int PATH, int AS, int LN>
DEV void sw_fused_step(StW &z0, StW &z1, int32_t (&L)[8], int32_t (&R)[8], uint64_t limit, uint32_t &trunc, uint32_t nq,
                       uint32_t as, uint8_t *dst, uint32_t nbase, bool al, uint32_t bs, bool sto, int64_t &pre0,
                       int64_t &pre1, uint32_t lane, lds_u32x4 *stg, bool odd, bool carry, SwLn &q) {
    /* source order is issue order here (the compiler keeps its MAC asm blocks in place): the
     * two cursor chains first, the MAC blocks between their dependent steps */
    const uint32_t w0 = br_peek(z0.b), w1 = br_peek(z1.b);
    const uint32_t q0 = ffbh(w0), q1 = ffbh(w1); /* ~0u for an empty window: slow */
    const bool sl0 = q0 >= z0.k32, sl1 = q1 >= z1.k32;
    const int32_t p0 = sw_shift<PATH>(z0, sw_mad(z0.c[0], z0.x[(T + 15) & 15], pre0));
    const int32_t p1 = sw_shift<PATH>(z1, sw_mad(z1.c[0], z1.x[(T + 15) & 15], pre1));
    uint32_t u0 = (q0 << z0.k) | __builtin_amdgcn_ubfe(w0, z0.km - q0, z0.k);
    uint32_t u1 = (q1 << z1.k) | __builtin_amdgcn_ubfe(w1, z1.km - q1, z1.k);
    const uint32_t laneb = lane << 4;
    st_adv_nc(z0.b, sl0 ? 0u : q0 + z0.k1, laneb);
    pre0 = sw_pre<T>(z0);
    st_adv_nc(z1.b, sl1 ? 0u : q1 + z1.k1, laneb);
    pre1 = sw_pre<T>(z1);
    /* landing check on even steps: the word read now and the one the next step reads */
    const bool ld0 = (T & 1) == 0 && z0.b.wi >= z0.b.vlim, ld1 = (T & 1) == 0 && z1.b.wi >= z1.b.vlim;
    st_next_word(z0.b);
    st_next_word(z1.b);
    if (__builtin_expect(any_lane(sl0 || sl1 || ld0 || ld1), 0)) {
        st_rare(z0, sl0, ld0, u0, limit, trunc, nq, lane);
        st_rare(z1, sl1, ld1, u1, limit, trunc, nq, lane);
    }
    const int32_t s0 = (int32_t)(((u0 >> 1) ^ (0u - (u0 & 1u))) + (uint32_t)p0);
    const int32_t s1 = (int32_t)(((u1 >> 1) ^ (0u - (u1 & 1u))) + (uint32_t)p1);
    z0.x[T] = s0;
    z1.x[T] = s1;
    L[T & 7] = (int32_t)((uint32_t)s0 << z0.wasted);
    R[T & 7] = (int32_t)((uint32_t)s1 << z1.wasted);
    if ((T & 7) == 7) {
#pragma unroll
        for (int i = 0; i < 8; i++) sw_decor<AS>(as, L[i], R[i]);
        if (LN) { /* FILEREADER line flush: units to the LDS slot / carry (sw_line_group) */
            uint32_t d[12];
            sw_pack24(L, R, d);
            sw_line_group(stg, lane, odd, carry, q, d, T >> 3, dst + (uint64_t)nbase * 6u);
        } else if (sto) {
            sw_emit8<FMT>(dst, nbase + (uint32_t)T - 7u, 8u, al, bs, L, R);
        }
    }
}

/* One sample of both channels on the general path (warm-up, partition headers, escapes, the
 * last partial chunk).  At T = 7 / 15 returns whether the aligned store path ran. */
template <int T, int FMT>
DEV bool sw_gen_step(StW &z0, StW &z1, int32_t (&L)[8], int32_t (&R)[8], uint64_t limit, uint32_t &trunc, uint32_t nst,
                     uint32_t as, uint8_t *dst, uint32_t n, bool valid, bool al, uint32_t bs, bool sto) {
    const bool v = valid && n < bs;
    int32_t s0 = 0, s1 = 0;
    if (v) {
        if (n < z0.order) s0 = z0.x[T];
        else s0 = (int32_t)((uint32_t)st_next(z0, limit, trunc, nst) + (uint32_t)sw_full<T, 2>(z0));
        if (n < z1.order) s1 = z1.x[T];
        else s1 = (int32_t)((uint32_t)st_next(z1, limit, trunc, nst) + (uint32_t)sw_full<T, 2>(z1));
        z0.x[T] = s0;
        z1.x[T] = s1;
    }
    L[T & 7] = (int32_t)((uint32_t)s0 << z0.wasted);
    R[T & 7] = (int32_t)((uint32_t)s1 << z1.wasted);
    bool stored = false;
    if ((T & 7) == 7) {
        const uint32_t nq = n - 7u;
        const uint32_t nv = (valid && nq < bs) ? min(8u, bs - nq) : 0u;
#pragma unroll
        for (int q = 0; q < 8; q++) decorrelate(as, L[q], R[q]);
        if (sto) stored = sw_emit8<FMT>(dst, nq, nv, al, bs, L, R);
    }
    return stored;
}

template <int FMT>
__global__ void __launch_bounds__(64, 2) k_decode_sw(const uint32_t *__restrict__ words, uint64_t nbytes,
                                                     uint32_t nframes, bnf_stream_params sp, uint32_t chn_lanes,
                                                     uint8_t *__restrict__ out, uint64_t out_bytes,
                                                     bnf_frame_info *__restrict__ info,
                                                     const uint32_t *__restrict__ perm, uint32_t ablate,
                                                     const uint32_t *__restrict__ crcp) {
    constexpr uint32_t SPG = sw_stores8<FMT>();
    /* 16 KB: both channels' bitstream rings; 4 KB: the flush tile (20 KB, 8 waves per CU) */
    __shared__ LDS_DMA_ALIGN uint32_t ring[2 * ST_RD * RING_LANE_DW + 1024]; /* the two rings, then the 4 KB flush tile */
    const uint32_t lane = threadIdx.x;
    const uint32_t slot = blockIdx.x * 64u + lane;
    const uint32_t f = (perm && slot < nframes) ? perm[slot] : slot;
    const uint64_t limit = nbytes * 8u;
    bnf_frame_info fi;
    const bool have = f < nframes;
    if (have) fi = info[f];
    const bool mine = have && fi.status == BNF_ST_OK && (fi.flags & BNF_FL_SW) && !(fi.flags & BNF_FL_REDO) &&
                      (!(ablate & BNF_MODE_WREDO) || (fi.flags & BNF_FL_WAVE_REDO));
    if (!__any(mine)) return;

    uint64_t stride = 8;
    bool ok = mine && fi.channels == 2 && chn_lanes >= 2 && sp.channels == 2;
    if (FMT == BNF_OUT_FILEREADER) { stride = 6; ok = ok && sp.bps == 24; }
    const uint32_t bs = ok ? fi.blocksize : 0u;
    const uint64_t os = ok ? fi.out_sample : 0u;
    ok = ok && (os + bs) * stride <= out_bytes;
    uint8_t *dst = out + os * stride;
    /* timing ablation 0x10000000: every wave stores into one 64 KB window (same store
     * instructions, an L2-resident footprint); output is wrong */
    const bool hot = (ablate & 0x10000000u) != 0 && out_bytes >= (1u << 20); /* the window needs 513 KB */
    if (hot) dst = out + (uint64_t)(blockIdx.x & 7u) * 65536u + lane * 1024u;
    const bool al = (((uintptr_t)dst) & 15u) == 0 && (FMT != BNF_OUT_PLANAR32 || (bs & 3u) == 0);
    const bool all_al = !any_lane(ok && !al); /* every run of the wave takes the 16-byte stores */

    StW z0, z1;
    lds_u32 *ring0 = (lds_u32 *)ring, *ring1 = (lds_u32 *)ring + ST_RD * RING_LANE_DW;
    br_init(z0.b, words, nbytes, ring0, lane, ST_RD);
    br_init(z1.b, words, nbytes, ring1, lane, ST_RD);
    if (ok) {
        br_seek(z0.b, fi.frame_off * 8u + fi.sub_start[0]);
        ok = sw_setup(z0, sub_bps(fi, 0), bs, limit);
    }
    if (ok) {
        br_seek(z1.b, fi.frame_off * 8u + fi.sub_start[1]);
        ok = sw_setup(z1, sub_bps(fi, 1), bs, limit);
    }
    const uint32_t as = ok ? fi.assignment : 0u;
    const uint32_t as_u = __builtin_amdgcn_readfirstlane(as);
    const bool as_uni = !any_lane(ok && as != as_u);
    const bool all_wide = !any_lane(ok && !(z0.wide && z1.wide));
    /* the fused chunks' compile-time variant: the 64-bit path everywhere and one assignment,
     * M/S (C3) or independent; anything else runs the per-lane variant */
    const int fix = (as_uni && all_wide && as_u <= 3u) ? (int)as_u : -1;

    uint32_t mybs = ok ? bs : 0u;
    for (int o = 32; o > 0; o >>= 1) mybs = max(mybs, (uint32_t)__shfl_xor(mybs, o));
    const uint32_t nchunks = (mybs + ST_CHK - 1) / ST_CHK;
    uint32_t trunc = 0;
    const bool sto = !(ablate & 2u);
    /* FILEREADER runs that start on a 64-byte line: the fused chunks flush whole lines
     * (sw_line_flush); the slots sit past the two rings (the 4 KB staging tile).
     * Ablation bit 0x20000000 (exact): per-lane 16-byte stores instead */
    const bool line = FMT == BNF_OUT_FILEREADER && sto && !hot && all_al && !(ablate & 0x20000000u) &&
                      !any_lane(ok && (((uintptr_t)dst) & 63u) != 0);
    lds_u32x4 *stg = (lds_u32x4 *)((lds_u32 *)ring + 2u * ST_RD * RING_LANE_DW);
    static_assert(sizeof(ring) >= (2 * ST_RD * RING_LANE_DW + 1024) * 4, "the flush's 4 KB staging tile lies past the two rings");
    static_assert(sizeof(ring) >= (2u * ST_RD * RING_LANE_DW + 1024u) * 4u, "line slots past the rings");
    SwLn q;
    SwRuns runs;
    if (line) sw_runs(runs, ok ? (uint64_t)(uintptr_t)dst : 0ull, bs, lane);
    bool carry = false, cvalid = false; /* carry: an even chunk left its half line (wave-uniform) */
    uint32_t carry_b = 0;                /* its byte offset in the runs */
    wait_vm(); /* setup loads done: the store count starts from zero */
    uint32_t nst = 0; /* vector-memory ops (PCM stores) issued by this wave since the last refill's DMAs (a lower bound) */
    for (uint32_t kc = 0; kc < nchunks; kc++) {
        const uint32_t n0 = kc * ST_CHK;
        const bool valid = ok && n0 < bs;
        bool fast = valid && n0 >= 16u && n0 + ST_CHK <= bs && !(ablate & 12u);
        if (fast) { /* partition headers at the chunk boundary (aligned partitions) */
            if (z0.left == 0 && z0.pidx < z0.nparts) st_partition(z0);
            if (z1.left == 0 && z1.pidx < z1.nparts) st_partition(z1);
            fast = !z0.esc && !z1.esc && z0.left >= ST_CHK && z1.left >= ST_CHK;
        }
        const bool fused = !any_lane(valid && !fast);
        const bool odd = (kc & 1u) != 0;
        const bool ln = line && fused && any_lane(valid);
        if (carry) { /* a carried half line that this chunk does not take: stored directly */
            const bool take = ln && odd;
            const bool d = cvalid && !(take && valid);
            if (d) {
                gst128((uint64_t)(uintptr_t)dst + carry_b, q.c0);
                gst128((uint64_t)(uintptr_t)dst + carry_b + 16u, q.c1);
            }
            if (any_lane(d)) nst += 2u;
            if (!take) carry = false;
        }
        if (fused) {
            if (valid) {
                int64_t pre0 = sw_pre<15>(z0), pre1 = sw_pre<15>(z1); /* older taps of the chunk's first sample */
                st_resync(z0.b, lane);
                st_resync(z1.b, lane);
                auto chunk = [&](auto pc, auto ac, auto lc) {
                    constexpr int PATH = decltype(pc)::value, AS = decltype(ac)::value, LN = decltype(lc)::value;
#pragma unroll 1
                    for (uint32_t h = 0; h < ST_CHK / 16; h++) {
                        int32_t L[8], R[8];
                        const uint32_t nb = hot ? (n0 + h * 16u) & 127u : n0 + h * 16u;
                        const uint32_t nqa = nst + (!LN && all_al && sto ? h * 2u * SPG : 0u);
                        const uint32_t nqb = nqa + (LN ? 0u : (all_al && sto ? SPG : 0u));
#define SWS(T, NQ) sw_fused_step<T, FMT, PATH, AS, LN>(z0, z1, L, R, limit, trunc, NQ, as, dst, nb, al, bs, sto, pre0, pre1, lane, stg, odd, carry, q)
                        SWS(0, nqa); SWS(1, nqa); SWS(2, nqa); SWS(3, nqa); SWS(4, nqa); SWS(5, nqa); SWS(6, nqa); SWS(7, nqa);
                        SWS(8, nqb); SWS(9, nqb); SWS(10, nqb); SWS(11, nqb); SWS(12, nqb); SWS(13, nqb); SWS(14, nqb); SWS(15, nqb);
#undef SWS
                    }
                };
                using I0 = std::integral_constant<int, 0>;
                using I1 = std::integral_constant<int, 1>;
                bool done = false;
                if constexpr (FMT == BNF_OUT_FILEREADER) {
                    if (ln) {
                        if (fix == 3) chunk(I0(), std::integral_constant<int, 3>(), I1());
                        else if (fix == 0) chunk(I0(), I0(), I1());
                        else chunk(std::integral_constant<int, 2>(), std::integral_constant<int, -1>(), I1());
                        done = true;
                    }
                }
                if (!done) {
                    if (fix == 3) chunk(I0(), std::integral_constant<int, 3>(), I0());
                    else if (fix == 0) chunk(I0(), I0(), I0());
                    else chunk(std::integral_constant<int, 2>(), std::integral_constant<int, -1>(), I0());
                }
                z0.left -= ST_CHK;
                z1.left -= ST_CHK;
            }
            if (ln) { /* every lane active: the chunk's lines (sw_line_flush) */
                if (!odd) {
                    nst += sw_line_flush(stg, runs, n0, 0, lane);
                    carry = true;
                    cvalid = valid;
                    carry_b = n0 * 6u + 64u; /* units c0, c1: bytes 64..95 of the chunk */
                } else {
                    if (!carry) nst += 2u; /* the direct half line (sw_line_group) */
                    if (carry) nst += sw_line_flush(stg, runs, n0, -32, lane);
                    lds_u32x4 *my = stg + lane * 4u;
                    my[0] = q.h0; my[1] = q.h1; my[2] = q.h2; my[3] = q.h3;
                    nst += sw_line_flush(stg, runs, n0, 32, lane);
                    carry = false;
                }
            } else if (all_al && sto && any_lane(valid)) {
                nst += (ST_CHK / 8) * SPG;
            }
        } else {
#pragma unroll 1
            for (uint32_t h = 0; h < ST_CHK / 16; h++) {
                int32_t L[8], R[8];
                const uint32_t nb = n0 + h * 16u;
                bool st0, st1;
#define SWG(T) sw_gen_step<T, FMT>(z0, z1, L, R, limit, trunc, nst, as, dst, nb + T, valid, al, bs, sto)
                SWG(0); SWG(1); SWG(2); SWG(3); SWG(4); SWG(5); SWG(6);
                st0 = SWG(7);
                if (any_lane(st0)) nst += SPG;
                SWG(8); SWG(9); SWG(10); SWG(11); SWG(12); SWG(13); SWG(14);
                st1 = SWG(15);
                if (any_lane(st1)) nst += SPG;
#undef SWG
            }
        }
        /* refill: wait for the previous refill's DMAs (the stores since stay in flight), then
         * issue the next groups */
        {
            const bool want = valid && n0 + ST_CHK < bs;
            wait_vm_n(nst);
            z0.b.vendw = z0.b.iend * 4u;
            z1.b.vendw = z1.b.iend * 4u;
            st_refill_issue(z0.b, want);
            st_refill_issue(z1.b, want);
            nst = 0;
        }
    }

    if (carry && cvalid) { /* the last chunk was even: its half line */
        gst128((uint64_t)(uintptr_t)dst + carry_b, q.c0);
        gst128((uint64_t)(uintptr_t)dst + carry_b + 16u, q.c1);
    }

    /* ---- end of the last subframe, zero padding, CRC-16 (read_frame_ tail) */
    uint32_t crc_read = 0;
    uint64_t end_byte = 0, resume = 0;
    if (ok && trunc) ok = false;
    if (ok) {
        while (z1.pidx < z1.nparts) { /* finish_partitions */
            const uint32_t kk = br_read(z1.b, z1.plen);
            if (kk >= z1.pesc) br_read(z1.b, 5);
            z1.pidx++;
        }
        const uint32_t padbits = (uint32_t)((8u - (br_pos(z1.b) & 7u)) & 7u);
        const uint32_t zp = br_read(z1.b, padbits);
        if (br_pos(z1.b) > limit || zp != 0) ok = false;
        end_byte = br_pos(z1.b) >> 3;
        crc_read = br_read(z1.b, 16);
        if (br_pos(z1.b) > limit) ok = false;
        resume = br_pos(z1.b);
    }
    uint32_t crc = crc_read;
    /* the table-free zero test over frame + footer (round 6: 9.40 -> 9.23 ms on C3, same box) */
    if (ok && !(ablate & 1u) && !st_crc16_frame((const uint8_t *)words, crcp, f, fi.frame_off, end_byte + 2u)) ok = false;
    if (ok && crc != crc_read) ok = false;
    if (ok) {
        info[f].resume_bit = resume;
        info[f].crc16_read = crc_read;
        info[f].crc16_calc = crc;
        info[f].crc_ok = 1u;
    } else if (mine) {
        info[f].flags = fi.flags | BNF_FL_REDO;
    }
}
#endif /* BNF_TU == 7 */
#endif /* BNF_TU == 3 || BNF_TU == 4 || BNF_TU == 7 */

/* ------------------------------------------------------------- host launchers */
/* The library is built from this file three times (BNF_TU 0: sync scan + k_parse + shared
 * launchers, 1: k_decode<8>, 2: k_decode<32>), so the instances compile in parallel.  Each
 * TU is its own code object: the __constant__ tables are uploaded into every one. */
/* mode switches are read by launching threads while a test or tool may set them: atomics */
static std::atomic<uint32_t> g_ablate{0xFFFFFFFFu};
static uint32_t ablate_flags() {
    uint32_t v = g_ablate.load(std::memory_order_relaxed);
    if (v == 0xFFFFFFFFu) {
        const char *e = getenv("BNFLAC_ABLATE"); /* timing experiments only: results are wrong */
        v = e ? (uint32_t)strtoul(e, nullptr, 0) : 0u;
        g_ablate.store(v, std::memory_order_relaxed);
    }
    return v;
}
static hipError_t upload_tables(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_crc8_tab), crc8, 256);
    if (e != hipSuccess) return e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_crc16_tab), crc16x8, 8 * 256 * sizeof(uint16_t));
    if (e != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_crc16_xpow), xpow, 40 * sizeof(uint16_t));
}

#define TU_FN(name) TU_FN2(name, BNF_TU)
#define TU_FN2(name, n) TU_FN3(name, n)
#define TU_FN3(name, n) name##_tu##n
#if BNF_TU == 1 || BNF_TU == 2 || BNF_TU == 5
#define DEC_W (BNF_TU == 1 ? 8 : (BNF_TU == 5 ? 16 : 32))
#define DEC_RD 8 /* ring slots (16 for k_decode<32> measured: LDS then caps it at 6 waves per CU) */
extern "C" {
hipError_t TU_FN(bnf_upload_tables)(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    return upload_tables(crc8, crc16x8, xpow);
}
void TU_FN(bnf_set_ablate)(uint32_t v) { g_ablate.store(v, std::memory_order_relaxed); }
hipError_t TU_FN(bnf_stats)(uint64_t *out16, int reset) {
    uint64_t v[16];
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stats), sizeof v);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 16; i++) out16[i] += v[i];
    if (reset) {
        static const uint64_t z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z);
    }
    return e;
}
/* seg: k_order's bucket ends (W = 16 / 32 only, with perm): blocks outside the class leave first */
hipError_t TU_FN(bnf_launch_decode)(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                    uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                    const uint32_t *perm, uint32_t mode, const uint32_t *seg, hipStream_t s) {
    const uint32_t fpb = DEC_LANES / chn_lanes;
    const uint32_t nb = (nframes + fpb - 1) / fpb;
    if (!perm || (DEC_W == 8 && !(mode & (BNF_MODE_NOST | BNF_MODE_STREDO)))) seg = nullptr;
    hipLaunchKernelGGL((k_decode<DEC_W, 32, DEC_RD>), dim3(nb), dim3(DEC_LANES), 0, s, words, nbytes, nframes, sp, chn_lanes,
                       fmt, out, out_bytes, info, perm, ablate_flags() | mode, seg);
    return hipGetLastError();
}
#if BNF_TU == 2
/* k_decode_sys's hand-back list (W = 32: every order); nframes bounds the list */
hipError_t bnf_launch_decode_list_tu2(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                      uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                      const uint32_t *list, uint32_t mode, hipStream_t s) {
    const uint32_t fpb = DEC_LANES / chn_lanes;
    const uint32_t nb = std::min<uint32_t>((nframes + fpb - 1) / fpb, 512u);
    hipLaunchKernelGGL((k_decode_list<DEC_W, 32, DEC_RD>), dim3(std::max(nb, 1u)), dim3(DEC_LANES), 0, s, words, nbytes, sp,
                       chn_lanes, fmt, out, out_bytes, info, list, ablate_flags() | mode);
    return hipGetLastError();
}
/* the W16 + W32 segment of the decode order (k_decode_seg; perm and seg required) */
hipError_t bnf_launch_decode_seg_tu2(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                     uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                     const uint32_t *perm, uint32_t mode, const uint32_t *seg, hipStream_t s) {
    const uint32_t fpb = DEC_LANES / chn_lanes;
    const uint32_t nb = std::min<uint32_t>((nframes + fpb - 1) / fpb, 512u);
    hipLaunchKernelGGL((k_decode_seg<DEC_W, 32, DEC_RD>), dim3(std::max(nb, 1u)), dim3(DEC_LANES), 0, s, words, nbytes,
                       nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, ablate_flags() | mode | BNF_MODE_SEG, seg);
    return hipGetLastError();
}
#endif
} /* extern "C" */
#endif

#if BNF_TU == 3 || BNF_TU == 4
/* TU 3: k_decode_st<FLACDECODER>; TU 4: the other layouts */
extern "C" {
hipError_t TU_FN(bnf_upload_tables)(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    return upload_tables(crc8, crc16x8, xpow);
}
void TU_FN(bnf_set_ablate)(uint32_t v) { g_ablate.store(v, std::memory_order_relaxed); }
hipError_t TU_FN(bnf_stats)(uint64_t *out16, int reset) {
    uint64_t v[16];
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stats), sizeof v);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 16; i++) out16[i] += v[i];
    if (reset) {
        static const uint64_t z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z);
    }
    return e;
}
/* stereo fast path; launched before k_decode<8> (it hands frames back to it) */
hipError_t TU_FN(bnf_launch_decode)(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                    uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                    const uint32_t *perm, uint32_t mode, const uint32_t *crcp, hipStream_t s) {
    const dim3 grid((nframes + 63) / 64);
    const uint32_t ab = ablate_flags() | mode;
    if (ab & 0x400u) return hipSuccess; /* timing ablation: everything to k_decode<8> */
#if BNF_TU == 3
    (void)fmt;
    hipLaunchKernelGGL(k_decode_st<BNF_OUT_FLACDECODER>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
#else
    switch (fmt) {
    case BNF_OUT_PLANAR32:
        hipLaunchKernelGGL(k_decode_st<BNF_OUT_PLANAR32>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    case BNF_OUT_INTERLEAVED32:
        hipLaunchKernelGGL(k_decode_st<BNF_OUT_INTERLEAVED32>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    default:
        hipLaunchKernelGGL(k_decode_st<BNF_OUT_FILEREADER>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    }
#endif
    return hipGetLastError();
}
} /* extern "C" */
#endif

#if BNF_TU == 7
extern "C" {
hipError_t TU_FN(bnf_upload_tables)(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    return upload_tables(crc8, crc16x8, xpow);
}
void TU_FN(bnf_set_ablate)(uint32_t v) { g_ablate.store(v, std::memory_order_relaxed); }
hipError_t TU_FN(bnf_stats)(uint64_t *out16, int reset) {
    uint64_t v[16];
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stats), sizeof v);
    if (e != hipSuccess) return e;
    for (int i = 0; i < 16; i++) out16[i] += v[i];
    if (reset) {
        static const uint64_t z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z);
    }
    return e;
}
/* stereo frames above 16 bits; launched before k_decode<8>/<16>/<32> (it hands frames back to k_decode<16>) */
hipError_t bnf_launch_decode_sw_tu7(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                                    uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                                    const uint32_t *perm, uint32_t mode, const uint32_t *crcp, hipStream_t s) {
    const dim3 grid((nframes + 63) / 64);
    const uint32_t ab = ablate_flags() | mode;
    switch (fmt) {
    case BNF_OUT_PLANAR32:
        hipLaunchKernelGGL(k_decode_sw<BNF_OUT_PLANAR32>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    case BNF_OUT_INTERLEAVED32:
        hipLaunchKernelGGL(k_decode_sw<BNF_OUT_INTERLEAVED32>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    case BNF_OUT_FILEREADER:
        hipLaunchKernelGGL(k_decode_sw<BNF_OUT_FILEREADER>, grid, dim3(64), 0, s, words, nbytes, nframes, sp, chn_lanes, out, out_bytes, info, perm, ab, crcp);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
} /* extern "C" */
#endif

#if BNF_TU == 0
extern "C" {
hipError_t bnf_upload_tables_tu3(const uint8_t *, const uint16_t *, const uint16_t *);
hipError_t bnf_upload_tables_tu4(const uint8_t *, const uint16_t *, const uint16_t *);
void bnf_set_ablate_tu3(uint32_t);
void bnf_set_ablate_tu4(uint32_t);
hipError_t bnf_stats_tu3(uint64_t *, int);
hipError_t bnf_stats_tu4(uint64_t *, int);
hipError_t bnf_launch_decode_tu3(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                 uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
hipError_t bnf_launch_decode_tu4(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                 uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
hipError_t bnf_launch_decode_sw_tu7(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                    uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
hipError_t bnf_upload_tables_tu5(const uint8_t *, const uint16_t *, const uint16_t *);
void bnf_set_ablate_tu5(uint32_t);
hipError_t bnf_stats_tu5(uint64_t *, int);
hipError_t bnf_launch_decode_tu5(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                 uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
hipError_t bnf_upload_tables_tu1(const uint8_t *, const uint16_t *, const uint16_t *);
hipError_t bnf_upload_tables_tu2(const uint8_t *, const uint16_t *, const uint16_t *);
hipError_t bnf_upload_tables_tu7(const uint8_t *, const uint16_t *, const uint16_t *);
void bnf_set_ablate_tu7(uint32_t);
hipError_t bnf_stats_tu7(uint64_t *, int);
hipError_t bnf_upload_tables_tu8(const uint8_t *, const uint16_t *, const uint16_t *);
hipError_t bnf_stats_tu8(uint64_t *, int);
void bnf_set_ablate_tu8(uint32_t);
hipError_t bnf_launch_decode_sys_tu8(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                     uint64_t, bnf_frame_info *, const uint32_t *, uint32_t *, uint32_t, hipStream_t);
hipError_t bnf_launch_decode_list_tu2(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                      uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, hipStream_t);
hipError_t bnf_launch_decode_seg_tu2(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                     uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
void bnf_set_ablate_tu1(uint32_t);
void bnf_set_ablate_tu2(uint32_t);
hipError_t bnf_stats_tu1(uint64_t *, int);
hipError_t bnf_stats_tu2(uint64_t *, int);
hipError_t bnf_launch_decode_tu1(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                 uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);
hipError_t bnf_launch_decode_tu2(const uint32_t *, uint64_t, uint32_t, bnf_stream_params, uint32_t, int, uint8_t *,
                                 uint64_t, bnf_frame_info *, const uint32_t *, uint32_t, const uint32_t *, hipStream_t);

hipError_t bnf_upload_tables(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow) {
    hipError_t e = upload_tables(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu1(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu2(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu3(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu4(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu5(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu7(crc8, crc16x8, xpow);
    if (e == hipSuccess) e = bnf_upload_tables_tu8(crc8, crc16x8, xpow);
    return e;
}

hipError_t bnf_launch_sync_scan(const uint8_t *d, uint64_t n, uint32_t *d_block_counts, uint32_t *d_total,
                                uint64_t *d_out, uint32_t cap, hipStream_t s) {
    const uint64_t per_block = (uint64_t)SCAN_THREADS * SCAN_BYTES_PER_THREAD;
    const uint32_t nblocks = (uint32_t)((n + per_block - 1) / per_block);
    if (nblocks == 0) return hipMemsetAsync(d_total, 0, sizeof(uint32_t), s);
    hipLaunchKernelGGL(k_sync_count, dim3(nblocks), dim3(SCAN_THREADS), 0, s, d, n, d_block_counts);
    hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, d_block_counts, nblocks, d_total);
    hipLaunchKernelGGL(k_sync_write, dim3(nblocks), dim3(SCAN_THREADS), 0, s, d, n, d_block_counts, d_out, cap);
    return hipGetLastError();
}

uint32_t bnf_scan_blocks(uint64_t n) {
    const uint64_t per_block = (uint64_t)SCAN_THREADS * SCAN_BYTES_PER_THREAD;
    return (uint32_t)((n + per_block - 1) / per_block);
}

void bnf_set_ablate(uint32_t v) {
    g_ablate.store(v, std::memory_order_relaxed);
    bnf_set_ablate_tu1(v);
    bnf_set_ablate_tu2(v);
    bnf_set_ablate_tu3(v);
    bnf_set_ablate_tu4(v);
    bnf_set_ablate_tu5(v);
    bnf_set_ablate_tu7(v);
    bnf_set_ablate_tu8(v);
}

hipError_t bnf_stats(uint64_t *out16, int reset) {
    for (int i = 0; i < 16; i++) out16[i] = 0;
    hipError_t e = bnf_stats_tu1(out16, reset);
    if (e == hipSuccess) e = bnf_stats_tu2(out16, reset);
    if (e == hipSuccess) e = bnf_stats_tu3(out16, reset);
    if (e == hipSuccess) e = bnf_stats_tu5(out16, reset);
    if (e == hipSuccess) e = bnf_stats_tu7(out16, reset);
    if (e == hipSuccess) e = bnf_stats_tu8(out16, reset);
    return e == hipSuccess ? bnf_stats_tu4(out16, reset) : e;
}

/* words: 16-byte aligned; the allocation must cover round_up(nbytes, 16) bytes. */
} /* extern "C" */

/* Frame orders: counting sorts that put similar frames into the same wave (lane- and
 * wave-serial work is bounded by the longest frame of a wave).  Frames land in their bucket
 * in any order: each frame's output and record depend on that frame only.
 *  - decode order (MODE 0): decode class (k_parse's flags), then blocksize, descending;
 *  - parse order (MODE 1): the subframe walk's length, blocksize x (channels - 1), read
 *    from the frame header bytes (a heuristic: a bad header only lands in another bucket). */
#define ORDER_NB 256
DEV uint32_t order_bucket(uint32_t work) { return 63u - min(work >> 8, 63u); } /* larger first */
template <int MODE>
DEV uint32_t order_key(const bnf_frame_info *__restrict__ info, const uint8_t *__restrict__ bytes, uint64_t nbytes,
                       const uint64_t *__restrict__ offs, uint32_t f) {
    if (MODE == 0) {
        const uint32_t st = info[f].status, fl = info[f].flags, bs = info[f].blocksize;
        const uint32_t c = st != BNF_ST_OK ? 1u : (fl & BNF_FL_W32) ? 3u : (fl & BNF_FL_W16) ? 2u : (fl & BNF_FL_ST) ? 0u : 1u;
        return c * 64u + order_bucket(bs ? bs - 1u : 0u);
    }
    const uint64_t o = offs[f];
    if (o + 16u > nbytes) return 63u;
    const uint32_t code = bytes[o + 2] >> 4, chc = bytes[o + 3] >> 4;
    const uint32_t C = chc < 8u ? chc + 1u : 2u;
    uint32_t bs = 0;
    if (code == 1u) bs = 192u;
    else if (code >= 2u && code <= 5u) bs = 576u << (code - 2u);
    else if (code >= 8u) bs = 256u << (code - 8u);
    else if (code == 6u || code == 7u) { /* 8 / 16 bits after the UTF-8 coded number */
        const uint32_t lead = bytes[o + 4];
        const uint32_t n = lead < 0x80u ? 1u : (uint32_t)__builtin_clz(~(lead << 24)); /* leading ones */
        const uint64_t q = o + 4u + min(n, 7u);
        bs = (code == 6u ? bytes[q] : ((uint32_t)bytes[q] << 8 | bytes[q + 1])) + 1u;
    }
    return order_bucket((bs * (C > 1u ? C - 1u : 1u)) >> 1);
}
template <int MODE>
__global__ void __launch_bounds__(256) k_order_count(const bnf_frame_info *__restrict__ info,
                                                     const uint8_t *__restrict__ bytes, uint64_t nbytes,
                                                     const uint64_t *__restrict__ offs, uint32_t nframes,
                                                     uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[ORDER_NB];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    if (f < nframes) atomicAdd(&h[order_key<MODE>(info, bytes, nbytes, offs, f)], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
/* exclusive, in place; cls (host memory, optional): the W16 and W32 class sizes, which
 * bnf_launch_decode reads back one batch later to choose the side grids */
__global__ void __launch_bounds__(ORDER_NB) k_order_scan(uint32_t *__restrict__ hist, uint32_t *__restrict__ cls) {
    __shared__ uint32_t t[ORDER_NB];
    const uint32_t i = threadIdx.x;
    const uint32_t v = hist[i];
    t[i] = v;
    __syncthreads();
    for (uint32_t o = 1; o < ORDER_NB; o <<= 1) {
        const uint32_t a = i >= o ? t[i - o] : 0u;
        __syncthreads();
        t[i] += a;
        __syncthreads();
    }
    hist[i] = t[i] - v;
    if (cls && i == ORDER_NB - 1u) {
        cls[0] = t[3u * 64u - 1u] - t[2u * 64u - 1u];
        cls[1] = t[4u * 64u - 1u] - t[3u * 64u - 1u];
        cls[2] = t[ORDER_NB - 1u]; /* every frame of the order */
        cls[3] = t[2u * 64u - 1u] - t[64u - 1u]; /* class 1: narrow non-stereo frames (and failed ones) */
    }
}
template <int MODE>
__global__ void __launch_bounds__(256) k_order_place(const bnf_frame_info *__restrict__ info,
                                                     const uint8_t *__restrict__ bytes, uint64_t nbytes,
                                                     const uint64_t *__restrict__ offs, uint32_t nframes,
                                                     uint32_t *__restrict__ off, uint32_t *__restrict__ perm) {
    __shared__ uint32_t h[ORDER_NB], base[ORDER_NB];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t f = blockIdx.x * 256u + threadIdx.x;
    uint32_t k = 0, r = 0;
    if (f < nframes) {
        k = order_key<MODE>(info, bytes, nbytes, offs, f);
        r = atomicAdd(&h[k], 1u); /* rank within this block's share of the bucket */
    }
    __syncthreads();
    if (h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&off[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (f < nframes) perm[base[k] + r] = f;
}
/* order: ORDER_NB + nframes words of scratch; returns the permutation inside it */
template <int MODE>
static hipError_t launch_order(const bnf_frame_info *info, const uint8_t *bytes, uint64_t nbytes, const uint64_t *offs,
                               uint32_t nframes, uint32_t *order, const uint32_t **perm, hipStream_t s,
                               uint32_t *cls = nullptr) {
    uint32_t *hist = order, *pm = order + ORDER_NB;
    hipError_t e = hipMemsetAsync(hist, 0, ORDER_NB * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const dim3 g((nframes + 255) / 256);
    hipLaunchKernelGGL(k_order_count<MODE>, g, dim3(256), 0, s, info, bytes, nbytes, offs, nframes, hist);
    hipLaunchKernelGGL(k_order_scan, dim3(1), dim3(ORDER_NB), 0, s, hist, cls);
    hipLaunchKernelGGL(k_order_place<MODE>, g, dim3(256), 0, s, info, bytes, nbytes, offs, nframes, hist, pm);
    *perm = pm;
    return hipGetLastError();
}

/* The side streams of the current device for the W = 16 and W = 32 decode instances
 * (created on first use, kept for the process), and the decode order
 * (BNFLAC_DECODE_SERIAL=1: every decode instance on the caller's stream). */
struct SideQ {
    hipStream_t st[3]; /* W16, W32, the W8 instance's class-1 launch */
    hipEvent_t fork, join[3];
    uint32_t *cls; /* host memory: the last decode order's W16 / W32 class sizes, its frame count and its class 1 size (k_order_scan) */
};
static std::mutex g_side_mu;
static std::atomic<uint64_t> g_seg_launches{0}; /* k_decode_seg launches (bnf_decode_seg_launches) */
static SideQ g_side[64];
static int decode_fork_mode() { /* 0 serial; 1 fork after k_decode_st; 2 fork before it (default) */
    static const int m = [] {
        const char *e = getenv("BNFLAC_DECODE_SERIAL");
        if (e && atoi(e) != 0) return 0;
        const char *f = getenv("BNFLAC_DECODE_FORK");
        return (f && atoi(f) == 1) ? 1 : 2;
    }();
    return m;
}
static SideQ *side_queue() { /* under g_side_mu; nullptr: decode serially */
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    SideQ &q = g_side[dev];
    if (!q.st[1]) {
        SideQ n = {};
        bool ok = hipEventCreateWithFlags(&n.fork, hipEventDisableTiming) == hipSuccess;
        for (int i = 0; i < 3 && ok; i++)
            ok = hipStreamCreateWithFlags(&n.st[i], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&n.join[i], hipEventDisableTiming) == hipSuccess;
        if (ok && hipHostMalloc((void **)&n.cls, 64, hipHostMallocCoherent) != hipSuccess) n.cls = nullptr;
        if (n.cls) n.cls[0] = n.cls[1] = n.cls[2] = n.cls[3] = ~0u; /* unknown: the full grids */
        if (!ok) {
            for (int i = 0; i < 3; i++) {
                if (n.join[i]) (void)hipEventDestroy(n.join[i]);
                if (n.st[i]) (void)hipStreamDestroy(n.st[i]);
            }
            if (n.fork) (void)hipEventDestroy(n.fork);
            return nullptr;
        }
        q = n;
    }
    return &q;
}

/* Parse kernel choice: k_parse_wave (a wave per frame) for launches too small to fill the
 * chip with lane-per-frame waves, k_parse otherwise.  BNFLAC_PARSE_WAVE=0 never, 1 always.
 * Default, from tools/pw_stats.py on one box (lane walk vs wave scan, ms): C2 1,024 frames
 * 0.47 vs 0.12, 4,096 0.47 vs 0.21, 16,384 0.47 vs 0.62; C3 8,192 0.94 vs 0.19; C5 469 3.53 vs
 * 0.32, 3,752 3.33 vs 0.53; C4 4,096 2.56 vs 1.69.  The lane walk only wins once there are
 * ~256 lane-waves of short-partition frames: wave up to 8,192 frames, and up to 32,768 for
 * streams whose subframes are long (above 16 bits or more than 2 channels). */
static std::atomic<int> g_parse_wave{-1};
static bool use_parse_wave(uint32_t nframes, const bnf_stream_params &sp) {
    int m = g_parse_wave.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *e = getenv("BNFLAC_PARSE_WAVE");
        m = e ? (atoi(e) ? 1 : 0) : 2;
        g_parse_wave.store(m, std::memory_order_relaxed);
    }
    if (m != 2) return m == 1;
    return nframes <= 8192u || (nframes <= 32768u && (sp.bps > 16u || sp.channels > 2u));
}

/* k_decode_sys (systolic restore, every frame class) or the lane kernels by class.  The lane
 * kernels run one subframe per lane (k_decode_st: one stereo frame), so a launch of few frames is
 * a few waves, each as long as one lane's serial chain; k_decode_sys spreads each subframe over a
 * producer lane and a restore quad.  Auto: k_decode_sys while the lane kernels would have fewer
 * than SYS_AUTO_WAVES subframe waves (BNFLAC_SYS_WAVES overrides).
 * BNFLAC_DECODE_SYS=0 never, 1 always; bnf_set_decode_sys overrides. */
#define SYS_AUTO_WAVES 1024u
static std::atomic<int> g_decode_sys{-1};
static bool use_decode_sys(uint32_t nframes, const bnf_stream_params &sp, uint32_t chn_lanes) {
    int m = g_decode_sys.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *e = getenv("BNFLAC_DECODE_SYS");
        m = e ? (atoi(e) ? 1 : 0) : 2;
        g_decode_sys.store(m, std::memory_order_relaxed);
    }
    if (chn_lanes > 8u || m == 0) return false;
    if (m == 1) return true;
    static const uint32_t lim = [] {
        const char *e = getenv("BNFLAC_SYS_WAVES");
        return e ? (uint32_t)strtoul(e, nullptr, 0) : SYS_AUTO_WAVES;
    }();
    /* A variable-blocksize stream's lane waves last as long as its longest frames while most
     * frames are short, so the lane kernels need that many more frames to pay: the limit
     * scales with max_blocksize / 2048 (tools/sys_crossover.sh, profiles/r6_sys_crossover.txt:
     * C4, blocksizes 192-16384, sys 5.2 / 10.7 / 15.6 / 20.4 ms against the lanes' 15.8 / 17.2 /
     * 17.6 / 18.0 at 8 / 32 / 48 / 64 copies of 4,096 frames; C2 and C3, fixed blocksizes, cross
     * between 16 and 32 copies of 1,024 frames, where the unscaled limit already is) */
    uint64_t scale = 1;
    if (sp.has_stream_info && sp.max_blocksize > sp.min_blocksize && sp.max_blocksize > 4096u) scale = sp.max_blocksize / 2048u;
    return (uint64_t)nframes * chn_lanes < (uint64_t)lim * 64u * scale;
}

/* The CRC-16 hand-off (crcp, CRCP_WORDS): 0 none (the decode tails read every frame again),
 * 1 k_parse folds channel 0's lines from its ring while walking (the prefix), 2 and the rest of
 * the span to the next frame at its end (the verdict), 3 (default) 1 where it pays (below).
 * Env BNFLAC_CRC_MODE; bnf_set_crc_mode. */
static std::atomic<int> g_crc_mode{-1};
static int crc_mode() {
    int m = g_crc_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char *e = getenv("BNFLAC_CRC_MODE");
        m = e ? std::min(std::max(atoi(e), 0), 3) : 3;
        g_crc_mode.store(m, std::memory_order_relaxed);
    }
    return m;
}

extern "C" {
int bnf_crc_mode() { return crc_mode(); }
void bnf_set_crc_mode(int mode) { g_crc_mode.store(mode < 0 ? -1 : std::min(mode, 3), std::memory_order_relaxed); } /* -1: env */
uint64_t bnf_decode_seg_launches() { return g_seg_launches.load(std::memory_order_relaxed); }
void bnf_set_decode_sys(int mode) { g_decode_sys.store(mode < 0 ? 2 : (mode ? 1 : 0), std::memory_order_relaxed); } /* -1: auto */
void bnf_set_parse_wave(int mode) { g_parse_wave.store(mode < 0 ? 2 : (mode ? 1 : 0), std::memory_order_relaxed); } /* -1: auto */
hipError_t bnf_parse_wave_stats(uint64_t *out8, int reset) { /* debug counters of k_parse_wave (BNFLAC_PW_STATS=1) */
    hipError_t e = hipMemcpyFromSymbol(out8, HIP_SYMBOL(g_pw_stats), 8 * sizeof(uint64_t));
    if (e == hipSuccess && reset) {
        static const uint64_t z[8] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_pw_stats), z, sizeof z);
    }
    return e;
}
hipError_t bnf_launch_parse(const uint32_t *words, uint64_t nbytes, const uint64_t *frame_offs, uint32_t nframes,
                            bnf_stream_params sp, const uint64_t *out_sample_in, uint64_t base_sample,
                            bnf_frame_info *info, uint32_t *order, uint32_t *crcp, bool *handed, hipStream_t s) {
    if (handed) *handed = false;
    if (!nframes || !nbytes) return hipSuccess;
    if (use_parse_wave(nframes, sp)) { /* no CRC-16 hand-off from the wave walk */
        static const uint32_t pws = getenv("BNFLAC_PW_STATS") ? 1u : 0u;
        static const int seg = [] { const char *e = getenv("BNFLAC_PW_SEG"); return e ? atoi(e) : 0; }();
        hipLaunchKernelGGL(k_parse_wave, dim3(nframes), dim3(64), 0, s, words, nbytes, frame_offs, nframes, sp,
                           out_sample_in, base_sample, info, pws, seg);
        return hipGetLastError();
    }
    /* (Round 5: k_parse's occupancy is 5 waves per SIMD, LDS-bound; 4 or 3, by padding the LDS
     * to 10 / 13 KB, measured the same on C2-C4.)
     * the parse order (walk length from the header bytes): a fixed-blocksize stream's frames
     * all walk the same length (the last one aside), so the order only costs its three
     * launches there (C2: 0.12 ms per 1,024 batches) */
    const uint32_t *perm = nullptr;
    const bool fixed_bs = sp.has_stream_info && sp.min_blocksize == sp.max_blocksize;
    if (order && !fixed_bs) {
        hipError_t e = launch_order<1>(nullptr, (const uint8_t *)words, nbytes, frame_offs, nframes, order, &perm, s);
        if (e != hipSuccess) return e;
    }
    /* the CRC-16 hand-off (crcp; crc_mode).  It only pays where the stereo decode tails are on
     * the launch's critical path: not for a 16-bit stream whose previous decode order on this
     * device (one batch behind, as for the segment grid) had a quarter or more W16 / W32
     * frames, whose side instances then outlast k_decode_st (C4: k_parse +0.6 ms for no
     * decode gain) */
    int cm = crcp ? crc_mode() : 0;
    if (cm == 3 && sp.bps <= 16u) {
        std::lock_guard<std::mutex> lk(g_side_mu);
        const SideQ *sq = side_queue();
        if (sq && sq->cls) {
            const uint32_t w16 = __atomic_load_n(&sq->cls[0], __ATOMIC_RELAXED), w32 = __atomic_load_n(&sq->cls[1], __ATOMIC_RELAXED),
                           n = __atomic_load_n(&sq->cls[2], __ATOMIC_RELAXED);
            if (w16 != ~0u && w32 != ~0u && n != ~0u && 4ull * ((uint64_t)w16 + w32) >= n && n) cm = 0;
        }
    }
    if (cm == 3) cm = 1;
    if (handed) *handed = cm != 0;
    const dim3 g((nframes + 63) / 64);
    if (cm == 2)
        hipLaunchKernelGGL(k_parse<2>, g, dim3(64), 0, s, words, nbytes, frame_offs, nframes, sp, out_sample_in,
                           base_sample, info, ablate_flags(), perm, crcp);
    else if (cm == 1)
        hipLaunchKernelGGL(k_parse<1>, g, dim3(64), 0, s, words, nbytes, frame_offs, nframes, sp, out_sample_in,
                           base_sample, info, ablate_flags(), perm, crcp);
    else
        hipLaunchKernelGGL(k_parse<0>, g, dim3(64), 0, s, words, nbytes, frame_offs, nframes, sp, out_sample_in,
                           base_sample, info, ablate_flags(), perm, nullptr);
    return hipGetLastError();
}

/* k_fill_bad over a decoded batch (the batch API; not the stream API's candidate windows,
 * whose failed candidates share the next frame's slot) */
hipError_t bnf_launch_fill_bad(const bnf_frame_info *info, uint32_t nframes, bnf_stream_params sp, int fmt,
                               uint8_t *out, uint64_t out_bytes, hipStream_t s) {
    if (!nframes) return hipSuccess;
    hipLaunchKernelGGL(k_fill_bad, dim3((nframes + 63) / 64), dim3(64), 0, s, info, nframes, sp, fmt, out, out_bytes);
    return hipGetLastError();
}

hipError_t bnf_launch_decode(const uint32_t *words, uint64_t nbytes, uint32_t nframes, bnf_stream_params sp,
                             uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes, bnf_frame_info *info,
                             uint32_t *order, const uint32_t *crcp, hipStream_t s) {
    if (!nframes || !nbytes) return hipSuccess;
    uint32_t mode = 0;
    /* every frame through k_decode_sys (decode order by class and blocksize), then its
     * hand-backs through k_decode_list; order scratch: 256 + nframes (perm) + 4 + nframes (list) */
    if (order && use_decode_sys(nframes, sp, chn_lanes)) {
        const uint32_t *perm = nullptr;
        uint32_t *list = order + 256u + nframes;
        hipError_t e = hipMemsetAsync(list, 0, 16, s);
        if (e == hipSuccess) e = launch_order<0>(info, nullptr, 0, nullptr, nframes, order, &perm, s);
        if (e == hipSuccess)
            e = bnf_launch_decode_sys_tu8(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, list, mode, s);
        if (e == hipSuccess)
            e = bnf_launch_decode_list_tu2(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, list, mode, s);
        return e;
    }
    /* the class segments of the decode order (bucket ends), for the W16 / W32 grids */
    static const bool seg_on = [] { const char *e = getenv("BNFLAC_DECODE_SEG"); return !e || atoi(e) != 0; }();
    /* k_decode_st -> k_decode<8> on s (k_decode<8> takes k_decode_st's hand-backs);
     * k_decode<16> and k_decode<32> each on a side stream of the device, forked from s
     * before k_decode_st (default) or after it (BNFLAC_DECODE_FORK=1), and joined before
     * anything that reads the whole batch: the classes are disjoint frame sets.  Forking
     * before overlaps all four (C4 35.7 -> 27.8 ms).  While k_decode<32> had a 16-slot ring
     * (25.6 KB of LDS) its early-exiting workgroups slowed a batch with no W16/W32 frames
     * (C2's k_decode_st +4%), so the fork came after k_decode_st; with the 8-slot ring
     * (17 KB) C2 measures the same either way (3 A/B rounds).  The fork/join is enqueued under
     * one lock, so concurrent callers sharing the side streams keep their event pairs in
     * order. */
    /* Above 16 bits there are no stereo fast-path frames and LPC frames are W16/W32, so one
     * instance does nearly all the work; forking would only add the other instances'
     * early-exiting launches beside it (C3's k_decode<16>: 13.4 -> 15.0 ms) */
    const int fm = sp.bps > 16 ? 0 : decode_fork_mode();
    /* stereo frames above 16 bits: k_decode_sw first (serial above 16 bits), the other
     * instances then take only its hand-backs among them */
    const bool sw = sp.bps > 16 && sp.bps <= 24 && fmt != BNF_OUT_FLACDECODER && !(ablate_flags() & BNF_ABLATE_NO_SW);
    std::unique_lock<std::mutex> lk(g_side_mu, std::defer_lock);
    SideQ *sq = nullptr;
    if (fm) {
        lk.lock();
        sq = side_queue();
    }
    /* W16 / W32 grids: the full-size side grids, or -- when the previous decode order on this
     * device had neither class (read from host memory one batch behind, no sync; a stale or
     * wrong guess only costs time) -- k_decode_seg over both classes after k_decode<8> */
    uint32_t *cls = (sq && seg_on && order) ? sq->cls : nullptr;
    const bool seg_only = cls && __atomic_load_n(&cls[0], __ATOMIC_RELAXED) == 0u &&
                          __atomic_load_n(&cls[1], __ATOMIC_RELAXED) == 0u;
    const uint32_t *perm = nullptr;
    hipError_t e = hipSuccess;
    if (order) e = launch_order<0>(info, nullptr, 0, nullptr, nframes, order, &perm, s, cls);
    const uint32_t *seg = (perm && seg_on) ? order : nullptr;
    if (seg_only) { /* no fork */
        sq = nullptr;
        lk.unlock();
    }
    /* The W = 8 instance's two jobs as two launches when the previous decode order on this
     * device had class-1 frames (narrow non-stereo: VERBATIM / CONSTANT subframes; C4): those
     * on a third side stream beside k_decode_st, and after k_decode_st only its hand-backs.
     * One launch after k_decode_st put both on the stream's critical path (C4 at 32 copies:
     * k_decode_st 11.7 ms, then k_decode<8> 6.3 ms, while the W16 / W32 grids ended at 10.9). */
    const bool w8split = sq && seg && cls && __atomic_load_n(&cls[3], __ATOMIC_RELAXED) != 0u &&
                         !(ablate_flags() & BNF_ABLATE_NO_W8SPLIT);
    const int nside = w8split ? 3 : 2;
    auto fork = [&]() -> hipError_t {
        hipError_t r = hipEventRecord(sq->fork, s);
        for (int i = 0; i < nside && r == hipSuccess; i++) r = hipStreamWaitEvent(sq->st[i], sq->fork, 0);
        if (r == hipSuccess)
            r = bnf_launch_decode_tu2(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, seg, sq->st[1]);
        if (r == hipSuccess)
            r = bnf_launch_decode_tu5(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, seg, sq->st[0]);
        if (r == hipSuccess && w8split)
            r = bnf_launch_decode_tu1(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm,
                                      mode | BNF_MODE_NOST, seg, sq->st[2]);
        for (int i = 0; i < nside && r == hipSuccess; i++) r = hipEventRecord(sq->join[i], sq->st[i]);
        return r;
    };
    if (sq && fm == 2 && e == hipSuccess) e = fork();
    if (sw) {
        if (e == hipSuccess) e = bnf_launch_decode_sw_tu7(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, crcp, s);
        mode |= BNF_MODE_SW;
    }
    if (e == hipSuccess)
        e = fmt == BNF_OUT_FLACDECODER
                ? bnf_launch_decode_tu3(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, crcp, s)
                : bnf_launch_decode_tu4(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, crcp, s);
    if (sq && fm == 1 && e == hipSuccess) e = fork();
    if (e == hipSuccess)
        e = w8split ? bnf_launch_decode_tu1(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm,
                                            mode | BNF_MODE_STREDO, seg, s)
                    : bnf_launch_decode_tu1(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, nullptr, s);
    if (sq) {
        for (int i = 0; i < nside; i++) { /* joined even if a launch failed */
            const hipError_t ej = hipStreamWaitEvent(s, sq->join[i], 0);
            if (e == hipSuccess) e = ej;
        }
        lk.unlock();
    } else if (seg_only) {
        g_seg_launches.fetch_add(1, std::memory_order_relaxed);
        if (e == hipSuccess)
            e = bnf_launch_decode_seg_tu2(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, seg, s);
    } else {
        if (e == hipSuccess) e = bnf_launch_decode_tu5(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, seg, s);
        if (e == hipSuccess) e = bnf_launch_decode_tu2(words, nbytes, nframes, sp, chn_lanes, fmt, out, out_bytes, info, perm, mode, seg, s);
    }
    return e;
}

/* Frame chain over ncand parsed candidates (see k_gap_crc).  Scratch (device): gap_crc,
 * mark, pos: ncand u32 each; jump: levels * ncand i32; bs: ncand u64; small: 64 bytes.
 * *nframes (device) receives the chain length after the EOS rule (may exceed cap). */
hipError_t bnf_launch_chain(const uint8_t *bytes, uint64_t nbytes, const uint64_t *cand, uint32_t ncand,
                            const bnf_frame_info *info, uint64_t first_off, bnf_stream_params sp, uint32_t *gap_crc,
                            int32_t *jump, uint32_t levels, uint32_t *mark, uint32_t *pos, uint64_t *bs, uint8_t *small,
                            uint64_t *d_offs, uint64_t *d_os, bnf_frame_info *d_info, uint32_t cap, uint32_t *nframes,
                            hipStream_t s) {
    int32_t *head = (int32_t *)small;
    uint32_t *chain_len = (uint32_t *)(small + 8);
    uint64_t *samples = (uint64_t *)(small + 16);
    hipError_t e = hipMemsetAsync(head, 0x7f, 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(mark, 0, sizeof(uint32_t) * (size_t)ncand, s);
    if (e != hipSuccess) return e;
    const dim3 g256((ncand + 255) / 256);
    if (ncand) {
        hipLaunchKernelGGL(k_gap_crc, dim3((ncand + 3) / 4), dim3(256), 0, s, bytes, nbytes, cand, ncand, gap_crc);
        hipLaunchKernelGGL(k_chain_keys, dim3(1), dim3(1024), 0, s, gap_crc, ncand, info);
        hipLaunchKernelGGL(k_chain_succ, g256, dim3(256), 0, s, cand, ncand, gap_crc, first_off, jump, head);
        for (uint32_t k = 0; k + 1 < levels; k++)
            hipLaunchKernelGGL(k_chain_jump, g256, dim3(256), 0, s, jump + (size_t)k * ncand,
                               jump + (size_t)(k + 1) * ncand, ncand);
        hipLaunchKernelGGL(k_chain_mark, g256, dim3(256), 0, s, jump, mark, ncand, head, 1);
        for (int k = (int)levels - 1; k >= 0; k--)
            hipLaunchKernelGGL(k_chain_mark, g256, dim3(256), 0, s, jump + (size_t)k * ncand, mark, ncand, head, 0);
        e = hipMemcpyAsync(pos, mark, sizeof(uint32_t) * (size_t)ncand, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, pos, ncand, chain_len);
    hipLaunchKernelGGL(k_chain_compact, g256, dim3(256), 0, s, cand, ncand, info, mark, pos, bs, ncand);
    hipLaunchKernelGGL(k_scan_u64, dim3(1), dim3(1024), 0, s, bs, chain_len, ncand, samples);
    e = hipMemcpyAsync(nframes, chain_len, 4, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    if (ncand)
        hipLaunchKernelGGL(k_chain_emit, g256, dim3(256), 0, s, cand, ncand, info, mark, pos, bs, sp, d_offs, d_os,
                           d_info, cap, nframes);
    return hipGetLastError();
}

hipError_t bnf_launch_scan_u32(uint32_t *v, uint32_t n, uint32_t *total, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, v, n, total);
    return hipGetLastError();
}
} /* extern "C" */
#endif
