/*
 * bnflac_runtime.cpp -- host side of libbnflac.so.
 *
 *  - bnflac_* batched API: thin, asynchronous launchers over the HIP kernels.
 *  - FLAC__stream_decoder_*: libFLAC 1.2.1-compatible stream decoder.  Metadata and
 *    the libFLAC state machine (find_metadata_, frame_sync_, the per-frame error and
 *    write sequence of read_frame_, LibFlac.dll@0x10010130/0x10011760/0x100118c0) are
 *    replayed on the host from per-frame records; every frame body is decoded on the
 *    GPU in windows of many frames at once.  Read-ahead changes when the client's read
 *    callback is called, never what the write/error callbacks receive.
 *
 * The product path has no CPU decode: if no GPU is usable the decoder fails loudly
 * (init returns MEMORY_ALLOCATION_ERROR and bnflac_last_error() says why).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../../include/bnflac.h"
#include "bnflac_device.h"
#include "bnflac_md5.h"

static_assert(sizeof(bnflac_frame_info) == sizeof(bnf_frame_info), "frame info layout");
static_assert(sizeof(bnf_frame_info) == 128, "frame info is 128 bytes");
static_assert(offsetof(FLAC__FrameHeader, number) == 24, "FrameHeader.FrameOrSampleNumber @24 (LibFLACSharp.cs:232)");
static_assert(offsetof(FLAC__FrameHeader, crc) == 32, "FrameHeader.Crc @32 (LibFLACSharp.cs:233)");
static_assert(offsetof(FLAC__StreamMetadata, data) == 16, "StreamMetadata.data @16 (LibFLACSharp.cs:299)");
static_assert(offsetof(FLAC__StreamMetadata, data.stream_info.sample_rate) == 32, "sample_rate @32");
static_assert(offsetof(FLAC__StreamMetadata, data.stream_info.total_samples) == 48, "total_samples @48");

extern "C" {
hipError_t bnf_upload_tables(const uint8_t *crc8, const uint16_t *crc16x8, const uint16_t *xpow);
hipError_t bnf_launch_sync_scan(const uint8_t *d, uint64_t n, uint32_t *d_block_counts, uint32_t *d_total,
                                uint64_t *d_out, uint32_t cap, hipStream_t s);
uint32_t bnf_scan_blocks(uint64_t n);
void bnf_set_ablate(uint32_t v);
hipError_t bnf_stats(uint64_t *out16, int reset);
hipError_t bnf_launch_parse(const uint32_t *words, uint64_t nbytes, const uint64_t *frame_offs,
                            uint32_t nframes, bnf_stream_params sp, const uint64_t *out_sample_in,
                            uint64_t base_sample, bnf_frame_info *info, uint32_t *order, uint32_t *crcp,
                            bool *handed, hipStream_t s);
/* order: nullptr, or 256 + nframes words of device scratch for the frame order (k_order_*);
 * crcp: nullptr, or k_parse's CRC-16 hand-off for these frames (8 words per frame) */
hipError_t bnf_launch_decode(const uint32_t *words, uint64_t nbytes, uint32_t nframes,
                             bnf_stream_params sp, uint32_t chn_lanes, int fmt, uint8_t *out, uint64_t out_bytes,
                             bnf_frame_info *info, uint32_t *order, const uint32_t *crcp, hipStream_t s);
hipError_t bnf_launch_fill_bad(const bnf_frame_info *info, uint32_t nframes, bnf_stream_params sp, int fmt,
                               uint8_t *out, uint64_t out_bytes, hipStream_t s);
hipError_t bnf_launch_chain(const uint8_t *bytes, uint64_t nbytes, const uint64_t *cand, uint32_t ncand,
                            const bnf_frame_info *info, uint64_t first_off, bnf_stream_params sp, uint32_t *gap_crc,
                            int32_t *jump, uint32_t levels, uint32_t *mark, uint32_t *pos, uint64_t *bs, uint8_t *small,
                            uint64_t *d_offs, uint64_t *d_os, bnf_frame_info *d_info, uint32_t cap, uint32_t *nframes,
                            hipStream_t s);
}

/* ------------------------------------------------------------------ errors */
static thread_local std::string g_err;
static int fail(const std::string &m, int code = -1) {
    g_err = m;
    return code;
}
extern "C" BNFLAC_API const char *bnflac_last_error(void) { return g_err.c_str(); }

/* ------------------------------------------------------------ CRC tables */
static void build_tables(uint8_t *c8, uint16_t *c16, uint16_t *xp) {
    for (int i = 0; i < 256; i++) {
        uint8_t c = (uint8_t)i;
        for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
        c8[i] = c;
        uint16_t w = (uint16_t)(i << 8);
        for (int b = 0; b < 8; b++) w = (uint16_t)((w & 0x8000) ? (w << 1) ^ 0x8005 : (w << 1));
        c16[i] = w;
    }
    for (int k = 1; k < 8; k++)
        for (int i = 0; i < 256; i++) {
            uint16_t p = c16[(k - 1) * 256 + i];
            c16[k * 256 + i] = (uint16_t)((p << 8) ^ c16[p >> 8]);
        }
    /* x^(8*2^j) mod P */
    auto mulmod = [](uint32_t a, uint32_t b) {
        uint32_t r = 0;
        for (int i = 15; i >= 0; i--) {
            r = (r & 0x8000u) ? ((r << 1) ^ 0x8005u) & 0xffffu : (r << 1);
            if ((b >> i) & 1u) r ^= a;
        }
        return r;
    };
    uint32_t v = 0x0100; /* x^8 */
    for (int j = 0; j < 40; j++) {
        xp[j] = (uint16_t)v;
        v = mulmod(v, v);
    }
}

/* The caller's current HIP device is restored on scope exit (the library never leaves the
 * thread on another device). */
struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

static std::mutex g_dev_mu;
static bool g_tables_ready[64];

static int ensure_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail("bnflac: no HIP device available (the decode path is GPU-only)");
    if (dev < 0 || dev >= n || dev >= 64) return fail("bnflac: bad device index");
    std::lock_guard<std::mutex> lk(g_dev_mu);
    DevGuard g(dev);
    if (!g_tables_ready[dev]) {
        uint8_t c8[256];
        uint16_t c16[8 * 256], xp[40];
        build_tables(c8, c16, xp);
        if (bnf_upload_tables(c8, c16, xp) != hipSuccess) return fail("bnflac: table upload failed");
        g_tables_ready[dev] = true;
    }
    return 0;
}

/* Timing experiments only (bench.py --ablate): skip parts of the kernels.  Results are
 * wrong while non-zero.  bit0 CRC-16, bit1 PCM stores, bit2 restore, bit3 Rice decode,
 * bit4 k_parse subframe walk.  0x2000 is an exact A/B switch: the 24-bit FLACFileReader
 * wide flush (pack_wide24) off. */
extern "C" BNFLAC_API void bnflac_debug_set_ablate(uint32_t flags) { bnf_set_ablate(flags); }
extern "C" void bnf_set_parse_wave(int mode);
/* parse kernel: -1 auto (k_parse_wave for small launches), 0 k_parse, 1 k_parse_wave (tests, A/B) */
extern "C" BNFLAC_API void bnflac_debug_set_parse_wave(int mode) { bnf_set_parse_wave(mode); }
extern "C" void bnf_set_decode_sys(int mode);
/* k_decode_sys (systolic restore, every frame class): -1 auto (BNFLAC_DECODE_SYS), 0 the lane
 * kernels by class, 1 always (tests, A/B) */
extern "C" BNFLAC_API void bnflac_debug_set_decode_sys(int mode) { bnf_set_decode_sys(mode); }
extern "C" int bnf_crc_mode();
extern "C" void bnf_set_crc_mode(int mode);
/* the CRC-16 hand-off: -1 env BNFLAC_CRC_MODE (default 3), 0 none, 1 k_parse's prefix, 2 + its verdict,
 * 3 the prefix where it pays (bnf_launch_parse) */
extern "C" BNFLAC_API void bnflac_debug_set_crc_mode(int mode) { bnf_set_crc_mode(mode); }
extern "C" uint64_t bnf_decode_seg_launches();
extern "C" BNFLAC_API uint64_t bnflac_debug_decode_seg_launches(void) { return bnf_decode_seg_launches(); }
extern "C" hipError_t bnf_parse_wave_stats(uint64_t *out8, int reset);
/* k_parse_wave's debug counters (collected when BNFLAC_PW_STATS is set): passes, splice rounds,
 * serial fallbacks, partitions, frames, wave-cycles in scans.  out8: 8 values. */
extern "C" BNFLAC_API int bnflac_debug_parse_wave_stats(uint64_t *out8, int reset) {
    return bnf_parse_wave_stats(out8, reset) == hipSuccess ? 0 : -1;
}
extern "C" BNFLAC_API int bnflac_debug_stats(uint64_t *out16, int reset) {
    return bnf_stats(out16, reset) == hipSuccess ? 0 : fail("bnflac_debug_stats failed");
}

extern "C" BNFLAC_API int bnflac_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

/* ----------------------------------------------------------------- context */
struct CtxBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool grow(size_t n) {
        if (n <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, n) != hipSuccess) return false;
        cap = n;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct bnflac_ctx {
    int device;
    uint32_t *d_block_counts = nullptr;
    uint32_t block_cap = 0;
    /* bnflac_index_stream scratch */
    CtxBuf cand, info, gap, jump, mark, pos, bs, small;
    CtxBuf order, porder; /* decode / parse order: histogram + permutation (k_order_*) */
    /* k_parse's CRC-16 hand-off of the last bnflac_parse_frames batch (8 words per frame), and
     * the batch they belong to: bnflac_decode_parsed uses them only for that same batch */
    CtxBuf crcp;
    const void *crcp_bytes = nullptr, *crcp_info = nullptr;
    uint64_t crcp_nbytes = 0;
    uint32_t crcp_n = 0;
};

/* crc mode 0: no CRC-16 hand-off, the decode tails check the whole frame (1 / 2 choose who
 * computes it: bnf_launch_parse) */
static bool crc_prefix_on() { return bnf_crc_mode() != 0; }

extern "C" BNFLAC_API int bnflac_ctx_create(int device, bnflac_ctx **out) {
    *out = nullptr;
    if (ensure_device(device)) return -1;
    bnflac_ctx *c = new bnflac_ctx();
    c->device = device;
    *out = c;
    return 0;
}

/* Debug: the CRC-16 hand-off of the ctx's last bnflac_parse_frames (8 words per frame, see
 * CRCP_WORDS in bnflac_kernels.hip), synchronously; -1 when there is none for nframes frames */
extern "C" BNFLAC_API int bnflac_debug_crc_handoff(bnflac_ctx *ctx, uint32_t *out, uint32_t nframes) {
    if (!ctx || !out) return fail("bnflac_debug_crc_handoff: null argument");
    if (!ctx->crcp_bytes || ctx->crcp_n != nframes) return fail("bnflac_debug_crc_handoff: no hand-off for this batch");
    DevGuard dg(ctx->device);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(out, ctx->crcp.p, 32ull * nframes, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("bnflac_debug_crc_handoff: HIP error");
    return 0;
}

extern "C" BNFLAC_API void bnflac_ctx_destroy(bnflac_ctx *ctx) {
    if (!ctx) return;
    if (ctx->d_block_counts) (void)hipFree(ctx->d_block_counts);
    for (CtxBuf *b : {&ctx->cand, &ctx->info, &ctx->gap, &ctx->jump, &ctx->mark, &ctx->pos, &ctx->bs, &ctx->small,
                      &ctx->order, &ctx->porder, &ctx->crcp})
        b->release();
    delete ctx;
}

static uint32_t lanes_for(uint32_t channels) {
    uint32_t l = 1;
    while (l < channels) l <<= 1;
    return l > 8 ? 8 : l;
}

extern "C" BNFLAC_API uint32_t bnflac_out_stride(int fmt, const bnflac_stream_params *sp) {
    switch (fmt) {
    case BNFLAC_OUT_PLANAR32:
    case BNFLAC_OUT_INTERLEAVED32: return 4u * sp->channels;
    case BNFLAC_OUT_FLACDECODER: return sp->channels == 2 ? 4u : 2u;
    default: return sp->channels * (sp->bps == 24 ? 3u : 2u);
    }
}

extern "C" BNFLAC_API int bnflac_md5_interleaved32(const int32_t *pcm, uint64_t nsamples, uint32_t channels,
                                                   uint32_t bps, uint8_t out_md5[16]) {
    if ((!pcm && nsamples) || !out_md5) return fail("bnflac_md5_interleaved32: null pointer");
    if (channels < 1 || channels > FLAC__MAX_CHANNELS || bps < 4 || bps > 32)
        return fail("bnflac_md5_interleaved32: bad channels/bps");
    Md5 m;
    md5_init(m);
    const int32_t *chan[FLAC__MAX_CHANNELS];
    for (uint32_t c = 0; c < channels; c++) chan[c] = pcm + c;
    md5_accumulate(m, chan, channels, nsamples, channels, (bps + 7) / 8);
    md5_final(m, out_md5);
    return 0;
}

extern "C" BNFLAC_API int bnflac_index_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                              uint64_t *d_offsets, uint32_t cap, uint32_t *d_count, void *hs) {
    if (!ctx) return fail("bnflac_index_frames: null ctx");
    DevGuard dg(ctx->device); /* launches and scratch on the context's device */
    if (((uintptr_t)d_bytes) & 3u) return fail("bnflac_index_frames: d_bytes must be 4-byte aligned");
    const uint32_t nb = bnf_scan_blocks(nbytes);
    if (nb > ctx->block_cap) {
        if (ctx->d_block_counts) (void)hipFree(ctx->d_block_counts);
        ctx->d_block_counts = nullptr;
        if (hipMalloc(&ctx->d_block_counts, sizeof(uint32_t) * (size_t)std::max(nb, 1u)) != hipSuccess)
            return fail("bnflac_index_frames: out of device memory");
        ctx->block_cap = nb;
    }
    hipError_t e = bnf_launch_sync_scan(d_bytes, nbytes, ctx->d_block_counts, d_count, d_offsets, cap, (hipStream_t)hs);
    return e == hipSuccess ? 0 : fail(std::string("bnflac_index_frames: ") + hipGetErrorString(e));
}

static int check_args(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, const bnflac_stream_params *sp,
                      const char *who) {
    if (!ctx || !sp) return fail(std::string(who) + ": null argument");
    if (((uintptr_t)d_bytes) & 15u) return fail(std::string(who) + ": d_bytes must be 16-byte aligned");
    if (sp->channels < 1 || sp->channels > 8) return fail(std::string(who) + ": channels must be 1..8");
    if (nbytes >= (1ull << 34)) return fail(std::string(who) + ": buffer larger than 16 GiB");
    return 0;
}

extern "C" BNFLAC_API int bnflac_parse_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                              const uint64_t *d_frame_offsets, uint32_t nframes,
                                              const bnflac_stream_params *sp, const uint64_t *d_out_sample,
                                              uint64_t base_sample, bnflac_frame_info *d_info, void *hs) {
    if (check_args(ctx, d_bytes, nbytes, sp, "bnflac_parse_frames")) return -1;
    DevGuard dg(ctx->device); /* launches and scratch on the context's device */
    bnf_stream_params p;
    memcpy(&p, sp, sizeof p);
    if (!ctx->porder.grow(sizeof(uint32_t) * (256u + (size_t)nframes)))
        return fail("bnflac_parse_frames: out of device memory (parse-order scratch)");
    ctx->crcp_bytes = ctx->crcp_info = nullptr; /* no prefixes until this launch is enqueued */
    const bool pre = crc_prefix_on() && ctx->crcp.grow(32u * std::max<size_t>(nframes, 1u));
    bool handed = false;
    hipError_t e = bnf_launch_parse((const uint32_t *)d_bytes, nbytes, d_frame_offsets,
                                    nframes, p, d_out_sample, base_sample, (bnf_frame_info *)d_info,
                                    (uint32_t *)ctx->porder.p, pre ? (uint32_t *)ctx->crcp.p : nullptr, &handed,
                                    (hipStream_t)hs);
    if (e == hipSuccess && pre && handed) {
        ctx->crcp_bytes = d_bytes;
        ctx->crcp_info = d_info;
        ctx->crcp_nbytes = nbytes;
        ctx->crcp_n = nframes;
    }
    return e == hipSuccess ? 0 : fail(std::string("k_parse: ") + hipGetErrorString(e));
}

extern "C" BNFLAC_API int bnflac_decode_parsed(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes, uint32_t nframes,
                                               const bnflac_stream_params *sp, int out_format, uint8_t *d_out,
                                               uint64_t out_bytes, bnflac_frame_info *d_info, void *hs) {
    if (check_args(ctx, d_bytes, nbytes, sp, "bnflac_decode_parsed")) return -1;
    DevGuard dg(ctx->device); /* launches and scratch on the context's device */
    if (out_format < 0 || out_format > 3) return fail("bnflac_decode_parsed: bad out_format");
    bnf_stream_params p;
    memcpy(&p, sp, sizeof p);
    /* decode order (256 + nframes) + k_decode_sys's hand-back list (4 + nframes) */
    if (!ctx->order.grow(sizeof(uint32_t) * (260u + 2u * (size_t)nframes)))
        return fail("bnflac_decode_parsed: out of device memory (decode-order scratch)");
    /* the parse of this same batch on this context handed over its CRC-16 work (used once) */
    const bool pre = ctx->crcp_bytes == d_bytes && ctx->crcp_info == d_info && ctx->crcp_nbytes == nbytes &&
                     ctx->crcp_n == nframes;
    ctx->crcp_bytes = ctx->crcp_info = nullptr;
    hipError_t e = bnf_launch_decode((const uint32_t *)d_bytes, nbytes, nframes, p,
                                     lanes_for(sp->channels), out_format, d_out, out_bytes, (bnf_frame_info *)d_info,
                                     (uint32_t *)ctx->order.p, pre ? (const uint32_t *)ctx->crcp.p : nullptr,
                                     (hipStream_t)hs);
    if (e == hipSuccess) /* a non-OK frame's range: zeros (include/bnflac.h) */
        e = bnf_launch_fill_bad((const bnf_frame_info *)d_info, nframes, p, out_format, d_out, out_bytes, (hipStream_t)hs);
    return e == hipSuccess ? 0 : fail(std::string("k_decode: ") + hipGetErrorString(e));
}

extern "C" BNFLAC_API int bnflac_decode_frames(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                               const uint64_t *d_frame_offsets, uint32_t nframes,
                                               const bnflac_stream_params *sp, const uint64_t *d_out_sample,
                                               uint64_t base_sample, int out_format, uint8_t *d_out, uint64_t out_bytes,
                                               bnflac_frame_info *d_info, void *hs) {
    if (out_format < 0 || out_format > 3) return fail("bnflac_decode_frames: bad out_format");
    int rc = bnflac_parse_frames(ctx, d_bytes, nbytes, d_frame_offsets, nframes, sp, d_out_sample, base_sample, d_info, hs);
    if (rc) return rc;
    return bnflac_decode_parsed(ctx, d_bytes, nbytes, nframes, sp, out_format, d_out, out_bytes, d_info, hs);
}

extern "C" BNFLAC_API int bnflac_index_stream(bnflac_ctx *ctx, const uint8_t *d_bytes, uint64_t nbytes,
                                              uint64_t first_offset, const bnflac_stream_params *sp,
                                              uint64_t *d_frame_offsets, uint64_t *d_out_sample,
                                              bnflac_frame_info *d_info, uint32_t cap, uint32_t *d_nframes, void *hs) {
    if (check_args(ctx, d_bytes, nbytes, sp, "bnflac_index_stream")) return -1;
    DevGuard dg(ctx->device); /* launches and scratch on the context's device */
    if (!d_frame_offsets || !d_nframes) return fail("bnflac_index_stream: null output");
    hipStream_t s = (hipStream_t)hs;
    /* 1. sync candidates (one host sync for their count) */
    uint32_t ccap = (uint32_t)std::min<uint64_t>(nbytes / 1024 + 4096, 1u << 30), ncand = 0;
    for (int attempt = 0;; attempt++) {
        if (!ctx->cand.grow(sizeof(uint64_t) * ccap) || !ctx->small.grow(64))
            return fail("bnflac_index_stream: out of device memory");
        if (bnflac_index_frames(ctx, d_bytes, nbytes, (uint64_t *)ctx->cand.p, ccap, (uint32_t *)ctx->small.p, hs))
            return -1;
        if (hipMemcpyAsync(&ncand, ctx->small.p, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return fail("bnflac_index_stream: HIP error reading the candidate count");
        if (ncand <= ccap) break;
        if (attempt) return fail("bnflac_index_stream: candidate count changed");
        ccap = ncand;
    }
    if (ncand >= (1u << 30)) return fail("bnflac_index_stream: too many sync candidates");
    uint32_t levels = 1;
    while ((1ull << levels) <= ncand) levels++;
    const size_t n = std::max<uint32_t>(ncand, 1u);
    if (!ctx->info.grow(sizeof(bnf_frame_info) * n) || !ctx->gap.grow(4 * n) || !ctx->jump.grow(4 * n * levels) ||
        !ctx->mark.grow(4 * n) || !ctx->pos.grow(4 * n) || !ctx->bs.grow(8 * n))
        return fail("bnflac_index_stream: out of device memory");
    bnf_stream_params p;
    memcpy(&p, sp, sizeof p);
    ctx->crcp_bytes = ctx->crcp_info = nullptr; /* the records this writes carry no CRC-16 hand-off */
    /* 2. header, CRC-8 and subframe walk of every candidate */
    hipError_t e = bnf_launch_parse((const uint32_t *)d_bytes, nbytes, (const uint64_t *)ctx->cand.p, ncand, p, nullptr,
                                    0, (bnf_frame_info *)ctx->info.p, nullptr, nullptr, nullptr, s);
    /* 3. successor chain, EOS rule, compaction */
    if (e == hipSuccess)
        e = bnf_launch_chain(d_bytes, nbytes, (const uint64_t *)ctx->cand.p, ncand, (const bnf_frame_info *)ctx->info.p,
                             first_offset, p, (uint32_t *)ctx->gap.p, (int32_t *)ctx->jump.p, levels,
                             (uint32_t *)ctx->mark.p, (uint32_t *)ctx->pos.p, (uint64_t *)ctx->bs.p,
                             (uint8_t *)ctx->small.p + 16, d_frame_offsets, d_out_sample, (bnf_frame_info *)d_info, cap,
                             d_nframes, s);
    return e == hipSuccess ? 0 : fail(std::string("bnflac_index_stream: ") + hipGetErrorString(e));
}

/* ====================================================================== */
/*                 libFLAC-compatible stream decoder                       */
/* ====================================================================== */

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool grow(size_t n) {
        if (n <= cap) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(n, 1 << 16);
        c = c + c / 4;
        if (hipMalloc(&p, c) != hipSuccess) return false;
        cap = c;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

} // namespace

struct FLAC__StreamDecoder {
    FLAC__StreamDecoderState state = FLAC__STREAM_DECODER_UNINITIALIZED;
    FLAC__StreamDecoderReadCallback read_cb = nullptr;
    FLAC__StreamDecoderSeekCallback seek_cb = nullptr;
    FLAC__StreamDecoderTellCallback tell_cb = nullptr;
    FLAC__StreamDecoderLengthCallback length_cb = nullptr;
    FLAC__StreamDecoderEofCallback eof_cb = nullptr;
    FLAC__StreamDecoderWriteCallback write_cb = nullptr;
    FLAC__StreamDecoderMetadataCallback metadata_cb = nullptr;
    FLAC__StreamDecoderErrorCallback error_cb = nullptr;
    void *client = nullptr;
    FILE *file = nullptr;
    bool ignore_write_status = false;

    /* bytes delivered by the read callback, stream offsets [buf_base, buf_base + buf.size());
     * pos = consumed (absolute).  Bytes below the frame being decoded are dropped once they
     * pile up (trim_consumed); a seek repositions the client and restarts the buffer there. */
    std::vector<uint8_t> buf;
    uint64_t buf_base = 0;
    uint64_t pos = 0;
    uint64_t bitpos_meta = 0; /* bit cursor used while reading metadata */
    bool cached = false;
    uint8_t lookahead = 0;
    uint8_t header_warmup[2] = {0, 0};
    int client_done = 0; /* 1: client reported end of stream, 2: abort */

    bool has_stream_info = false;
    FLAC__StreamMetadata stream_info;
    uint64_t samples_decoded = 0;
    unsigned fixed_block_size = 0, next_fixed_block_size = 0;
    uint64_t first_frame_offset = 0;
    bool is_seeking = false;
    /* MD5 of the decoded PCM vs STREAMINFO md5sum (stream_decoder.c md5_checking /
     * do_md5_checking / md5context); off unless set_md5_checking(true) before init */
    bool md5_checking = false, do_md5 = false;
    Md5 md5;
    uint64_t seek_target = 0;
    int seek_done = 0;
    /* SEEKTABLE points (read_metadata_seektable_): sample number, byte offset from the first
     * frame header, frame samples; placeholders dropped.  Only narrows a seek's search. */
    struct SeekPoint { uint64_t sample, offset; uint32_t frame_samples; };
    std::vector<SeekPoint> seek_table;

    FLAC__Frame frame;
    std::vector<int32_t> output[FLAC__MAX_CHANNELS];
    unsigned output_capacity = 0, output_channels = 0;

    unsigned channels = 0, bits_per_sample = 0, sample_rate = 0, blocksize = 0;
    FLAC__ChannelAssignment channel_assignment = FLAC__CHANNEL_ASSIGNMENT_INDEPENDENT;

    /* GPU window */
    int device = 0;
    bool gpu_ready = false;
    hipStream_t stream = nullptr;
    bnflac_ctx *ctx = nullptr;
    DevBuf d_bytes, d_cand, d_count, d_info, d_pcm;
    uint64_t win_base = 0, win_end = 0;
    bool win_valid = false;
    std::vector<uint64_t> cand;
    std::vector<bnf_frame_info> info;
    std::vector<int32_t> pcm;
    uint32_t pcm_ch = 1;                    /* planar slots per sample in pcm: the window's widest frame */
    uint64_t read_ahead = 32ull << 20;      /* window read-ahead cap */
    uint64_t read_ahead_cur = 256ull << 10; /* grows x2 per window up to the cap: the first frame comes quickly */
};

namespace {

using Dec = FLAC__StreamDecoder;

uint64_t bend(const Dec *d) { return d->buf_base + d->buf.size(); } /* one past the last buffered byte */
uint8_t bat(const Dec *d, uint64_t p) { return d->buf[(size_t)(p - d->buf_base)]; }


/* read_callback_ (stream_decoder.c) semantics, without touching the decoder state:
 * 0 = got bytes, 1 = end of stream, 2 = abort. */
int fill_raw(Dec *d, size_t want = 65536) {
    if (d->client_done) {
        /* libFLAC would ask again: the eof callback answers first */
        if (d->client_done == 2) return 2;
        if (d->eof_cb && d->eof_cb(d, d->client)) return 1;
    }
    for (int spins = 0; spins < 1000000; spins++) {
        if (d->eof_cb && d->eof_cb(d, d->client)) return 1;
        size_t old = d->buf.size();
        size_t bytes = want;
        d->buf.resize(old + bytes);
        FLAC__StreamDecoderReadStatus st = d->read_cb(d, d->buf.data() + old, &bytes, d->client);
        if (bytes > want) bytes = want;
        d->buf.resize(old + bytes);
        if (st == FLAC__STREAM_DECODER_READ_STATUS_ABORT) return 2;
        if (bytes == 0) {
            if (st == FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM || (d->eof_cb && d->eof_cb(d, d->client))) return 1;
            continue;
        }
        return 0;
    }
    return 2;
}

/* the decoder genuinely needs bytes [.., upto): failure sets END_OF_STREAM / ABORTED */
bool need_bytes(Dec *d, uint64_t upto) {
    while (bend(d) < upto) {
        int r = fill_raw(d);
        if (r) {
            if (!d->client_done) d->client_done = r;
            d->state = (r == 2) ? FLAC__STREAM_DECODER_ABORTED : FLAC__STREAM_DECODER_END_OF_STREAM;
            return false;
        }
    }
    return true;
}

/* read ahead for the GPU window; hitting the client's end is remembered, not reported */
void read_ahead(Dec *d, uint64_t upto) {
    while (bend(d) < upto && !d->client_done) {
        int r = fill_raw(d);
        if (r) d->client_done = r;
    }
}

/* metadata bit reader on the host buffer */
bool mb_read(Dec *d, uint32_t *v, unsigned bits) {
    if (bits == 0) {
        *v = 0;
        return true;
    }
    uint64_t end = d->bitpos_meta + bits;
    if (!need_bytes(d, (end + 7) / 8)) return false;
    uint64_t x = 0;
    for (uint64_t p = d->bitpos_meta; p < end; p++) x = (x << 1) | ((bat(d, p >> 3) >> (7 - (p & 7))) & 1u);
    d->bitpos_meta = end;
    *v = (uint32_t)x;
    return true;
}

bool mb_byte(Dec *d, uint32_t *x) {
    if (d->cached) {
        *x = d->lookahead;
        d->cached = false;
        return true;
    }
    return mb_read(d, x, 8);
}

void send_error(Dec *d, FLAC__StreamDecoderErrorStatus st) {
    if (!d->is_seeking) d->error_cb(d, st, d->client);
}

bool skip_id3v2(Dec *d) {
    uint32_t x, skip = 0;
    if (!mb_read(d, &x, 24)) return false;
    for (int i = 0; i < 4; i++) {
        if (!mb_read(d, &x, 8)) return false;
        skip = (skip << 7) | (x & 0x7f);
    }
    uint64_t end = d->bitpos_meta + (uint64_t)skip * 8;
    if (!need_bytes(d, end / 8)) return false;
    d->bitpos_meta = end;
    return true;
}

/* find_metadata_ */
bool find_metadata(Dec *d) {
    static const uint8_t sync[4] = {'f', 'L', 'a', 'C'};
    static const uint8_t id3[3] = {'I', 'D', '3'};
    uint32_t x;
    unsigned i = 0, id = 0;
    bool first = true;
    while (i < 4) {
        if (!mb_byte(d, &x)) return false;
        if (x == sync[i]) {
            first = true;
            i++;
            id = 0;
            continue;
        }
        if (x == id3[id]) {
            id++;
            i = 0;
            if (id == 3 && !skip_id3v2(d)) return false;
            continue;
        }
        id = 0;
        if (x == 0xff) {
            d->header_warmup[0] = (uint8_t)x;
            if (!mb_read(d, &x, 8)) return false;
            if (x == 0xff) {
                d->lookahead = (uint8_t)x;
                d->cached = true;
            } else if (x >> 2 == 0x3e) {
                d->header_warmup[1] = (uint8_t)x;
                d->pos = d->bitpos_meta / 8;
                d->state = FLAC__STREAM_DECODER_READ_FRAME;
                return true;
            }
        }
        i = 0;
        if (first) {
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            first = false;
        }
    }
    d->state = FLAC__STREAM_DECODER_READ_METADATA;
    return true;
}

/* read_metadata_ (STREAMINFO reported; every other block skipped, as libFLAC's default
 * metadata_respond set does) */
bool read_metadata(Dec *d) {
    uint32_t last, type, length;
    if (!mb_read(d, &last, 1) || !mb_read(d, &type, 7) || !mb_read(d, &length, 24)) return false;
    if (type == FLAC__METADATA_TYPE_STREAMINFO) {
        FLAC__StreamMetadata &m = d->stream_info;
        FLAC__StreamMetadata_StreamInfo &si = m.data.stream_info;
        uint32_t v, hi, lo;
        memset(&m, 0, sizeof m);
        m.type = FLAC__METADATA_TYPE_STREAMINFO;
        m.is_last = last ? 1 : 0;
        m.length = length;
        if (!mb_read(d, &v, 16)) return false;
        si.min_blocksize = v;
        if (!mb_read(d, &v, 16)) return false;
        si.max_blocksize = v;
        if (!mb_read(d, &v, 24)) return false;
        si.min_framesize = v;
        if (!mb_read(d, &v, 24)) return false;
        si.max_framesize = v;
        if (!mb_read(d, &v, 20)) return false;
        si.sample_rate = v;
        if (!mb_read(d, &v, 3)) return false;
        si.channels = v + 1;
        if (!mb_read(d, &v, 5)) return false;
        si.bits_per_sample = v + 1;
        if (!mb_read(d, &hi, 4) || !mb_read(d, &lo, 32)) return false;
        si.total_samples = ((uint64_t)hi << 32) | lo;
        for (int i = 0; i < 16; i++) {
            if (!mb_read(d, &v, 8)) return false;
            si.md5sum[i] = (uint8_t)v;
        }
        uint64_t end = d->bitpos_meta + (uint64_t)(uint32_t)(length - 34u) * 8;
        if (!need_bytes(d, end / 8)) return false;
        d->bitpos_meta = end;
        d->has_stream_info = true;
        /* an all-zero md5sum means "not computed": nothing to check against */
        bool zero = true;
        for (int i = 0; i < 16; i++) zero = zero && si.md5sum[i] == 0;
        if (zero) d->do_md5 = false;
        if (d->metadata_cb && !d->is_seeking) d->metadata_cb(d, &m, d->client);
    } else if (type == FLAC__METADATA_TYPE_SEEKTABLE) {
        /* read_metadata_seektable_: length / 18 points of (sample 64, offset 64, samples 16),
         * kept whatever the respond set (libFLAC's seek uses them; no callback here, as the
         * reference leaves metadata_respond at its STREAMINFO-only default) */
        const uint64_t end = d->bitpos_meta + (uint64_t)length * 8;
        d->seek_table.clear();
        for (uint32_t i = 0; i < length / 18u; i++) {
            uint32_t a, b, c, e, f;
            if (!mb_read(d, &a, 32) || !mb_read(d, &b, 32) || !mb_read(d, &c, 32) || !mb_read(d, &e, 32) ||
                !mb_read(d, &f, 16))
                return false;
            const uint64_t sample = ((uint64_t)a << 32) | b;
            if (sample == ~0ull) continue; /* FLAC__STREAM_METADATA_SEEKPOINT_PLACEHOLDER */
            d->seek_table.push_back({sample, ((uint64_t)c << 32) | e, f});
        }
        if (!need_bytes(d, end / 8)) return false;
        d->bitpos_meta = end;
    } else {
        uint64_t end = d->bitpos_meta + (uint64_t)length * 8;
        if (!need_bytes(d, end / 8)) return false;
        d->bitpos_meta = end;
    }
    if (last) {
        d->pos = d->bitpos_meta / 8;
        d->first_frame_offset = d->pos;
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    }
    return true;
}

bool byte_at(Dec *d, uint64_t p, uint32_t *x) {
    if (!need_bytes(d, p + 1)) return false;
    *x = bat(d, p);
    return true;
}

/* Drop consumed bytes once they pile up: everything below `keep` (the frame being decoded)
 * is no longer needed -- decoded windows live on the GPU and in info/pcm, and a seek
 * refills through the client's seek callback. */
void trim_consumed(Dec *d, uint64_t keep) {
    if (keep <= d->buf_base) return;
    const uint64_t drop = std::min<uint64_t>(keep - d->buf_base, d->buf.size());
    if (drop < (16ull << 20) || drop * 2 < d->buf.size()) return;
    d->buf.erase(d->buf.begin(), d->buf.begin() + (ptrdiff_t)drop);
    d->buf_base += drop;
}

/* frame_sync_ (@0x10011760) over the host buffer */
bool frame_sync(Dec *d) {
    bool first = true;
    uint64_t total = d->has_stream_info ? d->stream_info.data.stream_info.total_samples : 0;
    if (total > 0 && d->samples_decoded >= total) {
        d->state = FLAC__STREAM_DECODER_END_OF_STREAM;
        return true;
    }
    for (;;) {
        uint32_t x;
        if (d->cached) {
            x = d->lookahead;
            d->cached = false;
        } else {
            if (!byte_at(d, d->pos, &x)) return false;
            d->pos++;
        }
        if (x == 0xff) {
            d->header_warmup[0] = (uint8_t)x;
            if (!byte_at(d, d->pos, &x)) return false;
            d->pos++;
            if (x == 0xff) {
                d->lookahead = (uint8_t)x;
                d->cached = true;
            } else if (x >> 2 == 0x3e) {
                d->header_warmup[1] = (uint8_t)x;
                d->state = FLAC__STREAM_DECODER_READ_FRAME;
                return true;
            }
        }
        if (first) {
            send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_LOST_SYNC);
            first = false;
        }
    }
}

bool gpu_init(Dec *d) {
    if (d->gpu_ready) return true;
    const char *dev = getenv("BNFLAC_DEVICE");
    int cur = 0;
    if (!dev && hipGetDevice(&cur) != hipSuccess) cur = 0;
    d->device = dev ? atoi(dev) : cur; /* the caller's device (a torchrun rank's), unless overridden */
    if (bnflac_ctx_create(d->device, &d->ctx) != 0) return false;
    DevGuard g(d->device);
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) return fail("bnflac: stream create failed") == 0;
    d->gpu_ready = true;
    return true;
}

void gpu_free(Dec *d) {
    if (!d->gpu_ready) return;
    DevGuard g(d->device);
    d->d_bytes.release();
    d->d_cand.release();
    d->d_count.release();
    d->d_info.release();
    d->d_pcm.release();
    if (d->stream) (void)hipStreamDestroy(d->stream);
    d->stream = nullptr;
    bnflac_ctx_destroy(d->ctx);
    d->ctx = nullptr;
    d->gpu_ready = false;
}

/* Decode every candidate frame in buf[base, buf.size()) on the GPU. */
bool decode_window(Dec *d, uint64_t base) {
    if (!gpu_init(d)) {
        d->state = FLAC__STREAM_DECODER_MEMORY_ALLOCATION_ERROR;
        return false;
    }
    DevGuard g(d->device);
    const uint64_t n = bend(d) - base;
    const size_t padded = (size_t)((n + 3) & ~3ull) + 16;
    if (!d->d_bytes.grow(padded)) goto oom;
    if (hipMemsetAsync((uint8_t *)d->d_bytes.p + (n & ~3ull), 0, padded - (n & ~3ull), d->stream) != hipSuccess) goto hip_fail;
    if (hipMemcpyAsync(d->d_bytes.p, d->buf.data() + (base - d->buf_base), n, hipMemcpyHostToDevice, d->stream) != hipSuccess) goto hip_fail;
    {
        uint32_t cap = (uint32_t)std::min<uint64_t>(n / 2 + 16, 1u << 30);
        cap = std::min<uint32_t>(cap, (uint32_t)(n / 64 + 4096));
        for (int attempt = 0; attempt < 2; attempt++) {
            if (!d->d_cand.grow(sizeof(uint64_t) * cap) || !d->d_count.grow(16)) goto oom;
            if (bnflac_index_frames(d->ctx, (const uint8_t *)d->d_bytes.p, n, (uint64_t *)d->d_cand.p, cap,
                                    (uint32_t *)d->d_count.p, d->stream) != 0)
                goto hip_fail;
            uint32_t cnt = 0;
            if (hipMemcpyAsync(&cnt, d->d_count.p, 4, hipMemcpyDeviceToHost, d->stream) != hipSuccess) goto hip_fail;
            if (hipStreamSynchronize(d->stream) != hipSuccess) goto hip_fail;
            if (cnt <= cap) {
                cap = cnt;
                break;
            }
            cap = cnt;
        }
        const uint32_t ncand = cap;
        d->cand.resize(ncand);
        d->info.resize(ncand);
        if (ncand) {
            if (hipMemcpyAsync(d->cand.data(), d->d_cand.p, sizeof(uint64_t) * ncand, hipMemcpyDeviceToHost, d->stream) != hipSuccess)
                goto hip_fail;
            bnf_stream_params sp;
            memset(&sp, 0, sizeof sp);
            if (d->has_stream_info) {
                const FLAC__StreamMetadata_StreamInfo &si = d->stream_info.data.stream_info;
                sp.has_stream_info = 1;
                sp.min_blocksize = si.min_blocksize;
                sp.max_blocksize = si.max_blocksize;
                sp.sample_rate = si.sample_rate;
                sp.channels = si.channels;
                sp.bps = si.bits_per_sample;
                sp.total_samples = si.total_samples;
            }
            if (!d->d_info.grow(sizeof(bnf_frame_info) * ncand)) goto oom;
            if (bnf_launch_parse((const uint32_t *)d->d_bytes.p, n, (const uint64_t *)d->d_cand.p, ncand, sp,
                                 nullptr, 0, (bnf_frame_info *)d->d_info.p, nullptr, nullptr, nullptr, d->stream) != hipSuccess)
                goto hip_fail;
            if (hipMemcpyAsync(d->info.data(), d->d_info.p, sizeof(bnf_frame_info) * ncand, hipMemcpyDeviceToHost, d->stream) != hipSuccess)
                goto hip_fail;
            if (hipStreamSynchronize(d->stream) != hipSuccess) goto hip_fail;
            uint64_t tot = 0;
            uint32_t pcm_ch = 1; /* planar slots per sample: the window's widest frame */
            for (auto &fi : d->info) {
                fi.out_sample = tot;
                if (fi.status == BNF_ST_OK) {
                    tot += fi.blocksize;
                    pcm_ch = std::max(pcm_ch, std::min<uint32_t>(fi.channels, 8u));
                }
            }
            d->pcm_ch = pcm_ch;
            if (!d->d_pcm.grow(sizeof(int32_t) * (size_t)std::max<uint64_t>(tot, 1) * pcm_ch)) goto oom;
            if (hipMemcpyAsync(d->d_info.p, d->info.data(), sizeof(bnf_frame_info) * ncand, hipMemcpyHostToDevice, d->stream) != hipSuccess)
                goto hip_fail;
            bnf_stream_params spd = sp;
            spd.channels = pcm_ch;
            if (bnf_launch_decode((const uint32_t *)d->d_bytes.p, n, ncand, spd, lanes_for(pcm_ch), BNF_OUT_PLANAR32,
                                  (uint8_t *)d->d_pcm.p, (uint64_t)std::max<uint64_t>(tot, 1) * pcm_ch * 4,
                                  (bnf_frame_info *)d->d_info.p, nullptr, nullptr, d->stream) != hipSuccess)
                goto hip_fail;
            d->pcm.resize((size_t)tot * pcm_ch);
            if (tot && hipMemcpyAsync(d->pcm.data(), d->d_pcm.p, sizeof(int32_t) * (size_t)tot * pcm_ch, hipMemcpyDeviceToHost, d->stream) != hipSuccess)
                goto hip_fail;
            if (hipMemcpyAsync(d->info.data(), d->d_info.p, sizeof(bnf_frame_info) * ncand, hipMemcpyDeviceToHost, d->stream) != hipSuccess)
                goto hip_fail;
            if (hipStreamSynchronize(d->stream) != hipSuccess) goto hip_fail;
        }
    }
    d->win_base = base;
    d->win_end = bend(d);
    d->win_valid = true;
    d->read_ahead_cur = std::min(d->read_ahead, d->read_ahead_cur * 2);
    return true;
oom:
    fail("bnflac: out of device memory");
    d->state = FLAC__STREAM_DECODER_MEMORY_ALLOCATION_ERROR;
    return false;
hip_fail:
    fail(std::string("bnflac: HIP error in decode window: ") + hipGetErrorString(hipGetLastError()));
    d->state = FLAC__STREAM_DECODER_MEMORY_ALLOCATION_ERROR;
    return false;
}

const bnf_frame_info *lookup(Dec *d, uint64_t p) {
    if (!d->win_valid || p < d->win_base || p >= d->win_end) return nullptr;
    uint64_t rel = p - d->win_base;
    auto it = std::lower_bound(d->cand.begin(), d->cand.end(), rel);
    if (it == d->cand.end() || *it != rel) return nullptr;
    return &d->info[(size_t)(it - d->cand.begin())];
}

void allocate_output(Dec *d, unsigned size, unsigned ch) {
    if (size <= d->output_capacity && ch <= d->output_channels) return;
    for (unsigned i = 0; i < FLAC__MAX_CHANNELS; i++) d->output[i].clear();
    /* twice the capacity: a client that copies more than the frame (FLACFileReader copies
     * the first frame's blocksize from a trimmed seek frame, FLACFileReader.cs:287) reads
     * stale values instead of running off the allocation */
    for (unsigned i = 0; i < ch; i++) d->output[i].assign(2u * (size ? size : 1), 0);
    d->output_capacity = size;
    d->output_channels = ch;
}

/* read_frame_ (@0x100118c0) replay for the frame whose sync starts at d->pos - 2 */
bool read_frame(Dec *d, bool *got) {
    *got = false;
    const uint64_t p = d->pos - 2;
    const bnf_frame_info *fi = nullptr;
    for (int tries = 0;; tries++) {
        fi = lookup(d, p);
        if (fi && fi->status != BNF_ST_TRUNC) break;
        if (tries > 200) {
            fail("bnflac: frame window did not converge");
            d->state = FLAC__STREAM_DECODER_ABORTED;
            return false;
        }
        if (d->client_done) {
            /* no more bytes will come: a truncated frame makes libFLAC's reader fail here */
            if ((fi && fi->status == BNF_ST_TRUNC) ||
                (d->win_valid && d->win_base == p && d->win_end == bend(d))) {
                need_bytes(d, bend(d) + 1);
                return false;
            }
        } else {
            const uint64_t have = bend(d) > p ? bend(d) - p : 0;
            read_ahead(d, p + std::max<uint64_t>(d->read_ahead_cur, 2 * have + 4096));
        }
        if (!decode_window(d, p)) return false;
    }
    if (!fi) {
        d->state = FLAC__STREAM_DECODER_ABORTED;
        return false;
    }
    if (fi->status == BNF_ST_SKIPPED) {
        fail("bnflac: frame not decodable with the configured lanes");
        d->state = FLAC__STREAM_DECODER_ABORTED;
        return false;
    }
    const uint64_t abs_resume = d->win_base * 8 + fi->resume_bit;
    if (fi->status == BNF_ST_ERROR) {
        send_error(d, (FLAC__StreamDecoderErrorStatus)fi->err);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        d->pos = (abs_resume + 7) / 8;
        if (fi->cached >= 0) {
            d->cached = true;
            d->lookahead = (uint8_t)fi->cached;
        }
        return true;
    }
    /* header -> FLAC__Frame, frame/sample number conversion (@0x1001231f-0x100123ca) */
    FLAC__FrameHeader &h = d->frame.header;
    memset(&d->frame, 0, sizeof d->frame);
    h.blocksize = fi->blocksize;
    h.sample_rate = fi->sample_rate;
    h.channels = fi->channels;
    h.channel_assignment = (FLAC__ChannelAssignment)fi->assignment;
    h.bits_per_sample = fi->bps;
    h.crc = (FLAC__uint8)fi->crc8;
    d->next_fixed_block_size = 0;
    bool unparseable = false;
    if (fi->number_type == 0) {
        const uint32_t fn = (uint32_t)fi->number;
        h.number_type = FLAC__FRAME_NUMBER_TYPE_SAMPLE_NUMBER;
        if (d->fixed_block_size) {
            h.number.sample_number = (uint64_t)d->fixed_block_size * fn;
        } else if (d->has_stream_info) {
            const FLAC__StreamMetadata_StreamInfo &si = d->stream_info.data.stream_info;
            if (si.min_blocksize == si.max_blocksize) {
                h.number.sample_number = (uint64_t)si.min_blocksize * fn;
                d->next_fixed_block_size = si.max_blocksize;
            } else {
                unparseable = true;
            }
        } else if (fn == 0) {
            h.number.sample_number = 0;
            d->next_fixed_block_size = h.blocksize;
        } else {
            h.number.sample_number = (uint64_t)h.blocksize * fn;
        }
    } else {
        h.number_type = FLAC__FRAME_NUMBER_TYPE_SAMPLE_NUMBER;
        h.number.sample_number = fi->number;
    }
    if (unparseable) {
        send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_UNPARSEABLE_STREAM);
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        /* libFLAC stops right after the header's CRC-8 byte */
        d->pos = fi->frame_off + d->win_base + 2; /* conservative: resync just past the sync */
        return true;
    }
    d->frame.footer.crc = (FLAC__uint16)fi->crc16_read;
    allocate_output(d, h.blocksize, h.channels);
    const int32_t *src = d->pcm.data() + (size_t)fi->out_sample * d->pcm_ch;
    for (unsigned c = 0; c < h.channels; c++)
        memcpy(d->output[c].data(), src + (size_t)c * h.blocksize, sizeof(int32_t) * h.blocksize);
    if (!fi->crc_ok) send_error(d, FLAC__STREAM_DECODER_ERROR_STATUS_FRAME_CRC_MISMATCH); /* output already zeroed */
    *got = true;
    if (d->next_fixed_block_size) d->fixed_block_size = d->next_fixed_block_size;
    d->channels = h.channels;
    d->channel_assignment = h.channel_assignment;
    d->bits_per_sample = h.bits_per_sample;
    d->sample_rate = h.sample_rate;
    d->blocksize = h.blocksize;
    d->samples_decoded = h.number.sample_number + h.blocksize;
    d->pos = abs_resume / 8;
    trim_consumed(d, p);
    const FLAC__int32 *bufs[FLAC__MAX_CHANNELS];
    for (unsigned c = 0; c < FLAC__MAX_CHANNELS; c++) bufs[c] = c < d->output_channels ? d->output[c].data() : nullptr;
    if (d->is_seeking) {
        /* write_audio_frame_to_client_ while seeking: deliver only the frame holding the
         * target sample, trimmed so it starts there */
        const uint64_t sn = h.number.sample_number;
        if (d->seek_target >= sn && d->seek_target < sn + h.blocksize) {
            const unsigned delta = (unsigned)(d->seek_target - sn);
            FLAC__Frame fr = d->frame;
            fr.header.blocksize -= delta;
            fr.header.number.sample_number += delta;
            const FLAC__int32 *nb[FLAC__MAX_CHANNELS];
            for (unsigned c = 0; c < FLAC__MAX_CHANNELS; c++) nb[c] = bufs[c] ? bufs[c] + delta : nullptr;
            d->is_seeking = false;
            /* the callback runs in READ_FRAME, as libFLAC's; it may itself seek again */
            FLAC__StreamDecoderWriteStatus ws = d->write_cb(d, &fr, nb, d->client);
            if (ws != FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE && !d->ignore_write_status) {
                d->seek_done = -1;
                return false; /* state stays READ_FRAME */
            }
            d->seek_done = 1;
            d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
            return true;
        }
        d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
        return true;
    }
    /* write_audio_frame_to_client_: no STREAMINFO -> no sum to compare, stop hashing */
    if (!d->has_stream_info) d->do_md5 = false;
    if (d->do_md5) md5_accumulate(d->md5, bufs, h.channels, h.blocksize, 1, (h.bits_per_sample + 7) / 8);
    FLAC__StreamDecoderWriteStatus ws = d->write_cb(d, &d->frame, bufs, d->client);
    if (ws != FLAC__STREAM_DECODER_WRITE_STATUS_CONTINUE && !d->ignore_write_status) return false; /* state stays READ_FRAME */
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    return true;
}

void reset_fields(Dec *d) {
    d->buf.clear();
    d->buf_base = 0;
    d->pos = 0;
    d->bitpos_meta = 0;
    d->cached = false;
    d->client_done = 0;
    d->has_stream_info = false;
    d->seek_table.clear();
    d->samples_decoded = 0;
    d->fixed_block_size = d->next_fixed_block_size = 0;
    d->first_frame_offset = 0;
    d->win_valid = false;
    d->cand.clear();
    d->info.clear();
    d->pcm.clear();
    d->is_seeking = false;
    d->do_md5 = d->md5_checking;
    d->read_ahead_cur = std::min<uint64_t>(d->read_ahead, 256ull << 10);
    md5_init(d->md5);
}

/* Sample number of a decoded window frame (the header number conversion of read_frame). */
uint64_t frame_first_sample(const Dec *d, const bnf_frame_info &fi) {
    if (fi.number_type == 1) return fi.number;
    if (d->fixed_block_size) return (uint64_t)d->fixed_block_size * fi.number;
    if (d->has_stream_info) {
        const FLAC__StreamMetadata_StreamInfo &si = d->stream_info.data.stream_info;
        if (si.min_blocksize == si.max_blocksize) return (uint64_t)si.min_blocksize * fi.number;
    }
    return (uint64_t)fi.blocksize * fi.number;
}

/* Frame of the decoded window that holds `target` (intact frames only: header, CRC-16).
 * Returns 1 found (*off = its absolute offset), 0 the window's frames all lie before it
 * (lo_off/lo_s = the last one), -1 they all lie after it (hi_off/hi_s = the first one),
 * -2 the window has no intact frame. */
int window_find(const Dec *d, uint64_t target, uint64_t *off, uint64_t *lo_off, uint64_t *lo_s, uint64_t *hi_off,
                uint64_t *hi_s) {
    bool any = false;
    uint64_t f_off = 0, f_s = 0, l_off = 0, l_s = 0;
    for (size_t i = 0; i < d->info.size(); i++) {
        const bnf_frame_info &fi = d->info[i];
        if (fi.status != BNF_ST_OK || !fi.crc_ok) continue;
        const uint64_t sn = frame_first_sample(d, fi), o = d->win_base + d->cand[i];
        if (sn <= target && target < sn + fi.blocksize) {
            *off = o;
            return 1;
        }
        if (!any) { f_off = o; f_s = sn; }
        l_off = o;
        l_s = sn + fi.blocksize;
        any = true;
    }
    if (!any) return -2;
    if (target < f_s) { *hi_off = f_off; *hi_s = f_s; return -1; }
    *lo_off = l_off;
    *lo_s = l_s;
    return 0;
}

/* Reposition the client at `at` and decode one window from there. */
bool window_at(Dec *d, uint64_t at, uint64_t bytes) {
    if (d->seek_cb(d, at, d->client) != FLAC__STREAM_DECODER_SEEK_STATUS_OK) return false;
    d->buf.clear();
    d->buf_base = at;
    d->client_done = 0;
    d->win_valid = false;
    d->cached = false;
    read_ahead(d, at + bytes);
    if (bend(d) <= at) return false;
    return decode_window(d, at);
}

/* Byte offset of the frame holding `target`: the current window when it is there and its
 * bytes are still buffered; otherwise an interpolation search between known (offset,
 * sample) points, each probe one client seek + one GPU window (O(window) per probe,
 * O(log) probes), like libFLAC's seek_to_absolute_sample_ but over decoded windows. */
bool seek_search(Dec *d, uint64_t target, uint64_t length, uint64_t *start, bool use_table);

bool seek_position(Dec *d, uint64_t target, uint64_t length, uint64_t *start) {
    uint64_t off = 0, lo_off = d->first_frame_offset, lo_s = 0, hi_off = length, hi_s = 0;
    if (d->win_valid && window_find(d, target, &off, &lo_off, &lo_s, &hi_off, &hi_s) == 1 && off >= d->buf_base) {
        *start = off;
        return true;
    }
    /* a SEEKTABLE only narrows the search; one that misleads it (offsets past the stream,
     * points out of order) costs a second, table-free search, never different output */
    if (!d->seek_table.empty() && seek_search(d, target, length, start, true)) return true;
    return seek_search(d, target, length, start, false);
}

/* seek_to_absolute_sample_ over decoded windows; use_table: bracket the target between the
 * SEEKTABLE points around it (libFLAC's lower/upper bound from the table) */
bool seek_search(Dec *d, uint64_t target, uint64_t length, uint64_t *start, bool use_table) {
    uint64_t off = 0, lo_off, lo_s, hi_off, hi_s;
    const FLAC__uint64 total = FLAC__stream_decoder_get_total_samples(d);
    lo_off = d->first_frame_offset;
    lo_s = 0;
    hi_off = length;
    hi_s = total ? total : ~0ull;
    if (use_table) {
        for (const auto &p : d->seek_table) {
            if (p.frame_samples == 0 || (total && p.sample >= total)) continue;
            const uint64_t o = d->first_frame_offset + p.offset;
            if (p.offset > length || o >= length) continue;
            if (p.sample <= target && p.sample >= lo_s && o >= lo_off) {
                lo_s = p.sample;
                lo_off = o;
            } else if (p.sample > target && p.sample < hi_s && o < hi_off) {
                hi_s = p.sample;
                hi_off = o;
            }
        }
        if (hi_off <= lo_off) return false;
    }
    const uint32_t maxfs = d->has_stream_info ? d->stream_info.data.stream_info.max_framesize : 0;
    const uint64_t win = std::max<uint64_t>(1ull << 20, 4ull * (maxfs ? maxfs : 65536));
    for (int probe = 0; probe < 64; probe++) {
        if (hi_off <= lo_off) return false;
        uint64_t est = lo_off;
        if (hi_s != ~0ull && hi_s > lo_s && target > lo_s)
            est = lo_off + (uint64_t)((double)(target - lo_s) / (double)(hi_s - lo_s) * (double)(hi_off - lo_off));
        est = (est > lo_off + win / 2) ? est - win / 2 : lo_off; /* aim the window's middle at the target */
        if (!window_at(d, est, win)) return false;
        const int r = window_find(d, target, &off, &lo_off, &lo_s, &hi_off, &hi_s);
        if (r == 1) {
            *start = off;
            return true;
        }
        if (r == -2) { /* nothing intact here: shrink the range from above */
            if (est == lo_off) return false;
            hi_off = est;
        } else if (r == -1 && est <= lo_off) {
            return false; /* the first frame at/after the range start is already past the target */
        }
    }
    return false;
}

/* file callbacks (stream_decoder.c file_*_callback_) */
FLAC__StreamDecoderReadStatus file_read(const FLAC__StreamDecoder *dec, FLAC__byte buffer[], size_t *bytes, void *) {
    FILE *f = dec->file;
    if (*bytes > 0) {
        *bytes = fread(buffer, 1, *bytes, f);
        if (ferror(f)) return FLAC__STREAM_DECODER_READ_STATUS_ABORT;
        if (*bytes == 0) return FLAC__STREAM_DECODER_READ_STATUS_END_OF_STREAM;
        return FLAC__STREAM_DECODER_READ_STATUS_CONTINUE;
    }
    return FLAC__STREAM_DECODER_READ_STATUS_ABORT;
}
FLAC__StreamDecoderSeekStatus file_seek(const FLAC__StreamDecoder *dec, FLAC__uint64 off, void *) {
    return fseeko(dec->file, (off_t)off, SEEK_SET) < 0 ? FLAC__STREAM_DECODER_SEEK_STATUS_ERROR : FLAC__STREAM_DECODER_SEEK_STATUS_OK;
}
FLAC__StreamDecoderTellStatus file_tell(const FLAC__StreamDecoder *dec, FLAC__uint64 *off, void *) {
    off_t p = ftello(dec->file);
    if (p < 0) return FLAC__STREAM_DECODER_TELL_STATUS_ERROR;
    *off = (FLAC__uint64)p;
    return FLAC__STREAM_DECODER_TELL_STATUS_OK;
}
FLAC__StreamDecoderLengthStatus file_length(const FLAC__StreamDecoder *dec, FLAC__uint64 *len, void *) {
    struct stat st;
    if (fstat(fileno(dec->file), &st) != 0) return FLAC__STREAM_DECODER_LENGTH_STATUS_ERROR;
    *len = (FLAC__uint64)st.st_size;
    return FLAC__STREAM_DECODER_LENGTH_STATUS_OK;
}
FLAC__bool file_eof(const FLAC__StreamDecoder *dec, void *) { return feof(dec->file) ? 1 : 0; }

} // namespace

/* ---------------------------------------------------------------- exports */
extern "C" {

BNFLAC_API FLAC__StreamDecoder *FLAC__stream_decoder_new(void) {
    Dec *d = new (std::nothrow) Dec();
    if (!d) return nullptr;
    memset(&d->stream_info, 0, sizeof d->stream_info);
    memset(&d->frame, 0, sizeof d->frame);
    const char *ra = getenv("BNFLAC_READ_AHEAD_MB");
    if (ra) d->read_ahead = (uint64_t)std::max(1, atoi(ra)) << 20;
    return d;
}

static int init_common(Dec *d) {
    reset_fields(d);
    if (!gpu_init(d)) return FLAC__STREAM_DECODER_INIT_STATUS_MEMORY_ALLOCATION_ERROR;
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_METADATA;
    return FLAC__STREAM_DECODER_INIT_STATUS_OK;
}

BNFLAC_API int FLAC__stream_decoder_init_stream(FLAC__StreamDecoder *d, FLAC__StreamDecoderReadCallback read,
                                                FLAC__StreamDecoderSeekCallback seek, FLAC__StreamDecoderTellCallback tell,
                                                FLAC__StreamDecoderLengthCallback length, FLAC__StreamDecoderEofCallback eof,
                                                FLAC__StreamDecoderWriteCallback write,
                                                FLAC__StreamDecoderMetadataCallback metadata,
                                                FLAC__StreamDecoderErrorCallback error, void *client) {
    if (!d) return FLAC__STREAM_DECODER_INIT_STATUS_MEMORY_ALLOCATION_ERROR;
    if (d->state != FLAC__STREAM_DECODER_UNINITIALIZED) return FLAC__STREAM_DECODER_INIT_STATUS_ALREADY_INITIALIZED;
    if (!read || !write || !error || (seek && (!tell || !length || !eof)))
        return FLAC__STREAM_DECODER_INIT_STATUS_INVALID_CALLBACKS;
    d->read_cb = read; d->seek_cb = seek; d->tell_cb = tell; d->length_cb = length; d->eof_cb = eof;
    d->write_cb = write; d->metadata_cb = metadata; d->error_cb = error; d->client = client;
    d->ignore_write_status = false;
    return init_common(d);
}

BNFLAC_API int FLAC__stream_decoder_init_file(FLAC__StreamDecoder *d, const char *filename,
                                              FLAC__StreamDecoderWriteCallback write,
                                              FLAC__StreamDecoderMetadataCallback metadata,
                                              FLAC__StreamDecoderErrorCallback error, void *client) {
    if (!d) return FLAC__STREAM_DECODER_INIT_STATUS_MEMORY_ALLOCATION_ERROR;
    if (d->state != FLAC__STREAM_DECODER_UNINITIALIZED) return FLAC__STREAM_DECODER_INIT_STATUS_ALREADY_INITIALIZED;
    if (!write || !error) return FLAC__STREAM_DECODER_INIT_STATUS_INVALID_CALLBACKS;
    FILE *f = filename ? fopen(filename, "rb") : stdin;
    if (!f) return FLAC__STREAM_DECODER_INIT_STATUS_ERROR_OPENING_FILE;
    d->file = f;
    d->read_cb = file_read; d->seek_cb = file_seek; d->tell_cb = file_tell; d->length_cb = file_length; d->eof_cb = file_eof;
    d->write_cb = write; d->metadata_cb = metadata; d->error_cb = error; d->client = client;
    /* LibFLACSharp.cs:205-206 declares this write callback void: its return register is
     * garbage, so it is treated as CONTINUE (BNFLAC_STRICT_WRITE_STATUS=1 honours it). */
    const char *strict = getenv("BNFLAC_STRICT_WRITE_STATUS");
    d->ignore_write_status = !(strict && atoi(strict));
    int rc = init_common(d);
    if (rc != FLAC__STREAM_DECODER_INIT_STATUS_OK) {
        fclose(f);
        d->file = nullptr;
    }
    return rc;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_finish(FLAC__StreamDecoder *d) {
    if (!d) return 0;
    if (d->state == FLAC__STREAM_DECODER_UNINITIALIZED) return 1;
    if (d->file && d->file != stdin) fclose(d->file);
    d->file = nullptr;
    bool md5_failed = false;
    if (d->do_md5) {
        uint8_t sum[16];
        md5_final(d->md5, sum);
        md5_failed = memcmp(sum, d->stream_info.data.stream_info.md5sum, 16) != 0;
    }
    reset_fields(d);
    for (unsigned i = 0; i < FLAC__MAX_CHANNELS; i++) d->output[i].clear();
    d->output_capacity = d->output_channels = 0;
    d->md5_checking = false; /* set_defaults_ */
    d->state = FLAC__STREAM_DECODER_UNINITIALIZED;
    return md5_failed ? 0 : 1;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_set_md5_checking(FLAC__StreamDecoder *d, FLAC__bool value) {
    if (!d || d->state != FLAC__STREAM_DECODER_UNINITIALIZED) return 0;
    d->md5_checking = value != 0;
    return 1;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_get_md5_checking(const FLAC__StreamDecoder *d) {
    return (d && d->md5_checking) ? 1 : 0;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_delete(FLAC__StreamDecoder *d) {
    if (!d) return 1;
    FLAC__stream_decoder_finish(d);
    gpu_free(d);
    delete d;
    return 1;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_process_single(FLAC__StreamDecoder *d) {
    if (!d) return 0;
    bool got;
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
            if (!read_frame(d, &got)) return 0;
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

BNFLAC_API FLAC__bool FLAC__stream_decoder_process_until_end_of_metadata(FLAC__StreamDecoder *d) {
    if (!d) return 0;
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

BNFLAC_API FLAC__bool FLAC__stream_decoder_process_until_end_of_stream(FLAC__StreamDecoder *d) {
    if (!d) return 0;
    bool got;
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
            if (!read_frame(d, &got)) return 0;
            break;
        case FLAC__STREAM_DECODER_END_OF_STREAM:
        case FLAC__STREAM_DECODER_ABORTED:
            return 1;
        default:
            return 0;
        }
    }
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_seek_absolute(FLAC__StreamDecoder *d, FLAC__uint64 sample) {
    /* stream_decoder.c FLAC__stream_decoder_seek_absolute: states 0-4, a seek callback, the
     * target below STREAMINFO's total; is_seeking and MD5-off come BEFORE the metadata pass
     * (a seek before it suppresses the STREAMINFO callback), then the length callback. */
    if (!d) return 0;
    if (d->state > FLAC__STREAM_DECODER_END_OF_STREAM) return 0;
    if (!d->seek_cb) return 0;
    FLAC__uint64 total = FLAC__stream_decoder_get_total_samples(d);
    if (total > 0 && sample >= total) return 0;
    d->is_seeking = true;
    d->do_md5 = false; /* a seek turns MD5 checking off */
    FLAC__uint64 length = 0;
    if (d->length_cb(d, &length, d->client) != FLAC__STREAM_DECODER_LENGTH_STATUS_OK) {
        d->is_seeking = false;
        return 0;
    }
    if (d->state <= FLAC__STREAM_DECODER_READ_METADATA) {
        if (!FLAC__stream_decoder_process_until_end_of_metadata(d)) {
            d->is_seeking = false;
            return 0;
        }
        total = FLAC__stream_decoder_get_total_samples(d);
        if (total > 0 && sample >= total) {
            d->is_seeking = false;
            return 0;
        }
    }
    /* seek_to_absolute_sample_: find the frame holding `sample` (one decoded window when it
     * is already there, else an interpolation search over client seeks, each step one GPU
     * window), then decode from it: only that frame reaches the write callback, trimmed. */
    uint64_t start = 0;
    if (!seek_position(d, sample, length, &start)) {
        d->is_seeking = false;
        d->state = FLAC__STREAM_DECODER_SEEK_ERROR;
        return 0;
    }
    d->seek_target = sample;
    d->seek_done = 0;
    d->pos = start;
    d->cached = false;
    d->samples_decoded = 0;
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC;
    bool got;
    for (int guard = 0; guard < 100000000 && !d->seek_done; guard++) {
        if (d->state == FLAC__STREAM_DECODER_SEARCH_FOR_FRAME_SYNC) {
            if (!frame_sync(d)) break;
        } else if (d->state == FLAC__STREAM_DECODER_READ_FRAME) {
            if (!read_frame(d, &got)) break;
        } else {
            break;
        }
    }
    d->is_seeking = false;
    if (d->seek_done == 1) return 1;
    d->state = FLAC__STREAM_DECODER_SEEK_ERROR;
    return 0;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_get_decode_position(const FLAC__StreamDecoder *d, FLAC__uint64 *position) {
    if (!d || !d->tell_cb) return 0;
    if (d->tell_cb(d, position, d->client) != FLAC__STREAM_DECODER_TELL_STATUS_OK) return 0;
    const uint64_t unconsumed = bend(d) - std::min<uint64_t>(d->pos, bend(d));
    *position -= unconsumed;
    return 1;
}

BNFLAC_API FLAC__uint64 FLAC__stream_decoder_get_total_samples(const FLAC__StreamDecoder *d) {
    return (d && d->has_stream_info) ? d->stream_info.data.stream_info.total_samples : 0;
}
BNFLAC_API unsigned FLAC__stream_decoder_get_channels(const FLAC__StreamDecoder *d) { return d ? d->channels : 0; }
BNFLAC_API unsigned FLAC__stream_decoder_get_bits_per_sample(const FLAC__StreamDecoder *d) { return d ? d->bits_per_sample : 0; }
BNFLAC_API unsigned FLAC__stream_decoder_get_sample_rate(const FLAC__StreamDecoder *d) { return d ? d->sample_rate : 0; }
BNFLAC_API FLAC__StreamDecoderState FLAC__stream_decoder_get_state(const FLAC__StreamDecoder *d) {
    return d ? d->state : FLAC__STREAM_DECODER_UNINITIALIZED;
}

BNFLAC_API FLAC__bool FLAC__stream_decoder_reset(FLAC__StreamDecoder *d) {
    if (!d || d->state == FLAC__STREAM_DECODER_UNINITIALIZED) return 0;
    if (d->file == stdin) return 0;
    if (d->seek_cb && d->seek_cb(d, 0, d->client) == FLAC__STREAM_DECODER_SEEK_STATUS_ERROR) return 0;
    reset_fields(d);
    d->state = FLAC__STREAM_DECODER_SEARCH_FOR_METADATA;
    return 1;
}

} /* extern "C" */
