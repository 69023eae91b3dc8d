/*
 * bnflac_reader.cpp -- streaming PCM reader over a whole FLAC stream.
 *
 * The fast path under FLACDecoder.Read (FLACDecoder.cs:124-205) and the OpenAL buffer
 * fill (OpenALDemo/Program.cs:33-38, StreamingPlayer.cs:424-464): the caller asks for
 * `count` bytes of packed PCM at a time (4 x 16 KiB for OpenAL) and gets exactly the byte
 * sequence FLACDecoder.CopyTo would produce.
 *
 * On open the compressed stream goes to HBM once, bnflac_index_stream finds its frames and
 * one bnflac_decode_parsed launch decodes all of them (a stream is far too small to fill the
 * chip, so one launch costs what one window would).  The PCM then comes back in windows of
 * frames: window w+1 is copied into one slot of a pinned host ring while the caller drains
 * window w from the other.  Reads are memcpy from pinned memory; the D2H copies overlap
 * them.  Device buffers, pinned slots, the stream and its events are kept in a per-device
 * pool when a reader closes and reused by the next open (allocation dominated open/close).  A stream that is not intact (the frame chain ends before STREAMINFO's total, a
 * frame fails its CRC, or a frame needs the libFLAC error path) is refused at the point
 * it is reached, with bnflac_reader_last_error() saying why: the libFLAC stream API is the path
 * for damaged streams.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../../include/bnflac.h"

namespace {

thread_local std::string g_rerr;

/* run on the reader's device, restore the caller's on scope exit */
struct RDevGuard {
    int prev = -1;
    explicit RDevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~RDevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};
int rfail(const std::string &m) {
    g_rerr = m;
    return -1;
}

/* STREAMINFO and the first frame offset from the metadata blocks (read_metadata_) */
/* BNFLAC_READER_TRACE=1: open's phases to stderr (device-synchronised; development only) */
struct OpenTrace {
    bool on = getenv("BNFLAC_READER_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char *what, hipStream_t s) {
        if (!on) return;
        if (s) (void)hipStreamSynchronize(s);
        const auto n = std::chrono::steady_clock::now();
        fprintf(stderr, "reader_open %-14s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

bool parse_metadata(const uint8_t *d, uint64_t n, bnflac_stream_params &sp, uint64_t &first) {
    if (n < 8 || memcmp(d, "fLaC", 4) != 0) return false;
    uint64_t p = 4;
    bool have = false;
    for (;;) {
        if (p + 4 > n) return false;
        const uint32_t hdr = d[p], len = ((uint32_t)d[p + 1] << 16) | ((uint32_t)d[p + 2] << 8) | d[p + 3];
        if ((hdr & 0x7F) == 0 && len >= 34 && p + 4 + 34 <= n) {
            const uint8_t *s = d + p + 4;
            sp.has_stream_info = 1;
            sp.min_blocksize = ((uint32_t)s[0] << 8) | s[1];
            sp.max_blocksize = ((uint32_t)s[2] << 8) | s[3];
            uint64_t x = 0;
            for (int i = 10; i < 18; i++) x = (x << 8) | s[i];
            sp.sample_rate = (uint32_t)(x >> 44);
            sp.channels = (uint32_t)((x >> 41) & 7) + 1;
            sp.bps = (uint32_t)((x >> 36) & 31) + 1;
            sp.total_samples = x & ((1ull << 36) - 1);
            have = true;
        }
        p += 4 + (uint64_t)len;
        if (hdr & 0x80) break;
    }
    first = p;
    return have && p <= n;
}

/* A frame header at byte p that read_frame_header_ would accept (sync, codes, UTF-8
 * number, CRC-8; FLAC format / LibFlac.dll@0x10011d70); its coded number in *num. */
bool header_ok(const uint8_t *d, uint64_t n, uint64_t p, uint64_t *num, uint32_t *is_sample) {
    if (p + 6 > n || d[p] != 0xFF || (d[p + 1] >> 1) != 0x7C) return false;
    const uint32_t b2 = d[p + 2], b3 = d[p + 3];
    if ((b2 >> 4) == 0 || (b2 & 15) == 15 || (b3 >> 4) >= 11 || ((b3 >> 1) & 7) == 3 || ((b3 >> 1) & 7) == 7 || (b3 & 1))
        return false;
    uint64_t q = p + 4, v = d[q];
    int extra;
    if (!(v & 0x80)) extra = 0;
    else if ((v & 0xE0) == 0xC0) { extra = 1; v &= 0x1F; }
    else if ((v & 0xF0) == 0xE0) { extra = 2; v &= 0x0F; }
    else if ((v & 0xF8) == 0xF0) { extra = 3; v &= 0x07; }
    else if ((v & 0xFC) == 0xF8) { extra = 4; v &= 0x03; }
    else if ((v & 0xFE) == 0xFC) { extra = 5; v &= 0x01; }
    else if (v == 0xFE) { extra = 6; v = 0; }
    else return false;
    q++;
    for (int i = 0; i < extra; i++, q++) {
        if (q >= n || (d[q] & 0xC0) != 0x80) return false;
        v = (v << 6) | (d[q] & 0x3F);
    }
    if ((b2 >> 4) == 6) q += 1;
    else if ((b2 >> 4) == 7) q += 2;
    if ((b2 & 15) == 12) q += 1;
    else if ((b2 & 15) == 13 || (b2 & 15) == 14) q += 2;
    if (q >= n) return false;
    uint8_t c = 0; /* CRC-8, poly 0x07 */
    for (uint64_t i = p; i < q; i++) {
        c ^= d[i];
        for (int b = 0; b < 8; b++) c = (uint8_t)((c & 0x80) ? (c << 1) ^ 0x07 : (c << 1));
    }
    if (c != d[q]) return false;
    *num = v;
    *is_sample = d[p + 1] & 1;
    return true;
}

} // namespace

struct bnflac_reader {
    bnflac_ctx *ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    /* allocation sizes of the pooled buffers below (device: bytes, offs, os, info, out, n) */
    size_t cap_bytes = 0, cap_offs = 0, cap_os = 0, cap_info = 0, cap_out = 0, cap_ring = 0, cap_hinfo = 0;
    bnflac_frame_info *h_info = nullptr; /* pinned: every frame's record after the decode */
    bnflac_stream_params sp{};
    int fmt = BNFLAC_OUT_FLACDECODER;
    uint32_t stride = 0;
    uint64_t nbytes = 0;
    void *d_bytes = nullptr, *d_offs = nullptr, *d_os = nullptr, *d_info = nullptr, *d_out = nullptr, *d_n = nullptr;
    uint32_t nframes = 0;
    std::vector<uint64_t> os; /* out_sample per frame, + end */
    uint32_t window = 256;    /* frames per window */
    uint32_t nwin = 0;
    /* pinned ring: two slots, each one window of PCM */
    uint8_t *ring[2] = {nullptr, nullptr};
    size_t slot_bytes = 0;
    hipEvent_t done[2] = {nullptr, nullptr};
    uint32_t slot_win[2] = {~0u, ~0u}; /* window held (or in flight) in each slot */
    uint32_t cur = 0;                  /* window being read */
    uint64_t cur_pos = 0;              /* bytes of it already returned */
    uint64_t total_bytes = 0, returned = 0;
    bool failed = false;
    /* FLACFileReader compat mode (bnflac_reader_read_filereader): the C# reader's state */
    int mode = 0;                 /* 0 unused, 1 byte reads (bnflac_reader_read), 2 FLACFileReader reads */
    uint32_t fr_next = 0;         /* next frame "ProcessSingle" decodes */
    bool fr_landed = false;       /* window r->cur has landed (compat mode) */
    uint32_t spc = 0;             /* m_samplesPerChannel: the first frame's blocksize */
    uint32_t fr_idx = 0;          /* m_flacSampleIndex */
    std::vector<uint8_t> image;   /* m_flacSamples, packed: spc sample frames x channels x bytes */
    bool eos = false;             /* decoder state reached EndOfStream */
};

namespace {

uint64_t win_bytes(const bnflac_reader *r, uint32_t w) {
    const uint32_t f0 = w * r->window, f1 = std::min(r->nframes, f0 + r->window);
    return (r->os[f1] - r->os[f0]) * r->stride;
}

/* copy window w's PCM into its slot; asynchronous on r->stream (the decode of every frame
 * was queued on it at open) */
int issue_window(bnflac_reader *r, uint32_t w) {
    if (w >= r->nwin) return 0;
    const uint32_t slot = w & 1u;
    const uint32_t f0 = w * r->window;
    const uint64_t b0 = r->os[f0] * r->stride, nb = win_bytes(r, w);
    if (nb && hipMemcpyAsync(r->ring[slot], (const uint8_t *)r->d_out + b0, nb, hipMemcpyDeviceToHost, r->stream) != hipSuccess)
        return rfail("bnflac_reader: D2H copy failed");
    if (hipEventRecord(r->done[slot], r->stream) != hipSuccess) return rfail("bnflac_reader: event record failed");
    r->slot_win[slot] = w;
    return 0;
}

/* wait for window w and check every frame of it decoded cleanly */
int land_window(bnflac_reader *r, uint32_t w) {
    const uint32_t slot = w & 1u;
    if (r->slot_win[slot] != w) return rfail("bnflac_reader: window not issued");
    if (hipEventSynchronize(r->done[slot]) != hipSuccess) return rfail("bnflac_reader: HIP error while decoding");
    const uint32_t f0 = w * r->window, f1 = std::min(r->nframes, f0 + r->window);
    for (uint32_t i = f0; i < f1; i++) {
        const bnflac_frame_info &fi = r->h_info[i];
        if (fi.status == 3 && (fi.flags & 4u))
            return rfail("bnflac_reader: frame at byte " + std::to_string(fi.frame_off) +
                         " cannot be carried by this output layout");
        if (fi.status != 0 || !fi.crc_ok)
            return rfail("bnflac_reader: frame at byte " + std::to_string(fi.frame_off) +
                         " is damaged (use the libFLAC stream API for damaged streams)");
    }
    return 0;
}

/* per-device pool of one reader's resources (a closed reader's, for the next open) */
std::mutex g_pool_mu;
std::vector<bnflac_reader *> g_pool;

void free_resources(bnflac_reader *r) {
    for (void *p : {r->d_bytes, r->d_offs, r->d_os, r->d_info, r->d_out, r->d_n})
        if (p) (void)hipFree(p);
    for (int i = 0; i < 2; i++) {
        if (r->ring[i]) (void)hipHostFree(r->ring[i]);
        if (r->done[i]) (void)hipEventDestroy(r->done[i]);
    }
    if (r->h_info) (void)hipHostFree(r->h_info);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->ctx) bnflac_ctx_destroy(r->ctx);
}

/* a reader for `device`, with the pooled resources of an earlier one when there are any */
bnflac_reader *take_reader(int device) {
    bnflac_reader *r = new bnflac_reader();
    r->device = device;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); i++) {
        bnflac_reader *p = g_pool[i];
        if (p->device != device) continue;
        g_pool.erase(g_pool.begin() + (long)i);
        r->ctx = p->ctx;
        r->stream = p->stream;
        r->d_bytes = p->d_bytes; r->cap_bytes = p->cap_bytes;
        r->d_offs = p->d_offs; r->cap_offs = p->cap_offs;
        r->d_os = p->d_os; r->cap_os = p->cap_os;
        r->d_info = p->d_info; r->cap_info = p->cap_info;
        r->d_out = p->d_out; r->cap_out = p->cap_out;
        r->d_n = p->d_n;
        r->ring[0] = p->ring[0]; r->ring[1] = p->ring[1]; r->cap_ring = p->cap_ring;
        r->done[0] = p->done[0]; r->done[1] = p->done[1];
        r->h_info = p->h_info; r->cap_hinfo = p->cap_hinfo;
        delete p;
        break;
    }
    return r;
}

bool dgrow(void *&p, size_t &cap, size_t n) { /* device buffer of at least n bytes */
    if (p && cap >= n) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) return false;
    cap = n;
    return true;
}
template <typename T> bool hgrow(T *&p, size_t &cap, size_t n) { /* pinned host buffer */
    if (p && cap >= n) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    if (hipHostMalloc((void **)&p, n, hipHostMallocDefault) != hipSuccess) return false;
    cap = n;
    return true;
}

/* Pool policy.  Only what open/close churn costs is worth keeping: the stream, events, ctx,
 * index scratch and small buffers.  Buffers sized by the stream (the compressed copy, the PCM,
 * the pinned ring slots and records) are kept only up to BNFLAC_READER_POOL_CAP bytes each
 * (default 64 MiB), so a closed reader never pins a large stream's HBM or host memory for the
 * life of the process; BNFLAC_READER_POOL=0 disables pooling; bnflac_reader_pool_release()
 * frees everything pooled. */
size_t pool_cap() {
    static const size_t c = [] {
        const char *e = getenv("BNFLAC_READER_POOL_CAP");
        return e ? (size_t)strtoull(e, nullptr, 0) : (size_t)64 << 20;
    }();
    return c;
}
bool pool_on() {
    static const bool on = [] {
        const char *e = getenv("BNFLAC_READER_POOL");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
void trim_for_pool(bnflac_reader *p) {
    const size_t cap = pool_cap();
    auto dtrim = [&](void *&b, size_t &c) {
        if (b && c > cap) { (void)hipFree(b); b = nullptr; c = 0; }
    };
    dtrim(p->d_bytes, p->cap_bytes);
    dtrim(p->d_out, p->cap_out);
    dtrim(p->d_offs, p->cap_offs);
    dtrim(p->d_os, p->cap_os);
    dtrim(p->d_info, p->cap_info);
    if (p->cap_ring > cap) {
        for (int i = 0; i < 2; i++)
            if (p->ring[i]) { (void)hipHostFree(p->ring[i]); p->ring[i] = nullptr; }
        p->cap_ring = 0;
    }
    if (p->h_info && p->cap_hinfo > cap) { (void)hipHostFree(p->h_info); p->h_info = nullptr; p->cap_hinfo = 0; }
}

/* close: the resources go back to the pool (one set per device) unless the reader failed
 * in a way that may have left the stream in error */
void release(bnflac_reader *r, bool keep = true) {
    bool ok = !r->stream || hipStreamSynchronize(r->stream) == hipSuccess;
    if (keep && ok && pool_on() && r->ctx && r->stream && r->done[0] && r->done[1]) {
        trim_for_pool(r);
        std::lock_guard<std::mutex> lk(g_pool_mu);
        bool have = false;
        for (bnflac_reader *p : g_pool) have = have || p->device == r->device;
        if (!have) {
            bnflac_reader *p = new bnflac_reader();
            *p = std::move(*r);
            g_pool.push_back(p);
            delete r;
            return;
        }
    }
    free_resources(r);
    delete r;
}

} // namespace

extern "C" {

BNFLAC_API const char *bnflac_reader_last_error(void) { return g_rerr.c_str(); }

BNFLAC_API int bnflac_reader_open(int device, const uint8_t *bytes, uint64_t nbytes, int out_format,
                                  uint32_t window_frames, bnflac_reader **out) {
    if (!out) return rfail("bnflac_reader_open: null out");
    *out = nullptr;
    if (!bytes) return rfail("bnflac_reader_open: null bytes");
    if (out_format < 0 || out_format > 3) return rfail("bnflac_reader_open: bad out_format");
    if (device < 0 || device >= bnflac_device_count()) return rfail("bnflac_reader_open: bad device index");
    RDevGuard dg(device);
    OpenTrace tr;
    bnflac_stream_params sp{};
    uint64_t first = 0;
    if (!parse_metadata(bytes, nbytes, sp, first))
        return rfail("bnflac_reader_open: no fLaC marker / STREAMINFO (use the libFLAC stream API)");
    if (sp.channels < 1 || sp.channels > 8) return rfail("bnflac_reader_open: bad channel count");
    if (out_format == BNFLAC_OUT_FLACDECODER && sp.bps != 16) /* FLACDecoder.cs:526-529 aborts on these */
        return rfail("bnflac_reader_open: FLACDecoder layout needs 16-bit samples, stream has " + std::to_string(sp.bps));
    bnflac_reader *r = take_reader(device);
    r->sp = sp;
    r->fmt = out_format;
    if (window_frames) r->window = window_frames;
    if (!r->ctx && bnflac_ctx_create(device, &r->ctx)) {
        const std::string e = bnflac_last_error();
        r->ctx = nullptr;
        release(r, false);
        return rfail("bnflac_reader_open: " + e);
    }
    r->stride = bnflac_out_stride(out_format, &r->sp);
    r->nbytes = nbytes;
    const size_t padded = (size_t)((nbytes + 15) & ~15ull) + 16;
    /* Frame records.  A frame is >= 9 bytes, so nbytes / 8 bounds the chain, but at 128 B a
     * record that bound is 16x the stream (171 MB for a 10.7 MB C2 stream): past the pool cap,
     * so every open allocated it and every close paid a 0.2 ms hipFree.  STREAMINFO's total
     * and minimum blocksize give the usual count (frames past the total are dropped by the
     * index); a chain longer than that re-indexes at the full bound below. */
    const uint32_t cap_full = (uint32_t)std::min<uint64_t>(nbytes / 8 + 16, 1u << 30);
    uint32_t cap = cap_full;
    if (r->sp.total_samples && r->sp.min_blocksize >= 16)
        cap = (uint32_t)std::min<uint64_t>(cap_full, r->sp.total_samples / r->sp.min_blocksize + 16);
    size_t cap_n = 16;
    if ((!r->stream && hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) ||
        !dgrow(r->d_bytes, r->cap_bytes, padded) || !dgrow(r->d_offs, r->cap_offs, 8ull * cap) ||
        !dgrow(r->d_os, r->cap_os, 8ull * cap) || !dgrow(r->d_info, r->cap_info, sizeof(bnflac_frame_info) * cap) ||
        (!r->d_n && !dgrow(r->d_n, cap_n, 16)) ||
        (!r->done[0] && hipEventCreateWithFlags(&r->done[0], hipEventDisableTiming) != hipSuccess) ||
        (!r->done[1] && hipEventCreateWithFlags(&r->done[1], hipEventDisableTiming) != hipSuccess)) {
        release(r, false);
        return rfail("bnflac_reader_open: out of device memory");
    }
    tr.mark("ctx+alloc", r->stream);
    /* one H2D of the whole stream; the tail padding is zero */
    if (hipMemsetAsync((uint8_t *)r->d_bytes + (nbytes & ~15ull), 0, padded - (nbytes & ~15ull), r->stream) != hipSuccess ||
        hipMemcpyAsync(r->d_bytes, bytes, nbytes, hipMemcpyHostToDevice, r->stream) != hipSuccess) {
        release(r, false);
        return rfail("bnflac_reader_open: H2D copy failed");
    }
    tr.mark("h2d", r->stream);
    uint32_t nf = 0;
    for (;;) {
        if (bnflac_index_stream(r->ctx, (const uint8_t *)r->d_bytes, nbytes, first, &r->sp, (uint64_t *)r->d_offs,
                                (uint64_t *)r->d_os, (bnflac_frame_info *)r->d_info, cap, (uint32_t *)r->d_n,
                                r->stream)) {
            const std::string e = bnflac_last_error();
            release(r, false);
            return rfail("bnflac_reader_open: " + e);
        }
        if (hipMemcpyAsync(&nf, r->d_n, 4, hipMemcpyDeviceToHost, r->stream) != hipSuccess ||
            hipStreamSynchronize(r->stream) != hipSuccess || (nf > cap && cap == cap_full)) {
            release(r, false);
            return rfail("bnflac_reader_open: frame index failed");
        }
        if (nf <= cap) break;
        /* more frames than STREAMINFO implies: index again with room for any chain */
        cap = cap_full;
        if (!dgrow(r->d_offs, r->cap_offs, 8ull * cap) || !dgrow(r->d_os, r->cap_os, 8ull * cap) ||
            !dgrow(r->d_info, r->cap_info, sizeof(bnflac_frame_info) * cap)) {
            release(r, false);
            return rfail("bnflac_reader_open: out of device memory");
        }
    }
    tr.mark("index", r->stream);
    r->nframes = nf;
    r->os.resize((size_t)nf + 1);
    /* the running sample counts, and the last frame's record (its blocksize ends the stream) */
    bnflac_frame_info last{};
    uint64_t last_off = 0;
    if (nf && (hipMemcpy(r->os.data(), r->d_os, 8ull * nf, hipMemcpyDeviceToHost) != hipSuccess ||
               hipMemcpy(&last, (bnflac_frame_info *)r->d_info + (nf - 1), sizeof last, hipMemcpyDeviceToHost) != hipSuccess ||
               hipMemcpy(&last_off, (uint64_t *)r->d_offs + (nf - 1), 8, hipMemcpyDeviceToHost) != hipSuccess)) {
        release(r, false);
        return rfail("bnflac_reader_open: D2H copy failed");
    }
    const uint64_t end = nf ? r->os[nf - 1] + last.blocksize : 0;
    r->os[nf] = end;
    if (r->sp.total_samples && end != r->sp.total_samples) {
        release(r);
        return rfail("bnflac_reader_open: the frame chain covers " + std::to_string(end) + " of " +
                     std::to_string(r->sp.total_samples) + " samples (damaged stream: use the libFLAC stream API)");
    }
    tr.mark("index-readback", r->stream);
    r->total_bytes = end * r->stride;
    r->nwin = (nf + r->window - 1) / r->window;
    size_t slot_bytes = 16;
    for (uint32_t w = 0; w < r->nwin; w++) slot_bytes = std::max<size_t>(slot_bytes, win_bytes(r, w));
    size_t c0 = r->cap_ring, c1 = r->cap_ring; /* the two slots are sized together */
    if (!dgrow(r->d_out, r->cap_out, std::max<uint64_t>(r->total_bytes, 16)) || !hgrow(r->ring[0], c0, slot_bytes) ||
        !hgrow(r->ring[1], c1, slot_bytes) ||
        !hgrow(r->h_info, r->cap_hinfo, sizeof(bnflac_frame_info) * std::max(nf, 1u))) {
        r->cap_ring = std::min(c0, c1);
        release(r, false);
        return rfail("bnflac_reader_open: out of memory");
    }
    r->cap_ring = std::min(c0, c1);
    tr.mark("alloc-out", r->stream);
    /* every frame in one decode launch, the records back to pinned memory, then the first
     * two windows of PCM */
    if (nf && (bnflac_decode_parsed(r->ctx, (const uint8_t *)r->d_bytes, r->nbytes, nf, &r->sp, r->fmt,
                                    (uint8_t *)r->d_out, r->total_bytes, (bnflac_frame_info *)r->d_info, r->stream) ||
               hipMemcpyAsync(r->h_info, r->d_info, sizeof(bnflac_frame_info) * nf, hipMemcpyDeviceToHost, r->stream) !=
                   hipSuccess)) {
        const std::string e = bnflac_last_error();
        release(r, false);
        return rfail("bnflac_reader_open: " + e);
    }
    if (!r->sp.total_samples && nf) {
        /* length unknown (STREAMINFO total 0): a damaged frame would end the chain early with
         * every chained frame intact.  Refuse when an acceptable header numbered past the
         * chain's last frame follows it (trailing tags and metadata are allowed).  The scan
         * starts where the last frame ends (its decoded record's resume bit: after the CRC-16
         * footer), so a header-like byte pattern inside that frame's own payload is never taken
         * for a following frame; this needs the decode, so these streams sync once here. */
        if (hipStreamSynchronize(r->stream) != hipSuccess) {
            release(r, false);
            return rfail("bnflac_reader_open: HIP error while decoding");
        }
        const bnflac_frame_info &lf = r->h_info[nf - 1];
        const uint64_t scan0 = (lf.status == 0 && lf.resume_bit / 8 > last_off) ? lf.resume_bit / 8 : last_off + 2;
        const uint64_t last_no = last.number_type ? r->os[nf - 1] : last.number;
        for (uint64_t p = scan0; p + 1 < nbytes; p++) {
            uint64_t no = 0;
            uint32_t is_sample = 0;
            if (bytes[p] != 0xFF || !header_ok(bytes, nbytes, p, &no, &is_sample)) continue;
            const uint64_t room = (nbytes - p) / 16 + 1; /* frames that could still follow */
            const bool plausible = is_sample ? (no >= end && no <= end + room * 65536ull)
                                             : (no > last_no && no <= last_no + 1 + room);
            if (plausible) {
                release(r);
                return rfail("bnflac_reader_open: the frame chain ends at byte " + std::to_string(last_off) +
                             " but a frame header follows at byte " + std::to_string(p) +
                             " (damaged stream: use the libFLAC stream API)");
            }
        }
    }
    if (issue_window(r, 0) || issue_window(r, 1)) {
        release(r, false);
        return -1;
    }
    tr.mark("decode+windows", r->stream);
    *out = r;
    return 0;
}

BNFLAC_API int bnflac_reader_params(const bnflac_reader *r, bnflac_stream_params *sp, uint64_t *total_bytes,
                                    uint32_t *nframes) {
    if (!r) return rfail("bnflac_reader_params: null reader");
    if (sp) *sp = r->sp;
    if (total_bytes) *total_bytes = r->total_bytes;
    if (nframes) *nframes = r->nframes;
    return 0;
}

BNFLAC_API int64_t bnflac_reader_read(bnflac_reader *r, uint8_t *buf, uint64_t count) {
    if (!r) return rfail("bnflac_reader_read: null reader");
    RDevGuard dg(r->device);
    if (r->failed) return rfail("bnflac_reader_read: reader failed earlier");
    if (r->mode == 2) return rfail("bnflac_reader_read: this reader is in FLACFileReader mode");
    r->mode = 1;
    if (!buf && count) return rfail("bnflac_reader_read: null buffer");
    uint64_t done = 0;
    while (done < count && r->cur < r->nwin) {
        const uint32_t w = r->cur, slot = w & 1u;
        if (r->cur_pos == 0 && land_window(r, w)) {
            r->failed = true;
            return -1;
        }
        const uint64_t wb = win_bytes(r, w), take = std::min<uint64_t>(count - done, wb - r->cur_pos);
        memcpy(buf + done, r->ring[slot] + r->cur_pos, take);
        done += take;
        r->cur_pos += take;
        if (r->cur_pos == wb) { /* window drained: its slot takes the window after the next */
            r->cur++;
            r->cur_pos = 0;
            if (issue_window(r, w + 2)) {
                r->failed = true;
                return -1;
            }
        }
    }
    r->returned += done;
    return (int64_t)done;
}

/* ---- FLACFileReader compat mode: FLACFileReader.Read(buffer, offset, numBytes) replayed over
 * the decoded frames (FLACFileReader.cs:145-174, 208-254, 267-301). */

/* ProcessSingle: the next frame's packed bytes (FILEREADER layout, bs sample frames) */
int fr_next_frame(bnflac_reader *r, const uint8_t **bytes, uint32_t *bs) {
    if (r->fr_next >= r->nframes) return 0;
    const uint32_t f = r->fr_next, w = f / r->window;
    while (r->cur < w) { /* the window before is done: its slot takes the window after the next */
        if (issue_window(r, r->cur + 2)) return -1;
        r->cur++;
        r->fr_landed = false;
    }
    if (!r->fr_landed) {
        if (land_window(r, w)) return -1;
        r->fr_landed = true;
    }
    const uint64_t f0 = (uint64_t)w * r->window;
    *bytes = r->ring[w & 1u] + (r->os[f] - r->os[f0]) * r->stride;
    *bs = (uint32_t)(r->os[f + 1] - r->os[f]);
    r->fr_next++;
    return 1;
}

/* FLAC_WriteCallback: the first frame fixes m_samplesPerChannel; every frame overwrites the
 * first min(bs, spc) samples of m_flacSamples (libFLAC's buffers keep the rest: a short
 * frame leaves the previous frames' samples behind, a long one is truncated) */
void fr_write(bnflac_reader *r, const uint8_t *bytes, uint32_t bs) {
    const uint32_t sf = r->stride; /* bytes per sample frame: channels x (2 | 3) */
    if (!r->spc) {
        r->spc = bs;
        r->image.assign((size_t)bs * sf, 0);
        r->fr_idx = 0;
    }
    memcpy(r->image.data(), bytes, (size_t)std::min(bs, r->spc) * sf);
}

/* CopyFlacBufferToNAudioBuffer: sample-major, channel-minor, until the buffer's LENGTH
 * (not offset + numBytes); returns bytes copied or -1 (IndexOutOfRange: a sample that does
 * not fit, after its leading bytes were written, as the C# byte loop does) */
int64_t fr_copy(bnflac_reader *r, uint8_t *buf, uint64_t len, uint64_t &noff) {
    const uint64_t start = noff;
    const uint32_t C = r->sp.channels, fb = r->sp.bps == 24 ? 3u : 2u;
    bool full = noff >= len;
    for (; r->fr_idx < r->spc && !full; r->fr_idx++) {
        for (uint32_t ch = 0; ch < C && !full; ch++) {
            const uint8_t *smp = r->image.data() + ((size_t)r->fr_idx * C + ch) * fb;
            for (uint32_t k = 0; k < fb; k++) {
                if (noff >= len) return -1;
                buf[noff++] = smp[k];
            }
            full = noff >= len;
        }
    }
    if (r->fr_idx >= r->spc) r->fr_idx = 0;
    return (int64_t)(noff - start);
}

/* FLACFileReader.Position / seek_absolute (FLACFileReader.cs:109-137,295-299): the next read
 * starts at sample `sample` (per channel).  The frame holding it is found in the index
 * (binary search over the running sample counts); its window and the next are copied
 * again and the reader resumes inside the first. */
BNFLAC_API int bnflac_reader_seek(bnflac_reader *r, uint64_t sample) {
    if (!r) return rfail("bnflac_reader_seek: null reader");
    RDevGuard dg(r->device);
    if (r->mode == 2) return rfail("bnflac_reader_seek: not available in FLACFileReader mode");
    if (r->failed) return rfail("bnflac_reader_seek: reader failed earlier");
    const uint64_t total = r->os[r->nframes];
    if (sample >= total) return rfail("bnflac_reader_seek: sample past the end of the stream");
    if (hipStreamSynchronize(r->stream) != hipSuccess) return rfail("bnflac_reader_seek: HIP error");
    const uint32_t f = (uint32_t)(std::upper_bound(r->os.begin(), r->os.begin() + r->nframes, sample) - r->os.begin()) - 1u;
    const uint32_t w = f / r->window;
    r->slot_win[0] = r->slot_win[1] = ~0u;
    if (issue_window(r, w) || issue_window(r, w + 1)) {
        r->failed = true;
        return -1;
    }
    r->cur = w;
    r->cur_pos = 0;
    if (land_window(r, w)) {
        r->failed = true;
        return -1;
    }
    r->cur_pos = (sample - r->os[(size_t)w * r->window]) * r->stride;
    r->returned = sample * r->stride;
    return 0;
}

/* FLACFileReader.Read(buffer, offset, numBytes) with buffer.Length = buffer_length
 * (FLACFileReader.cs:145-174): drain the carried-over samples, then "ProcessSingle" +
 * copy until numBytes are reached or the stream ends; the copy runs to the end of the
 * buffer, so the return may exceed numBytes.  Exceptions of the C# surface return -1 with
 * their message (bnflac_reader_last_error): IndexOutOfRange for a sample that does not fit
 * the buffer, NotSupported for bit depths other than 16 and 24.  Needs a reader opened with
 * the FILEREADER layout; byte reads and seeks are not mixed with it. */
BNFLAC_API int64_t bnflac_reader_read_filereader(bnflac_reader *r, uint8_t *buffer, uint64_t offset, uint64_t num_bytes,
                                                 uint64_t buffer_length) {
    if (!r) return rfail("bnflac_reader_read_filereader: null reader");
    RDevGuard dg(r->device);
    if (r->failed) return rfail("bnflac_reader_read_filereader: reader failed earlier");
    if (r->fmt != BNFLAC_OUT_FILEREADER) return rfail("bnflac_reader_read_filereader: reader not opened with the FILEREADER layout");
    if (r->mode == 1) return rfail("bnflac_reader_read_filereader: this reader already serves byte reads");
    if (!buffer && buffer_length) return rfail("bnflac_reader_read_filereader: null buffer");
    r->mode = 2;
    uint64_t noff = offset;
    int64_t copied = 0;
    if (r->fr_idx > 0) {
        if (r->sp.bps != 16 && r->sp.bps != 24) return rfail("Input FLAC bit depth is not supported!");
        const int64_t c = fr_copy(r, buffer, buffer_length, noff);
        if (c < 0) return rfail("Index was outside the bounds of the array.");
        copied = c;
    }
    while ((uint64_t)copied < num_bytes) {
        if (r->eos) break;
        if (r->sp.bps != 16 && r->sp.bps != 24) {
            /* ProcessSingle decodes the frame; CopyFlacBufferToNAudioBuffer throws from its
             * sample loop (FLACFileReader.cs:239-240), which runs only while the offset is
             * inside the buffer (:211-214): at or past buffer.Length it copies 0 bytes and
             * Read keeps decoding to the end of the stream */
            if (r->fr_next >= r->nframes) {
                r->eos = true;
                break;
            }
            r->fr_next++;
            if (noff < buffer_length) return rfail("Input FLAC bit depth is not supported!");
            continue;
        }
        const uint8_t *fb = nullptr;
        uint32_t bs = 0;
        const int g = fr_next_frame(r, &fb, &bs);
        if (g < 0) {
            r->failed = true;
            return -1;
        }
        if (g == 0) { /* the decoder reached EndOfStream */
            r->eos = true;
            break;
        }
        fr_write(r, fb, bs);
        const int64_t c = fr_copy(r, buffer, buffer_length, noff);
        if (c < 0) return rfail("Index was outside the bounds of the array.");
        copied += c;
    }
    return copied;
}

BNFLAC_API void bnflac_reader_close(bnflac_reader *r) {
    if (!r) return;
    RDevGuard dg(r->device);
    release(r, !r->failed);
}

BNFLAC_API int bnflac_reader_pool_release(int device) {
    std::vector<bnflac_reader *> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size();) {
            if (device < 0 || g_pool[i]->device == device) {
                drop.push_back(g_pool[i]);
                g_pool.erase(g_pool.begin() + (long)i);
            } else {
                i++;
            }
        }
    }
    for (bnflac_reader *p : drop) {
        RDevGuard dg(p->device);
        free_resources(p);
        delete p;
    }
    return (int)drop.size();
}

} /* extern "C" */
