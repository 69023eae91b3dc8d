/* Streaming-reader timing from C (no Python in the loop): open (H2D, frame index,
 * decode-ahead) + bnflac_reader_read in fixed pieces until the end, repeated; prints the
 * best open / read / close split and the samples per second of the whole pass.
 *   gcc -O2 tools/reader_bench.c -Iinclude -Lbirdnest/audio_amd/lib -lbnflac \
 *       -Wl,-rpath,'$ORIGIN/../birdnest/audio_amd/lib' -o tools/reader_bench
 *   tools/reader_bench <stream.flac> [reps=10] [piece=16384] [format=2] [window=0] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "bnflac.h"

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s stream.flac [reps] [piece] [format] [window]\n", argv[0]);
        return 2;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const size_t piece = argc > 3 ? (size_t)atol(argv[3]) : 16384;
    const int fmt = argc > 4 ? atoi(argv[4]) : BNFLAC_OUT_FLACDECODER;
    const uint32_t window = argc > 5 ? (uint32_t)atoi(argv[5]) : 0;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *bytes = malloc((size_t)n), *buf = malloc(piece);
    if (!bytes || !buf || fread(bytes, 1, (size_t)n, f) != (size_t)n) return 2;
    fclose(f);
    double best_open = 1e30, best_read = 1e30, best_close = 1e30, best_all = 1e30;
    uint64_t total = 0, samples = 0;
    for (int i = 0; i < reps; i++) {
        bnflac_reader *r = NULL;
        const double t0 = now_ms();
        if (bnflac_reader_open(0, bytes, (uint64_t)n, fmt, window, &r)) {
            fprintf(stderr, "open: %s\n", bnflac_reader_last_error());
            return 1;
        }
        const double t1 = now_ms();
        uint64_t got = 0;
        for (;;) {
            const int64_t k = bnflac_reader_read(r, buf, piece);
            if (k < 0) {
                fprintf(stderr, "read: %s\n", bnflac_reader_last_error());
                return 1;
            }
            if (k == 0) break;
            got += (uint64_t)k;
        }
        const double t2 = now_ms();
        bnflac_stream_params sp;
        uint64_t tb = 0;
        uint32_t nf = 0;
        bnflac_reader_params(r, &sp, &tb, &nf);
        bnflac_reader_close(r);
        const double t3 = now_ms();
        total = got;
        samples = sp.total_samples * sp.channels;
        if (t1 - t0 < best_open) best_open = t1 - t0;
        if (t2 - t1 < best_read) best_read = t2 - t1;
        if (t3 - t2 < best_close) best_close = t3 - t2;
        if (t3 - t0 < best_all) best_all = t3 - t0;
    }
    printf("{\"bytes\": %llu, \"samples\": %llu, \"piece\": %zu, \"open_ms\": %.3f, \"read_ms\": %.3f, "
           "\"close_ms\": %.3f, \"total_ms\": %.3f, \"MSamples_per_s\": %.1f}\n",
           (unsigned long long)total, (unsigned long long)samples, piece, best_open, best_read, best_close, best_all,
           samples / best_all / 1e3);
    return 0;
}
