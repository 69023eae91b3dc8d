/* Host-side floor of the streaming reader's Read(): memcpy of a C2 stream's PCM (16.8 MB) in
 * 16 KiB pieces into one reused buffer, from pinned host memory a D2H copy just wrote (what
 * bnflac_reader_read does) and from ordinary memory, plus the D2H itself.  Calibration only.
 *   hipcc -O2 tools/memcpy_probe.cpp -o tools/memcpy_probe && tools/memcpy_probe */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

static volatile uint32_t g_sink;
static double drain(const uint8_t *src, size_t n, uint8_t *buf, size_t piece) {
    const double t0 = now_ms();
    uint32_t acc = 0;
    for (size_t o = 0; o < n; o += piece) {
        memcpy(buf, src + o, n - o < piece ? n - o : piece);
        acc += buf[(o >> 7) & (piece - 1)]; /* the caller looks at what it got */
        __asm__ volatile("" ::"r"(buf) : "memory");
    }
    g_sink = acc;
    return now_ms() - t0;
}

int main(void) {
    const size_t n = 16777216, piece = 16384;
    uint8_t *pin = NULL, *dev = NULL, *buf = (uint8_t *)malloc(piece), *plain = (uint8_t *)malloc(n);
    if (hipHostMalloc((void **)&pin, n, hipHostMallocDefault) != hipSuccess || hipMalloc((void **)&dev, n) != hipSuccess)
        return 1;
    memset(plain, 1, n);
    (void)hipMemset(dev, 3, n);
    (void)hipDeviceSynchronize();
    for (int rep = 0; rep < 3; rep++) {
        double t0 = now_ms();
        (void)hipMemcpy(pin, dev, n, hipMemcpyDeviceToHost);
        const double d2h = now_ms() - t0;
        const double a = drain(pin, n, buf, piece); /* just written by the DMA */
        const double b = drain(pin, n, buf, piece); /* again (cache-warm where it fits) */
        const double c = drain(plain, n, buf, piece);
        printf("D2H %.3f ms (%.1f GB/s); memcpy 16 KiB pieces: pinned after DMA %.3f ms (%.1f GB/s), "
               "pinned again %.3f ms, malloc'd %.3f ms\n",
               d2h, n / d2h / 1e6, a, n / a / 1e6, b, c);
    }
    /* the D2H split over k streams (k copy engines, if the runtime spreads them) */
    hipStream_t st[4];
    for (int i = 0; i < 4; i++) (void)hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
    for (int k = 1; k <= 4; k *= 2)
        for (int rep = 0; rep < 3; rep++) {
            const double t0 = now_ms();
            for (int i = 0; i < k; i++) (void)hipMemcpyAsync(pin + i * (n / k), dev + i * (n / k), n / k, hipMemcpyDeviceToHost, st[i]);
            for (int i = 0; i < k; i++) (void)hipStreamSynchronize(st[i]);
            const double t = now_ms() - t0;
            printf("D2H on %d stream(s): %.3f ms (%.1f GB/s)\n", k, t, n / t / 1e6);
        }
    /* 4 MiB windows one after another on one stream, as the reader issues them */
    for (int rep = 0; rep < 3; rep++) {
        const double t0 = now_ms();
        for (int w = 0; w < 4; w++) (void)hipMemcpyAsync(pin + w * (n / 4), dev + w * (n / 4), n / 4, hipMemcpyDeviceToHost, st[0]);
        (void)hipStreamSynchronize(st[0]);
        const double t = now_ms() - t0;
        printf("D2H 4 x 4 MiB on one stream: %.3f ms (%.1f GB/s)\n", t, n / t / 1e6);
    }
    return (int)buf[0] & 0;
}
