// Microbenchmark: TCP->TCC write requests for scattered 64-byte vs 128-byte runs per store
// instruction (4 vs 8 lanes x 16 B per frame run).  Calibration only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int RUN>  // bytes per frame run within one store instruction (64 or 128)
__global__ void __launch_bounds__(64) k(uint4 *out, uint32_t iters, uint32_t stride_runs) {
    const uint32_t lane = threadIdx.x;
    constexpr uint32_t LPR = RUN / 16;            // lanes per run
    const uint32_t fr = lane / LPR, unit = lane % LPR;
    uint4 v = make_uint4(lane, iters, 1, 2);
    for (uint32_t it = 0; it < iters; it++) {
        // frame fr of this wave's 64/LPR frames; runs spread far apart like per-frame PCM
        const uint64_t run = ((uint64_t)blockIdx.x * (64 / LPR) + fr) * stride_runs + it;
        out[run * LPR + unit] = v;
        v.x += 1;
    }
}
int main() {
    const uint32_t blocks = 4096, iters = 256;
    for (int r = 0; r < 2; r++) {
        const uint32_t lpr = r ? 8 : 4;
        const uint32_t runs_per_block = 64 / lpr;
        const uint64_t stride_runs = iters;  // each frame's runs are contiguous over iterations
        const size_t bytes = (size_t)blocks * runs_per_block * stride_runs * lpr * 16;
        uint4 *d;
        if (hipMalloc(&d, bytes) != hipSuccess) return 1;
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            if (r) hipLaunchKernelGGL(k<128>, dim3(blocks), dim3(64), 0, 0, d, iters, (uint32_t)stride_runs);
            else hipLaunchKernelGGL(k<64>, dim3(blocks), dim3(64), 0, 0, d, iters, (uint32_t)stride_runs);
            hipEventRecord(e1);
            hipDeviceSynchronize();
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("run=%dB bytes=%.1f MB time=%.3f ms -> %.1f GB/s\n", r ? 128 : 64, bytes / 1e6, ms, bytes / ms / 1e6);
        }
        hipFree(d);
    }
    return 0;
}
