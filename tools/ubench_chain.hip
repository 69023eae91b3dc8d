// Microbenchmark: cycles per step of a Rice-cursor-like dependent chain, per wave, at
// several waves/SIMD; optionally with one ds_read per step (ring word).  Calibration only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int LDSREAD>
__global__ void __launch_bounds__(64) k(uint32_t *out, int iters, uint32_t seed) {
    __shared__ uint32_t ring[2048];
    const uint32_t lane = threadIdx.x;
    for (int i = lane; i < 2048; i += 64) ring[i] = i * 2654435761u;
    __syncthreads();
    uint32_t hi = seed ^ lane, lo = seed * 3 + lane, s = lane & 31, wi = lane, nx = 0x12345;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, s);
        const uint32_t q = w ? (uint32_t)__builtin_clz(w) : 32u;
        const uint32_t len = min(q + 4u, 32u);
        const int32_t t = (int32_t)s - (int32_t)len;
        const bool c = t < 0;
        s = (uint32_t)t & 31u;
        hi = c ? lo : hi;
        lo = c ? __builtin_bswap32(nx) : lo;
        wi += c ? 1u : 0u;
        if (LDSREAD) nx = ring[((wi & 31u) << 6) + lane];
        else nx = nx * 1664525u + 1013904223u;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) { out[blockIdx.x * 2] = (uint32_t)(t1 - t0); }
    out[blockIdx.x * 2 + 1] ^= hi ^ lo ^ s;
}
int main() {
    uint32_t *d;
    hipMalloc(&d, 1 << 24);
    const int iters = 4096;
    for (int lds = 0; lds < 2; lds++)
        for (int wps : {1, 2, 4, 8}) {
            const int blocks = 256 * 4 * wps; // 256 CUs x 4 SIMDs x waves/SIMD
            hipMemset(d, 0, 1 << 24);
            hipEvent_t e0, e1;
            hipEventCreate(&e0); hipEventCreate(&e1);
            if (lds) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, d, iters, 7u);
            else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, d, iters, 7u);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            if (lds) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, d, iters, 7u);
            else hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, d, iters, 7u);
            hipEventRecord(e1);
            hipDeviceSynchronize();
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            uint32_t h[2];
            hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
            printf("lds=%d waves/SIMD=%d: kernel %.3f ms, per-wave memtime %.1f ticks/step, %.1f ns/step/wave\n", lds, wps,
                   ms, h[0] / (double)iters, ms * 1e6 / iters);
        }
    return 0;
}
