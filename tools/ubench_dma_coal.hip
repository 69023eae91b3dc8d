// Microbenchmark (calibration only): LDS-DMA refills of 64-byte runs of many streams, the same
// bytes and instruction count moved two ways -- SCATTERED: each lane its own stream, the run in
// four instructions of one 16-byte piece per lane (k_decode_sys's producer today); COALESCED:
// four lanes per stream, each instruction moving whole 64-byte runs of 16 streams.  Every lane
// of every instruction is active; each stream advances 64 bytes per refill, streams 1 MiB apart.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gvoid;
template <bool COAL, int WAIT>
__global__ void __launch_bounds__(64) k(const uint8_t *src, uint32_t *out, uint32_t chunks, uint64_t span) {
    __shared__ __attribute__((aligned(1024))) uint32_t ring[8 * 256];
    const uint32_t lane = threadIdx.x;
    const uint64_t s0 = (uint64_t)blockIdx.x * 64u;  // this wave's first stream
    for (uint32_t c = 0; c < chunks; c++) {
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            uint64_t stream, piece;
            if (COAL) { stream = s0 + 16u * u + (lane >> 2); piece = lane & 3u; }
            else { stream = s0 + lane; piece = u; }
            const uint64_t off = (stream * (1u << 20) + (uint64_t)c * 64u + piece * 16u) % span;
            __builtin_amdgcn_global_load_lds((gvoid *)(src + off), (lds_void *)(ring + ((c & 1u) * 4u + u) * 256u), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(WAIT) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0) out[blockIdx.x] = ring[lane * 4 + 1];
}
int main() {
    const uint64_t span = 1ull << 32;  // 4 GiB
    uint8_t *src;
    uint32_t *out;
    if (hipMalloc(&src, span) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    (void)hipMemset(src, 1, span);
    const uint32_t chunks = 256;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (uint32_t blocks : {64u, 512u, 2048u})
        for (int rep = 0; rep < 2; rep++)
            for (int m = 0; m < 4; m++) {
                (void)hipEventRecord(e0);
                switch (m) {
                case 0: hipLaunchKernelGGL((k<false, 4>), dim3(blocks), dim3(64), 0, 0, src, out, chunks, span); break;
                case 1: hipLaunchKernelGGL((k<true, 4>), dim3(blocks), dim3(64), 0, 0, src, out, chunks, span); break;
                case 2: hipLaunchKernelGGL((k<false, 0>), dim3(blocks), dim3(64), 0, 0, src, out, chunks, span); break;
                default: hipLaunchKernelGGL((k<true, 0>), dim3(blocks), dim3(64), 0, 0, src, out, chunks, span); break;
                }
                (void)hipEventRecord(e1);
                (void)hipDeviceSynchronize();
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                const double bytes = (double)blocks * 64 * 64 * chunks;
                printf("waves=%4u %-9s wait=%s: %.3f ms, %.1f GB/s, %.0f ns per refill (4 instr)\n", blocks,
                       (m & 1) ? "coalesced" : "scattered", m < 2 ? "1 behind" : "each   ", ms, bytes / ms / 1e6,
                       ms * 1e6 / chunks);
            }
    return 0;
}
