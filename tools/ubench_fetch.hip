// Calibration of rocprofv3 FETCH_SIZE for the decoders' read shapes (known bytes in,
// counter out).  Each kernel reads exactly `bytes` distinct bytes from a 4 GiB buffer
// (far beyond the 256 MiB Infinity Cache):
//   coalesced  -- 16 B per lane, 1 KiB contiguous per wave instruction (the guide's
//                 calibration case: FETCH_SIZE = half the bytes on gfx950);
//   lane64     -- every lane its own stream, 64-byte groups = 4 x 16-byte LDS-DMA into one
//                 half cache line (k_decode_st's ring refill, bnflac_kernels.hip st_refill_issue);
//   lane16     -- every lane its own stream, one 16-byte LDS-DMA per step (scattered pieces).
// Run under rocprofv3 --pmc FETCH_SIZE; the kernel names carry the mode.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_fetch.hip -o tools/ubench_fetch
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gvoid;

#define STEPS 256 /* 16-byte pieces per lane (lane modes) / KiB per wave (coalesced) */

__global__ void __launch_bounds__(64) k_coalesced(const uint32_t *src, uint32_t *out) {
    __shared__ uint32_t ring[4 * 256];
    const uint64_t base = (uint64_t)blockIdx.x * STEPS * 256; /* words: STEPS KiB per wave */
    for (int it = 0; it < STEPS; it++) {
        __builtin_amdgcn_global_load_lds((gvoid *)(src + base + (uint64_t)it * 256 + threadIdx.x * 4),
                                         (lds_void *)(ring + (it & 3) * 256), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ring[1];
}

__global__ void __launch_bounds__(64) k_lane64(const uint32_t *src, uint32_t *out) {
    __shared__ uint32_t ring[8 * 256];
    /* lane streams STEPS*16 bytes long, back to back: no two lanes share a line */
    const uint64_t base = ((uint64_t)blockIdx.x * 64 + threadIdx.x) * STEPS * 4;
    for (int it = 0; it < STEPS; it += 4) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            __builtin_amdgcn_global_load_lds((gvoid *)(src + base + (uint64_t)(it + k) * 4),
                                             (lds_void *)(ring + ((it + k) & 7) * 256), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ring[1];
}

__global__ void __launch_bounds__(64) k_lane16(const uint32_t *src, uint32_t *out) {
    __shared__ uint32_t ring[8 * 256];
    const uint64_t base = ((uint64_t)blockIdx.x * 64 + threadIdx.x) * STEPS * 4;
    for (int it = 0; it < STEPS; it++) {
        __builtin_amdgcn_global_load_lds((gvoid *)(src + base + (uint64_t)it * 4), (lds_void *)(ring + (it & 7) * 256),
                                         16, 0, 0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = ring[1];
}

int main() {
    const uint64_t words = 1ull << 30; /* 4 GiB */
    uint32_t *src, *out;
    if (hipMalloc(&src, words * 4) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
    (void)hipMemset(src, 1, words * 4);
    const uint32_t blocks = (uint32_t)(words * 4 / (64ull * STEPS * 16)); /* every byte read once */
    const double bytes = (double)blocks * 64 * STEPS * 16;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int m = 0; m < 3; m++) {
        (void)hipEventRecord(e0);
        if (m == 0) hipLaunchKernelGGL(k_coalesced, dim3(blocks), dim3(64), 0, 0, src, out);
        if (m == 1) hipLaunchKernelGGL(k_lane64, dim3(blocks), dim3(64), 0, 0, src, out);
        if (m == 2) hipLaunchKernelGGL(k_lane16, dim3(blocks), dim3(64), 0, 0, src, out);
        (void)hipEventRecord(e1);
        (void)hipDeviceSynchronize();
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s bytes read %.0f (%.3f GiB)  %.3f ms  %.1f GB/s\n", m == 0 ? "coalesced" : (m == 1 ? "lane64" : "lane16"),
               bytes, bytes / (1 << 30), ms, bytes / ms / 1e6);
    }
    return 0;
}
