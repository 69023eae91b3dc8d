// Microbenchmark: cost of scattered LDS-DMA (global_load_lds_dwordx4) instructions by active
// lanes per instruction, at a fixed number of 16-byte pieces moved.  Calibration only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gvoid;
template <int ACTIVE>  // active lanes per instruction (64 / ACTIVE instructions per 64 pieces)
__global__ void __launch_bounds__(64) k(const uint32_t *src, uint32_t *out, uint32_t iters, uint64_t span_words) {
    __shared__ uint32_t ring[4 * 256];
    const uint32_t lane = threadIdx.x;
    uint64_t pos = ((uint64_t)blockIdx.x * 64 + lane) * 4096;  // each lane its own stream, 16 KiB apart
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int g = 0; g < 64 / ACTIVE; g++) {
            if ((lane / ACTIVE) == (uint32_t)g)
                __builtin_amdgcn_global_load_lds((gvoid *)(src + (pos % span_words)), (lds_void *)(ring + (it & 3) * 256), 16, 0, 0);
        }
        pos += 4;  // next 16 bytes of this lane's stream
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0) out[blockIdx.x] = ring[lane * 4 + 1];
}
int main() {
    const uint64_t span = 1ull << 28;  // 1 GiB of words
    uint32_t *src, *out;
    if (hipMalloc(&src, span * 4) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    (void)hipMemset(src, 1, span * 4);
    const uint32_t blocks = 2048, iters = 512;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++)
        for (int a : {64, 16, 8, 4}) {
            (void)hipEventRecord(e0);
            switch (a) {
            case 64: hipLaunchKernelGGL(k<64>, dim3(blocks), dim3(64), 0, 0, src, out, iters, span); break;
            case 16: hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(64), 0, 0, src, out, iters, span); break;
            case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(64), 0, 0, src, out, iters, span); break;
            default: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, src, out, iters, span); break;
            }
            (void)hipEventRecord(e1);
            (void)hipDeviceSynchronize();
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double pieces = (double)blocks * 64 * iters;
            printf("active=%2d lanes/instr (%2d instr per 64 pieces): %.3f ms, %.1f GB/s of 16-B pieces\n", a, 64 / a, ms,
                   pieces * 16 / ms / 1e6);
        }
    return 0;
}
