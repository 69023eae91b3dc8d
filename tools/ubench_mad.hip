// Throughput of the LPC multiply-accumulate forms on gfx950: v_mad_i64_i32 (exact 64-bit,
// libFLAC's wide restore) vs v_mad_i32_i24 (the 12-bit split forms), 8 independent chains
// per lane.  hipcc --offload-arch=gfx950 -O3 tools/ubench_mad.hip -o tools/ubench_mad
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
__global__ void k64(const int32_t *in, int64_t *out) {
    int32_t c = in[threadIdx.x & 63], x = in[64 + (threadIdx.x & 63)];
    int64_t a[8];
    for (int i = 0; i < 8; i++) a[i] = i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(a[i]) : "v"(c), "v"(x + i) : "vcc");
    }
    int64_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k24(const int32_t *in, int64_t *out) {
    int32_t c = in[threadIdx.x & 63], x = in[64 + (threadIdx.x & 63)];
    int32_t a[8];
    for (int i = 0; i < 8; i++) a[i] = i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a[i]) : "v"(c), "v"(x + i));
    }
    int64_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k64dep(const int32_t *in, int64_t *out) { /* one dependent chain: latency */
    int32_t c = in[threadIdx.x & 63], x = in[64 + (threadIdx.x & 63)];
    int64_t a = 1;
    for (int it = 0; it < ITERS * 8; it++) asm volatile("v_mad_i64_i32 %0, vcc, %1, %2, %0" : "+v"(a) : "v"(c), "v"(x) : "vcc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
__global__ void k24dep(const int32_t *in, int64_t *out) {
    int32_t c = in[threadIdx.x & 63], x = in[64 + (threadIdx.x & 63)];
    int32_t a = 1;
    for (int it = 0; it < ITERS * 8; it++) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a) : "v"(c), "v"(x));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
int main() {
    int32_t *in; int64_t *out;
    hipMalloc(&in, 512); hipMalloc(&out, 8 << 20); hipMemset(in, 1, 512);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    struct { const char *n; void (*k)(const int32_t *, int64_t *); int grid; int blk; } ks[] = {
        {"mad_i64_i32 8 chains, full chip", k64, 2048, 256}, {"mad_i32_i24 8 chains, full chip", k24, 2048, 256},
        {"mad_i64_i32 1 chain, 1 wave/SIMD", k64dep, 1024, 64}, {"mad_i32_i24 1 chain, 1 wave/SIMD", k24dep, 1024, 64}};
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.k, dim3(k.grid), dim3(k.blk), 0, 0, in, out);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(k.grid), dim3(k.blk), 0, 0, in, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double waveinstr = (double)k.grid * k.blk / 64 * ITERS * 8;
        printf("%-36s %8.3f ms  %.3f wave-instr/ns  (%.2f cycles per wave-instr per SIMD at 2.4 GHz)\n", k.n, ms,
               waveinstr / (ms * 1e6), 1024.0 * 2.4 * ms * 1e6 / waveinstr);
    }
    return 0;
}
