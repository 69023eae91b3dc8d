// Does an exec-masked global_load_lds_dwordx4 leave inactive lanes' LDS entries alone?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gvoid;
__global__ void __launch_bounds__(64) k(const uint32_t *src, uint32_t *out, int pattern) {
    __shared__ uint32_t buf[256];
    const uint32_t lane = threadIdx.x;
    for (int i = 0; i < 4; i++) buf[lane * 4 + i] = 0xAA000000u | (lane << 8) | i;
    __syncthreads();
    bool act = pattern == 0 ? (lane & 1) : pattern == 1 ? (lane < 16) : (lane >= 40);
    if (act) __builtin_amdgcn_global_load_lds((gvoid *)(src + lane * 4), (lds_void *)(lds_u32 *)buf, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = 0; i < 4; i++) out[lane * 4 + i] = buf[lane * 4 + i];
}
int main() {
    uint32_t h[256], *ds, *dout, r[256];
    for (int i = 0; i < 256; i++) h[i] = 0xBB000000u | i;
    hipMalloc(&ds, 1024); hipMalloc(&dout, 1024);
    hipMemcpy(ds, h, 1024, hipMemcpyHostToDevice);
    for (int p = 0; p < 3; p++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout, p);
        hipMemcpy(r, dout, 1024, hipMemcpyDeviceToHost);
        printf("pattern %d:\n", p);
        for (int l = 0; l < 64; l++) printf("  lane %2d: %08x %08x %08x %08x\n", l, r[l*4], r[l*4+1], r[l*4+2], r[l*4+3]);
    }
    return 0;
}
