// Where does global_load_lds_dwordx4 with an instruction offset put its data in LDS?
// Each lane's four consecutive 16-byte blocks (global address a + 16 k, k = 0..3) are loaded
// with one base address and offset:16k; mode 0 passes the slot base as the LDS pointer, mode 1
// the slot base - 16k (compensating an offset that also moves the LDS destination).  Prints,
// per mode and slot, whether lane l's 16 bytes landed at slot k + 16 l.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gvoid;
template <int OFF>
__device__ void ld(const uint32_t *g, lds_u32 *l) { __builtin_amdgcn_global_load_lds((gvoid *)g, (lds_void *)l, 16, OFF, 0); }
__global__ void __launch_bounds__(64) k(const uint32_t *src, uint32_t *out, int mode) {
    __shared__ __attribute__((aligned(1024))) uint32_t buf[5 * 256];
    const uint32_t lane = threadIdx.x;
    for (int i = 0; i < 20; i++) buf[lane * 20 + i] = 0xAA000000u | (lane * 20 + i);
    __syncthreads();
    const uint32_t *g = src + lane * 16; /* lane's 64 bytes */
    lds_u32 *b = (lds_u32 *)buf;
    if (mode == 0) {
        ld<0>(g, b + 0 * 256); ld<16>(g, b + 1 * 256); ld<32>(g, b + 2 * 256); ld<48>(g, b + 3 * 256);
    } else {
        ld<0>(g, b + 0 * 256); ld<16>(g, b + 1 * 256 - 4); ld<32>(g, b + 2 * 256 - 8); ld<48>(g, b + 3 * 256 - 12);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = 0; i < 20; i++) out[lane * 20 + i] = buf[lane * 20 + i];
}
int main() {
    static uint32_t h[64 * 16], r[5 * 256];
    uint32_t *ds, *dout;
    for (int i = 0; i < 64 * 16; i++) h[i] = 0xBB000000u | i;
    hipMalloc(&ds, sizeof h);
    hipMalloc(&dout, sizeof r);
    hipMemcpy(ds, h, sizeof h, hipMemcpyHostToDevice);
    for (int m = 0; m < 2; m++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dout, m);
        if (hipMemcpy(r, dout, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) { printf("error\n"); return 1; }
        for (int s = 0; s < 4; s++) {
            int good = 0;
            for (int l = 0; l < 64; l++) {
                bool ok = true;
                for (int w = 0; w < 4; w++) ok = ok && r[s * 256 + l * 4 + w] == (0xBB000000u | (l * 16 + s * 4 + w));
                good += ok;
            }
            printf("mode %d slot %d: %2d/64 lanes in place; lane0 %08x %08x lane1 %08x; word at slot+16k: %08x\n", m, s, good,
                   r[s * 256], r[s * 256 + 1], r[s * 256 + 4], r[s * 256 + 4 * s]);
        }
    }
    return 0;
}
