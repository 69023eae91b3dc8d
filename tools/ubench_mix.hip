// Issue rate of k_decode_st's VALU mix on gfx950 (VERDICT r4 "next" 1a): each instruction
// class alone, 8 independent chains per lane (throughput) and 1 dependent chain (latency),
// at 1, 2, 4 and 8 waves per SIMD, plus a blended mix in k_decode_st's proportions.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mix.hip -o tools/ubench_mix && tools/ubench_mix
// Each wave stamps s_memtime around its loop; cycles per wave-instruction per SIMD =
// (mean wave cycles) / (instructions per wave) / (waves per SIMD) -- the SIMD's issue interval.
// The wall-clock figure (at an assumed 2.4 GHz) is printed beside it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// one asm statement per iteration (the compiler adds a wait state after each asm statement):
// 8 instructions on 8 independent registers a0..a7 (throughput), operands x, y, s (mask)
#define IND_KERNEL(name, INS)                                                                   \
    __global__ __launch_bounds__(256) void name(const uint32_t *in, uint32_t *out, uint64_t *cyc) { \
        uint32_t x = in[threadIdx.x & 63], y = in[64 + (threadIdx.x & 63)];                     \
        uint32_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7; \
        uint64_t s = (uint64_t)in[128] | ((uint64_t)in[129] << 32);                              \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
        for (int it = 0; it < ITERS; it++) {                                                     \
            asm volatile(INS("%0") INS("%1") INS("%2") INS("%3") INS("%4") INS("%5") INS("%6") INS("%7") \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(x), "v"(y), "s"(s));                                             \
        }                                                                                        \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
        if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }
// one dependent chain: 8 instructions per iteration, each reading the previous result
#define DEP_KERNEL(name, INS)                                                                   \
    __global__ __launch_bounds__(256) void name(const uint32_t *in, uint32_t *out, uint64_t *cyc) { \
        uint32_t x = in[threadIdx.x & 63], y = in[64 + (threadIdx.x & 63)];                     \
        uint32_t a0 = x, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                 \
        uint64_t s = (uint64_t)in[128] | ((uint64_t)in[129] << 32);                              \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
        for (int it = 0; it < ITERS; it++) {                                                     \
            asm volatile(INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(x), "v"(y), "s"(s));                                             \
        }                                                                                        \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;       \
        if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }

// operands: %N = the chain register, %8 = x, %9 = y, %10 = s (64-bit SGPR pair)
#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n\t"
#define I_XOR(r) "v_xor_b32 " r ", " r ", %8\n\t"
#define I_LSHL(r) "v_lshlrev_b32 " r ", 3, " r "\n\t"
#define I_ALIGNBIT(r) "v_alignbit_b32 " r ", " r ", %8, %9\n\t"
#define I_FFBH(r) "v_ffbh_u32 " r ", " r "\n\t"
#define I_BFE(r) "v_bfe_u32 " r ", " r ", %8, %9\n\t"
#define I_DOT2(r) "v_dot2_i32_i16 " r ", " r ", %8, %9\n\t"
#define I_PERM(r) "v_perm_b32 " r ", " r ", %8, %9\n\t"
#define I_CND(r) "v_cndmask_b32_e64 " r ", " r ", %8, %10\n\t"
#define I_ADD3(r) "v_add3_u32 " r ", " r ", %8, %9\n\t"
#define I_LSHLADD(r) "v_lshl_add_u32 " r ", " r ", 2, %8\n\t"
#define I_MAD24(r) "v_mad_u32_u24 " r ", " r ", %8, %9\n\t"
#define I_MULLO(r) "v_mul_lo_u32 " r ", " r ", %8\n\t"
#define I_MED3(r) "v_med3_i32 " r ", " r ", %8, %9\n\t"
#define I_SUBREV(r) "v_sub_u32 " r ", %8, " r "\n\t"
// k_decode_st's fused pair step in miniature: window, length, field, advance, predictor, pack,
// select, xor.  The throughput form issues each instruction for all 8 registers in turn.
#define ALL8(I) I("%0") I("%1") I("%2") I("%3") I("%4") I("%5") I("%6") I("%7")
#define SEQ(r) I_ALIGNBIT(r) I_FFBH(r) I_BFE(r) I_ADD(r) I_DOT2(r) I_PERM(r) I_CND(r) I_XOR(r)
#define MIX_IND(r) ALL8(I_ALIGNBIT) ALL8(I_FFBH) ALL8(I_BFE) ALL8(I_ADD) ALL8(I_DOT2) ALL8(I_PERM) ALL8(I_CND) ALL8(I_XOR)
#define KPAIR(tag, INS) IND_KERNEL(ind_##tag, INS) DEP_KERNEL(dep_##tag, INS)
KPAIR(add, I_ADD)
KPAIR(xor, I_XOR)
KPAIR(lshl, I_LSHL)
KPAIR(alignbit, I_ALIGNBIT)
KPAIR(ffbh, I_FFBH)
KPAIR(bfe, I_BFE)
KPAIR(dot2, I_DOT2)
KPAIR(perm, I_PERM)
KPAIR(cndmask, I_CND)
KPAIR(add3, I_ADD3)
KPAIR(lshl_add, I_LSHLADD)
KPAIR(mad_u24, I_MAD24)
KPAIR(mul_lo, I_MULLO)
KPAIR(med3, I_MED3)
KPAIR(sub, I_SUBREV)
__global__ __launch_bounds__(256) void ind_mix8(const uint32_t *in, uint32_t *out, uint64_t *cyc) {
    uint32_t x = in[threadIdx.x & 63], y = in[64 + (threadIdx.x & 63)];
    uint32_t a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
    uint64_t s = (uint64_t)in[128] | ((uint64_t)in[129] << 32);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; it++) {
        asm volatile(MIX_IND(0)
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(x), "v"(y), "s"(s));
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

#define SEQ8(r) SEQ("%0") SEQ("%0") SEQ("%0") SEQ("%0") SEQ("%0") SEQ("%0") SEQ("%0") SEQ("%0")
#define SEQ1(r) SEQ(r)
DEP_KERNEL(dep_mix8, SEQ1)

typedef void (*kfn)(const uint32_t *, uint32_t *, uint64_t *);
struct K { const char *n; kfn ind, dep; int per_iter; };

int main() {
    uint32_t *in, *out; uint64_t *cyc;
    hipMalloc(&in, 1024); hipMalloc(&out, 64 << 20); hipMalloc(&cyc, 8 << 20);
    uint32_t hin[256];
    for (int i = 0; i < 256; i++) hin[i] = 0x9e3779b9u * (i + 1);
    hin[128] = 0x5555aaaau; hin[129] = 0xaaaa5555u;
    for (int i = 0; i < 64; i++) hin[64 + i] = (hin[64 + i] & 0x1f) | 0x00020000u;  // bfe/alignbit shift operand
    hipMemcpy(in, hin, sizeof hin, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    static uint64_t hc[1 << 20];
    K ks[] = {
#define E(t) {#t, ind_##t, dep_##t, 8},
        E(add) E(xor) E(lshl) E(alignbit) E(ffbh) E(bfe) E(dot2) E(perm) E(cndmask) E(add3) E(lshl_add)
        E(mad_u24) E(mul_lo) E(med3) E(sub)
#undef E
        {"mix8 (alignbit ffbh bfe add dot2 perm cndmask xor)", ind_mix8, dep_mix8, 64},
    };
    printf("%-52s %5s %6s %9s %12s %12s\n", "instruction", "mode", "w/SIMD", "ms", "cyc/instr/SIMD", "wall cyc@2.4");
    for (auto &k : ks) {
        for (int dep = 0; dep < 2; dep++) {
            for (int w : {1, 2, 4, 8}) {
                int grid = 256 * w, blk = 256;  // 4 waves per workgroup: one per SIMD
                kfn f = dep ? k.dep : k.ind;
                hipLaunchKernelGGL(f, dim3(grid), dim3(blk), 0, 0, in, out, cyc);
                hipDeviceSynchronize();
                hipEventRecord(e0);
                hipLaunchKernelGGL(f, dim3(grid), dim3(blk), 0, 0, in, out, cyc);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                int nw = grid * blk / 64;
                hipMemcpy(hc, cyc, nw * 8, hipMemcpyDeviceToHost);
                double m = 0; for (int i = 0; i < nw; i++) m += hc[i]; m /= nw;
                double ipw = (double)ITERS * k.per_iter;  // instructions per wave
                double wall = 1024.0 * 2.4e6 * ms / (ipw * nw);
                printf("%-52s %5s %6d %9.4f %12.2f %12.2f\n", k.n, dep ? "dep" : "ind", w, ms, m / ipw / w, wall);
            }
        }
    }
    return 0;
}
