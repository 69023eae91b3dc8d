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
        uint64_t w64 = x; uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
        for (int it = 0; it < ITERS; it++) {                                                     \
            asm volatile(INS("%0") INS("%1") INS("%2") INS("%3") INS("%4") INS("%5") INS("%6") INS("%7") \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
                         [w] "+v"(w64) : "v"(x), "v"(y), "s"(s) : "vcc", "s0");                                             \
        }                                                                                        \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)w64;       \
        if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }
// one dependent chain: 8 instructions per iteration, each reading the previous result
#define DEP_KERNEL(name, INS)                                                                   \
    __global__ __launch_bounds__(256) void name(const uint32_t *in, uint32_t *out, uint64_t *cyc) { \
        uint32_t x = in[threadIdx.x & 63], y = in[64 + (threadIdx.x & 63)];                     \
        uint32_t a0 = x, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                 \
        uint64_t s = (uint64_t)in[128] | ((uint64_t)in[129] << 32);                              \
        uint64_t w64 = x; uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
        for (int it = 0; it < ITERS; it++) {                                                     \
            asm volatile(INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") INS("%0") \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), \
                         [w] "+v"(w64) : "v"(x), "v"(y), "s"(s) : "vcc", "s0");                                             \
        }                                                                                        \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)w64;       \
        if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }

#define KPAIR(tag, INS) IND_KERNEL(ind_##tag, INS) DEP_KERNEL(dep_##tag, INS)
// operands: %N = the chain register, %8 = the 64-bit register w, %9 = x, %10 = y, %11 = s (64-bit SGPR pair)
#define I_and(r) "v_and_b32 " r ", " r ", %9\n\t"
KPAIR(and, I_and)
#define I_or(r) "v_or_b32 " r ", " r ", %9\n\t"
KPAIR(or, I_or)
#define I_mov(r) "v_mov_b32 " r ", %9\n\t"
KPAIR(mov, I_mov)
#define I_max_i32(r) "v_max_i32 " r ", " r ", %9\n\t"
KPAIR(max_i32, I_max_i32)
#define I_min_u32(r) "v_min_u32 " r ", " r ", %9\n\t"
KPAIR(min_u32, I_min_u32)
#define I_cndmask_e32(r) "v_cndmask_b32 " r ", " r ", %9, vcc\n\t"
KPAIR(cndmask_e32, I_cndmask_e32)
#define I_lshrrev(r) "v_lshrrev_b32 " r ", %9, " r "\n\t"
KPAIR(lshrrev, I_lshrrev)
#define I_ashrrev(r) "v_ashrrev_i32 " r ", %9, " r "\n\t"
KPAIR(ashrrev, I_ashrrev)
#define I_lshlrev_v(r) "v_lshlrev_b32 " r ", %9, " r "\n\t"
KPAIR(lshlrev_v, I_lshlrev_v)
#define I_bfi(r) "v_bfi_b32 " r ", " r ", %9, %10\n\t"
KPAIR(bfi, I_bfi)
#define I_and_or(r) "v_and_or_b32 " r ", " r ", %9, %10\n\t"
KPAIR(and_or, I_and_or)
#define I_lshl_or(r) "v_lshl_or_b32 " r ", " r ", %9, %10\n\t"
KPAIR(lshl_or, I_lshl_or)
#define I_xad(r) "v_xad_u32 " r ", " r ", %9, %10\n\t"
KPAIR(xad, I_xad)
#define I_max3(r) "v_max3_i32 " r ", " r ", %9, %10\n\t"
KPAIR(max3, I_max3)
#define I_or3(r) "v_or3_b32 " r ", " r ", %9, %10\n\t"
KPAIR(or3, I_or3)
#define I_dot2c(r) "v_dot2c_i32_i16 " r ", %9, %10\n\t"
KPAIR(dot2c, I_dot2c)
#define I_pk_add_u16(r) "v_pk_add_u16 " r ", " r ", %9\n\t"
KPAIR(pk_add_u16, I_pk_add_u16)
#define I_pk_max_i16(r) "v_pk_max_i16 " r ", " r ", %9\n\t"
KPAIR(pk_max_i16, I_pk_max_i16)
#define I_bfe_i32(r) "v_bfe_i32 " r ", " r ", %9, %10\n\t"
KPAIR(bfe_i32, I_bfe_i32)
#define I_add_co(r) "v_add_co_u32 " r ", vcc, " r ", %9\n\t"
KPAIR(add_co, I_add_co)
#define I_addc(r) "v_addc_co_u32 " r ", vcc, " r ", %9, vcc\n\t"
KPAIR(addc, I_addc)
#define I_cmp_lt(r) "v_cmp_lt_u32 vcc, " r ", %9\n\t"
KPAIR(cmp_lt, I_cmp_lt)
#define I_mad_i64(r) "v_mad_i64_i32 %[w], vcc, " r ", %9, %[w]\n\t"
KPAIR(mad_i64, I_mad_i64)
#define I_mul_u32_u24(r) "v_mul_u32_u24 " r ", " r ", %9\n\t"
KPAIR(mul_u32_u24, I_mul_u32_u24)
#define I_sad_u32(r) "v_sad_u32 " r ", " r ", %9, %10\n\t"
KPAIR(sad_u32, I_sad_u32)
#define I_perm_e(r) "v_perm_b32 " r ", " r ", %9, %10\n\t"
KPAIR(perm_e, I_perm_e)
#define I_lshrrev_b64(r) "v_lshrrev_b64 %[w], %9, %[w]\n\t"
KPAIR(lshrrev_b64, I_lshrrev_b64)
#define I_alignbyte(r) "v_alignbyte_b32 " r ", " r ", %9, %10\n\t"
KPAIR(alignbyte, I_alignbyte)
#define I_bcnt(r) "v_bcnt_u32_b32 " r ", " r ", %9\n\t"
KPAIR(bcnt, I_bcnt)
#define I_sub_co(r) "v_sub_co_u32 " r ", vcc, " r ", %9\n\t"
KPAIR(sub_co, I_sub_co)
#define I_readfirstlane(r) "v_readfirstlane_b32 s0, " r "\n\t"
KPAIR(readfirstlane, I_readfirstlane)

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
        E(and) E(or) E(mov) E(max_i32) E(min_u32) E(cndmask_e32) E(lshrrev) E(ashrrev) E(lshlrev_v) E(bfi) E(and_or) E(lshl_or) E(xad) E(max3) E(or3) E(dot2c) E(pk_add_u16) E(pk_max_i16) E(bfe_i32) E(add_co) E(addc) E(cmp_lt) E(mad_i64) E(mul_u32_u24) E(sad_u32) E(perm_e) E(lshrrev_b64) E(alignbyte) E(bcnt) E(sub_co) E(readfirstlane)
#undef E
    };
    printf("%-52s %5s %6s %9s %12s %12s\n", "instruction", "mode", "w/SIMD", "ms", "cyc/instr/SIMD", "wall cyc@2.4");
    for (auto &k : ks) {
        for (int dep = 0; dep < 1; dep++) {
            for (int w : {2, 8}) {
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
