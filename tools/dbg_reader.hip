// Standalone check of the LDS-ring bit reader (BR in bnflac_kernels.hip) against a plain
// bit extractor.  Build: hipcc --offload-arch=gfx950 -O3 -I include tools/dbg_reader.hip
#include "../birdnest/audio_amd/csrc/bnflac_kernels.hip"
#include <cstdio>
#include <vector>

DEV uint32_t ref_bits(const uint8_t *d, uint64_t nbytes, uint64_t pos, uint32_t n) {
    uint32_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t p = pos + i;
        const uint32_t bit = (p >> 3) < nbytes ? (d[p >> 3] >> (7 - (p & 7))) & 1u : 0u;
        v = (v << 1) | bit;
    }
    return v;
}

__global__ void __launch_bounds__(64) k_test(const uint32_t *words, uint64_t nbytes, uint32_t *res, int mode) {
    __shared__ uint32_t ring[RING_MAX * RING_LANE_DW];
    BR b;
    const uint32_t lane = threadIdx.x;
    br_init(b, words, nbytes, (lds_u32 *)ring, lane, RING_MAX);
    uint64_t pos = (uint64_t)lane * 4099u + 5u + blockIdx.x * 100003u;
    br_seek(b, pos);
    uint32_t bad = 0, first = 0xffffffffu, got0 = 0, exp0 = 0;
    uint32_t rbad = 0, rinfo = 0, rgot = 0, rexp = 0;
    for (uint32_t i = 0; i < 4000; i++) {
        if ((mode == 0 || mode == 4) && (i & 7) == 0) br_refill(b);
        if (mode == 3 && (i & 7) == 0) {
            br_refill(b);
            const uint32_t need = b.wi >> 2;
            for (uint32_t j = need; j < b.vendw / 4; j++)
                for (uint32_t q = 0; q < 4; q++) {
                    const uint32_t w = j * 4 + q;
                    const uint32_t g = ring_word(b, w);
                    const uint32_t e = w < b.nw ? b.w[w] : 0u;
                    if (g != e) { if (!rbad) { rinfo = (i << 16) | ((j - need) << 8) | (b.vendw / 4 - need); rgot = g; rexp = e; } rbad++; }
                }
        }
        if (mode == 1 && (i & 31) == 0 && lane < 32) br_refill(b);
        const uint32_t n = 1u + ((i * 7u + lane) % 23u);
        if (br_pos(b) != pos) { bad++; if (first == 0xffffffffu) { first = i | 0x80000000u; } }
        const uint32_t v = br_read(b, n);
        if (mode == 4) {
            const uint32_t e2 = b.wi < b.nw ? b.w[b.wi] : 0u;
            if (b.nx != e2 && !rbad) { rbad = 1; rinfo = i; rgot = b.wi - ((uint32_t)(pos >> 5)); rexp = (b.vendw << 16) | (b.iend - (b.wi >> 2)); }
        }
        const uint32_t e = ref_bits((const uint8_t *)words, nbytes, pos, n);
        if (v != e) { bad++; if (first == 0xffffffffu) { first = i; got0 = v; exp0 = e; } }
        pos += n;
        if (i % 997 == 996) { br_skip(b, 333); pos += 333; }
    }
    uint32_t *r = res + (blockIdx.x * 64 + lane) * 4;
    r[0] = bad; r[1] = first; r[2] = got0; r[3] = exp0;
    if (mode == 3 || mode == 4) { r[0] = rbad; r[1] = rinfo; r[2] = rgot; r[3] = rexp; }
}

int main() {
    const uint64_t nbytes = 4u << 20;
    std::vector<uint8_t> h(nbytes + 64);
    uint32_t x = 12345;
    for (auto &c : h) { x = x * 1664525u + 1013904223u; c = (uint8_t)(x >> 24); }
    uint32_t *d_words, *d_res;
    hipMalloc(&d_words, nbytes + 64);
    hipMemcpy(d_words, h.data(), nbytes + 64, hipMemcpyHostToDevice);
    const int nb = 32;
    hipMalloc(&d_res, nb * 64 * 16);
    int fails = 0;
    for (int mode = 0; mode < 5; mode++) {
        hipMemset(d_res, 0, nb * 64 * 16);
        hipLaunchKernelGGL(k_test, dim3(nb), dim3(64), 0, 0, d_words, nbytes, d_res, mode);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
        std::vector<uint32_t> r(nb * 64 * 4);
        hipMemcpy(r.data(), d_res, r.size() * 4, hipMemcpyDeviceToHost);
        int nbad = 0;
        for (int l = 0; l < nb * 64; l++)
            if (r[l * 4]) {
                if (nbad < 5) printf("mode %d lane %d: bad=%u first=%x got=%08x exp=%08x\n", mode, l, r[l * 4],
                                     r[l * 4 + 1], r[l * 4 + 2], r[l * 4 + 3]);
                nbad++;
            }
        printf("mode %d: %d/%d lanes with mismatches\n", mode, nbad, nb * 64);
        fails += nbad;
    }
    return fails ? 1 : 0;
}
