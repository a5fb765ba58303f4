// op_rates.hip — issue cost of the VALU ops the HighwayHash update uses, on
// gfx950: 8 independent chains per lane, 8 waves per SIMD, reported as SIMD
// cycles per wave-instruction (2.0 = full rate for a wave64 op on SIMD32).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t* out, uint64_t seed) {
    const uint32_t seed_s = (uint32_t)seed;
    uint64_t a[8];
    uint32_t b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + i + 1); b[i] = (uint32_t)(a[i] >> 7) | 1u; }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
            if constexpr (OP == 1) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(a[i]) : "v"(b[i]) : "vcc");
            if constexpr (OP == 2) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "v"(0x05020C03u));
            if constexpr (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 4) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %1, vcc" : "+v"(b[i]), "+v"(b[(i + 4) & 7]) ,"+v"(b[(i+2)&7]) : : "vcc");
            if constexpr (OP == 5) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 7) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 8) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "s"(seed_s));
            if constexpr (OP == 9) asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 10) asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(b[i]) : "s"(seed_s));
            if constexpr (OP == 11) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "v"(b[(i + 3) & 7]));
            if constexpr (OP == 12) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "s"(seed_s));
            if constexpr (OP == 13) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(b[i]));
            if constexpr (OP == 14) asm volatile("v_bfe_u32 %0, %0, 3, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 15) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "v"(b[(i + 3) & 7]));
            if constexpr (OP == 16) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a[i]) : "s"(seed));
            if constexpr (OP == 17) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(b[i]) : "s"(seed_s));
            if constexpr (OP == 18) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
            if constexpr (OP == 19) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "v"(b[(i + 3) & 7]));
            if constexpr (OP == 20) asm volatile("v_and_b32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
        }
    }
    uint64_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i] ^ b[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
float run(uint64_t* d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<OP><<<blocks, 256>>>(d, 3);
    hipEventRecord(a);
    k<OP><<<blocks, 256>>>(d, 5);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char** argv) {
    // default 8 blocks of 4 waves per CU = 8 waves per SIMD; argv[1] = waves per SIMD
    const int wps = argc > 1 ? atoi(argv[1]) : 8;
    const int blocks = 256 * wps;
    uint64_t* d;
    CK(hipMalloc(&d, (size_t)blocks * 256 * 8));
    const char* names[] = {"v_lshl_add_u64 v,v", "v_mad_u64_u32", "v_perm_b32 v,v,v", "v_xor_b32 v,v", "add_co+addc (2 ops)",
                           "v_mov_b32_dpp", "v_mul_lo_u32", "v_mul_hi_u32", "v_perm_b32 v,v,s", "v_perm_b32 x,x,v",
                           "v_perm_b32 s,s,v", "v_add3_u32 v,v,v", "v_and_or_b32 v,v,s", "v_lshrrev_b32 imm", "v_bfe_u32",
                           "v_xad_u32 v,v,v", "v_lshl_add_u64 s,v", "v_xor_b32 s,v", "v_perm_b32 v0,v0,v",
                           "v_bitop3_b32 xor3", "v_and_b32 v,v"};
    float ms[21] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks),
                    run<5>(d, blocks), run<6>(d, blocks), run<7>(d, blocks), run<8>(d, blocks), run<9>(d, blocks),
                    run<10>(d, blocks), run<11>(d, blocks), run<12>(d, blocks), run<13>(d, blocks), run<14>(d, blocks),
                    run<15>(d, blocks), run<16>(d, blocks), run<17>(d, blocks), run<18>(d, blocks), run<19>(d, blocks), run<20>(d, blocks)};
    const double waves_per_simd = wps, clk = 2.1e9;
    for (int i = 0; i < 21; ++i) {
        const double ops = waves_per_simd * ITERS * 8;  // wave-ops per SIMD
        printf("%-22s %.3f ms  ~%.2f SIMD cycles per wave-op (at %.1f GHz)\n", names[i], ms[i], ms[i] * 1e-3 * clk / ops,
               clk / 1e9);
    }
    return 0;
}
