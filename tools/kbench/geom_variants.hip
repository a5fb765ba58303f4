// geom_variants.hip — microbenchmark of GF matrix-apply variants for a given
// geometry (compile with -DKK=16 -DMM=4 -DSS=65536), n stripes device-resident,
// interleaved timing in one process.  Checks every variant's parity against the
// library kernel.  Not part of the product.
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stddef.h>

#include <algorithm>
#include <functional>
#include <vector>

#ifndef KK
#define KK 16
#endif
#ifndef MM
#define MM 4
#endif
#ifndef SS
#define SS 65536
#endif

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

// Rolled over inputs in groups of G, next group's loads issued before the
// current group's arithmetic; tables indexed by the (scalar) loop counter.
template <int R, int G>
__global__ __launch_bounds__(256) void k_loop(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    uint4 x[G], y[G];
#pragma unroll
    for (int g = 0; g < G; ++g) x[g] = ld16(sbase + p.in_off[g] + off);
    const uint32_t C = p.C;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < C; c0 += G) {
        if (c0 + G < C) {
#pragma unroll
            for (int g = 0; g < G; ++g) y[g] = ld16(sbase + p.in_off[c0 + G + g] + off);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t c = c0 + g;
            const uint32_t w[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u;
                const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
                const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(p.tab[r][c], s0, s1, s2);
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) x[g] = y[g];
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

// Table dwords of coefficient (r, c) loaded where used: an opaque zero offset
// stops the compiler hoisting all C*R*5 dwords into (spilled) SGPRs.
// (Read straight from the kernel-argument segment: taking &p.tab of the by-value
// parameter would copy the whole struct to scratch.)
__device__ __forceinline__ const uint32_t* tab_at(const GfApplyParams&, int r, int c) {
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
    const uint8_t* ka = (const uint8_t*)__builtin_amdgcn_kernarg_segment_ptr();
    return (const uint32_t*)(ka + offsetof(GfApplyParams, tab) + ((size_t)(r * kMaxC + c) * 5) * 4 + z);
}

template <int C0, int CN, int R>
__device__ __forceinline__ void gf_acc_late(const GfApplyParams& p, const uint4* x, uint32_t (&acc)[R][4]) {
#pragma unroll
    for (int i = 0; i < CN; ++i) {
        const int c = C0 + i;
        const uint32_t w[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
        const uint32_t* tb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) tb[r] = tab_at(p, r, c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t s0 = w[q] & 0x07070707u;
            const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
            const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(tb[r], s0, s1, s2);
        }
    }
}

// Two halves of a 512-thread block split the inputs (C0 = C/2 each) of the
// same 16-byte units; the upper half hands its partial sums over LDS.
template <int C, int R>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_split(const GfApplyParams p) {
    constexpr int H = C / 2;
    __shared__ uint32_t part[R * 4][256];
    const uint32_t half = threadIdx.x >> 8, t = threadIdx.x & 255u;
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + t;
    const bool ok = u < p.units;
    const uint64_t off = (uint64_t)(ok ? u : 0) * 16u;
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    uint4 x[H];
    if (__builtin_amdgcn_readfirstlane(half) == 0) {
#pragma unroll
        for (int i = 0; i < H; ++i) x[i] = ld16(sbase + p.in_off[i] + off);
        gf_acc_late<0, H, R>(p, x, acc);
    } else {
#pragma unroll
        for (int i = 0; i < H; ++i) x[i] = ld16(sbase + p.in_off[H + i] + off);
        gf_acc_late<H, H, R>(p, x, acc);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) part[r * 4 + q][t] = acc[r][q];
    }
    __syncthreads();
    if (half == 0 && ok) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] ^= part[r * 4 + q][t];
        gf_store<R>(p, obase, off, acc, stripe);
    }
}

// Compile-time C, 8-byte units (uint2): 32 VGPRs of inputs at C = 16.
template <int C, int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_narrow(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / (p.chunks_per_stripe * 2);
    const uint32_t chunk = blockIdx.x - stripe * (p.chunks_per_stripe * 2);
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;  // 8-byte unit
    if (u >= p.units * 2) return;
    const uint64_t off = (uint64_t)u * 8u;
    uint2 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = *(const uint2*)(sbase + p.in_off[c] + off);
    uint32_t acc[R][2];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = 0u;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t w[2] = {x[c].x, x[c].y};
        const uint32_t* tb[R];
#pragma unroll
        for (int r = 0; r < R; ++r) tb[r] = tab_at(p, r, c);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t s0 = w[q] & 0x07070707u;
            const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
            const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(tb[r], s0, s1, s2);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) *(uint2*)(obase + p.out_off[r] + off) = make_uint2(acc[r][0], acc[r][1]);
}

// Compile-time C, rolled groups of G (fully unrolled by the compiler).
template <int C, int R, int G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_cloop(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    uint4 x[G], y[G];
#pragma unroll
    for (int g = 0; g < G; ++g) x[g] = ld16(sbase + p.in_off[g] + off);
#pragma unroll
    for (int c0 = 0; c0 < C; c0 += G) {
        if (c0 + G < C) {
#pragma unroll
            for (int g = 0; g < G; ++g) y[g] = ld16(sbase + p.in_off[c0 + G + g] + off);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int c = c0 + g;
            const uint32_t w[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
            const uint32_t* tb[R];
#pragma unroll
            for (int r = 0; r < R; ++r) tb[r] = tab_at(p, r, c);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u;
                const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
                const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(tb[r], s0, s1, s2);
            }
        }
        if (c0 + G < C) {
#pragma unroll
            for (int g = 0; g < G; ++g) x[g] = y[g];
        }
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) { if (b & 1) r ^= a; b >>= 1; a = (a << 1) ^ ((a & 0x80) ? 0x1d : 0); }
    return r;
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 15;
    const uint64_t S = SS, STRIDE = (uint64_t)(KK + MM) * S;
    uint8_t* d;
    CK(hipMalloc(&d, n * STRIDE));
    k_fill<<<4096, 256>>>(d, n * STRIDE, 7);
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < KK; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < MM; ++r) p.out_off[r] = (KK + r) * S;
    for (int r = 0; r < MM; ++r)
        for (int c = 0; c < KK; ++c) {
            const uint8_t co = (uint8_t)(0x1b + 37 * r + 11 * c);  // arbitrary nonzero coefficients
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = KK; p.R = MM; p.mode = GF_MODE_STORE; p.units = S / 16;
    p.chunks_per_stripe = (p.units + 255) / 256;
    const uint32_t blocks = p.chunks_per_stripe * n;
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {
        {"library vec", [&] { CK(launch_gf_apply_vec(p, n, 0)); }},
        {"loop G=2", [&] { k_loop<MM, 2><<<blocks, 256>>>(p); }},
        {"loop G=4", [&] { k_loop<MM, 4><<<blocks, 256>>>(p); }},
        {"loop G=8", [&] { k_loop<MM, 8><<<blocks, 256>>>(p); }},
        {"split 512", [&] { k_split<KK, MM><<<blocks, 512>>>(p); }},
        {"narrow 8B", [&] { k_narrow<KK, MM><<<blocks * 2, 256>>>(p); }},
        {"cloop G=4", [&] { k_cloop<KK, MM, 4><<<blocks, 256>>>(p); }},
        {"cloop G=8", [&] { k_cloop<KK, MM, 8><<<blocks, 256>>>(p); }},
    };
    std::vector<uint8_t> ref(MM * S), got(MM * S);
    vs[0].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), d + (n - 1) * STRIDE + KK * S, MM * S, hipMemcpyDeviceToHost));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> t(vs.size());
    for (int it = 0; it < iters; ++it)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(a));
            vs[v].f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it) t[v].push_back(ms);
            if (!it) {
                CK(hipMemcpy(got.data(), d + (n - 1) * STRIDE + KK * S, MM * S, hipMemcpyDeviceToHost));
                if (memcmp(got.data(), ref.data(), MM * S)) printf("%s: MISMATCH\n", vs[v].name);
            }
        }
    const double alg = (double)n * STRIDE;
    printf("RS(%d,%d) S=%llu n=%llu\n", KK, MM, (unsigned long long)S, (unsigned long long)n);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("%-14s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", vs[v].name, x[x.size() / 2], x[0],
               alg / (x[x.size() / 2] * 1e-3) / 1e9, 100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
