// xor3_variants.hip — GF(2^8) matrix-apply with the gfx950 three-input XOR
// (v_bitop3_b32, truth table 0x96) folding the three v_perm lookups of each
// word x coefficient into the accumulator: 1.5 ops per input-row instead of 3
// v_xor.  Production kernels against their xor3 variants, interleaved timing
// in one process, outputs compared byte for byte.  Not part of the product.
// Usage: xor3_variants n [iters]
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

template <int C, int R>
__global__ __launch_bounds__(256) void k_vec_x3(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint32_t acc[R][4], pend[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t w[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t* t = p.tab[r][c];
                const uint32_t p0 = __builtin_amdgcn_perm(t[1], t[0], s0), p1 = __builtin_amdgcn_perm(t[3], t[2], s1),
                               p2 = __builtin_amdgcn_perm(t[4], t[4], s2);
                if (c % 2 == 0) {
                    acc[r][q] = x3(acc[r][q], p0, p1);
                    pend[r][q] = p2;
                } else {
                    acc[r][q] = x3(acc[r][q], pend[r][q], p0);
                    acc[r][q] = x3(acc[r][q], p1, p2);
                }
            }
        }
    }
    if (C % 2) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] ^= pend[r][q];
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

template <int R>
__global__ __launch_bounds__(256) void k_loop_x3(const GfApplyParams p) {
    constexpr int G = 4;
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    const uint32_t C = p.C;  // multiple of 2 here
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    uint4 x[G], y[G];
#pragma unroll
    for (int g = 0; g < G; ++g)
        if ((uint32_t)g < C) x[g] = ld16(sbase + p.in_off[g] + off);
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < C; c0 += G) {
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (c0 + G + g < C) y[g] = ld16(sbase + p.in_off[c0 + G + g] + off);
        uint32_t pend[R][4];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t c = c0 + g;
            if (c >= C) break;
            const uint32_t w[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t* t = p.tab[r][c];
                    const uint32_t p0 = __builtin_amdgcn_perm(t[1], t[0], s0), p1 = __builtin_amdgcn_perm(t[3], t[2], s1),
                                   p2 = __builtin_amdgcn_perm(t[4], t[4], s2);
                    if (g % 2 == 0) {
                        acc[r][q] = x3(acc[r][q], p0, p1);
                        pend[r][q] = p2;
                    } else {
                        acc[r][q] = x3(acc[r][q], pend[r][q], p0);
                        acc[r][q] = x3(acc[r][q], p1, p2);
                    }
                }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) x[g] = y[g];
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

// RS(16,4) candidates.  V2: groups of 8 inputs in flight (next group's loads
// issued before the current group's arithmetic), arithmetic in halves of 4 so
// the tables of one half (80 dwords) fit in SGPRs.
template <int R>
__global__ __launch_bounds__(256) void k_loop8(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    const uint32_t C = p.C;  // multiple of 8 here
    uint32_t acc[R][4], pend[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    uint4 x[8], y[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) x[g] = ld16(sbase + p.in_off[g] + off);
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < C; c0 += 8) {
        if (c0 + 8 < C) {
#pragma unroll
            for (int g = 0; g < 8; ++g) y[g] = ld16(sbase + p.in_off[c0 + 8 + g] + off);
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const uint32_t c = c0 + g;
            const uint32_t w[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t* t = p.tab[r][c];
                    gf_fold(g & 1, acc[r][q], pend[r][q], __builtin_amdgcn_perm(t[1], t[0], s0),
                            __builtin_amdgcn_perm(t[3], t[2], s1), __builtin_amdgcn_perm(t[4], t[4], s2));
                }
            }
        }
#pragma unroll
        for (int g = 0; g < 8; ++g) x[g] = y[g];
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

// V3: all C inputs loaded up front (unrolled), tables re-read from the
// kernel-argument segment per input behind an accumulator fence (scalar
// loads), so they never pile up in VGPRs.
template <int C, int R>
__global__ __launch_bounds__(256) void k_unroll_s(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 256u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint32_t acc[R][4], pend[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3]));
        uint32_t z;
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        const uint32_t* tc = &p.tab[0][c][0] + z;
        const uint32_t w[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t* t = tc + r * (kMaxC * 5);
                gf_fold(c & 1, acc[r][q], pend[r][q], __builtin_amdgcn_perm(t[1], t[0], s0),
                        __builtin_amdgcn_perm(t[3], t[2], s1), __builtin_amdgcn_perm(t[4], t[4], s2));
            }
        }
    }
    if (C % 2) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] ^= pend[r][q];
    }
    gf_store<R>(p, obase, off, acc, stripe);
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) { if (b & 1) r ^= a; b >>= 1; a = (a << 1) ^ ((a & 0x80) ? 0x1d : 0); }
    return r;
}

static void setup(GfApplyParams& p, uint8_t* d, int K, int M, uint64_t S) {
    memset(&p, 0, sizeof(p));
    const uint64_t STRIDE = (K + M) * S;
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            const uint8_t co = (uint8_t)(0x1d * (r + 1) + 7 * c + 3);
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE;
    p.units = (uint32_t)(S / 16);
    p.chunks_per_stripe = (p.units + 255) / 256;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 12;
    const uint64_t bytes = n * (8 + 4) * 131072ull;
    uint8_t* d;
    CK(hipMalloc(&d, bytes));
    k_fill<<<4096, 256>>>(d, bytes, 5);
    GfApplyParams p84, p164;
    setup(p84, d, 8, 4, 131072);
    setup(p164, d, 16, 4, 65536);
    const uint32_t b84 = (uint32_t)(p84.chunks_per_stripe * n), b164 = (uint32_t)(p164.chunks_per_stripe * n);
    struct V { const char* name; std::function<void()> f; double alg; int geo; };
    std::vector<V> vs = {
        {"RS(8,4) vec (prod)", [&] { k_gf_apply_vec<8, 4><<<b84, 256>>>(p84); }, n * 12.0 * 131072, 0},
        {"RS(8,4) vec xor3", [&] { k_vec_x3<8, 4><<<b84, 256>>>(p84); }, n * 12.0 * 131072, 0},
        {"RS(16,4) loop (prod)", [&] { k_gf_apply_loop<4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(16,4) loop xor3", [&] { k_loop_x3<4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(16,4) loop (prod)", [&] { k_gf_apply_loop<4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(16,4) loop8", [&] { k_loop8<4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(16,4) loop (prod)", [&] { k_gf_apply_loop<4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(16,4) unroll sload", [&] { k_unroll_s<16, 4><<<b164, 256>>>(p164); }, n * 20.0 * 65536, 1},
        {"RS(8,4) vec (prod)", [&] { k_gf_apply_vec<8, 4><<<b84, 256>>>(p84); }, n * 12.0 * 131072, 0},
        {"RS(8,4) unroll sload", [&] { k_unroll_s<8, 4><<<b84, 256>>>(p84); }, n * 12.0 * 131072, 0},
    };
    // correctness: each variant's parity against the production kernel of its geometry
    std::vector<uint8_t> ref, got;
    for (size_t v = 0; v < vs.size(); ++v) {
        const uint64_t S = vs[v].geo ? 65536 : 131072, K = vs[v].geo ? 16 : 8;
        const uint64_t stride = (K + 4) * S, last = (n - 1) * stride + K * S;
        CK(hipMemset(d + last, 0, 4 * S));
        vs[v].f();
        CK(hipDeviceSynchronize());
        std::vector<uint8_t>& dst = (v % 2 == 0) ? ref : got;
        dst.resize(4 * S);
        CK(hipMemcpy(dst.data(), d + last, 4 * S, hipMemcpyDeviceToHost));
        if (v % 2 == 1) printf("%s: parity %s\n", vs[v].name, memcmp(ref.data(), got.data(), 4 * S) ? "MISMATCH" : "ok");
    }
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
        }
    // back-to-back launches (as bench.py times them): 20 in a row, events between
    for (size_t v : {(size_t)0, (size_t)5}) {
        std::vector<hipEvent_t> ev(21);
        for (auto& e : ev) CK(hipEventCreate(&e));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ev[0]));
        for (int i = 0; i < 20; ++i) {
            vs[v].f();
            CK(hipEventRecord(ev[i + 1]));
        }
        CK(hipEventSynchronize(ev[20]));
        float tot = 0, mx = 0;
        for (int i = 0; i < 20; ++i) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            tot += ms;
            mx = std::max(mx, ms);
        }
        printf("%-22s back-to-back x20: avg %.4f ms max %.4f\n", vs[v].name, tot / 20, mx);
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("%-22s med %.4f ms min %.4f -> %.1f GB/s (%.1f%% of 8 TB/s)\n", vs[v].name, med, x[0],
               vs[v].alg / (med * 1e-3) / 1e9, 100 * vs[v].alg / (med * 1e-3) / 8e12);
    }
    return 0;
}
