// recon_variants.hip — reconstruct-shaped GF apply (C = 8 survivors, R = 1..2
// rebuilt shards) with 1 or 2 16-byte units per thread: with few outputs the
// kernel holds few registers, so more bytes per lane can be in flight.
// Outputs compared byte for byte with the production kernel.  Not part of the
// product.  Usage: recon_variants n [iters]
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

// U units per thread, unit u at chunk*256*U + u*256 + t (coalesced per unit)
template <int C, int R, int U>
__global__ __launch_bounds__(256) void k_vec_u(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    uint4 x[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t unit = (chunk * U + u) * 256u + threadIdx.x;
        if (unit < p.units) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[u][c] = ld16(sbase + p.in_off[c] + (uint64_t)unit * 16u);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t unit = (chunk * U + u) * 256u + threadIdx.x;
        if (unit >= p.units) continue;
        uint32_t acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
        gf_accumulate<0, C, R>(p, x[u], acc);
        gf_store<R>(p, obase, (uint64_t)unit * 16u, acc, stripe);
    }
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

static void setup(GfApplyParams& p, uint8_t* d, int C, int R, uint64_t S) {
    memset(&p, 0, sizeof(p));
    const uint64_t STRIDE = 12 * S;
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < C; ++c) p.in_off[c] = (c + 1) * S;  // survivors 1..8 (shard 0 lost)
    for (int r = 0; r < R; ++r) p.out_off[r] = (r == 0 ? 0 : 9 + r) * S;
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < C; ++c) {
            const uint8_t co = (uint8_t)(0x53 * (r + 1) + 11 * c + 5);
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = C; p.R = R; p.mode = GF_MODE_STORE; p.units = (uint32_t)(S / 16);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t S = 131072, bytes = n * 12 * S;
    uint8_t* d;
    CK(hipMalloc(&d, bytes));
    k_fill<<<4096, 256>>>(d, bytes, 9);
    GfApplyParams p1, p2;
    setup(p1, d, 8, 1, S);
    setup(p2, d, 8, 2, S);
    auto grid = [&](GfApplyParams& p, int U) { p.chunks_per_stripe = (p.units + 256 * U - 1) / (256 * U); return (uint32_t)(p.chunks_per_stripe * n); };
    struct V { const char* name; std::function<void()> f; double alg; int R; };
    std::vector<V> vs = {
        {"e1 prod", [&] { GfApplyParams q = p1; CK(launch_gf_apply_vec(q, n, 0)); }, n * 9.0 * S, 1},
        {"e1 U=2", [&] { GfApplyParams q = p1; uint32_t g = grid(q, 2); k_vec_u<8, 1, 2><<<g, 256>>>(q); }, n * 9.0 * S, 1},
        {"e2 prod", [&] { GfApplyParams q = p2; CK(launch_gf_apply_vec(q, n, 0)); }, n * 10.0 * S, 2},
        {"e2 U=2", [&] { GfApplyParams q = p2; uint32_t g = grid(q, 2); k_vec_u<8, 2, 2><<<g, 256>>>(q); }, n * 10.0 * S, 2},
    };
    for (size_t v = 0; v < vs.size(); v += 2) {
        const uint64_t last = (n - 1) * 12 * S;
        std::vector<uint8_t> a(S), b(S);
        CK(hipMemset(d + last, 0, S));
        vs[v].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(a.data(), d + last, S, hipMemcpyDeviceToHost));
        CK(hipMemset(d + last, 0, S));
        vs[v + 1].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(b.data(), d + last, S, hipMemcpyDeviceToHost));
        printf("%s vs %s: %s\n", vs[v].name, vs[v + 1].name, memcmp(a.data(), b.data(), S) ? "MISMATCH" : "ok");
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int it = 0; it < iters; ++it)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0));
            vs[v].f();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 2) t[v].push_back(ms);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("%-8s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", vs[v].name, med, x[0], vs[v].alg / (med * 1e-3) / 1e9,
               100 * vs[v].alg / (med * 1e-3) / 8e12);
    }
    return 0;
}
