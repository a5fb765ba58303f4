// bs_variants.hip — bit-sliced GF(2^8) encode (gf_bitslice.h) against the
// production table kernels, interleaved timing in one process, parity compared
// byte for byte.  Not part of the product.
// Usage: bs_variants n [iters]
#include "../../rustfs_amd/csrc/rs_kernels.hip"
#include "../../rustfs_amd/csrc/gf_bitslice.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

template <int K, int M>
__global__ __launch_bounds__(256) void k_bs(const GfApplyParams p) {
    constexpr bs::Terms<K, M> T{};
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t col = chunk * 4u + (threadIdx.x >> 6);  // 2 KiB column of this wave
    if (col >= p.units) return;
    const uint64_t off = (uint64_t)col * 2048u + (threadIdx.x & 63u) * 16u;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    uint32_t Q[K][8];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint4 a = ld16(sbase + p.in_off[c] + off), b = ld16(sbase + p.in_off[c] + off + 1024);
        Q[c][0] = a.x; Q[c][1] = a.y; Q[c][2] = a.z; Q[c][3] = a.w;
        Q[c][4] = b.x; Q[c][5] = b.y; Q[c][6] = b.z; Q[c][7] = b.w;
        bs::transpose(Q[c], m4, m2, m1);
    }
    const uint32_t* P = &Q[0][0];
#pragma unroll
    for (int r = 0; r < M; ++r) {
        uint32_t o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            constexpr int NMAX = K * 8;
            const int n = T.n[r][i];
            uint32_t a = n ? P[T.idx[r][i][0]] : 0u;
#pragma unroll
            for (int t = 1; t < NMAX; t += 2) {
                if (t + 1 < n) a = x3(a, P[T.idx[r][i][t]], P[T.idx[r][i][t + 1]]);
                else if (t < n) a ^= P[T.idx[r][i][t]];
            }
            o[i] = a;
        }
        bs::transpose(o, m4, m2, m1);
        st16(obase + p.out_off[r] + off, make_uint4(o[0], o[1], o[2], o[3]));
        st16(obase + p.out_off[r] + off + 1024, make_uint4(o[4], o[5], o[6], o[7]));
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

static void setup(GfApplyParams& p, uint8_t* d, int K, int M, uint64_t S, const uint8_t* rows) {
    memset(&p, 0, sizeof(p));
    const uint64_t STRIDE = (K + M) * S;
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            const uint8_t co = rows[r * K + c];
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE;
}

struct Geo {
    int K, M;
    uint64_t S;
    GfApplyParams pt, pb;
    uint32_t bt, bb;
    std::function<void()> prod, bsk;
};

template <int K, int M>
static Geo make_geo(uint8_t* d, uint64_t n, uint64_t S) {
    constexpr bs::EncodeRows<K, M> E{};
    Geo g;
    g.K = K; g.M = M; g.S = S;
    setup(g.pt, d, K, M, S, &E.g[0][0]);
    g.pb = g.pt;
    g.pt.units = (uint32_t)(S / 16);
    g.pt.chunks_per_stripe = (g.pt.units + 255) / 256;
    g.bt = (uint32_t)(g.pt.chunks_per_stripe * n);
    g.pb.units = (uint32_t)(S / 2048);
    g.pb.chunks_per_stripe = (g.pb.units + 3) / 4;
    g.bb = (uint32_t)(g.pb.chunks_per_stripe * n);
    return g;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 12;
    const uint64_t bytes = n * (8 + 8) * 131072ull;  // largest geometry: RS(8,8) 1 MiB stripes
    uint8_t* d;
    CK(hipMalloc(&d, bytes));
    k_fill<<<4096, 256>>>(d, bytes, 5);
    std::vector<Geo> gs;
    gs.push_back(make_geo<8, 4>(d, n, 131072));
    gs.push_back(make_geo<16, 4>(d, n, 65536));
    gs.push_back(make_geo<8, 8>(d, n, 131072));
    gs.push_back(make_geo<4, 4>(d, n, 262144));
    gs.push_back(make_geo<2, 2>(d, n, 524288));
    for (auto& g : gs) {
        GfApplyParams* pt = &g.pt; GfApplyParams* pb = &g.pb;
        uint32_t bt = g.bt, bb = g.bb;
        const int K = g.K, M = g.M;
        g.prod = [=] { hipLaunchKernelGGL(pick_vec(K, M), dim3(bt), dim3(256), 0, 0, *pt); };
        if (K == 8 && M == 4) g.bsk = [=] { k_bs<8, 4><<<bb, 256>>>(*pb); };
        if (K == 16 && M == 4) g.bsk = [=] { k_bs<16, 4><<<bb, 256>>>(*pb); };
        if (K == 8 && M == 8) g.bsk = [=] { k_bs<8, 8><<<bb, 256>>>(*pb); };
        if (K == 4 && M == 4) g.bsk = [=] { k_bs<4, 4><<<bb, 256>>>(*pb); };
        if (K == 2 && M == 2) g.bsk = [=] { k_bs<2, 2><<<bb, 256>>>(*pb); };
    }
    // correctness: parity of the last stripe, every geometry
    for (auto& g : gs) {
        const uint64_t stride = (g.K + g.M) * g.S, last = (n - 1) * stride + g.K * g.S, pb = g.M * g.S;
        std::vector<uint8_t> ref(pb), got(pb);
        CK(hipMemset(d + last, 0, pb));
        g.prod();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), d + last, pb, hipMemcpyDeviceToHost));
        CK(hipMemset(d + last, 0, pb));
        g.bsk();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), d + last, pb, hipMemcpyDeviceToHost));
        printf("RS(%d,%d) bitsliced parity %s\n", g.K, g.M, memcmp(ref.data(), got.data(), pb) ? "MISMATCH" : "ok");
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> t(gs.size() * 2);
    for (int it = 0; it < iters; ++it)
        for (size_t v = 0; v < t.size(); ++v) {
            CK(hipEventRecord(a));
            if (v % 2) gs[v / 2].bsk(); else gs[v / 2].prod();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t[v].push_back(ms);
        }
    for (size_t v = 0; v < t.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        const Geo& g = gs[v / 2];
        const double alg = (double)n * (g.K + g.M) * g.S, med = x[x.size() / 2];
        printf("RS(%2d,%d) %-10s med %.4f ms min %.4f -> %.1f GB/s (%.1f%% of 8 TB/s)\n", g.K, g.M,
               v % 2 ? "bitsliced" : "table", med, x[0], alg / (med * 1e-3) / 1e9, 100 * alg / (med * 1e-3) / 8e12);
    }
    return 0;
}
