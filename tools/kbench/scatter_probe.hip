// scatter_probe.hip — does HBM throughput depend on how many stripes are
// streamed at once (piece size per shard per visit)?  The production encode
// kernel with the block -> (stripe, column) mapping changed: G consecutive
// 1 KiB columns of one stripe per group of blocks, groups round-robin over the
// stripes (G = S / 1 KiB: the production order, one stripe at a time; G = 1:
// every stripe advanced 1 KiB at a time, like a kernel that walks all stripes
// in lockstep).  Measurement code.  Usage: scatter_probe [n]
#include "../../rustfs_amd/csrc/rs_kernels.hip"
#include "../../rustfs_amd/csrc/gf_bitslice.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

// one wave per block: 64 lanes x 16 B = 1 KiB column of every shard; PIECE
// bytes per lane-group: lanes cover PIECE-byte runs of 1024/PIECE stripes
template <int C, int R>
__global__ __launch_bounds__(64) void k_probe(const GfApplyParams p, uint32_t n, uint32_t cols, uint32_t G,
                                             uint32_t piece) {
    // group g = blockIdx / G; within a group, column = (g / n_groups_per_col)..
    const uint32_t b = blockIdx.x;
    const uint32_t per_piece_stripes = 1024u / piece;  // stripes one block touches
    const uint32_t sgroups = n / per_piece_stripes;
    const uint32_t colpieces = cols * (1024u / piece);  // piece-columns per stripe
    // block -> (stripe group sg, piece column pc): G consecutive piece columns per stripe group
    const uint32_t grp = b / G, within = b % G;
    const uint32_t sg = grp % sgroups, pc = (grp / sgroups) * G + within;
    if (pc >= colpieces) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t stripe = sg * per_piece_stripes + lane / (piece / 16u);
    const uint64_t off = (uint64_t)pc * piece + (lane % (piece / 16u)) * 16u;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    gf_accumulate<0, C, R>(p, x, acc);
    gf_store<R>(p, obase, off, acc, stripe);
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    constexpr int K = 8, M = 4;
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    const uint64_t S = 131072, STRIDE = (K + M) * S;
    uint8_t* d;
    CK(hipMalloc(&d, (uint64_t)n * STRIDE));
    k_fill<<<4096, 256>>>(d, (uint64_t)n * STRIDE, 3);
    constexpr bs::EncodeRows<K, M> E{};
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            const uint8_t co = E.g[r][c];
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE; p.units = S / 16;
    const uint32_t cols = S / 1024;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Cfg { uint32_t piece, G; };
    std::vector<Cfg> cfgs;
    for (uint32_t piece : {1024u, 512u, 256u})
        for (uint32_t G : {1u, 2u, 4u, 16u, 128u * (1024u / piece)}) cfgs.push_back({piece, G});
    std::vector<std::vector<float>> t(cfgs.size() + 1);
    for (int it = 0; it < 10; ++it) {
        for (size_t v = 0; v < cfgs.size(); ++v) {
            const uint32_t blocks = n * cols;  // one block per 1 KiB of every shard per stripe
            CK(hipEventRecord(a));
            k_probe<K, M><<<blocks, 64>>>(p, n, cols, cfgs[v].G, cfgs[v].piece);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t[v].push_back(ms);
        }
        CK(hipEventRecord(a));
        CK(launch_gf_apply_vec(p, n, 0));
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it > 1) t[cfgs.size()].push_back(ms);
    }
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v <= cfgs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        if (v < cfgs.size()) printf("piece %4u G %4u", cfgs[v].piece, cfgs[v].G);
        else printf("production      ");
        printf("  med %.4f ms -> %.1f GB/s (%.1f%%)\n", x[x.size() / 2], alg / (x[x.size() / 2] * 1e-3) / 1e9,
               100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
