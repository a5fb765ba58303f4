// skew_probe.hip — is the stripe-walking pattern's HBM deficit address
// aliasing?  The walk of walk_probe.hip (every wave streams one stripe's
// 8 data shards in and 4 parity shards out, 1 KiB per shard per step) over
// layouts whose shard pitch and stripe stride are padded by a skew, so the
// thousands of walks in flight stop landing on the same HBM channel/bank
// offsets.  Also the production sweep-order encode kernel on the same
// layouts.  Measurement code.  Usage: skew_probe [n]
#include "../../rustfs_amd/csrc/rs_kernels.hip"
#include "../../rustfs_amd/csrc/gf_bitslice.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;
constexpr int K = 8, M = 4;
constexpr uint32_t S = 131072;

__global__ __launch_bounds__(256) void k_walk(uint8_t* base, uint32_t n, uint64_t pitch, uint64_t stride) {
    const uint32_t stripe = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (stripe >= n) return;
    uint8_t* sb = base + (uint64_t)stripe * stride + lane * 16u;
    constexpr uint32_t P = 1024, steps = S / P;
    uint4 a[K], b[K];
    auto load = [&](uint4 (&x)[K], uint32_t st) {
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = *(const uint4*)(sb + c * pitch + st * P);
    };
    auto work = [&](uint4 (&x)[K], uint32_t st) {
#pragma unroll
        for (int r = 0; r < M; ++r) {
            uint4 v = x[r];
            v.x ^= x[r + 4].x; v.y ^= x[r + 4].y; v.z ^= x[r + 4].z; v.w ^= x[r + 4].w;
            *(uint4*)(sb + (K + r) * pitch + st * P) = v;
        }
    };
    load(a, 0);
    for (uint32_t st = 0; st < steps; st += 2) {
        if (st + 1 < steps) load(b, st + 1);
        work(a, st);
        if (st + 1 >= steps) break;
        if (st + 2 < steps) load(a, st + 2);
        work(b, st + 1);
    }
}


// W waves per stripe, wave w streams KiB column (step*W + w): the workgroup's
// step covers W contiguous KiB of every shard.  LDS pads the occupancy.
template <int W>
__global__ __launch_bounds__(64 * W) void k_walk_w(uint8_t* base, uint32_t n) {
    extern __shared__ uint8_t pad[];
    if (n == 0xFFFFFFFFu) pad[threadIdx.x] = 0;
    const uint32_t stripe = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint8_t* sb = base + (uint64_t)stripe * ((K + M) * (uint64_t)S) + w * 1024u + lane * 16u;
    constexpr uint32_t P = 1024 * W, steps = S / P;
    uint4 a[K], b[K];
    auto load = [&](uint4 (&x)[K], uint32_t st) {
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = *(const uint4*)(sb + c * (uint64_t)S + st * P);
    };
    auto work = [&](uint4 (&x)[K], uint32_t st) {
#pragma unroll
        for (int r = 0; r < M; ++r) {
            uint4 v = x[r];
            v.x ^= x[r + 4].x; v.y ^= x[r + 4].y; v.z ^= x[r + 4].z; v.w ^= x[r + 4].w;
            *(uint4*)(sb + (K + r) * (uint64_t)S + st * P) = v;
        }
    };
    load(a, 0);
    for (uint32_t st = 0; st < steps; st += 2) {
        if (st + 1 < steps) load(b, st + 1);
        work(a, st);
        if (st + 1 >= steps) break;
        if (st + 2 < steps) load(a, st + 2);
        work(b, st + 1);
    }
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + seed) * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    struct Cfg { uint64_t pad_shard, pad_stripe; };
    std::vector<Cfg> cfgs = {{0, 0}};
    const uint64_t maxb = (uint64_t)n * ((K + M) * (S + 4096) + 65536);
    uint8_t* d;
    CK(hipMalloc(&d, maxb));
    k_fill<<<4096, 256>>>(d, maxb, 3);
    CK(hipDeviceSynchronize());
    constexpr bs::EncodeRows<K, M> E{};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double alg = (double)n * (K + M) * S;
    for (auto& c : cfgs) {
        const uint64_t pitch = S + c.pad_shard, stride = (K + M) * pitch + c.pad_stripe;
        GfApplyParams p;
        memset(&p, 0, sizeof(p));
        p.base = d; p.out_base = d; p.stripe_stride = stride; p.out_stripe_stride = stride;
        for (int i = 0; i < K; ++i) p.in_off[i] = i * pitch;
        for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * pitch;
        for (int r = 0; r < M; ++r)
            for (int i = 0; i < K; ++i) {
                const uint8_t co = E.g[r][i];
                auto pack = [&](int sh, int f) { uint32_t v = 0; for (int q = 0; q < 4; ++q) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + q) << sh)) << (8 * q); return v; };
                p.tab[r][i][0] = pack(0, 0); p.tab[r][i][1] = pack(0, 4); p.tab[r][i][2] = pack(3, 0); p.tab[r][i][3] = pack(3, 4); p.tab[r][i][4] = pack(6, 0);
            }
        p.C = K; p.R = M; p.mode = GF_MODE_STORE; p.units = S / 16;
        std::vector<float> tw, te;
        for (int it = 0; it < 10; ++it) {
            float ms;
            CK(hipEventRecord(a));
            k_walk<<<(n + 3) / 4, 256>>>(d, n, pitch, stride);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) tw.push_back(ms);
            CK(hipEventRecord(a));
            CK(launch_gf_apply_vec(p, n, 0));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) te.push_back(ms);
        }
        std::sort(tw.begin(), tw.end());
        std::sort(te.begin(), te.end());
        const float mw = tw[tw.size() / 2], me = te[te.size() / 2];
        printf("shard pad %5llu stripe pad %5llu: walk %.4f ms (%.1f%%)  encode-sweep %.4f ms (%.1f%%)\n",
               (unsigned long long)c.pad_shard, (unsigned long long)c.pad_stripe, mw, 100 * alg / (mw * 1e-3) / 8e12, me,
               100 * alg / (me * 1e-3) / 8e12);
    }
    // W waves per stripe, LDS-limited residency
    {
        struct WC { int W; uint32_t lds; };
        std::vector<WC> wcs;
        for (int W : {1, 2, 4, 8, 16})
            for (uint32_t lds : {160u << 10, 80u << 10, 40u << 10, 20u << 10, 0u}) wcs.push_back({W, lds});
        auto pick = [](int W) -> void (*)(uint8_t*, uint32_t) {
            switch (W) { case 1: return k_walk_w<1>; case 2: return k_walk_w<2>; case 4: return k_walk_w<4>;
                         case 8: return k_walk_w<8>; default: return k_walk_w<16>; }
        };
        for (int W : {1, 2, 4, 8, 16})
            CK(hipFuncSetAttribute((const void*)pick(W), hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10));
        for (auto& c : wcs) {
            std::vector<float> tw;
            for (int it = 0; it < 8; ++it) {
                float ms;
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(pick(c.W), dim3(n), dim3(64 * c.W), c.lds, 0, d, n);
                CK(hipGetLastError());
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                if (it > 1) tw.push_back(ms);
            }
            std::sort(tw.begin(), tw.end());
            int nb = 0;
            CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pick(c.W), 64 * c.W, c.lds));
            const float mw = tw[tw.size() / 2];
            printf("walk W=%2d waves/stripe (%2d KiB per shard per step), %3d stripes per CU: %.4f ms (%.1f%%)\n", c.W,
                   c.W, nb, mw, 100 * alg / (mw * 1e-3) / 8e12);
        }
    }
    return 0;
}
