// walk_probe.hip — HBM rate of the fused kernel's memory pattern without its
// arithmetic: every wave walks ONE stripe front to back in steps of P bytes
// per shard (8 data loads, 4 parity stores per step, next step's loads in
// flight), W waves per CU (LDS pads the occupancy), so W x 256 stripes are
// streamed at once.  Measurement code.  Usage: walk_probe [n]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int K = 8, M = 4;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint64_t S = 131072, STRIDE = (K + M) * S;

template <int U, int MODE>  // U x 1 KiB per shard per step; MODE 0 rw, 1 reads only, 2 writes only
__global__ __launch_bounds__(256) void k_walk(uint8_t* base, uint32_t n, uint32_t pad) {
    extern __shared__ uint8_t dummy[];
    if (pad == 12345) dummy[threadIdx.x] = 0;  // occupancy limiter only
    const uint32_t stripe = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (stripe >= n) return;
    uint8_t* sb = base + (uint64_t)stripe * STRIDE + lane * 16u;
    constexpr uint32_t P = 1024 * U;
    const uint32_t steps = S / P;
    uint4 a[K][U], b[K][U];
    uint4 sink = make_uint4(0, 0, 0, 0);
    auto load = [&](uint4 (&x)[K][U], uint32_t st) {
        if (MODE == 2) {
#pragma unroll
            for (int c = 0; c < K; ++c)
#pragma unroll
                for (int u = 0; u < U; ++u) x[c][u] = make_uint4(st, c, u, lane);
            return;
        }
#pragma unroll
        for (int c = 0; c < K; ++c)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (MODE == 4) {
                    const v4u w = __builtin_nontemporal_load((const v4u*)(sb + c * S + st * P + u * 1024));
                    x[c][u] = make_uint4(w.x, w.y, w.z, w.w);
                } else {
                    x[c][u] = *(const uint4*)(sb + c * S + st * P + u * 1024);
                }
    };
    auto work = [&](uint4 (&x)[K][U], uint32_t st) {
#pragma unroll
        for (int r = 0; r < M; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint4 v = x[r][u];
                v.x ^= x[r + 4][u].x; v.y ^= x[r + 4][u].y; v.z ^= x[r + 4][u].z; v.w ^= x[r + 4][u].w;
                if (MODE == 1) {
                    sink.x ^= v.x; sink.y ^= v.y; sink.z ^= v.z; sink.w ^= v.w;
                } else if (MODE >= 3) {
                    v4u w = {v.x, v.y, v.z, v.w};
                    __builtin_nontemporal_store(w, (v4u*)(sb + (K + r) * S + st * P + u * 1024));
                } else {
                    *(uint4*)(sb + (K + r) * S + st * P + u * 1024) = v;
                }
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
    if (MODE == 1 && (sink.x ^ sink.y ^ sink.z ^ sink.w) == 0x12345678u) *(uint4*)sb = sink;
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + seed) * 0x9E3779B97F4A7C15ull;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    uint8_t* d;
    CK(hipMalloc(&d, (uint64_t)n * STRIDE));
    k_fill<<<4096, 256>>>(d, (uint64_t)n * STRIDE, 3);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Cfg { int U; uint32_t lds; int mode; };
    // LDS per 4-wave block: 160 KiB -> 1 block (4 waves) per CU, 80 -> 2, 40 -> 4, 20 -> 8
    std::vector<Cfg> cfgs;
    for (int mode : {0, 3, 4})
        for (int U : {1, 2})
            for (uint32_t lds : {80u << 10, 16u << 10}) cfgs.push_back({U, lds, mode});
    auto pick = [](const Cfg& c) {
        if (c.mode == 0) return c.U == 1 ? k_walk<1, 0> : k_walk<2, 0>;
        if (c.mode == 3) return c.U == 1 ? k_walk<1, 3> : k_walk<2, 3>;
        return c.U == 1 ? k_walk<1, 4> : k_walk<2, 4>;
    };
    for (auto& c : cfgs) {
        auto f = pick(c);
        CK(hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10));
    }
    std::vector<std::vector<float>> t(cfgs.size());
    for (int it = 0; it < 8; ++it)
        for (size_t v = 0; v < cfgs.size(); ++v) {
            auto f = pick(cfgs[v]);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(f, dim3((n + 3) / 4), dim3(256), cfgs[v].lds, 0, d, n, 0u);
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t[v].push_back(ms);
        }
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v < cfgs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        auto f = pick(cfgs[v]);
        int nb = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 256, cfgs[v].lds));
        const double bytes = alg;
        printf("%s step %2d KiB/shard, %3d stripes per CU at once: med %.4f ms -> %.1f GB/s (%.1f%%)\n",
               cfgs[v].mode == 0 ? "rw      " : cfgs[v].mode == 3 ? "rw ntst " : "rw ntall", cfgs[v].U, 4 * nb,
               x[x.size() / 2], bytes / (x[x.size() / 2] * 1e-3) / 1e9, 100 * bytes / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
