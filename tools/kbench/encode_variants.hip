// encode_variants.hip — standalone microbenchmark of RS(8,4) encode kernel
// variants on device-resident 1 MiB stripes (n = 4096), interleaved timing in
// one process (cdna_hip_programming.md §5.4 rule 24).  Not part of the product;
// the winner is ported into rustfs_amd/csrc/rs_kernels.hip.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o encode_variants encode_variants.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <functional>

#include "../../rustfs_amd/csrc/rs_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int K = 8, M = 4;
constexpr uint64_t S = 131072;
constexpr uint64_t STRIDE = (K + M) * S;

struct Tabs { uint32_t t[M][K][5]; };

__device__ __forceinline__ uint32_t mulw(const uint32_t* t, uint32_t s0, uint32_t s1, uint32_t s2) {
    return __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^ __builtin_amdgcn_perm(t[4], t[4], s2);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint8_t* p) {
    if constexpr (NT) {
        u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *(const uint4*)p;
    }
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t* p, uint4 v) {
    if constexpr (NT) {
        u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (u32x4*)p);
    } else {
        *(uint4*)p = v;
    }
}

template <bool NT>
__device__ __forceinline__ void compute(const Tabs& T, const uint4* x, uint4* o) {
    uint32_t acc[M][4];
#pragma unroll
    for (int r = 0; r < M; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint32_t w[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < M; ++r) acc[r][q] ^= mulw(T.t[r][c], s0, s1, s2);
        }
    }
#pragma unroll
    for (int r = 0; r < M; ++r) o[r] = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}

// U units per thread, all loads issued before any compute; one block = 256*U units of one stripe.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_blocked(uint8_t* base, const Tabs T, uint32_t chunks) {
    const uint32_t stripe = blockIdx.x / chunks, chunk = blockIdx.x - stripe * chunks;
    uint8_t* sb = base + (uint64_t)stripe * STRIDE;
    uint4 x[U][K];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t off = ((uint64_t)(chunk * U + j) * 256 + threadIdx.x) * 16;
#pragma unroll
        for (int c = 0; c < K; ++c) x[j][c] = ld<NT>(sb + c * S + off);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint64_t off = ((uint64_t)(chunk * U + j) * 256 + threadIdx.x) * 16;
        uint4 o[M];
        compute<NT>(T, x[j], o);
#pragma unroll
        for (int r = 0; r < M; ++r) st<NT>(sb + (K + r) * S + off, o[r]);
    }
}

// Persistent grid-stride: unit index over all stripes, software-pipelined by one unit.
template <bool NT>
__global__ __launch_bounds__(256) void k_persist(uint8_t* base, const Tabs T, uint64_t total_units) {
    const uint64_t units_per_stripe = S / 16;
    uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    if (u >= total_units) return;
    uint4 x[K];
    {
        const uint64_t s = u / units_per_stripe, c0 = u - s * units_per_stripe;
        const uint8_t* p = base + s * STRIDE + c0 * 16;
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = ld<NT>(p + c * S);
    }
    while (true) {
        const uint64_t un = u + step;
        uint4 y[K];
        if (un < total_units) {
            const uint64_t s = un / units_per_stripe, c0 = un - s * units_per_stripe;
            const uint8_t* p = base + s * STRIDE + c0 * 16;
#pragma unroll
            for (int c = 0; c < K; ++c) y[c] = ld<NT>(p + c * S);
        }
        uint4 o[M];
        compute<NT>(T, x, o);
        const uint64_t s = u / units_per_stripe, c0 = u - s * units_per_stripe;
        uint8_t* p = base + s * STRIDE + c0 * 16;
#pragma unroll
        for (int r = 0; r < M; ++r) st<NT>(p + (K + r) * S, o[r]);
        if (un >= total_units) break;
        u = un;
#pragma unroll
        for (int c = 0; c < K; ++c) x[c] = y[c];
    }
}

// Same traffic shape, trivial compute: the practical ceiling for 8-read/4-write streaming.
template <bool NT>
__global__ __launch_bounds__(256) void k_copyshape(uint8_t* base, uint32_t chunks) {
    const uint32_t stripe = blockIdx.x / chunks, chunk = blockIdx.x - stripe * chunks;
    uint8_t* sb = base + (uint64_t)stripe * STRIDE;
    const uint64_t off = ((uint64_t)chunk * 256 + threadIdx.x) * 16;
    uint4 x[K];
#pragma unroll
    for (int c = 0; c < K; ++c) x[c] = ld<NT>(sb + c * S + off);
#pragma unroll
    for (int r = 0; r < M; ++r) {
        uint4 a = x[2 * r], b = x[2 * r + 1];
        st<NT>(sb + (K + r) * S + off, make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w));
    }
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) { if (b & 1) p ^= a; b >>= 1; a = (a << 1) ^ ((a & 0x80) ? 0x1d : 0); }
    return p;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    // RS(8,4) parity rows
    const uint8_t rows[4][8] = {{0x1a, 0x84, 0xba, 0x33, 0xe7, 0x10, 0xc6, 0x27}, {0x84, 0x1a, 0x33, 0xba, 0x10, 0xe7, 0x27, 0xc6},
                                {0xba, 0x33, 0x1a, 0x84, 0xc6, 0x27, 0xe7, 0x10}, {0x33, 0xba, 0x84, 0x1a, 0x27, 0xc6, 0x10, 0xe7}};
    Tabs T;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(rows[r][c], (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            T.t[r][c][0] = pack(0, 0); T.t[r][c][1] = pack(0, 4); T.t[r][c][2] = pack(3, 0); T.t[r][c][3] = pack(3, 4); T.t[r][c][4] = pack(6, 0);
        }
    const uint64_t bytes = n * STRIDE;
    uint8_t* d;
    CK(hipMalloc(&d, bytes));
    k_fill<<<4096, 256>>>(d, bytes, 12345);
    CK(hipDeviceSynchronize());
    const uint32_t units = S / 16;
    std::vector<uint8_t> ref(M * S), got(M * S);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));

    struct V { const char* name; std::function<void()> f; bool check; };
    int nblk_persist = 256 * 8;
    std::vector<V> vs = {
        {"library vec", [&] {
             rsg::GfApplyParams p; memset(&p, 0, sizeof(p));
             p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
             for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
             for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
             memcpy(p.tab, T.t, sizeof(T.t)); // [4][8][5] -> [4][16][5] handled below
             for (int r = 0; r < M; ++r) for (int c = 0; c < K; ++c) for (int i = 0; i < 5; ++i) p.tab[r][c][i] = T.t[r][c][i];
             p.C = K; p.R = M; p.mode = 0; p.units = units;
             CK(rsg::launch_gf_apply_vec(p, n, 0)); }, true},
        {"blocked U1", [&] { k_blocked<1, false><<<(units / 256) * n, 256>>>(d, T, units / 256); }, true},
        {"blocked U2", [&] { k_blocked<2, false><<<(units / 512) * n, 256>>>(d, T, units / 512); }, true},
        {"blocked U4", [&] { k_blocked<4, false><<<(units / 1024) * n, 256>>>(d, T, units / 1024); }, true},
        {"blocked U1 nt", [&] { k_blocked<1, true><<<(units / 256) * n, 256>>>(d, T, units / 256); }, true},
        {"blocked U2 nt", [&] { k_blocked<2, true><<<(units / 512) * n, 256>>>(d, T, units / 512); }, true},
        {"persist 2048", [&] { k_persist<false><<<nblk_persist, 256>>>(d, T, (uint64_t)units * n); }, true},
        {"persist 1024 nt", [&] { k_persist<true><<<1024, 256>>>(d, T, (uint64_t)units * n); }, true},
        {"persist 4096 nt", [&] { k_persist<true><<<4096, 256>>>(d, T, (uint64_t)units * n); }, true},
        {"copyshape", [&] { k_copyshape<false><<<(units / 256) * n, 256>>>(d, units / 256); }, false},
        {"copyshape nt", [&] { k_copyshape<true><<<(units / 256) * n, 256>>>(d, units / 256); }, false},
    };
    // reference parity of the last stripe from variant 0
    vs[0].f();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
    // host spot check of a few bytes against scalar GF
    {
        std::vector<uint8_t> dat(K * S);
        CK(hipMemcpy(dat.data(), d + (n - 1) * STRIDE, K * S, hipMemcpyDeviceToHost));
        for (uint64_t bpos : {(uint64_t)0, (uint64_t)1, (uint64_t)4095, (uint64_t)77777, S - 1}) {
            for (int r = 0; r < M; ++r) {
                uint8_t v = 0;
                for (int c = 0; c < K; ++c) v ^= gmul(rows[r][c], dat[c * S + bpos]);
                if (v != ref[r * S + bpos]) { printf("SPOT CHECK FAIL r=%d b=%llu\n", r, (unsigned long long)bpos); return 1; }
            }
        }
    }
    std::vector<std::vector<float>> t(vs.size());
    for (int it = 0; it < iters; ++it) {
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(a));
            vs[v].f();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 0) t[v].push_back(ms);
            if (it == 0 && vs[v].check) {
                CK(hipMemcpy(got.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
                if (memcmp(got.data(), ref.data(), M * S)) { printf("%s: MISMATCH\n", vs[v].name); }
            }
        }
    }
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("%-18s med %.4f ms  min %.4f ms  -> %.1f GB/s (med), %.1f%% of 8 TB/s\n", vs[v].name, x[x.size() / 2], x[0],
               alg / (x[x.size() / 2] * 1e-3) / 1e9, 100.0 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
