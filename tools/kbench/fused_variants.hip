// fused_variants.hip — ablation microbenchmark of the fused encode + HH256S
// kernel on RS(8,4), 1 MiB stripes, n = 4096, interleaved timing in one
// process: full kernel, no GF arithmetic, no hashing, neither, and the
// unfused pair (encode kernel + quad hash kernel).  Not part of the product.
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;
constexpr int K = 8, M = 4;

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
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t S = 131072, STRIDE = (K + M) * S;
    uint8_t *d, *dig;
    CK(hipMalloc(&d, n * STRIDE));
    CK(hipMalloc(&dig, n * (K + M) * 32));
    k_fill<<<4096, 256>>>(d, n * STRIDE, 3);
    const uint8_t rows[4][8] = {{0x1a, 0x84, 0xba, 0x33, 0xe7, 0x10, 0xc6, 0x27}, {0x84, 0x1a, 0x33, 0xba, 0x10, 0xe7, 0x27, 0xc6},
                                {0xba, 0x33, 0x1a, 0x84, 0xc6, 0x27, 0xe7, 0x10}, {0x33, 0xba, 0x84, 0x1a, 0x27, 0xc6, 0x10, 0xe7}};
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(rows[r][c], (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE; p.units = S / kFusedChunk;
    HashParams h;
    memset(&h, 0, sizeof(h));
    const uint64_t key[4] = {0xcd8a238efa34e74bull, 0x528596bbe6833e26ull, 0x14449fa35d930f04ull, 0xa036de22139de097ull};
    memcpy(h.key, key, sizeof(key));
    h.out = dig;
    h.n = n;
    const size_t lds1 = (size_t)K * M * 32 + (size_t)(K + M) * kFusedPitch;
    const size_t lds4 = (size_t)K * M * 32 + (size_t)4 * (K + M) * kFusedPitch;
    const uint32_t g4 = (uint32_t)((n + 3) / 4);
    HashParams hq;
    memset(&hq, 0, sizeof(hq));
    hq.data = d; hq.len = S; hq.n = n * (K + M); hq.shards = K + M; hq.shard_pitch = S; hq.stripe_stride = STRIDE;
    memcpy(hq.key, key, sizeof(key));
    hq.out = dig;
    GfApplyParams pe = p;
    pe.units = S / 16;
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {
        {"fused spw4 (prod)", [&] { CK(launch_encode_hash_fused(p, h, S, n, 0)); }},
        {"fused spw1", [&] { k_encode_hash_fused<K, M, 1, 0><<<n, 128, lds1>>>(p, h); }},
        {"fused spw2", [&] { k_encode_hash_fused<K, M, 2, 0><<<(n + 1) / 2, 64 * 4, lds1 * 2 - K * M * 32>>>(p, h); }},
        {"spw4 no-GF", [&] { k_encode_hash_fused<K, M, 4, 1><<<g4, 448, lds4>>>(p, h); }},
        {"spw4 no-hash", [&] { k_encode_hash_fused<K, M, 4, 2><<<g4, 448, lds4>>>(p, h); }},
        {"spw4 neither", [&] { k_encode_hash_fused<K, M, 4, 3><<<g4, 448, lds4>>>(p, h); }},
        {"encode only", [&] { CK(launch_gf_apply_vec(pe, n, 0)); }},
        {"quad hash only", [&] { CK(launch_hh256(hq, 0)); }},
    };
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
    // where do the two waves of a workgroup run?  HW_ID bits [5:4] = SIMD, [11:8] = CU
    k_encode_hash_fused<K, M, 1, 8><<<n, 128, lds1>>>(p, h);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> hd(n * (K + M) * 32);
    CK(hipMemcpy(hd.data(), dig, hd.size(), hipMemcpyDeviceToHost));
    int pairs[4][4] = {};
    for (uint64_t s = 0; s < n; ++s) {
        const uint32_t* w = (const uint32_t*)(hd.data() + s * (K + M) * 32);
        pairs[(w[0] >> 4) & 3][(w[1] >> 4) & 3]++;
    }
    printf("encoder SIMD x hasher SIMD histogram (rows: encoder simd)\n");
    for (int a = 0; a < 4; ++a) printf("  %6d %6d %6d %6d\n", pairs[a][0], pairs[a][1], pairs[a][2], pairs[a][3]);
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("%-16s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", vs[v].name, x[x.size() / 2], x[0],
               alg / (x[x.size() / 2] * 1e-3) / 1e9, 100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
