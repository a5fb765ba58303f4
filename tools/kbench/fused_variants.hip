// fused_variants.hip — ablation microbenchmark of the fused encode + HH256S
// kernel on RS(8,4), 1 MiB stripes, n = 4096, interleaved timing in one
// process: full kernel, no GF arithmetic, no hashing, neither, and the
// unfused pair (encode kernel + quad hash kernel).  Not part of the product.
#define RSG_MEASUREMENT_BUILD 1  // the ablation variants of k_encode_hash_fused
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <type_traits>
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

// Variant: double-buffered LDS rows, one barrier per chunk, CH-byte chunks
// (CH = 256: 4 bytes per encoder lane per shard).  The encoder may run one
// chunk ahead of the hashers.
template <int C, int R, int SPW, int CH>
__global__ __launch_bounds__(64 * (SPW + (SPW * (C + R) + 15) / 16)) __attribute__((amdgpu_waves_per_eu(7)))
void k_fused_db(const GfApplyParams p, const HashParams h) {
    extern __shared__ uint8_t lds_all[];
    constexpr int T = C + R;
    constexpr uint32_t kPitch = CH + 32;
    constexpr uint32_t kStripeRows = T * kPitch;
    constexpr uint32_t kBuf = SPW * kStripeRows;
    constexpr uint32_t kTabBytes = C * R * 32;
    constexpr int BPL = CH / 64;  // bytes per encoder lane per shard (4 or 8)
    typedef typename std::conditional<BPL == 4, uint32_t, uint2>::type word_t;
    uint8_t* rows = lds_all + kTabBytes;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t chunks = p.units;  // S / CH
    for (uint32_t i = threadIdx.x; i < (uint32_t)(C * R); i += blockDim.x) {
        const int c = i / R, r = i % R;
        uint8_t* d = lds_all + i * 32;
        *(uint4*)d = make_uint4(p.tab[r][c][0], p.tab[r][c][1], p.tab[r][c][2], p.tab[r][c][3]);
        *(uint32_t*)(d + 16) = p.tab[r][c][4];
    }
    __syncthreads();
    if (wave < (uint32_t)SPW) {
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + wave;
        const bool live = stripe < n;
        uint8_t* sb = p.out_base + (live ? stripe : 0) * p.stripe_stride;
        const uint32_t m7 = vgpr_const(0x07070707u), m3 = vgpr_const(0x03030303u);
        word_t x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = *(const word_t*)(sb + p.in_off[c] + lane * BPL);
#pragma unroll 1
        for (uint32_t ch = 0; ch < chunks; ++ch) {
            const uint64_t off = (uint64_t)ch * CH + lane * BPL;
            uint32_t tz;
            asm volatile("s_mov_b32 %0, 0" : "=s"(tz));
            const uint8_t* tabs = lds_all + tz;
            constexpr int NW = BPL / 4;
            uint32_t acc[R][NW];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int w = 0; w < NW; ++w) acc[r][w] = 0u;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                uint32_t xw[NW];
                __builtin_memcpy(xw, &x[c], 4 * NW);
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    const uint32_t s0 = xw[w] & m7, s1 = (xw[w] >> 3) & m7, s2 = (xw[w] >> 6) & m3;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint8_t* tp = tabs + (c * R + r) * 32;
                        const uint4 t4 = *(const uint4*)tp;
                        const uint32_t t2 = *(const uint32_t*)(tp + 16);
                        acc[r][w] ^= __builtin_amdgcn_perm(t4.y, t4.x, s0) ^ __builtin_amdgcn_perm(t4.w, t4.z, s1) ^
                                     __builtin_amdgcn_perm(t2, t2, s2);
                    }
                }
            }
            if (live) {
#pragma unroll
                for (int r = 0; r < R; ++r) __builtin_memcpy(sb + p.out_off[r] + off, acc[r], 4 * NW);
            }
            word_t y[C];
            if (ch + 1 < chunks) {
#pragma unroll
                for (int c = 0; c < C; ++c) y[c] = *(const word_t*)(sb + p.in_off[c] + off + CH);
            }
            uint8_t* buf = rows + (ch & 1) * kBuf + wave * kStripeRows;
#pragma unroll
            for (int c = 0; c < C; ++c) *(word_t*)(buf + c * kPitch + lane * BPL) = x[c];
#pragma unroll
            for (int r = 0; r < R; ++r) __builtin_memcpy(buf + (C + r) * kPitch + lane * BPL, acc[r], 4 * NW);
            lds_barrier();  // rows of chunk ch ready in buffer ch&1
            if (ch + 1 < chunks) {
#pragma unroll
                for (int c = 0; c < C; ++c) x[c] = y[c];
            }
        }
    } else {
        const uint32_t g = (wave - SPW) * 16u + (lane >> 2);
        const uint32_t ls = g / T, shard = g - ls * T;
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + ls;
        const bool live = g < (uint32_t)(SPW * T) && stripe < n;
        const uint32_t roff = (live ? ls * kStripeRows + shard * kPitch : 0) + 8 * q;
        HHQuad st;
        hhq_init(st, h.key, q);
#pragma unroll 1
        for (uint32_t ch = 0; ch < chunks; ++ch) {
            lds_barrier();
            if (live) {
                const uint8_t* row = rows + (ch & 1) * kBuf + roff;
#pragma unroll
                for (int t = 0; t < (int)(CH / 32); ++t) {
                    const u32x2 v = *(const u32x2*)(row + t * 32);
                    hhq_update(st, __builtin_bit_cast(uint64_t, v));
                }
            }
        }
        if (live) hhq_finish(st, h.out + (stripe * T + shard) * 32u, q);
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
        {"db spw4 256", [&] { GfApplyParams q2 = p; q2.units = S / 256;
                               k_fused_db<K, M, 4, 256><<<g4, 448, K * M * 32 + 2 * 4 * (K + M) * (256 + 32)>>>(q2, h); }},
        {"db spw2 512", [&] { GfApplyParams q2 = p; q2.units = S / 512;
                               k_fused_db<K, M, 2, 512><<<(n + 1) / 2, 256, K * M * 32 + 2 * 2 * (K + M) * (512 + 32)>>>(q2, h); }},
        {"db spw4 512", [&] { GfApplyParams q2 = p; q2.units = S / 512;
                               k_fused_db<K, M, 4, 512><<<g4, 448, K * M * 32 + 2 * 4 * (K + M) * (512 + 32)>>>(q2, h); }},
        {"fused spw2", [&] { k_encode_hash_fused<K, M, 2, 0><<<(n + 1) / 2, 64 * 4, lds1 * 2 - K * M * 32>>>(p, h); }},
        {"prio spw4 hashers", [&] { k_encode_hash_fused<K, M, 4, 16><<<g4, 448, lds4>>>(p, h); }},
        {"prio spw4 encoders", [&] { k_encode_hash_fused<K, M, 4, 32><<<g4, 448, lds4>>>(p, h); }},
        {"spw4 no-GF", [&] { k_encode_hash_fused<K, M, 4, 1><<<g4, 448, lds4>>>(p, h); }},
        {"spw4 no-hash", [&] { k_encode_hash_fused<K, M, 4, 2><<<g4, 448, lds4>>>(p, h); }},
        {"spw4 neither", [&] { k_encode_hash_fused<K, M, 4, 3><<<g4, 448, lds4>>>(p, h); }},
        {"encode only", [&] { CK(launch_gf_apply_vec(pe, n, 0)); }},
        {"quad hash only", [&] { CK(launch_hh256(hq, 0)); }},
    };
    {   // correctness of the experimental variants against the production kernel
        const size_t nd = n * (K + M) * 32;
        std::vector<uint8_t> ref(nd), got(nd), pref(M * S), pgot(M * S);
        vs[0].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pref.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
        for (auto& v : vs) {
            if (strncmp(v.name, "db", 2) && strncmp(v.name, "prio", 4)) continue;
            CK(hipMemset(dig, 0, nd));
            CK(hipMemset(d + (n - 1) * STRIDE + K * S, 0, M * S));
            v.f();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), dig, nd, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pgot.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
            printf("%s: digests %s, parity %s\n", v.name, memcmp(ref.data(), got.data(), nd) ? "MISMATCH" : "ok",
                   memcmp(pref.data(), pgot.data(), M * S) ? "MISMATCH" : "ok");
        }
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
