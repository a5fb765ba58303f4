// fused_bs.hip — fused encode + HighwayHash with a bit-sliced encoder wave,
// against the production fused kernel (digests and parity compared byte for
// byte, interleaved timing in one process).  Not part of the product.
// Usage: fused_bs n [iters]
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

constexpr int K = 8, M = 4;

// SPW = 4 stripes per workgroup, 512-byte chunks.  Wave 0 encodes all four
// stripes bit-sliced (16 lanes per stripe, 32 bytes per lane per shard: two
// 16-byte pieces 256 B apart); data-shard hasher waves read their packets from
// global memory (prefetched one chunk ahead), parity hasher waves from the
// double-buffered LDS parity rows.  One barrier per chunk.
template <int K_, int M_, int ABL = 0>
__global__ __launch_bounds__(64 * (1 + (4 * (K_ + M_) + 15) / 16))
__attribute__((amdgpu_waves_per_eu(4)))
void k_fused_bs(const GfApplyParams p, const HashParams h) {
    constexpr int SPW = 4;
    constexpr uint32_t CH = 512, PITCH = CH + 32, SLOT = SPW * M_ * PITCH;
    // separate LDS objects: the compiler's wait insertion then knows the
    // parity-row accesses cannot alias the in-flight LDS-DMA into dslot
    __shared__ __attribute__((aligned(16))) uint8_t lds_all[2 * SLOT];
    __shared__ __attribute__((aligned(16))) uint8_t dslot[2 * K_ * 1024];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t chunks = p.units;
    if (wave == 0) {
        // ------------------------------ encoder ------------------------------
        // Data chunks arrive by LDS-DMA (global_load_lds_dwordx4) in a
        // wave-private slot, lane-linear: instruction (c, half) puts lane t's
        // 16 B at dslot + (2c + half) * 1 KiB + 16 t.  Chunk ch+1 is requested
        // right after chunk ch was read out, so its transfer overlaps the whole
        // step; no prefetch registers (P holds one chunk: 64 VGPRs).
        constexpr bs::PlaneMasks<K_, M_> PM{};
        const uint32_t g = lane >> 4, u = lane & 15u;
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + g;
        const bool live = stripe < n;
        uint8_t* wb = p.out_base + (uint64_t)blockIdx.x * SPW * p.stripe_stride;
        const uint32_t voff = (live ? g : 0u) * (uint32_t)p.stripe_stride + u * 16u;
        const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
        auto dma = [&](uint32_t ch) {
#pragma unroll
            for (int c = 0; c < K_; ++c) {
                const uint8_t* src = wb + p.in_off[c] + (uint64_t)ch * CH + voff;
                __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dslot + (2 * c) * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(src + 256), (__attribute__((address_space(3))) void*)(dslot + (2 * c + 1) * 1024), 16, 0, 0);
            }
        };
        dma(0);
#pragma unroll 1
        for (uint32_t ch = 0; ch < chunks; ++ch) {
            uint32_t P[K_][8];
#pragma unroll
            for (int c = 0; c < K_; ++c) {
                const uint4 a = *(const uint4*)(dslot + (2 * c) * 1024 + lane * 16u);
                const uint4 b = *(const uint4*)(dslot + (2 * c + 1) * 1024 + lane * 16u);
                P[c][0] = a.x; P[c][1] = a.y; P[c][2] = a.z; P[c][3] = a.w;
                P[c][4] = b.x; P[c][5] = b.y; P[c][6] = b.z; P[c][7] = b.w;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): slot read out
            if (ch + 1 < chunks) dma(ch + 1);
            if constexpr (!(ABL & 1)) {
#pragma unroll
                for (int c = 0; c < K_; ++c) bs::transpose(P[c], m4, m2, m1);
            }
            uint8_t* slot = lds_all + (ch & 1u) * SLOT;
#pragma unroll
            for (int r = 0; r < M_; ++r) {
                uint32_t o[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    if constexpr (ABL & 1) {
                        o[i] = P[r][i] ^ P[r + M_][i];
                        continue;
                    }
                    uint32_t acc = 0, pend = 0;
                    int cnt = 0;
#pragma unroll
                    for (int c = 0; c < K_; ++c) {
                        const uint32_t mk = PM.mask[r][c][i];
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (!((mk >> j) & 1u)) continue;
                            if (cnt == 0) acc = P[c][j];
                            else if (cnt & 1) pend = P[c][j];
                            else acc = x3(acc, pend, P[c][j]);
                            ++cnt;
                        }
                    }
                    if (cnt > 1 && (cnt & 1) == 0) acc ^= pend;
                    o[i] = acc;
                }
                if constexpr (!(ABL & 1)) bs::transpose(o, m4, m2, m1);
                const uint4 a = make_uint4(o[0], o[1], o[2], o[3]);
                const uint4 b = make_uint4(o[4], o[5], o[6], o[7]);
                {   // unconditional (straight-line vmcnt accounting): a dead
                    // stripe's lanes alias the workgroup's first stripe and
                    // store the very bytes its own lanes store
                    uint8_t* dst = wb + p.out_off[r] + (uint64_t)ch * CH + voff;
                    st16(dst, a);
                    st16(dst + 256, b);
                }
                uint8_t* row = slot + (g * M_ + r) * PITCH + u * 16u;
                *(uint4*)row = a;
                *(uint4*)(row + 256) = b;
            }
            lds_barrier();  // parity rows of chunk ch published in slot ch & 1
        }
    } else {
        const uint32_t gs = (wave - 1) * 16u + (lane >> 2);
        const bool is_data = gs < (uint32_t)(SPW * K_);  // wave-uniform when SPW*K % 16 == 0
        uint32_t ls, shard;
        if (is_data) {
            ls = gs / K_;
            shard = gs - ls * K_;
        } else {
            const uint32_t pp = gs - SPW * K_;
            ls = pp / M_;
            shard = K_ + (pp - ls * M_);
        }
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + ls;
        const bool live = gs < (uint32_t)(SPW * (K_ + M_)) && stripe < n;
        HHQuad st;
        hhq_init(st, h.key, q);
        if (is_data) {
            const uint8_t* msg = p.out_base + (live ? stripe : 0) * p.stripe_stride + p.in_off[live ? shard : 0] + 8 * q;
            uint64_t w0[16], w1[16];
            auto fetch = [&](uint64_t (&w)[16], uint32_t ch) {
#pragma unroll
                for (int t = 0; t < 16; ++t) w[t] = ld64_any(msg + (uint64_t)ch * CH + t * 32);
            };
            auto step = [&](uint64_t (&cur)[16], uint64_t (&nxt)[16], uint32_t ch) {
                lds_barrier();
                if (ch + 1 < chunks) fetch(nxt, ch + 1);
                if (live) {
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        if constexpr (ABL & 2) st.v0 ^= cur[t];
                        else hhq_update(st, cur[t]);
                    }
                }
            };
            fetch(w0, 0);
#pragma unroll 1
            for (uint32_t ch = 0; ch < chunks; ch += 2) {
                step(w0, w1, ch);
                if (ch + 1 >= chunks) break;
                step(w1, w0, ch + 1);
            }
        } else {
            const uint32_t roff = (ls * M_ + (shard - K_)) * PITCH + 8 * q;
#pragma unroll 1
            for (uint32_t ch = 0; ch < chunks; ++ch) {
                lds_barrier();
                if (live) {
                    const uint8_t* row = lds_all + (ch & 1u) * SLOT + roff;
                    uint64_t w[16];
#pragma unroll
                    for (int t = 0; t < 16; ++t) w[t] = *(const uint64_t*)(row + t * 32);
#pragma unroll
                    for (int t = 0; t < 16; ++t) {
                        if constexpr (ABL & 2) st.v0 ^= w[t];
                        else hhq_update(st, w[t]);
                    }
                }
            }
        }
        if (live) hhq_finish(st, h.out + (stripe * (K_ + M_) + shard) * 32u, q);
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

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t S = 131072, STRIDE = (K + M) * S;
    uint8_t *d, *dig;
    CK(hipMalloc(&d, n * STRIDE));
    CK(hipMalloc(&dig, n * (K + M) * 32));
    k_fill<<<4096, 256>>>(d, n * STRIDE, 3);
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
    p.C = K; p.R = M; p.mode = GF_MODE_STORE; p.units = S / kFusedChunk;
    HashParams h;
    memset(&h, 0, sizeof(h));
    const uint64_t key[4] = {0xcd8a238efa34e74bull, 0x528596bbe6833e26ull, 0x14449fa35d930f04ull, 0xa036de22139de097ull};
    memcpy(h.key, key, sizeof(key));
    h.out = dig;
    h.n = n;
    const uint32_t g4 = (uint32_t)((n + 3) / 4);
    const uint32_t thr = 64 * (1 + (4 * (K + M) + 15) / 16);
    const size_t lds_bs = 2ull * 4 * M * (512 + 32) + 4ull * K * 512;
    GfApplyParams pe = p;
    pe.units = S / 16;
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {
        {"fused (prod)", [&] { CK(launch_encode_hash_fused(p, h, S, n, 0)); }},
        {"fused bs", [&] { k_fused_bs<K, M, 0><<<g4, thr>>>(p, h); }},
        {"fused bs no-GF", [&] { k_fused_bs<K, M, 1><<<g4, thr>>>(p, h); }},
        {"fused bs no-hash", [&] { k_fused_bs<K, M, 2><<<g4, thr>>>(p, h); }},
        {"fused bs neither", [&] { k_fused_bs<K, M, 3><<<g4, thr>>>(p, h); }},
        {"encode only", [&] { CK(launch_gf_apply_vec(pe, n, 0)); }},
    };
    {
        const size_t nd = n * (K + M) * 32;
        std::vector<uint8_t> ref(nd), got(nd), pref(M * S), pgot(M * S);
        vs[0].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pref.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
        CK(hipMemset(dig, 0, nd));
        CK(hipMemset(d + (n - 1) * STRIDE + K * S, 0, M * S));
        vs[1].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pgot.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
        printf("%s: digests %s, parity %s\n", vs[1].name, memcmp(ref.data(), got.data(), nd) ? "MISMATCH" : "ok",
               memcmp(pref.data(), pgot.data(), M * S) ? "MISMATCH" : "ok");
        vs[0].f();  // restore parity for the timing runs
        CK(hipDeviceSynchronize());
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
            if (it > 1) t[v].push_back(ms);
        }
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("%-18s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", vs[v].name, x[x.size() / 2], x[0],
               alg / (x[x.size() / 2] * 1e-3) / 1e9, 100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
