// fused_v3.hip — fused encode + HighwayHash with bit-sliced encoder waves:
// SPW = 8 stripes per workgroup, 256-byte chunks, data by LDS-DMA three chunks
// deep, parity rows double-buffered in LDS, data-shard hashers reading global
// memory two chunks ahead.  Not part of the product.  Usage: fused_v3 n [iters]
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

namespace v3 {
constexpr int SPW = 8;            // stripes per workgroup
constexpr uint32_t CH = 256;      // bytes per shard per step
constexpr uint32_t PP = CH + 32;  // parity row pitch (conflict-free ds_read_b64)
constexpr int NSLOT = 3;          // LDS-DMA ring depth (chunks)
}  // namespace v3

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16 ds_read_b128 (1 KiB apart) and their lgkmcnt wait in ONE statement: the
// compiler neither sees these LDS reads (so it adds no vmcnt wait for the
// LDS-DMA it cannot order across waves) nor can it use the destinations early.
__device__ __forceinline__ void read_slot16(uint32_t a, u32x4 (&r)[16]) {
    asm volatile(
        "ds_read_b128 %0, %16 offset:0\n\t"
        "ds_read_b128 %1, %16 offset:1024\n\t"
        "ds_read_b128 %2, %16 offset:2048\n\t"
        "ds_read_b128 %3, %16 offset:3072\n\t"
        "ds_read_b128 %4, %16 offset:4096\n\t"
        "ds_read_b128 %5, %16 offset:5120\n\t"
        "ds_read_b128 %6, %16 offset:6144\n\t"
        "ds_read_b128 %7, %16 offset:7168\n\t"
        "ds_read_b128 %8, %16 offset:8192\n\t"
        "ds_read_b128 %9, %16 offset:9216\n\t"
        "ds_read_b128 %10, %16 offset:10240\n\t"
        "ds_read_b128 %11, %16 offset:11264\n\t"
        "ds_read_b128 %12, %16 offset:12288\n\t"
        "ds_read_b128 %13, %16 offset:13312\n\t"
        "ds_read_b128 %14, %16 offset:14336\n\t"
        "ds_read_b128 %15, %16 offset:15360\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]),
          "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
        : "v"(a)
        : "memory");
}

// Parity row r (compile time) from the bit planes P: 8 XOR chains, back to
// bytes.
template <int K_, int M_, int R>
__device__ __forceinline__ void bs_row(const uint32_t (&P)[K_][8], uint32_t (&o)[8], uint32_t m4, uint32_t m2,
                                       uint32_t m1) {
    constexpr bs::PlaneMasks<K_, M_> PM{};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t acc = 0, pend = 0;
        int cnt = 0;
#pragma unroll
        for (int c = 0; c < K_; ++c) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (!((PM.mask[R][c][i] >> j) & 1u)) continue;
                if (cnt == 0) acc = P[c][j];
                else if (cnt & 1) pend = P[c][j];
                else acc = x3(acc, pend, P[c][j]);
                ++cnt;
            }
        }
        if (cnt > 1 && (cnt & 1) == 0) acc ^= pend;
        o[i] = acc;
    }
    bs::transpose(o, m4, m2, m1);
}

template <int K_, int M_, int R0, int RN>
__device__ __forceinline__ void bs_rows(const uint32_t (&P)[K_][8], uint8_t* wb, const GfApplyParams& p, uint64_t coff,
                                        uint8_t* pr, uint32_t prow_off, uint32_t m4, uint32_t m2, uint32_t m1) {
    if constexpr (RN > 0) {
        uint32_t o[8];
        bs_row<K_, M_, R0>(P, o, m4, m2, m1);
        const uint4 a = make_uint4(o[0], o[1], o[2], o[3]), b = make_uint4(o[4], o[5], o[6], o[7]);
        uint8_t* dst = wb + p.out_off[R0] + coff;
        st16(dst, a);
        st16(dst + 128, b);
        uint8_t* row = pr + R0 * v3::PP + prow_off;
        *(uint4*)row = a;
        *(uint4*)(row + 128) = b;
        bs_rows<K_, M_, R0 + 1, RN - 1>(P, wb, p, coff, pr, prow_off, m4, m2, m1);
    }
}

template <int K_, int M_, int E>
__global__ __launch_bounds__(64 * (E + (K_ + M_) / 2))
void k_fused_v3(const GfApplyParams p, const HashParams h) {
    using namespace v3;
    static_assert(K_ == 8 && M_ % E == 0, "slot reader assumes 8 data shards x 2 halves");
    constexpr int HD = SPW * K_ / 16;         // data hasher waves (global loads)
    constexpr uint32_t DSLOT = K_ * 2 * 1024;  // one chunk of all data shards, lane-linear
    constexpr uint32_t PSLOT = SPW * M_ * PP;  // parity rows of one chunk
    constexpr int RPW = M_ / E;
    extern __shared__ __attribute__((aligned(16))) uint8_t dslot[];  // NSLOT * DSLOT (LDS-DMA ring)
    __shared__ __attribute__((aligned(16))) uint8_t prow[2 * PSLOT];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t chunks = p.units;  // S / CH, >= 2
    const uint64_t wbase = (uint64_t)blockIdx.x * SPW;
    if (wave < (uint32_t)E) {
        // ------------------------------ encoders ------------------------------
        // lane t: stripe g = t/8, u = t%8 holds bytes [16u, +16) and
        // [128 + 16u, +16) of every data shard's chunk (lane-linear in the DMA
        // slot); encoder e computes parity rows [e*RPW, (e+1)*RPW).  Wave 0
        // issues the DMA two chunks ahead and retires chunk ch+1 (counted
        // vmcnt) before barrier ch, so both encoders read it after that barrier.
        const uint32_t g = lane >> 3, u = lane & 7u;
        const bool live = wbase + g < n;  // a dead stripe re-reads stripe 0 and stores its bytes again
        uint8_t* wb = p.out_base + wbase * p.stripe_stride;
        const uint64_t voff = (uint64_t)(live ? g : 0u) * p.stripe_stride + u * 16u;
        const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
        auto dma = [&](uint32_t ch) {
            uint8_t* slot = dslot + (ch % NSLOT) * DSLOT;
#pragma unroll
            for (int c = 0; c < K_; ++c) {
                const uint8_t* src = wb + p.in_off[c] + (uint64_t)ch * CH + voff;
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (__attribute__((address_space(3))) void*)(slot + (2 * c) * 1024), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((const void*)(src + 128),
                                                 (__attribute__((address_space(3))) void*)(slot + (2 * c + 1) * 1024), 16, 0,
                                                 0);
            }
        };
        if (wave == 0) {
            dma(0);
            dma(1);
            __builtin_amdgcn_s_waitcnt(0x0F70 | 0x1);  // vmcnt(16): chunk 0 landed
        }
        lds_barrier();  // chunk 0 visible to both encoders
        const uint32_t prow_off = (g * M_) * PP + u * 16u;
#pragma unroll 1
        for (uint32_t ch = 0; ch < chunks; ++ch) {
            u32x4 v[16];
            read_slot16((uint32_t)(uintptr_t)(dslot + (ch % NSLOT) * DSLOT) + lane * 16u, v);
            if (wave == 0 && ch + 2 < chunks) dma(ch + 2);  // the slot read at step ch-1
            uint32_t P[K_][8];
#pragma unroll
            for (int c = 0; c < K_; ++c) {
                P[c][0] = v[2 * c].x; P[c][1] = v[2 * c].y; P[c][2] = v[2 * c].z; P[c][3] = v[2 * c].w;
                P[c][4] = v[2 * c + 1].x; P[c][5] = v[2 * c + 1].y; P[c][6] = v[2 * c + 1].z; P[c][7] = v[2 * c + 1].w;
                bs::transpose(P[c], m4, m2, m1);
            }
            uint8_t* pr = prow + (ch & 1u) * PSLOT;
            const uint64_t coff = (uint64_t)ch * CH + voff;
            if (wave == 0) bs_rows<K_, M_, 0, RPW>(P, wb, p, coff, pr, prow_off, m4, m2, m1);
            else if (wave == 1) bs_rows<K_, M_, (E > 1 ? RPW : 0), (E > 1 ? RPW : 0)>(P, wb, p, coff, pr, prow_off, m4, m2, m1);
            else if (wave == 2) bs_rows<K_, M_, (E > 2 ? 2 * RPW : 0), (E > 2 ? RPW : 0)>(P, wb, p, coff, pr, prow_off, m4, m2, m1);
            else bs_rows<K_, M_, (E > 3 ? 3 * RPW : 0), (E > 3 ? RPW : 0)>(P, wb, p, coff, pr, prow_off, m4, m2, m1);
            if (wave == 0 && ch + 1 < chunks) {
                // retire DMA(ch+1): after it came stores(ch-1), DMA(ch+2) if
                // issued, stores(ch) - 2*RPW stores per step
                if (ch + 2 < chunks) __builtin_amdgcn_s_waitcnt(0x0F70 | ((4 * RPW + 2 * K_) & 15) | (((4 * RPW + 2 * K_) >> 4) << 14));
                else __builtin_amdgcn_s_waitcnt(0x0F70 | ((4 * RPW) & 15) | (((4 * RPW) >> 4) << 14));
            }
            lds_barrier();  // B(ch): parity rows of ch published; data ch+1 visible
        }
    } else {
        // ------------------------------ hashers -------------------------------
        const uint32_t hw = wave - E;
        HHQuad st;
        hhq_init(st, h.key, q);
        lds_barrier();  // matches the encoders' prologue barrier
        if (hw < (uint32_t)HD) {
            // data streams: quad -> (stripe, shard), packets straight from HBM
            const uint32_t gs = hw * 16u + (lane >> 2), ls = gs / K_, shard = gs - ls * K_;
            const bool live = wbase + ls < n;
            const uint8_t* msg = p.out_base + (wbase + (live ? ls : 0)) * p.stripe_stride + p.in_off[shard] + 8 * q;
            uint64_t wa[8], wb2[8];
            auto fetch = [&](uint64_t (&w)[8], uint32_t ch) {
#pragma unroll
                for (int t = 0; t < 8; ++t) w[t] = ld64_any(msg + (uint64_t)ch * CH + t * 32);
            };
            auto step = [&](uint64_t (&cur)[8], uint64_t (&nxt)[8], uint32_t ch) {
                fetch(nxt, ch + 1 < chunks ? ch + 1 : ch);  // clamped: straight-line loads
#pragma unroll
                for (int t = 0; t < 8; ++t) hhq_update(st, cur[t]);
                lds_barrier();
            };
            fetch(wa, 0);
#pragma unroll 1
            for (uint32_t ch = 0; ch < chunks; ch += 2) {
                step(wa, wb2, ch);
                if (ch + 1 >= chunks) break;
                step(wb2, wa, ch + 1);
            }
            if (live) hhq_finish(st, h.out + ((wbase + ls) * (K_ + M_) + shard) * 32u, q);
        } else {
            // parity streams: rows from LDS after the encoders' barrier
            const uint32_t gs = (hw - HD) * 16u + (lane >> 2), ls = gs / M_, r = gs - ls * M_;
            const bool live = wbase + ls < n;
            const uint32_t roff = (ls * M_ + r) * PP + 8 * q;
#pragma unroll 1
            for (uint32_t ch = 0; ch < chunks; ++ch) {
                lds_barrier();  // B(ch)
                const uint8_t* row = prow + (ch & 1u) * PSLOT + roff;
                uint64_t w[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) w[t] = *(const uint64_t*)(row + t * 32);
#pragma unroll
                for (int t = 0; t < 8; ++t) hhq_update(st, w[t]);
            }
            if (live) hhq_finish(st, h.out + ((wbase + ls) * (K_ + M_) + K_ + r) * 32u, q);
        }
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
    const size_t lds_v3 = (size_t)v3::NSLOT * K * 2 * 1024;
    CK(hipFuncSetAttribute((const void*)k_fused_v3<K, M, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_v3));
    CK(hipFuncSetAttribute((const void*)k_fused_v3<K, M, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_v3));
    CK(hipFuncSetAttribute((const void*)k_fused_v3<K, M, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_v3));
    const uint32_t g8 = (uint32_t)((n + 7) / 8);
    GfApplyParams p3 = p;
    p3.units = S / v3::CH;
    GfApplyParams pe = p;
    pe.units = S / 16;
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {
        {"fused (prod)", [&] { CK(launch_encode_hash_fused(p, h, S, n, 0)); }},
        {"v3 E=2", [&] { k_fused_v3<K, M, 2><<<g8, 64 * (2 + (K + M) / 2), lds_v3>>>(p3, h); }},
        {"v3 E=1", [&] { k_fused_v3<K, M, 1><<<g8, 64 * (1 + (K + M) / 2), lds_v3>>>(p3, h); }},
        {"v3 E=4", [&] { k_fused_v3<K, M, 4><<<g8, 64 * (4 + (K + M) / 2), lds_v3>>>(p3, h); }},
        {"encode only", [&] { CK(launch_gf_apply_vec(pe, n, 0)); }},
    };
    {
        const size_t nd = n * (K + M) * 32;
        std::vector<uint8_t> ref(nd), got(nd), pref(M * S), pgot(M * S);
        vs[0].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pref.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
        for (size_t v = 1; v + 1 < vs.size(); ++v) {
            CK(hipMemset(dig, 0, nd));
            CK(hipMemset(d + (n - 1) * STRIDE + K * S, 0, M * S));
            vs[v].f();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), dig, nd, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pgot.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < nd; i += 32) bad += memcmp(&ref[i], &got[i], 32) != 0;
            printf("%s: digests %s (%zu bad of %zu), parity %s\n", vs[v].name, bad ? "MISMATCH" : "ok", bad, nd / 32,
                   memcmp(pref.data(), pgot.data(), M * S) ? "MISMATCH" : "ok");
        }
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
