// fused_r2.hip — round-2 fused encode + HighwayHash candidate, against the
// production fused kernel (digests and parity compared for every stripe,
// interleaved timing in one process).  Measurement code.
//
// Design (DESIGN.md "Fused encode + hash"): one workgroup per CU, SPW = 8
// stripes, 512-byte steps.  Data shards arrive by LDS-DMA
// (global_load_lds_dwordx4) into a D-slot ring, D-1 steps ahead; two
// bit-sliced encoder waves (4 stripes x 8 B per lane = 32 B per lane per shard)
// read the data rows, store parity to HBM and into a double-buffered parity
// row area; K/2 data-hasher waves hash the data rows straight out of the ring,
// M/2 parity-hasher waves the parity rows one step behind.  One barrier per
// step; every LDS row layout is bank-conflict free for the reads made of it.
//
// Usage: fused_r2 n [iters]
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

namespace r2 {
constexpr uint32_t CH = 512;            // bytes per shard per step
constexpr uint32_t IP = 2 * CH + 32;    // LDS pitch of one DMA instruction (rows of stripes i and i+4)
constexpr uint32_t PP = CH + 32;        // parity row pitch

// s_waitcnt vmcnt(min(n, 63)) only (gfx9 encoding)
constexpr uint32_t vmcnt_imm(int n) {
    return 0x0F70u | ((uint32_t)(n > 63 ? 63 : n) & 15u) | (((uint32_t)(n > 63 ? 63 : n) >> 4) & 3u) << 14;
}

// 4 x ds_read_b64 of one shard's four stripe rows and their lgkmcnt wait, as
// one asm statement: the compiler does not see LDS reads of the DMA ring, so
// it adds no vmcnt(0) for the in-flight LDS-DMA (the counted wait before
// each barrier retires it).
__device__ __forceinline__ void read4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t (&w)[8]) {
    uint2 x0, x1, x2, x3;
    asm volatile(
        "ds_read_b64 %0, %4\n\t"
        "ds_read_b64 %1, %5\n\t"
        "ds_read_b64 %2, %6\n\t"
        "ds_read_b64 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
        : "memory");
    w[0] = x0.x; w[1] = x0.y; w[2] = x1.x; w[3] = x1.y;
    w[4] = x2.x; w[5] = x2.y; w[6] = x3.x; w[7] = x3.y;
}

// 16 packets of one stream (8 B per lane, 32 B apart) from LDS, one asm.
__device__ __forceinline__ void read16(uint32_t a, uint64_t (&w)[16]) {
    asm volatile(
        "ds_read_b64 %0, %16 offset:0\n\t"
        "ds_read_b64 %1, %16 offset:32\n\t"
        "ds_read_b64 %2, %16 offset:64\n\t"
        "ds_read_b64 %3, %16 offset:96\n\t"
        "ds_read_b64 %4, %16 offset:128\n\t"
        "ds_read_b64 %5, %16 offset:160\n\t"
        "ds_read_b64 %6, %16 offset:192\n\t"
        "ds_read_b64 %7, %16 offset:224\n\t"
        "ds_read_b64 %8, %16 offset:256\n\t"
        "ds_read_b64 %9, %16 offset:288\n\t"
        "ds_read_b64 %10, %16 offset:320\n\t"
        "ds_read_b64 %11, %16 offset:352\n\t"
        "ds_read_b64 %12, %16 offset:384\n\t"
        "ds_read_b64 %13, %16 offset:416\n\t"
        "ds_read_b64 %14, %16 offset:448\n\t"
        "ds_read_b64 %15, %16 offset:480\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6]), "=&v"(w[7]),
          "=&v"(w[8]), "=&v"(w[9]), "=&v"(w[10]), "=&v"(w[11]), "=&v"(w[12]), "=&v"(w[13]), "=&v"(w[14]),
          "=&v"(w[15])
        : "v"(a)
        : "memory");
}

// acc[r][i] (^)= XOR of the input planes P[c][j] with bit j of
// mask[R0 + r][C0 + c][i], rows [R0, R0 + RN), shards [C0, C0 + NC), folded
// with v_bitop3 two terms at a time.
template <int K, int M, int R0, int RN, int C0, int NC, bool FIRST>
__device__ __forceinline__ void fold(uint32_t (&acc)[RN][8], const uint32_t (&P)[NC][8]) {
    constexpr bs::PlaneMasks<K, M> PM{};
#pragma unroll
    for (int r = 0; r < RN; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t t[1 + 8 * NC];
            int n = 0;
            if (!FIRST) t[n++] = acc[r][i];
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if ((PM.mask[R0 + r][C0 + c][i] >> j) & 1u) t[n++] = P[c][j];
            uint32_t v = n ? t[0] : 0u;
            int k = 1;
            for (; k + 1 < n; k += 2) v = x3(v, t[k], t[k + 1]);
            if (k < n) v ^= t[k];
            acc[r][i] = v;
        }
    }
}

// v_bfi_b32: (m & a) | (~m & b), one full-rate VALU op (the compiler builds
// the masked swap from v_and/v_and_or/v_or: ~5.5 ops instead of 4).
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// 8x8 bit transpose of 8 dwords (bs::transpose) with two shifts and two
// v_bfi_b32 per masked swap
__device__ __forceinline__ void swap_bfi(uint32_t& lo, uint32_t& hi, int s, uint32_t mask) {
    const uint32_t a = lo, b = hi;
    lo = bfi(mask, a, b << s);
    hi = bfi(mask, a >> s, b);
}
__device__ __forceinline__ void transpose_bfi(uint32_t (&w)[8], uint32_t m4, uint32_t m2, uint32_t m1) {
#pragma unroll
    for (int d = 0; d < 4; ++d) swap_bfi(w[d], w[d + 4], 4, m4);
    swap_bfi(w[0], w[2], 2, m2);
    swap_bfi(w[1], w[3], 2, m2);
    swap_bfi(w[4], w[6], 2, m2);
    swap_bfi(w[5], w[7], 2, m2);
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap_bfi(w[d], w[d + 1], 1, m1);
}

// Flag synchronisation (FS kernels): monotonic per-slot counters in LDS
// instead of workgroup barriers, so encoders and hashers run decoupled.
// signal(): the wave's earlier LDS accesses have completed (lgkmcnt(0)), then
// one lane bumps the counter; wait_ge(): poll (relaxed LDS load + s_sleep)
// until the counter reaches v; the empty asm keeps later LDS reads below it.
__device__ __forceinline__ void fs_signal(uint32_t* c) {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if ((threadIdx.x & 63u) == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (bounded: a wait gives up after ~2^20 polls so that a logic error ends the
// kernel with wrong bytes, never a hang)
__device__ __forceinline__ void fs_wait_ge(uint32_t* c, uint32_t v) {
    for (uint32_t i = 0; i < (1u << 20); ++i) {
        if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) break;
        __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
}

template <int K, int M, int D, int SPW>
struct Layout {
    static constexpr int HS = SPW / 2;                // a DMA instruction brings stripes i and i + HS
    static constexpr int NI = HS * K;                 // DMA instructions per step (1 KiB each)
    static constexpr uint32_t DSLOT = NI * IP;        // one step of all data rows
    static constexpr uint32_t PSLOT = SPW * M * PP;   // one step of all parity rows
};

// Encoder wave: stripe group g (stripes {2g, 2g+1, 2g+4, 2g+5}; lane L holds
// 8 B at column 8L of each: dwords [2j, 2j+1] of a shard = stripe j of the
// four), parity rows [H*RPW, (H+1)*RPW) where RPW = M / (EW/2).  It reads the
// data rows of ring slot s % D with plain LDS loads (it issues no LDS-DMA, so
// the compiler schedules and counts them freely), stores parity to HBM and to
// the parity rows of slot s & 1.
template <int K, int M, int D, int SPW, int EW, int H, int ABL, int NP = 2, bool FS = false, int NDH = 4, int NPH = 2>
__device__ __forceinline__ void encoder(const GfApplyParams& p, uint64_t n, uint32_t steps, uint64_t s0, uint32_t g,
                                        uint8_t* ring, uint8_t* prow, uint32_t* sync) {
    using L = Layout<K, M, D, SPW>;
    constexpr int HS = L::HS;
    constexpr int GW = EW / (SPW / 4);  // waves per stripe group
    constexpr int RPW = M / GW;         // parity rows per wave
    constexpr int R0 = H * RPW;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    const uint32_t mys[4] = {2 * g, 2 * g + 1, 2 * g + HS, 2 * g + HS + 1};
    uint8_t* const base = p.out_base;
    const uint64_t stride = p.stripe_stride;
    uint64_t pdst[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pdst[j] = (s0 + mys[j] < n ? s0 + mys[j] : 0) * stride + lane * 8u;
    if constexpr (ABL & 32) __builtin_amdgcn_s_setprio(1);
    lds_barrier();  // B(0): slot 0 landed (FS: counters initialised)
    uint32_t* const dready = sync;
    uint32_t* const dfree = sync + D;
    uint32_t* const pready = sync + 2 * D;
    uint32_t* const pfree = sync + 2 * D + NP;
#pragma unroll 1
    for (uint32_t s = 0; s < steps; ++s) {
        if constexpr (FS) fs_wait_ge(&dready[s % D], NDH * (s / D + 1));
        const uint8_t* slot = ring + (s % D) * L::DSLOT + 2 * g * IP + lane * 8u;
        uint32_t acc[RPW][8];
#pragma unroll
        for (int c = 0; c < K; c += 2) {
            uint32_t P[2][8];
#pragma unroll
            for (int cc = 0; cc < 2; ++cc) {
                const uint8_t* row = slot + HS * (c + cc) * IP;
                const uint2 a0 = *(const uint2*)row, a1 = *(const uint2*)(row + IP);
                const uint2 a2 = *(const uint2*)(row + CH), a3 = *(const uint2*)(row + IP + CH);
                P[cc][0] = a0.x; P[cc][1] = a0.y; P[cc][2] = a1.x; P[cc][3] = a1.y;
                P[cc][4] = a2.x; P[cc][5] = a2.y; P[cc][6] = a3.x; P[cc][7] = a3.y;
                if constexpr (!(ABL & 1)) { if constexpr (ABL & 16) bs::transpose(P[cc], m4, m2, m1); else transpose_bfi(P[cc], m4, m2, m1); }
            }
            if constexpr (ABL & 1) {
#pragma unroll
                for (int r = 0; r < RPW; ++r)
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        acc[r][i] = (c == 0 ? 0u : acc[r][i]) ^ P[0][i] ^ P[1][(i + r) & 7];
                continue;
            }
            if (c == 0) fold<K, M, R0, RPW, 0, 2, true>(acc, P);
            else if (c == 2) fold<K, M, R0, RPW, (K > 2 ? 2 : 0), 2, false>(acc, P);
            else if (c == 4) fold<K, M, R0, RPW, (K > 4 ? 4 : 0), 2, false>(acc, P);
            else fold<K, M, R0, RPW, (K > 6 ? 6 : 0), 2, false>(acc, P);
        }
        if constexpr (FS) {
            fs_signal(&dfree[s % D]);  // this wave is done reading the slot
            if (s >= (uint32_t)NP) fs_wait_ge(&pfree[s % NP], NPH * (s / NP));
        }
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if constexpr (!(ABL & 1)) { if constexpr (ABL & 16) bs::transpose(acc[r], m4, m2, m1); else transpose_bfi(acc[r], m4, m2, m1); }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint2 v = make_uint2(acc[r][2 * j], acc[r][2 * j + 1]);
                // a dead stripe's lanes computed stripe 0's parity from stripe
                // 0's data and store exactly the bytes stripe 0's lanes store
                *(uint2*)(base + pdst[j] + p.out_off[R0 + r] + (uint64_t)s * CH) = v;
                *(uint2*)(prow + (s % NP) * L::PSLOT + ((R0 + r) * SPW + mys[j]) * PP + lane * 8u) = v;
            }
        }
        if constexpr (FS) fs_signal(&pready[s % NP]);
        else lds_barrier();  // B(s+1): parity rows of step s published
    }
}

// HI streams per hasher quad (1 or 2): with 2, each quad advances two
// independent HighwayHash chains in one instruction stream (twice the ILP of
// the serial per-packet chain) and half as many hasher waves are needed.
template <int K, int M, int HI, int SPW>
struct Waves {
    static constexpr int DATA = (SPW * K) / (16 * HI);    // data-hasher waves
    static constexpr int PAR = (SPW * M + 16 * HI - 1) / (16 * HI);  // parity-hasher waves
};

template <int K, int M, int D, int EW = 4, int ABL = 0, int HI = 1, int SPW = 8, bool FS = false, int NP = 2>
__global__ __launch_bounds__(64 * (EW + Waves<K, M, HI, SPW>::DATA + Waves<K, M, HI, SPW>::PAR))
void k_fused_r2(const GfApplyParams p, const HashParams h) {
    static_assert(K % 2 == 0 && M % 2 == 0 && K <= 8 && M <= 4, "layout: pairs of shards per hasher wave");
    static_assert(EW == SPW / 2 || EW == SPW / 4, "one or two encoder waves per group of 4 stripes");
    static_assert((SPW * K) % (16 * HI) == 0, "whole data-hasher waves");
    using L = Layout<K, M, D, SPW>;
    using W = Waves<K, M, HI, SPW>;
    constexpr int HS = L::HS;
    constexpr int NG = SPW / 4;  // encoder stripe groups
    __shared__ __attribute__((aligned(16))) uint8_t ring[D * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t prow[NP * L::PSLOT];
    __shared__ uint32_t sync[2 * D + 2 * NP];  // FS counters: dready, dfree, pready, pfree
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    if (FS && threadIdx.x < 2 * D + 2 * NP) sync[threadIdx.x] = 0;
    const uint64_t n = h.n;
    const uint32_t steps = p.units;  // S / CH
    const uint64_t s0 = (uint64_t)blockIdx.x * SPW;
    const uint32_t ring_base = (uint32_t)(uintptr_t)ring;

    if (wave < (uint32_t)EW) {
        const uint32_t g = wave % NG;
        if (EW == NG || wave < (uint32_t)NG)
            encoder<K, M, D, SPW, EW, 0, ABL, NP, FS, W::DATA, W::PAR>(p, n, steps, s0, g, ring, prow, sync);
        else
            encoder<K, M, D, SPW, EW, (EW == 2 * NG ? 1 : 0), ABL, NP, FS, W::DATA, W::PAR>(p, n, steps, s0, g, ring,
                                                                                        prow, sync);
        return;
    }
    // --------------------------------- hashers ---------------------------------
    const uint32_t hw = wave - EW, j = lane >> 2;
    const bool is_data = hw < (uint32_t)W::DATA;
    constexpr int NDI = 16 * HI / 2;  // DMA instructions a data-hasher wave owns
    uint32_t stripe_l[HI], shard[HI], roff[HI];
    bool live[HI];
#pragma unroll
    for (int x = 0; x < HI; ++x) {
        if (is_data) {
            // data hasher hw owns DMA instructions [NDI hw, NDI (hw+1)): it
            // brings them into the ring D-1 steps ahead and hashes both halves
            // of each; stream x of quad j: instruction NDI hw + 8x + (j & 7),
            // half j >> 3 (conflict-free ds_read_b64: the 8 quads of a 32-lane
            // group read 8 rows whose bases differ by 32 B mod 256 B)
            const uint32_t idx = NDI * hw + 8 * x + (j & 7u), half = j >> 3;
            shard[x] = idx / HS;
            stripe_l[x] = idx % HS + HS * half;
            roff[x] = idx * IP + half * CH + 8 * q;
        } else {
            uint32_t pi = 16 * HI * (hw - W::DATA) + 16 * x + j;  // parity row index r * SPW + stripe
            if (pi >= (uint32_t)(SPW * M)) pi = 0;                 // idle quad (M*SPW not a multiple)
            shard[x] = K + pi / SPW;
            stripe_l[x] = pi % SPW;
            roff[x] = pi * PP + 8 * q;
        }
        live[x] = s0 + stripe_l[x] < n &&
                  (is_data || 16 * HI * (hw - W::DATA) + 16 * x + j < (uint32_t)(SPW * M));
    }
    HHQuad st[HI];
#pragma unroll
    for (int x = 0; x < HI; ++x) hhq_init(st[x], h.key, q);
    auto hash16 = [&](const uint32_t (&a)[HI]) {
        uint64_t w[HI][16];
#pragma unroll
        for (int x = 0; x < HI; ++x) read16(a[x], w[x]);
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int x = 0; x < HI; ++x) {
                if constexpr (ABL & 2) st[x].v0 ^= w[x][t];
                else hhq_update(st[x], w[x][t]);
            }
    };
    if constexpr (ABL & 64) __builtin_amdgcn_s_setprio(1);
    if (is_data) {
        // DMA instruction NDI hw + k: shard c = (NDI hw + k) / 4, stripe pair
        // i = k % 4: lanes 0-31 stripe i, lanes 32-63 stripe i + 4
        uint64_t dsrc[HS];
#pragma unroll
        for (int i = 0; i < HS; ++i) {
            const uint64_t sg = s0 + i + (lane >> 5) * HS;
            dsrc[i] = (sg < n ? sg : 0) * p.stripe_stride + (lane & 31u) * 16u;
        }
        const uint8_t* base = p.out_base;
        auto dma = [&](uint32_t step) {
#pragma unroll
            for (int k = 0; k < NDI; ++k) {
                const uint32_t c = (NDI * hw + k) / HS;  // wave-uniform
                const uint8_t* src = base + dsrc[k % HS] + p.in_off[c] + (uint64_t)step * CH;
                __builtin_amdgcn_global_load_lds(
                    (const void*)src,
                    (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT + (NDI * hw + k) * IP),
                    16, 0, 0);
            }
        };
        if constexpr (FS) {
            // decoupled: DMA(t) lands -> dready[t % D]; refilling the slot of
            // step t-1 waits until every encoder wave released it (dfree)
            uint32_t* const dready = sync;
            uint32_t* const dfree = sync + D;
            for (int d = 0; d < D - 1; ++d)
                if (d < (int)steps) dma(d);
            lds_barrier();  // counters initialised
#pragma unroll 1
            for (uint32_t s = 0; s < steps; ++s) {
                // DMA(s) landed: younger are DMA(s+1 .. min(s+D-2, steps-1))
                const uint32_t younger = min((uint32_t)(D - 2), steps - 1 - s);
                if (younger >= 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * NDI));
                else if (younger == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(NDI));
                else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
                fs_signal(&dready[s % D]);
                uint32_t a[HI];
#pragma unroll
                for (int x = 0; x < HI; ++x) a[x] = ring_base + (s % D) * L::DSLOT + roff[x];
                hash16(a);
                if (s + D - 1 < steps) {
                    if (s >= 1) fs_wait_ge(&dfree[(s - 1) % D], EW * ((s - 1) / D + 1));
                    dma(s + D - 1);
                }
            }
        } else {
#pragma unroll
            for (int d = 0; d < D - 1; ++d) dma(d < (int)steps ? d : steps - 1);
            __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * NDI));  // DMA(0) landed
            lds_barrier();  // B(0)
#pragma unroll 1
            for (uint32_t s = 0; s < steps; ++s) {
                dma(s + D - 1 < steps ? s + D - 1 : steps - 1);  // into the slot step s-1 used
                uint32_t a[HI];
#pragma unroll
                for (int x = 0; x < HI; ++x) a[x] = ring_base + (s % D) * L::DSLOT + roff[x];
                hash16(a);
                __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * NDI));  // DMA(s+1) landed
                lds_barrier();  // B(s+1)
            }
        }
    } else if constexpr (FS) {
        uint32_t* const pready = sync + 2 * D;
        uint32_t* const pfree = sync + 2 * D + NP;
        lds_barrier();  // counters initialised
#pragma unroll 1
        for (uint32_t s = 0; s < steps; ++s) {
            fs_wait_ge(&pready[s % NP], EW * (s / NP + 1));
            uint32_t a[HI];
#pragma unroll
            for (int x = 0; x < HI; ++x) a[x] = (uint32_t)(uintptr_t)prow + (s % NP) * L::PSLOT + roff[x];
            hash16(a);
            fs_signal(&pfree[s % NP]);
        }
    } else {
        lds_barrier();  // B(0)
#pragma unroll 1
        for (uint32_t s = 0; s <= steps; ++s) {
            if (s > 0) {  // parity rows of step s-1, published by B(s)
                uint32_t a[HI];
#pragma unroll
                for (int x = 0; x < HI; ++x) a[x] = (uint32_t)(uintptr_t)prow + ((s - 1) % NP) * L::PSLOT + roff[x];
                hash16(a);
            }
            if (s < steps) lds_barrier();  // B(s+1)
        }
    }
#pragma unroll
    for (int x = 0; x < HI; ++x)
        if (live[x]) hhq_finish(st[x], h.out + ((s0 + stripe_l[x]) * (K + M) + shard[x]) * 32u, q);
}

// ---------------------------------------------------------------------------
// r4: symmetric waves.  8 waves, each = one bit-sliced encoder unit (stripe
// group g = w & 1, ONE parity row r = w >> 1) + a DMA share (instructions
// [4w, 4w+4)) + 12 hash streams (the 8 data rows it brought in, 4 parity
// rows), all in one instruction stream so the hash chains' latency can be
// filled with the encoder's independent work.
template <int K, int M, int D, int ABL = 0>
__global__ __launch_bounds__(512)
void k_fused_r4(const GfApplyParams p, const HashParams h) {
    static_assert(K == 8 && M == 4, "r4 layout: 8 waves = 2 groups x 4 rows");
    constexpr int SPW = 8, HS = 4;
    using L = Layout<K, M, D, SPW>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[D * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t prow[2 * L::PSLOT];
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint32_t g = w & 1u, r = w >> 1, j = lane >> 2;
    const uint64_t n = h.n;
    const uint32_t steps = p.units;
    const uint64_t s0 = (uint64_t)blockIdx.x * SPW;
    const uint32_t ring_base = (uint32_t)(uintptr_t)ring, prow_base = (uint32_t)(uintptr_t)prow;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    const uint32_t mys[4] = {2 * g, 2 * g + 1, 2 * g + HS, 2 * g + HS + 1};
    uint8_t* const base = p.out_base;
    const uint64_t stride = p.stripe_stride;
    // hash streams of this lane's quad: j < 8 data (instruction 4w + (j & 3),
    // half j >> 2), 8 <= j < 12 parity row 4w + j - 8, j >= 12 idle
    const bool hdata = j < 8, hpar = j >= 8 && j < 12;
    uint32_t hshard, hstripe, hroff;
    if (hdata) {
        const uint32_t idx = 4 * w + (j & 3u), half = j >> 2;
        hshard = idx / HS;
        hstripe = idx % HS + HS * half;
        hroff = idx * IP + half * CH + 8 * q;
    } else {
        const uint32_t pi = hpar ? 4 * w + (j - 8) : 0;
        hshard = K + pi / SPW;
        hstripe = pi % SPW;
        hroff = pi * PP + 8 * q;
    }
    const bool hlive = (hdata || hpar) && s0 + hstripe < n;
    HHQuad st;
    hhq_init(st, h.key, q);
    // DMA: instruction 4w + k: shard c = (4w + k) / 4 = w, stripe pair k
    uint64_t dsrc;
    {
        const uint64_t sg = s0 + (lane >> 5) * HS;  // + k below
        dsrc = (lane & 31u) * 16u;
        (void)sg;
    }
    auto dma = [&](uint32_t step) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t sg = s0 + k + (lane >> 5) * HS;
            const uint8_t* src = base + (sg < n ? sg : 0) * stride + dsrc + p.in_off[w] + (uint64_t)step * CH;
            __builtin_amdgcn_global_load_lds(
                (const void*)src, (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT + (4 * w + k) * IP),
                16, 0, 0);
        }
    };
    uint64_t pdst[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) pdst[jj] = (s0 + mys[jj] < n ? s0 + mys[jj] : 0) * stride + lane * 8u;
#pragma unroll
    for (int d = 0; d < D - 1; ++d) dma(d < (int)steps ? d : steps - 1);
    __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * 4));
    lds_barrier();  // B(0)
    constexpr int ND = 4, NS = 4;
#pragma unroll 1
    for (uint32_t s = 0; s <= steps; ++s) {
        if (s < steps) {
            dma(s + D - 1 < steps ? s + D - 1 : steps - 1);
            // ---- encoder unit: row r of group g ----
            const uint8_t* slot = ring + (s % D) * L::DSLOT + 2 * g * IP + lane * 8u;
            uint32_t acc[1][8];
#pragma unroll
            for (int c = 0; c < K; c += 2) {
                uint32_t P[2][8];
#pragma unroll
                for (int cc = 0; cc < 2; ++cc) {
                    const uint8_t* row = slot + HS * (c + cc) * IP;
                    const uint2 a0 = *(const uint2*)row, a1 = *(const uint2*)(row + IP);
                    const uint2 a2 = *(const uint2*)(row + CH), a3 = *(const uint2*)(row + IP + CH);
                    P[cc][0] = a0.x; P[cc][1] = a0.y; P[cc][2] = a1.x; P[cc][3] = a1.y;
                    P[cc][4] = a2.x; P[cc][5] = a2.y; P[cc][6] = a3.x; P[cc][7] = a3.y;
                    if constexpr (!(ABL & 1)) transpose_bfi(P[cc], m4, m2, m1);
                }
                if constexpr (ABL & 1) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc[0][i] = (c == 0 ? 0u : acc[0][i]) ^ P[0][i] ^ P[1][i];
                    continue;
                }
                // row r is wave-uniform but a runtime value: one fold per row
                if (r == 0) {
                    if (c == 0) fold<K, M, 0, 1, 0, 2, true>(acc, P); else if (c == 2) fold<K, M, 0, 1, 2, 2, false>(acc, P);
                    else if (c == 4) fold<K, M, 0, 1, 4, 2, false>(acc, P); else fold<K, M, 0, 1, 6, 2, false>(acc, P);
                } else if (r == 1) {
                    if (c == 0) fold<K, M, 1, 1, 0, 2, true>(acc, P); else if (c == 2) fold<K, M, 1, 1, 2, 2, false>(acc, P);
                    else if (c == 4) fold<K, M, 1, 1, 4, 2, false>(acc, P); else fold<K, M, 1, 1, 6, 2, false>(acc, P);
                } else if (r == 2) {
                    if (c == 0) fold<K, M, 2, 1, 0, 2, true>(acc, P); else if (c == 2) fold<K, M, 2, 1, 2, 2, false>(acc, P);
                    else if (c == 4) fold<K, M, 2, 1, 4, 2, false>(acc, P); else fold<K, M, 2, 1, 6, 2, false>(acc, P);
                } else {
                    if (c == 0) fold<K, M, 3, 1, 0, 2, true>(acc, P); else if (c == 2) fold<K, M, 3, 1, 2, 2, false>(acc, P);
                    else if (c == 4) fold<K, M, 3, 1, 4, 2, false>(acc, P); else fold<K, M, 3, 1, 6, 2, false>(acc, P);
                }
            }
            if constexpr (!(ABL & 1)) transpose_bfi(acc[0], m4, m2, m1);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const uint2 v = make_uint2(acc[0][2 * jj], acc[0][2 * jj + 1]);
                *(uint2*)(base + pdst[jj] + p.out_off[r] + (uint64_t)s * CH) = v;
                *(uint2*)(prow + (s & 1u) * L::PSLOT + (r * SPW + mys[jj]) * PP + lane * 8u) = v;
            }
        }
        // ---- hash: data rows of step s, parity rows of step s-1 ----
        if (s < steps || hpar) {
            const uint32_t a = hdata ? ring_base + (s % D) * L::DSLOT + hroff
                                     : prow_base + ((s + 1) & 1u) * L::PSLOT + hroff;  // (s-1) & 1
            uint64_t wv[16];
            read16(a, wv);
            const bool go = hdata ? s < steps : (hpar && s > 0);
            if (go) {
#pragma unroll
                for (int t = 0; t < 16; ++t) {
                    if constexpr (ABL & 2) st.v0 ^= wv[t];
                    else hhq_update(st, wv[t]);
                }
            }
        }
        if (s < steps) {
            if (s + 1 >= (uint32_t)(D - 1)) __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * ND + (D - 1) * NS));
            else __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * ND + NS));
            lds_barrier();  // B(s+1)
        }
    }
    if (hlive) hhq_finish(st, h.out + ((s0 + hstripe) * (K + M) + hshard) * 32u, q);
}
}  // namespace r2

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

constexpr int K = 8, M = 4;

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096;
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t S = argc > 3 ? strtoull(argv[3], 0, 10) : 131072;
    const uint64_t STRIDE = (K + M) * S;
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
    const uint32_t g8 = (uint32_t)((n + 7) / 8);
    auto thr = [](int ew, int hi = 1, int spw = 8) {
        if (spw == 4) return 64u * (ew + r2::Waves<K, M, 1, 4>::DATA + r2::Waves<K, M, 1, 4>::PAR);
        return 64u * (ew + (hi == 1 ? r2::Waves<K, M, 1, 8>::DATA + r2::Waves<K, M, 1, 8>::PAR
                                    : r2::Waves<K, M, 2, 8>::DATA + r2::Waves<K, M, 2, 8>::PAR));
    };
    const uint32_t g4 = (uint32_t)((n + 3) / 4);
    GfApplyParams pr = p;
    pr.units = S / r2::CH;
    GfApplyParams pe = p;
    pe.units = S / 16;
    struct V { const char* name; std::function<void()> f; };
    std::vector<V> vs = {
        {"fused (prod)", [&] { CK(launch_encode_hash_fused(p, h, S, n, 0)); }},
        {"r4 D3", [&] { r2::k_fused_r4<K, M, 3, 0><<<g8, 512>>>(pr, h); }},
        {"r4 D2", [&] { r2::k_fused_r4<K, M, 2, 0><<<g8, 512>>>(pr, h); }},
        {"v8 bar D3", [&] { r2::k_fused_r2<K, M, 3, 4, 0, 1, 8, false, 2><<<g8, thr(4)>>>(pr, h); }},
        {"r4 D3 nohash", [&] { r2::k_fused_r4<K, M, 3, 2><<<g8, 512>>>(pr, h); }},
        {"r4 D3 noGF", [&] { r2::k_fused_r4<K, M, 3, 1><<<g8, 512>>>(pr, h); }},
        {"r4 D3 neither", [&] { r2::k_fused_r4<K, M, 3, 3><<<g8, 512>>>(pr, h); }},
        {"encode only", [&] { CK(launch_gf_apply_vec(pe, n, 0)); }},
    };
    {
        const size_t nd = n * (K + M) * 32;
        std::vector<uint8_t> ref(nd), got(nd), pref(n * STRIDE), pgot(n * STRIDE);
        vs[0].f();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pref.data(), d, n * STRIDE, hipMemcpyDeviceToHost));
        for (int v = 1; v <= 3; ++v) {
            CK(hipMemset(dig, 0, nd));
            for (uint64_t s = 0; s < n; ++s) CK(hipMemset(d + s * STRIDE + K * S, 0, M * S));
            vs[v].f();
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), dig, nd, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pgot.data(), d, n * STRIDE, hipMemcpyDeviceToHost));
            uint64_t bad_d = 0, bad_p = 0;
            for (uint64_t x = 0; x < n * (K + M); ++x) bad_d += memcmp(&ref[x * 32], &got[x * 32], 32) != 0;
            for (uint64_t s = 0; s < n; ++s) bad_p += memcmp(&pref[s * STRIDE], &pgot[s * STRIDE], STRIDE) != 0;
            printf("%s: digests %s (%llu bad), stripes %s (%llu bad)\n", vs[v].name, bad_d ? "MISMATCH" : "ok",
                   (unsigned long long)bad_d, bad_p ? "MISMATCH" : "ok", (unsigned long long)bad_p);
        }
        vs[0].f();
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
