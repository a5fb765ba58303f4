// rs_decode_net16.hip — the one-pass GET / heal kernel for RS(16,4) with its
// rows as compile-time XOR networks per erasure pattern
// (k_decode_records_net16<PID>; networks in the generated rs164_decode_nets.h,
// tools/gen_decode_nets.py --k 16).  Compiled RSG_NET_PARTS times (Makefile)
// like rs_decode_net.hip.  RS(12,4) has its own four-wave form
// (rs_decode_netq.hip).
//
// The table kernel's RS(16,4) workgroup (k_decode_records_dma<16,NF,4,TH>:
// 4 stripes, NF present record files DMA'd into a 3-slot LDS ring per
// 512-byte step, ceil(2 NF / 8) DMA + verify-hash waves) with its 4 table-GF
// waves (one per stripe, 16 survivors x 4 rows of v_perm lookups each)
// replaced by two network waves over the one 4-stripe group (8 bytes of
// each stripe per lane): the 16 survivors' 128 bit planes do not fit one
// wave beside the rows, so
//   wave B transposes survivors 8-15 and runs the pattern's net_hi (all R
//     rows over those 64 planes) and hands its 32 partial planes to
//     wave A through a double-buffered LDS area;
//   wave A transposes survivors 0-7, runs net_lo, and one interval later
//     XORs in B's half, transposes the rows back, stores the rebuilt rows
//     (heal: also into the target-row area for the target hashers, now two
//     steps behind the DMA) and compares the surplus rows it kept from the
//     ring.  Each copies its own data survivors through (GET).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <array>
#include <utility>

#include "rs_device.h"
#include "rs_kernels.h"
#include "rs_records.h"

#ifndef RSG_NET_PART
#error "RSG_NET_PART (0 .. RSG_NET_PARTS-1) is set by the Makefile"
#endif

namespace rsg {

#include "rs164_decode_nets.h"
namespace decnetk = decnet16;
constexpr int kNetK = 16;
constexpr int kNetA = 8;  // survivors of network wave A (the rest are B's)

template <int NF, int TH>
struct Net16Shape : RecRing<NF, 4, TH> {
    static constexpr int NG = 2;                   // network waves A (survivors 0-7) and B (8-15)
    static constexpr int WAVES = RecRing<NF, 4, TH>::HW + NG + RecRing<NF, 4, TH>::TW;
    static constexpr uint32_t XSLOT = 32 * 64 * 4;  // a step's exchanged partial planes, lane-major (<= 8 KiB)
    static constexpr int XB = TH ? 1 : 0;           // extra barrier: heal's target hashers trail by 2 steps
    static constexpr uint32_t LDS_REST = 4 * XSLOT + (TH ? 2 * RecRing<NF, 4, TH>::TSLOT : 16);
    static constexpr int RD = dma::D;  // ring slots (18-19 files: 3 is what the LDS holds)
};

__device__ __forceinline__ void put8_16(uint8_t* p, const uint2& v) { st64_any(p, u64_of(v)); }  // any alignment

// Network wave A (survivors 0-7) or B (8-15) of the 4-stripe group.  Each
// runs its half network for all R rows, keeps its half of the rows it
// finishes — A the stored rows [0, NST), B the compared rows [NST, R) — and
// hands its half of the other wave's rows over through a double-buffered LDS
// area; one interval later each XORs the other's half in, transposes its
// rows back and stores (A; heal: also into the target-row area) or compares
// them with the surplus rows it kept from the ring (B, which also writes the
// stripes' verdicts).  Splitting the finishing work by row kind keeps the
// two waves' issue about equal (a single finishing wave paired with a hash
// wave on its SIMD set the pace).
template <int PID, int NF, int TH, bool A>
__device__ __forceinline__ void net16_wave(const GfApplyParams& p, uint64_t n, uint32_t steps, uint64_t s0,
                                           const uint8_t* ring, uint8_t* xbuf, uint8_t* trow) {
    using dma::CH;
    using dma::IP;
    using dma::PP;
    using L = Net16Shape<NF, TH>;
    constexpr int D = L::RD;
    constexpr decnetk::Pattern pat = decnetk::kPatterns[PID];
    constexpr int R = pat.R, NST = pat.n_store, NCMP = R - NST, SPW = L::SPW, HS = L::HS;
    static_assert(pat.nf == NF && (pat.heal ? NST : 0) == TH && R <= 4 && NST <= R && HS == 2, "pattern shape");
    constexpr int C0 = A ? 0 : kNetA, NC = A ? kNetA : kNetK - kNetA;  // this wave's survivors [C0, C0 + NC)
    // heal (SF): A finishes the stored rows, B the compared ones; GET: A
    // finishes every row (B holding half the rows as well as GET's
    // copy-through spilled at the 256-VGPR cap)
    constexpr bool SF = TH > 0;
    constexpr int K0 = A ? 0 : NST, KN = A ? (SF ? NST : R) : (SF ? NCMP : 0);  // rows it finishes
    constexpr int G0 = A ? NST : 0, GN = A ? (SF ? NCMP : 0) : (SF ? NST : R);  // rows it gives away
    constexpr bool CMP = K0 + KN > NST;  // it finishes compared rows (keeps the surplus rows, writes verdicts)
    // xbuf: B -> A (its half of the stored rows) at +0, A -> B (its half of the
    // compared rows) at +2 XSLOT, each double-buffered by step parity
    constexpr uint32_t TO_A = 0, TO_B = L::XSLOT;
    if (p.wave_prio & kPrioGf) __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    const uint32_t cmask = p.copy_mask;
    // stripe j of the group at ring row + {0, IP, CH, IP + CH}
    bool live[4];  // wave-uniform: a dead stripe (past n) computes stripe 0's rows and stores nothing
    uint8_t* ob[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        live[j] = s0 + j < n;
        ob[j] = p.out_base + (live[j] ? s0 + j : 0) * p.out_stripe_stride + lane * 8u;
    }
    auto row4 = [&](const uint8_t* row, uint2 (&x)[4]) {
        x[0] = *(const uint2*)row;
        x[1] = *(const uint2*)(row + IP);
        x[2] = *(const uint2*)(row + CH);
        x[3] = *(const uint2*)(row + IP + CH);
    };
    uint32_t diff[4] = {0u, 0u, 0u, 0u};  // CMP: OR of this lane's surplus-parity differences
    const uint32_t tail = walk_tail(p.byte_end, steps);  // a ragged walk's last step: first tail bytes only
    uint32_t keep[32];                    // step t-1's half of the rows it finishes ([8 K0, 8 (K0 + KN))), held across B(t)
    uint2 cmp[NCMP ? NCMP : 1][4];        // CMP: step t-1's surplus rows, held across B(t)
    // the exchange slot (direction to, step t) as lane-major dwords
    auto xb_at = [&](uint32_t to, uint32_t t) { return (uint32_t*)(xbuf + 2 * to + (t & 1) * L::XSLOT) + lane; };
    // step t: this wave's 8 survivors -> planes -> its half of every row;
    // the other wave's rows out to LDS; copy-through of its data survivors (GET)
    auto half = [&](uint32_t t) {
        const uint8_t* slot = ring + (t % D) * L::DSLOT + lane * 8u;
        uint32_t P[64];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint2 a[4];
            row4(slot + (C0 + c) * HS * IP, a);
            uint32_t w[8] = {a[0].x, a[0].y, a[1].x, a[1].y, a[2].x, a[2].y, a[3].x, a[3].y};
            dma::transpose(w, m4, m2, m1);
#pragma unroll
            for (int j = 0; j < 8; ++j) P[8 * c + j] = w[j];
        }
        // the network writes every row straight into keep; the given-away
        // rows are stored to LDS from there and never read again
        if constexpr (A) decnetk::net_lo<PID>(P, keep);
        else decnetk::net_hi<PID>(P, keep);
        uint32_t* xo = xb_at(A ? TO_B : TO_A, t);
#pragma unroll
        for (int i = 0; i < 8 * GN; ++i) xo[64 * i] = keep[8 * G0 + i];
        if constexpr (CMP) {
#pragma unroll
            for (int r = 0; r < NCMP; ++r) row4(slot + (kNetK + r) * HS * IP, cmp[r]);
        }
        if (!TH && cmask) {  // GET: this wave's present data survivors copied through
            const bool part = t + 1 == steps && tail != CH;  // wave-uniform
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (!((cmask >> (C0 + c)) & 1u)) continue;  // wave-uniform
                uint2 x[4];
                row4(slot + (C0 + c) * HS * IP, x);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!live[j]) continue;
                    if (!part) put8_16(ob[j] + p.copy_off[C0 + c] + (uint64_t)t * CH, x[j]);
                    else st64_part(ob[j] + p.copy_off[C0 + c] + (uint64_t)t * CH, u64_of(x[j]), lane * 8u, tail);
                }
            }
        }
    };
    // step s (in interval s+1): the other wave's half in, rows back to bytes,
    // stores (A) / compares (B)
    auto finish = [&](uint32_t s) {
        const uint32_t* xi = xb_at(A ? TO_A : TO_B, s);
        const bool part = s + 1 == steps && tail != CH;  // wave-uniform
#pragma unroll
        for (int k = 0; k < KN; ++k) {
            const int r = K0 + k;  // the row (compile-time after unrolling)
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = keep[8 * r + i] ^ xi[64 * (8 * k + i)];
            dma::transpose(w, m4, m2, m1);
            if (r < NST) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint2 v = make_uint2(w[2 * j], w[2 * j + 1]);
                    if (live[j]) {
                        if (!part) put8_16(ob[j] + p.out_off[r] + (uint64_t)s * CH, v);
                        else st64_part(ob[j] + p.out_off[r] + (uint64_t)s * CH, u64_of(v), lane * 8u, tail);
                    }
                    if constexpr (TH > 0)
                        *(uint2*)(trow + (s & 1) * L::TSLOT + (r * SPW + j) * PP + lane * 8u) = v;
                }
            } else if (!part) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    diff[j] = or_diff(or_diff(diff[j], cmp[r - NST][j].x, w[2 * j]), cmp[r - NST][j].y,
                                      w[2 * j + 1]);
            } else {  // only the bytes before the ragged step's tail count
                const uint64_t keepm = part_mask8(lane * 8u, tail);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint64_t d =
                        (u64_of(cmp[r - NST][j]) ^ ((uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32))) & keepm;
                    diff[j] |= (uint32_t)d | (uint32_t)(d >> 32);
                }
            }
        }
    };
    lds_barrier();  // B(0)
    if constexpr (KN == 0) {  // GET's B: halves only
#pragma unroll 1
        for (uint32_t t = 0; t < steps; ++t) {
            half(t);
            lds_barrier();  // B(t+1)
        }
    } else {
        // interval t: finish step t-1 (the other half published by B(t)), then step t's half
#pragma unroll 1
        for (uint32_t t = 0; t <= steps; ++t) {
            if (t > 0) finish(t - 1);
            if (t < steps) {
                half(t);
                lds_barrier();  // B(t+1)
            }
        }
    }
#pragma unroll
    for (int b = 0; b < L::XB; ++b) lds_barrier();  // B(steps+1): the last target rows published
    if constexpr (CMP) {  // each stripe's surplus verdict, written whole
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool any_bad = __builtin_amdgcn_ballot_w64(diff[j] != 0u) != 0;
            if (live[j] && lane == 0) p.ok_flags[s0 + j] = any_bad ? 0 : 1;
        }
    }
}

template <int PID, int NF, int TH>
__global__ __launch_bounds__((64 * Net16Shape<NF, TH>::WAVES)) void k_decode_records_net16(const GfApplyParams p,
                                                                                           const HashParams h) {
    using L = Net16Shape<NF, TH>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[L::RD * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t xbuf[4 * L::XSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t trow[TH ? 2 * L::TSLOT : 16];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t steps = p.units;
    const uint64_t s0 = (uint64_t)blockIdx.x * L::SPW;
    if (TH && wave >= (uint32_t)(L::HW + L::NG)) {
        records_target_hasher<4, TH, 2>(p, h, trow, wave - L::HW - L::NG, steps, s0);
        return;
    }
    if (wave == (uint32_t)L::HW) {
        net16_wave<PID, NF, TH, true>(p, h.n, steps, s0, ring, xbuf, trow);
        return;
    }
    if (wave == (uint32_t)L::HW + 1) {
        net16_wave<PID, NF, TH, false>(p, h.n, steps, s0, ring, xbuf, trow);
        return;
    }
    records_hash_wave<NF, 4, L::XB, L::RD>(h, p.wave_prio, ring, wave, steps, s0);
}

static_assert(dma::D * 2 * 19 * dma::IP + 4 * Net16Shape<19, 0>::XSLOT + 16 <= 160 * 1024, "RS(16,4) GET fits");
static_assert(dma::D * 2 * 18 * dma::IP + 4 * Net16Shape<18, 2>::XSLOT + 2 * Net16Shape<18, 2>::TSLOT <= 160 * 1024,
              "RS(16,4) heal fits");
static_assert(dma::D * 2 * 19 * dma::IP + 4 * Net16Shape<19, 1>::XSLOT + 2 * Net16Shape<19, 1>::TSLOT <= 160 * 1024,
              "RS(16,4) heal of one shard fits");

using Net16Launch = void (*)(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream);

template <int PID>
static void launch_net16(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    constexpr decnetk::Pattern pat = decnetk::kPatterns[PID];
    constexpr int NF = pat.nf, TH = pat.heal ? pat.n_store : 0;
    hipLaunchKernelGGL((k_decode_records_net16<PID, NF, TH>), dim3((uint32_t)blocks),
                       dim3(64 * Net16Shape<NF, TH>::WAVES), 0, stream, p, h);
}

template <int PID>
constexpr Net16Launch pick_net16() {
    if constexpr (PID % RSG_NET_PARTS == RSG_NET_PART) return &launch_net16<PID>;
    else return nullptr;
}

template <size_t... I>
constexpr std::array<Net16Launch, sizeof...(I)> net16_table(std::index_sequence<I...>) {
    return {pick_net16<(int)I>()...};
}

static const std::array<Net16Launch, decnetk::kCount> kNet16Part =
    net16_table(std::make_index_sequence<decnetk::kCount>{});

#define RSG_NET16_CAT2(a, b, c) a##b##c
#define RSG_NET16_CAT(a, b, c) RSG_NET16_CAT2(a, b, c)

// This part's launcher (launch_records_net16_partN): false if pattern `pid`
// is instantiated elsewhere.
bool RSG_NET16_CAT(launch_records_net16_part, RSG_NET_PART, )(int pid, uint64_t blocks, const GfApplyParams& p,
                                                             const HashParams& h, hipStream_t stream) {
    if (pid < 0 || pid >= decnetk::kCount || !kNet16Part[pid]) return false;
    kNet16Part[pid](blocks, p, h, stream);
    return true;
}

#if RSG_NET_PART == 0
// The pattern whose coefficient rows equal the launch's (R x 16, row-major),
// or -1.
int records_net16_pattern(int heal, int nf, int R, int n_store, const uint8_t* coef) {
    for (int i = 0; i < decnetk::kCount; ++i) {
        const decnetk::Pattern& pt = decnetk::kPatterns[i];
        if (pt.heal != heal || pt.nf != nf || pt.R != R || pt.n_store != n_store) continue;
        bool eq = true;
        for (int r = 0; r < R && eq; ++r)
            for (int c = 0; c < kNetK && eq; ++c) eq = pt.coef[r][c] == coef[r * kNetK + c];
        if (eq) return i;
    }
    return -1;
}
#endif

}  // namespace rsg
