// rs_decode_netq.hip — the one-pass GET / heal kernel for RS(12,4), the
// default geometry of a 16-drive set (storageclass.rs:24-31), with FOUR
// network waves (k_decode_records_net12<PID>): its rows as compile-time XOR
// networks per erasure pattern in four parts of the survivors (generated
// rs124_decode_nets.h, tools/gen_decode_nets.py --k 12).  Compiled
// RSG_NET_PARTS times (Makefile, RSG_NETQ_K=12) like rs_decode_net.hip; and
// again for RS(10,4), the 14-drive default (RSG_NETQ_K=10,
// k_decode_records_net10, rs104_decode_nets.h: parts of 3, 3, 2, 2
// survivors).
//
// At 1 MiB blocks RS(12,4)'s shards are 87382 bytes, so its record walks are
// ragged (170 whole 512-byte steps and 342 bytes, rs_records.h walk_tail) and
// its records sit at every alignment (LDS-DMA takes unaligned sources).
//
// The workgroup is the table kernel's (k_decode_records_dma<12,NF,4,TH>: 4
// stripes, NF present record files DMA'd into an LDS ring per 512-byte step
// by DMA + verify-hash waves) with the GF work done by four network waves,
// one per SIMD beside a hash wave: wave q transposes survivors 3q..3q+2 of
// the 4-stripe group (8 bytes of each stripe per lane) into 24 bit planes,
// runs the pattern's net_q<PID, q> (its part of all R <= 4 rows), keeps its
// part of row q and XORs its parts of the other rows into their
// accumulators in a double-buffered LDS area (LDS atomic XOR, ds_xor_b32:
// 8 KiB a step, not 24 for the parts side by side); one interval later it
// XORs row q's accumulator in, transposes the row back and stores it (rows
// [0, NST): rebuilt data / heal targets, heal also into the target-row area
// for the target hashers) or compares it with the surplus parity row it kept
// from the ring.
//
// Ring depth and workgroups per CU: GET takes a 2-slot ring, so two
// workgroups (two hash and two network waves per SIMD) share a CU and each
// hides the other's dependent hash chains and network latency — 2 data lost
// 1.39 against 1.50 ms with one workgroup and a 4-slot ring (interleaved on
// one box, profiles/r04/k/).  The heal's target rows do not fit two
// workgroups' LDS; it keeps one and a 4-slot ring.  Two network waves over
// halves (rs_decode_net16.hip's shape) ran GET 2 lost at 1.52 ms
// (profiles/r04/d/): both shared a SIMD with a hash wave at ~600 VALU a step.
// The same four-wave form for RS(8,4) (2 survivors a wave, 4-stripe
// workgroups, two per CU) measured 3-4 % slower than rs_decode_net.hip's
// 8-stripe workgroups (profiles/r04/l/) and is not built.
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
#ifndef RSG_NET_ABLATE
#define RSG_NET_ABLATE 0
#endif
#ifndef RSG_NETQ_K
#error "RSG_NETQ_K (12 or 10) is set by the Makefile"
#endif

#define RSG_NETQ_CAT2(a, b) a##b
#define RSG_NETQ_CAT(a, b) RSG_NETQ_CAT2(a, b)
#if RSG_NETQ_K == 12
#define RSG_NETQ_TAG net12
#elif RSG_NETQ_K == 10
#define RSG_NETQ_TAG net10
#else
#error "RSG_NETQ_K is 12 or 10 (RS(8,4) in this form measured slower: see the header)"
#endif
// k_decode_records_net12, launch_records_net12_partN, records_net12_pattern
#define RSG_NETQ_NAME(pre, post) RSG_NETQ_CAT(RSG_NETQ_CAT(pre, RSG_NETQ_TAG), post)

namespace rsg {

#if RSG_NETQ_K == 12
#include "rs124_decode_nets.h"
namespace decq = decnet12;
#else
#include "rs104_decode_nets.h"
namespace decq = decnet10;
#endif

namespace {

constexpr int kKQ = RSG_NETQ_K, kNQ = 4;  // data shards, network waves
// network wave q's survivors [kPartC0[q], kPartC0[q] + kPartN[q]): RS(12,4)
// 3 + 3 + 3 + 3, RS(10,4) 3 + 3 + 2 + 2 (the generator's parts)
constexpr int kPartC0[4] = {0, 3, 6, kKQ == 12 ? 9 : 8};
constexpr int kPartN[4] = {3, 3, kKQ == 12 ? 3 : 2, kKQ == 12 ? 3 : 2};

// TR (target rows in their accumulators): the fused encode (ENC, all four
// parity rows) and a heal on a 2-slot ring (its TH target rows).  A target
// row's finisher writes its bytes over the accumulator it has just read and
// the target hasher clears it after hashing it, so the target rows take three
// accumulator slots (the hasher trails two steps) instead of two plus the
// double-buffered row area — what lets RS(12,4)'s and RS(10,4)'s heal fit two
// workgroups (two hash chains and two network waves per SIMD) in the LDS.
template <int NF, int TH, int RDX = 4, bool ENC = false>
struct NetQShape : RecRing<NF, 4, TH> {
    static constexpr bool TR = ENC || (TH > 0 && RDX == 2);
    // a TR heal whose last hash wave's idle quads cover the target streams
    // hashes its targets there (records_hash_target_wave): one wave fewer
    static constexpr bool MERGE =
        TR && !ENC && TH > 0 && 2 * (8 - RecRing<NF, 4, TH>::LAST) >= 4 * TH;
    static constexpr int WAVES = RecRing<NF, 4, TH>::HW + kNQ + (MERGE ? 0 : RecRing<NF, 4, TH>::TW);
    static constexpr int NT = TR ? (ENC ? 4 : TH) : 0;  // rows [0, NT) have a target area
    static constexpr uint32_t XROW_T = 4 * dma::PP;    // target row: accumulator, then its 4 stripes' bytes
    static constexpr uint32_t XROW_C = 8 * 64 * 4;     // accumulator: 8 planes, lane-major dwords (2 KiB)
    static constexpr int NTS = 3, NCS = 2;             // slots: target rows, the other rows
    static constexpr uint32_t TSLOTX = NT * XROW_T, CSLOTX = (4 - NT) * XROW_C;
    static constexpr uint32_t XBYTES = NTS * TSLOTX + NCS * CSLOTX;  // the exchange area
    static constexpr int XB = TH ? 1 : 0;          // extra barrier: heal's target hashers trail by 2 steps
    static constexpr int RD = RDX;                 // ring slots (RD - 1 steps of DMA in flight)
    static constexpr uint32_t LDS = RD * RecRing<NF, 4, TH>::DSLOT + XBYTES +
                                    (TH && !TR ? 2 * RecRing<NF, 4, TH>::TSLOT : 16) + 32;
    // waves per SIMD with two workgroups per CU on the 2-slot ring (the
    // register budget the compiler must meet)
    static constexpr int WPE = RDX == 2 ? (2 * WAVES + 3) / 4 : 1;
};

__device__ __forceinline__ void put8_q(uint8_t* p, const uint2& v) { st64_any(p, u64_of(v)); }  // any alignment

// Verdict of the compared rows, combined across the waves that finish them:
// per-stripe mismatch bits OR-ed in and a count of waves done; the last one
// writes each live stripe's verdict whole (no memset before the launch).
struct Verdict {
    uint32_t bad;
    uint32_t done;
};

// Network wave Q of the 4-stripe group (survivors 3Q..3Q+2).
template <int PID, int NF, int TH, int Q, int RDX, bool ENC>
__device__ __forceinline__ void netq_wave(const GfApplyParams& p, uint64_t n, uint32_t steps, uint64_t s0,
                                           const uint8_t* ring, uint8_t* xbuf, uint8_t* trow, Verdict* vd) {
    using dma::CH;
    using dma::IP;
    using dma::PP;
    using L = NetQShape<NF, TH, RDX, ENC>;
    constexpr int D = L::RD;
    constexpr decq::Pattern pat = decq::kPatterns[PID];
    constexpr int R = pat.R, NST = pat.n_store, NCMP = R - NST, SPW = L::SPW, HS = L::HS;
    static_assert(pat.nf == NF && (pat.heal ? NST : 0) == TH && R <= kNQ && NST <= R && HS == 2, "pattern shape");
    constexpr int C0 = kPartC0[Q], NC = kPartN[Q];  // this wave's survivors [C0, C0 + NC)
    constexpr bool FIN = Q < R;             // it finishes row Q
    constexpr bool CMP = FIN && Q >= NST;   // ... a compared one (keeps surplus row Q - NST from the ring)
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
    uint32_t keep[8];   // step t-1's part of row Q, held across B(t)
    uint2 cmp[4];       // CMP: step t-1's surplus row, held across B(t)
    // row r's accumulator of step t, lane-major (target rows: NTS slots, the rest NCS)
    auto xrow = [&](int r, uint32_t t) -> uint8_t* {
        return r < L::NT ? xbuf + (t % L::NTS) * L::TSLOTX + r * L::XROW_T
                         : xbuf + L::NTS * L::TSLOTX + (t % L::NCS) * L::CSLOTX + (r - L::NT) * L::XROW_C;
    };
    auto xb_at = [&](int r, uint32_t t) { return (uint32_t*)xrow(r, t) + lane; };
    // step t: this wave's 3 survivors -> 24 planes -> its part of every row;
    // the other rows' parts out to LDS; copy-through of its data survivors (GET)
    auto part = [&](uint32_t t) {
        const uint8_t* slot = ring + (t % D) * L::DSLOT + lane * 8u;
        uint32_t P[64];  // planes [0, 8 NC) only
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            uint2 a[4];
            row4(slot + (C0 + c) * HS * IP, a);
            uint32_t w[8] = {a[0].x, a[0].y, a[1].x, a[1].y, a[2].x, a[2].y, a[3].x, a[3].y};
#if !RSG_NET_ABLATE
            dma::transpose(w, m4, m2, m1);
#endif
#pragma unroll
            for (int j = 0; j < 8; ++j) P[8 * c + j] = w[j];
        }
        uint32_t O[32];
#if RSG_NET_ABLATE  // experiment builds only: no arithmetic, rows = survivors (2: no LDS exchange either)
#pragma unroll
        for (int i = 0; i < 32; ++i) O[i] = P[i % (8 * NC)];
#else
        decq::net_q<PID, Q>(P, O);
#endif
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r == Q || RSG_NET_ABLATE >= 2) continue;
            uint32_t* xo = xb_at(r, t);
#pragma unroll
            for (int i = 0; i < 8; ++i)
                __hip_atomic_fetch_xor(xo + 64 * i, O[8 * r + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (FIN) {
#pragma unroll
            for (int i = 0; i < 8; ++i) keep[i] = O[8 * Q + i];
        }
        if constexpr (CMP) row4(slot + (kKQ + Q - NST) * HS * IP, cmp);
        if (!TH && cmask) {  // GET: this wave's present data survivors copied through
            const bool ragged = t + 1 == steps && tail != CH;  // wave-uniform
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (!((cmask >> (C0 + c)) & 1u)) continue;  // wave-uniform
                uint2 x[4];
                row4(slot + (C0 + c) * HS * IP, x);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!live[j]) continue;
                    if (!ragged) put8_q(ob[j] + p.copy_off[C0 + c] + (uint64_t)t * CH, x[j]);
                    else st64_part(ob[j] + p.copy_off[C0 + c] + (uint64_t)t * CH, u64_of(x[j]), lane * 8u, tail);
                }
            }
        }
    };
    // step s (in interval s+1): the other waves' parts of row Q in (the
    // accumulator cleared for step s+2, whose parts come after B(s+2)), the
    // row back to bytes, stored or compared
    auto finish = [&](uint32_t s) {
        const bool ragged = s + 1 == steps && tail != CH;  // wave-uniform
        uint32_t* xa = xb_at(Q, s);
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = keep[i] ^ xa[64 * i];
        if constexpr (!(L::TR && Q < L::NT)) {  // a target row's area: the target hasher clears it
#pragma unroll
            for (int i = 0; i < 8; ++i) xa[64 * i] = 0u;
        }
#if !RSG_NET_ABLATE
        dma::transpose(w, m4, m2, m1);
#endif
        if constexpr (Q < NST) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint2 v = make_uint2(w[2 * j], w[2 * j + 1]);
                if (live[j]) {
                    if (!ragged) put8_q(ob[j] + p.out_off[Q] + (uint64_t)s * CH, v);
                    else st64_part(ob[j] + p.out_off[Q] + (uint64_t)s * CH, u64_of(v), lane * 8u, tail);
                }
                if constexpr (L::TR)  // over the accumulator just read
                    *(uint2*)(xrow(Q, s) + j * PP + lane * 8u) = v;
                else if constexpr (TH > 0)
                    *(uint2*)(trow + (s & 1) * L::TSLOT + (Q * SPW + j) * PP + lane * 8u) = v;
            }
            if constexpr (L::TR) {  // the accumulator's words the rows' pitch skips (the hasher clears the rest)
                static_assert(PP - dma::CH == 32 && L::XROW_T >= 8 * 64 * 4 && Q < L::NT, "row pitch against the plane words");
                if (lane < 24u) *(uint32_t*)(xrow(Q, s) + dma::CH + (lane / 8u) * PP + (lane % 8u) * 4u) = 0u;
            }
        } else if (!ragged) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                diff[j] = or_diff(or_diff(diff[j], cmp[j].x, w[2 * j]), cmp[j].y, w[2 * j + 1]);
        } else {  // only the bytes before the ragged step's tail count
            const uint64_t keepm = part_mask8(lane * 8u, tail);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t d = (u64_of(cmp[j]) ^ ((uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32))) & keepm;
                diff[j] |= (uint32_t)d | (uint32_t)(d >> 32);
            }
        }
    };
    if constexpr (FIN) {  // every accumulator of row Q starts cleared
#pragma unroll
        for (int b = 0; b < (Q < L::NT ? L::NTS : L::NCS); ++b)
#pragma unroll
            for (int i = 0; i < 8; ++i) xb_at(Q, b)[64 * i] = 0u;
    }
    lds_barrier();  // B(0)
    if constexpr (!FIN) {  // R = 3: wave 3 hands its parts over only
#pragma unroll 1
        for (uint32_t t = 0; t < steps; ++t) {
            part(t);
            lds_barrier();  // B(t+1)
        }
    } else {
        // interval t: finish step t-1 (the other parts published by B(t)), then step t's part
#pragma unroll 1
        for (uint32_t t = 0; t <= steps; ++t) {
            if (t > 0) finish(t - 1);
            if (t < steps) {
                part(t);
                lds_barrier();  // B(t+1)
            }
        }
    }
#pragma unroll
    for (int b = 0; b < L::XB; ++b) lds_barrier();  // B(steps+1): the last target rows published
    if constexpr (CMP) {
        uint32_t bad = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) bad |= (__builtin_amdgcn_ballot_w64(diff[j] != 0u) != 0 ? 1u : 0u) << j;
        if (lane == 0) {
            if (NCMP > 1) {
                __hip_atomic_fetch_or(&vd->bad, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (__hip_atomic_fetch_add(&vd->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) + 1 !=
                    (uint32_t)NCMP)
                    return;  // another compare wave writes the verdicts
                bad = __hip_atomic_load(&vd->bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (live[j]) p.ok_flags[s0 + j] = (bad >> j) & 1u ? 0 : 1;
        }
    }
}

// ENC: the fused encode + HH256S (k_encode_hash_net12 below): the heal of
// all four parity shards over a stripe buffer, every digest written to the
// batch digest layout.
template <int PID, int NF, int TH, bool ENC = false, int RDX = 4>
__global__ __launch_bounds__((64 * NetQShape<NF, TH, RDX, ENC>::WAVES))
__attribute__((amdgpu_waves_per_eu(NetQShape<NF, TH, RDX, ENC>::WPE))) void RSG_NETQ_NAME(k_decode_records_, )(
    const GfApplyParams p, const HashParams h) {
    using L = NetQShape<NF, TH, RDX, ENC>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[L::RD * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t xbuf[L::XBYTES];
    __shared__ __attribute__((aligned(16))) uint8_t trow[TH && !L::TR ? 2 * L::TSLOT : 16];
    __shared__ Verdict vd;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t steps = p.units;
    const uint64_t s0 = (uint64_t)blockIdx.x * L::SPW;
    if (TH && wave >= (uint32_t)(L::HW + kNQ)) {
        if constexpr (L::TR)  // the target rows in their exchange slots, cleared once hashed
            records_target_hasher<4, TH, 2, ENC, L::NTS, L::TSLOTX, true, L::WPE>(&karg_gf(), &karg_hash(), xbuf, wave - L::HW - kNQ, steps, s0);
        else
            records_target_hasher<4, TH, 2, false, 2, 0, false, L::WPE>(&karg_gf(), &karg_hash(), trow, wave - L::HW - kNQ, steps, s0);
        return;
    }
    if (wave >= (uint32_t)L::HW) {
        const uint32_t q = wave - L::HW;
        if (q == 0 && threadIdx.x % 64 == 0) vd = Verdict{0u, 0u};  // ordered before the compares by B(0)
        if (q == 0) netq_wave<PID, NF, TH, 0, RDX, ENC>(p, h.n, steps, s0, ring, xbuf, trow, &vd);
        else if (q == 1) netq_wave<PID, NF, TH, 1, RDX, ENC>(p, h.n, steps, s0, ring, xbuf, trow, &vd);
        else if (q == 2) netq_wave<PID, NF, TH, 2, RDX, ENC>(p, h.n, steps, s0, ring, xbuf, trow, &vd);
        else netq_wave<PID, NF, TH, 3, RDX, ENC>(p, h.n, steps, s0, ring, xbuf, trow, &vd);
        return;
    }
    if constexpr (L::MERGE) {
        if (wave == (uint32_t)(L::HW - 1)) {  // the last hash wave hashes the target rows too
            records_hash_target_wave<NF, 4, L::RD, TH, L::NTS, L::TSLOTX, 2, true, L::WPE>(&karg_gf(), &karg_hash(), ring, xbuf, wave, steps, s0);
            return;
        }
    }
    records_hash_wave<NF, 4, L::XB, L::RD, ENC, L::WPE>(&karg_hash(), p.wave_prio, ring, wave, steps, s0);
}

static_assert(NetQShape<13, 0, 2>::LDS <= 80 * 1024 && NetQShape<12, 2>::LDS <= 160 * 1024 &&
                  NetQShape<13, 1>::LDS <= 160 * 1024,
              "RS(10,4) GET (two workgroups per CU) and heal workgroups fit the LDS");
#if RSG_NETQ_K == 12
static_assert(NetQShape<15, 0>::LDS <= 160 * 1024 && NetQShape<14, 0>::LDS <= 160 * 1024 &&
                  NetQShape<15, 1>::LDS <= 160 * 1024 && NetQShape<14, 2>::LDS <= 160 * 1024,
              "RS(12,4) GET / heal workgroups fit the LDS");
static_assert(NetQShape<15, 0, 2>::LDS <= 80 * 1024 && NetQShape<14, 0, 2>::LDS <= 80 * 1024 &&
                  NetQShape<12, 4, 2, true>::LDS <= 80 * 1024,
              "RS(12,4) GET and fused encode with a 2-slot ring: two workgroups per CU");
static_assert(NetQShape<14, 2, 2>::LDS <= 80 * 1024 && NetQShape<13, 3, 2>::LDS <= 80 * 1024 &&
                  NetQShape<15, 1, 2>::LDS > 80 * 1024,
              "RS(12,4) heal of 2+ targets on a 2-slot ring: two workgroups per CU (1 target: one, 4 slots)");
#endif
static_assert(NetQShape<12, 2, 2>::LDS <= 80 * 1024 && NetQShape<13, 1, 2>::LDS <= 80 * 1024,
              "RS(10,4) heal on a 2-slot ring: two workgroups per CU");

// heal: a 2-slot ring and two workgroups per CU where its LDS (the target rows
// in their accumulators) fits half a CU, else one on a 4-slot ring
template <int NF, int TH>
constexpr int heal_rd() {
    return NetQShape<NF, TH, 2>::LDS <= 80 * 1024 ? 2 : 4;
}

using NetQLaunch = void (*)(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream);

template <int PID>
void launch_netq(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    constexpr decq::Pattern pat = decq::kPatterns[PID];
    constexpr int NF = pat.nf, TH = pat.heal ? pat.n_store : 0;
    // GET: a 2-slot ring and two workgroups per CU (RSG_NET12_RD=4: the
    // 4-slot form); heal: the same where its LDS fits (heal_rd)
    if constexpr (TH == 0) {
        if (!RSG_MEASUREMENT_BUILD || tuning().net12_rd == 2)
            hipLaunchKernelGGL((RSG_NETQ_NAME(k_decode_records_, )<PID, NF, TH, false, 2>), dim3((uint32_t)blocks),
                               dim3(64 * NetQShape<NF, TH, 2>::WAVES), 0, stream, p, h);
#if RSG_MEASUREMENT_BUILD  // the 4-slot A/B form
        else
            hipLaunchKernelGGL((RSG_NETQ_NAME(k_decode_records_, )<PID, NF, TH>), dim3((uint32_t)blocks),
                               dim3(64 * NetQShape<NF, TH>::WAVES), 0, stream, p, h);
#endif
    } else {
        constexpr int RD = heal_rd<NF, TH>();
        hipLaunchKernelGGL((RSG_NETQ_NAME(k_decode_records_, )<PID, NF, TH, false, RD>), dim3((uint32_t)blocks),
                           dim3(64 * NetQShape<NF, TH, RD>::WAVES), 0, stream, p, h);
    }
}

// RS(10,4) GETs with two shards lost are not built: the run-time-table
// kernel runs them 4-8 % faster (one box, interleaved: two data lost 1.544
// against 1.481 ms, data + parity 1.428 against 1.321 / 1.333;
// profiles/r06/rs104/), and 85 of RS(10,4)'s 201 network kernels' compile
// time goes with them.  Its one-loss GETs (network 13 % faster) and every
// heal (9-10 %) keep their networks; so does every RS(12,4) pattern.
template <int PID>
constexpr bool netq_built() {
    constexpr decq::Pattern pat = decq::kPatterns[PID];
    return !(kKQ == 10 && !pat.heal && pat.nf == kKQ + 4 - 2);
}

template <int PID>
constexpr NetQLaunch pick_netq() {
    if constexpr (PID % RSG_NET_PARTS == RSG_NET_PART && netq_built<PID>()) return &launch_netq<PID>;
    else return nullptr;
}

template <size_t... I>
constexpr std::array<NetQLaunch, sizeof...(I)> netq_table(std::index_sequence<I...>) {
    return {pick_netq<(int)I>()...};
}

const std::array<NetQLaunch, decq::kCount> kNetQPart =
    netq_table(std::make_index_sequence<decq::kCount>{});

}  // namespace

// This part's launcher (launch_records_net12_partN): false if pattern `pid`
// is instantiated elsewhere.
bool RSG_NETQ_NAME(launch_records_, RSG_NETQ_CAT(_part, RSG_NET_PART))(int pid, uint64_t blocks,
                                                                       const GfApplyParams& p, const HashParams& h,
                                                                       hipStream_t stream) {
    if (pid < 0 || pid >= decq::kCount || !kNetQPart[pid]) return false;
    kNetQPart[pid](blocks, p, h, stream);
    return true;
}

#if RSG_NET_PART == 0
// The fused encode + HH256S of RS(12,4) and RS(10,4) (BitrotWriter over an
// encoded block, bitrot.rs:464-510 after erasure encode): the heal kernel of
// all four parity shards (pattern kEncodePid, rows = the encode matrix)
// walking the data shards of a stripe buffer in place — K data rows DMA'd and
// hashed, 4 parity rows computed by the network waves, stored and hashed by
// the target hasher — every digest to h.out (stripe-major, K + 4 per stripe).
namespace {
constexpr int encode_pid() {
    for (int i = 0; i < decq::kCount; ++i)
        if (decq::kPatterns[i].heal && decq::kPatterns[i].absent == (0xFu << kKQ)) return i;
    return -1;
}
constexpr int kEncodePid = encode_pid();
static_assert(kEncodePid >= 0 && decq::kPatterns[kEncodePid].nf == kKQ && decq::kPatterns[kEncodePid].R == 4,
              "the generated header lists the heal of every parity shard");
static_assert(NetQShape<kKQ, 4, 2, true>::LDS <= 80 * 1024, "the fused encode: two workgroups per CU");
}  // namespace

const uint8_t* RSG_NETQ_NAME(encode_, _coef)() { return &decq::kPatterns[kEncodePid].coef[0][0]; }

// p: the encode's table-GF launch (in place: base == out_base, in_off = the
// data shards, out_off = the parity shards); h: key, out (digests).
hipError_t RSG_NETQ_NAME(launch_encode_hash_, )(GfApplyParams p, HashParams h, uint64_t shard_len,
                                                uint64_t n_stripes, hipStream_t stream) {
    using L = NetQShape<kKQ, 4, 2, true>;
    if (p.C != (uint32_t)kKQ || p.R != 4 || n_stripes == 0 || shard_len == 0 || p.base != p.out_base ||
        p.stripe_stride != p.out_stripe_stride || 5 * p.stripe_stride >= (1ull << 32) ||
        (n_stripes + L::SPW - 1) / L::SPW > 0x7fffffffull || (shard_len + dma::CH - 1) / dma::CH > 0xffffffffull)
        return hipErrorInvalidValue;
    p.n_store = 4;
    p.copy_mask = 0;
    p.wave_prio = (uint32_t)tuning().get_prio;  // as the GET / heal (RSG_DMA_PRIO)
    p.units = (uint32_t)((shard_len + dma::CH - 1) / dma::CH);
    p.byte_end = shard_len;
    h.len = shard_len;
    h.n = n_stripes;
    h.shards = kKQ + 4;
    h.stripe_stride = p.stripe_stride;
    h.nbases = kKQ;
    for (int c = 0; c < kKQ; ++c) h.base[c] = p.base + p.in_off[c];
    // two workgroups per CU on a 2-slot ring (RSG_NET12_RD=4, measurement builds: one, 4 slots)
    if (!RSG_MEASUREMENT_BUILD || tuning().net12_rd == 2)
        hipLaunchKernelGGL((RSG_NETQ_NAME(k_decode_records_, )<kEncodePid, kKQ, 4, true, 2>),
                           dim3((uint32_t)((n_stripes + L::SPW - 1) / L::SPW)), dim3(64 * L::WAVES), 0, stream, p, h);
#if RSG_MEASUREMENT_BUILD
    else
        hipLaunchKernelGGL((RSG_NETQ_NAME(k_decode_records_, )<kEncodePid, kKQ, 4, true, 4>),
                           dim3((uint32_t)((n_stripes + L::SPW - 1) / L::SPW)), dim3(64 * L::WAVES), 0, stream, p, h);
#endif
    return hipGetLastError();
}

#endif

#if RSG_NET_PART == 0
// The pattern whose coefficient rows equal the launch's (R x K, row-major),
// or -1 (records_net12_pattern).
int RSG_NETQ_NAME(records_, _pattern)(int heal, int nf, int R, int n_store, const uint8_t* coef) {
    for (int i = 0; i < decq::kCount; ++i) {
        const decq::Pattern& pt = decq::kPatterns[i];
        if (pt.heal != heal || pt.nf != nf || pt.R != R || pt.n_store != n_store) continue;
        bool eq = true;
        for (int r = 0; r < R && eq; ++r)
            for (int c = 0; c < kKQ && eq; ++c) eq = pt.coef[r][c] == coef[r * kKQ + c];
        if (eq) return i;
    }
    return -1;
}
#endif

}  // namespace rsg
