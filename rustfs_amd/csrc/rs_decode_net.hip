// rs_decode_net.hip — the one-pass GET / heal kernel for RS(8,4) and RS(6,4)
// (the default geometries of 12- and 10-drive sets, storageclass.rs:24-31)
// with its rows as a compile-time XOR network per erasure pattern
// (k_decode_records_net<PID> / _net6; the networks in the generated
// rs84_decode_nets.h / rs64_decode_nets.h, tools/gen_decode_nets.py [--k 6]).
// Compiled RSG_NET_PARTS times per geometry (Makefile: RSG_NET_K = 8 or 6), part
// RSG_NET_PART instantiating
// the patterns with PID % RSG_NET_PARTS == RSG_NET_PART, so the kernels
// build in parallel.
//
// Same workgroup as k_decode_records_dma (rs_decode.hip): 8 stripes, NF
// present record files DMA'd into a 3-slot LDS ring per 512-byte step,
// ceil(4 NF / 8) DMA + verify-hash waves (rs_records.h), heal's target rows
// hashed one step behind by ceil(8 TH / 16) target hashers — but the 8
// run-time-table GF waves (one per stripe: 3 v_perm + 1.5 XOR per word and
// coefficient, v_perm at half the XOR issue rate) become 2 network waves,
// one per 4-stripe group (stripes 2g, 2g+1, 2g+4, 2g+5: 8 bytes of each per
// lane, as the fused encoder's k_encode_hash_dma groups): each step the wave
// bit-transposes the 8 (6) survivor rows into 64 (48) planes, runs the pattern's
// network (all R rows at once: 173-244 three-input XORs), transposes the
// rows back, stores the rebuilt rows (and heal's LDS row copies), compares
// the surplus parity rows with the ring and copies GET's present data through.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <array>
#include <utility>

#include "rs_device.h"
#include "rs_kernels.h"
#include "rs_records.h"

#ifndef RSG_NET_ABLATE
#define RSG_NET_ABLATE 0
#endif
#ifndef RSG_NET_PART
#error "RSG_NET_PART (0 .. RSG_NET_PARTS-1) is set by the Makefile"
#endif
#ifndef RSG_NET_K
#define RSG_NET_K 8
#endif

#define RSG_NET_CAT2(a, b) a##b
#define RSG_NET_CAT(a, b) RSG_NET_CAT2(a, b)
#if RSG_NET_K == 8
#define RSG_NET_TAG  // k_decode_records_net, launch_records_net_partN, records_net_pattern
#elif RSG_NET_K == 6
#define RSG_NET_TAG 6  // k_decode_records_net6, launch_records_net6_partN, records_net6_pattern
#else
#error "RSG_NET_K is 8 or 6"
#endif
#define RSG_NET_NAME(pre, post) RSG_NET_CAT(RSG_NET_CAT(pre, RSG_NET_TAG), post)

namespace rsg {

#if RSG_NET_K == 8
#include "rs84_decode_nets.h"
#elif RSG_NET_K == 6
#include "rs64_decode_nets.h"
namespace decnet = decnet6;
#endif
constexpr int kNetC = RSG_NET_K;  // survivors (data shards)

// 8 output bytes per lane: plain (cached) stores by default — the L2 gathers
// the walk's 512-byte rows before they reach HBM (RS(8,4), n = 4096, GET with
// 2 data lost 2.01 -> 1.97 ms, heal neutral; profiles/r03/ab_net/) — or
// non-temporal (RSG_GET_CACHED=0)
__device__ __forceinline__ void put8(uint8_t* p, const uint2& v, bool cached) {  // any alignment
    if (cached) st64_any(p, u64_of(v));
    else st16_nt_half(p, v);
}

// LDS rows through 32-bit address-space-3 pointers (the low 32 bits of a
// generic LDS address are its LDS offset, as dma::read16 relies on).
typedef __attribute__((address_space(3))) const uint64_t lds_u2;
__device__ __forceinline__ const lds_u2* lds_at(const uint8_t* p) {
    return (const lds_u2*)(uintptr_t)(uint32_t)(uintptr_t)p;
}
__device__ __forceinline__ uint2 u2_of(uint64_t v) { return make_uint2((uint32_t)v, (uint32_t)(v >> 32)); }
// one 8-byte lane column of the group's 4 stripes, row at byte offset off:
// stripes at +0, +IP, +CH, +IP+CH
__device__ __forceinline__ void row4(const lds_u2* slot, uint32_t off, uint2 (&x)[4]) {
    x[0] = u2_of(slot[off / 8]);
    x[1] = u2_of(slot[(off + dma::IP) / 8]);
    x[2] = u2_of(slot[(off + dma::CH) / 8]);
    x[3] = u2_of(slot[(off + dma::IP + dma::CH) / 8]);
}

template <int NF, int TH>
struct NetShape : RecRing<NF, 8, TH> {
    static constexpr int NG = 2;  // network waves (4-stripe groups)
    static constexpr int WAVES = RecRing<NF, 8, TH>::HW + NG + RecRing<NF, 8, TH>::TW;
};

// Network wave of 4-stripe group g (stripes 2g, 2g+1, 2g+HS, 2g+HS+1 of the
// workgroup; lane = 8 bytes of each): pattern PID's R rows over the 8
// survivors (present files 0..7 of the launch).
template <int PID, int NF, int TH>
__device__ __forceinline__ void net_wave(const GfApplyParams& p, uint64_t n, uint32_t steps, uint64_t s0, uint32_t g,
                                         const uint8_t* ring, uint8_t* trow) {
    using dma::CH;
    using dma::D;
    using dma::IP;
    using dma::PP;
    using L = NetShape<NF, TH>;
    constexpr decnet::Pattern pat = decnet::kPatterns[PID];
    constexpr int C = kNetC, R = pat.R, NST = pat.n_store, SPW = L::SPW, HS = L::HS;
    static_assert(pat.nf == NF && (pat.heal ? NST : 0) == TH && R <= 4 && NST <= R, "pattern shape");
    if (p.wave_prio & kPrioGf) __builtin_amdgcn_s_setprio(2);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    const uint32_t mys[4] = {2 * g, 2 * g + 1, 2 * g + HS, 2 * g + HS + 1};
    const uint32_t cmask = p.copy_mask;
    const bool cached = p.cached_stores != 0;
    bool live[4];       // wave-uniform: a dead stripe (past n) computes stripe 0's rows and stores nothing
    uint8_t* ob[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        live[j] = s0 + mys[j] < n;
        ob[j] = p.out_base + (live[j] ? s0 + mys[j] : 0) * p.out_stripe_stride + lane * 8u;
    }
    // this group's 8-byte lane column of a ring row (file f: + f * HS * IP);
    // the 4 stripes sit at +0, +IP, +CH, +IP+CH
    const uint32_t goff = 2 * g * IP + lane * 8u;
    uint32_t diff[4] = {0u, 0u, 0u, 0u};  // OR of this lane's surplus-parity differences
    const uint32_t tail = walk_tail(p.byte_end, steps);  // a ragged walk's last step: first tail bytes only
    lds_barrier();  // B(0)
#pragma unroll 1
    for (uint32_t s = 0; s < steps; ++s) {
        // the step's ring slot as a 32-bit LDS address: the row reads fold
        // their constant offsets (ds_read2_b64 pairs) instead of one VALU
        // add per read through a generic pointer
        const lds_u2* slot = lds_at(ring + (s % D) * L::DSLOT + goff);
        uint32_t P[64];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            uint2 a[4];
            row4(slot, c * HS * IP, a);
            uint32_t w[8] = {a[0].x, a[0].y, a[1].x, a[1].y, a[2].x, a[2].y, a[3].x, a[3].y};
#if !RSG_NET_ABLATE
            dma::transpose(w, m4, m2, m1);
#endif
#pragma unroll
            for (int j = 0; j < 8; ++j) P[8 * c + j] = w[j];
        }
        const bool part = s + 1 == steps && tail != CH;  // wave-uniform
        uint32_t O[32];
#if RSG_NET_ABLATE  // experiment builds only (round 3, profiles/KERNEL_NOTES.md): no arithmetic, rows = survivors
#pragma unroll
        for (int i = 0; i < 32; ++i) O[i] = P[i];
#else
        decnet::net<PID>(P, O);
#endif
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = O[8 * r + i];
#if !RSG_NET_ABLATE
            dma::transpose(w, m4, m2, m1);
#endif
            if (r < NST) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint2 v = make_uint2(w[2 * j], w[2 * j + 1]);
                    if (live[j]) {
                        if (!part) put8(ob[j] + p.out_off[r] + (uint64_t)s * CH, v, cached);
                        else st64_part(ob[j] + p.out_off[r] + (uint64_t)s * CH, u64_of(v), lane * 8u, tail);
                    }
                    if constexpr (TH > 0)
                        *(uint2*)(trow + (s & 1) * L::TSLOT + (r * SPW + mys[j]) * PP + lane * 8u) = v;
                }
            } else {
                uint2 o[4];
                row4(slot, (C + (r - NST)) * HS * IP, o);
                if (!part) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        diff[j] = or_diff(or_diff(diff[j], o[j].x, w[2 * j]), o[j].y, w[2 * j + 1]);
                } else {  // only the bytes before the ragged step's tail count
                    const uint64_t keep = part_mask8(lane * 8u, tail);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint64_t d = (u64_of(o[j]) ^ ((uint64_t)w[2 * j] | ((uint64_t)w[2 * j + 1] << 32))) & keep;
                        diff[j] |= (uint32_t)d | (uint32_t)(d >> 32);
                    }
                }
            }
        }
        if (!TH && cmask) {  // GET: the present data survivors copied through
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (!((cmask >> c) & 1u)) continue;  // wave-uniform
                uint2 x[4];
                row4(slot, c * HS * IP, x);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!live[j]) continue;
                    if (!part) put8(ob[j] + p.copy_off[c] + (uint64_t)s * CH, x[j], cached);
                    else st64_part(ob[j] + p.copy_off[c] + (uint64_t)s * CH, u64_of(x[j]), lane * 8u, tail);
                }
            }
        }
        lds_barrier();  // B(s+1): done with slot s % D
    }
    // each stripe's surplus verdict, written whole (no memset before the launch)
    if constexpr (NST < R) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool any_bad = __builtin_amdgcn_ballot_w64(diff[j] != 0u) != 0;
            if (live[j] && lane == 0) p.ok_flags[s0 + mys[j]] = any_bad ? 0 : 1;
        }
    }
}

// ENC: the fused encode + HH256S (launch_encode_hash_net below): the heal of
// all four parity shards over a stripe buffer, every digest written to the
// batch digest layout (the hash waves: the data shards' digests; the target
// hashers: the parity shards').
template <int PID, int NF, int TH, bool ENC = false>
__global__ __launch_bounds__((64 * NetShape<NF, TH>::WAVES)) void RSG_NET_NAME(k_decode_records_net, )(const GfApplyParams p,
                                                                                       const HashParams h) {
    using L = NetShape<NF, TH>;
    __shared__ __attribute__((aligned(16))) uint8_t ring[dma::D * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t trow[TH ? 2 * L::TSLOT : 16];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t steps = p.units;
    const uint64_t s0 = (uint64_t)blockIdx.x * L::SPW;
    if (TH && wave >= (uint32_t)(L::HW + L::NG)) {
        records_target_hasher<8, TH, 1, ENC>(&karg_gf(), &karg_hash(), trow, wave - L::HW - L::NG, steps, s0);
        return;
    }
    if (wave >= (uint32_t)L::HW) {
        net_wave<PID, NF, TH>(p, h.n, steps, s0, wave - L::HW, ring, trow);
        return;
    }
    records_hash_wave<NF, 8, 0, dma::D, ENC>(&karg_hash(), p.wave_prio, ring, wave, steps, s0);
}

using NetLaunch = void (*)(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream);

template <int PID>
static void launch_net(uint64_t blocks, const GfApplyParams& p, const HashParams& h, hipStream_t stream) {
    constexpr decnet::Pattern pat = decnet::kPatterns[PID];
    constexpr int NF = pat.nf, TH = pat.heal ? pat.n_store : 0;
    hipLaunchKernelGGL((RSG_NET_NAME(k_decode_records_net, )<PID, NF, TH>), dim3((uint32_t)blocks), dim3(64 * NetShape<NF, TH>::WAVES),
                       0, stream, p, h);
}

template <int PID>
constexpr NetLaunch pick_net() {
    if constexpr (PID % RSG_NET_PARTS == RSG_NET_PART) return &launch_net<PID>;
    else return nullptr;
}

template <size_t... I>
constexpr std::array<NetLaunch, sizeof...(I)> net_table(std::index_sequence<I...>) {
    return {pick_net<(int)I>()...};
}

static const std::array<NetLaunch, decnet::kCount> kNetPart = net_table(std::make_index_sequence<decnet::kCount>{});

// This part's launcher: false if pattern `pid` is instantiated elsewhere.
bool RSG_NET_NAME(launch_records_net, RSG_NET_CAT(_part, RSG_NET_PART))(int pid, uint64_t blocks,
                                                                        const GfApplyParams& p, const HashParams& h,
                                                                        hipStream_t stream) {
    if (pid < 0 || pid >= decnet::kCount || !kNetPart[pid]) return false;
    kNetPart[pid](blocks, p, h, stream);
    return true;
}

#if RSG_NET_PART == 0
// The fused encode + HH256S of RS(8,4) / RS(6,4) (BitrotWriter over
// an encoded block, bitrot.rs:464-510 after erasure encode): the heal kernel
// of all four parity shards (pattern kEncodePid, rows = the encode matrix)
// walking the data shards of a stripe buffer in place, as
// rs_decode_netq.hip's for RS(12,4) / RS(10,4).
namespace {
constexpr int encode_pid() {
    for (int i = 0; i < decnet::kCount; ++i)
        if (decnet::kPatterns[i].heal && decnet::kPatterns[i].absent == (0xFu << kNetC)) return i;
    return -1;
}
constexpr int kEncodePid = encode_pid();
static_assert(kEncodePid >= 0 && decnet::kPatterns[kEncodePid].nf == kNetC && decnet::kPatterns[kEncodePid].R == 4,
              "the generated header lists the heal of every parity shard");
}  // namespace

const uint8_t* RSG_NET_NAME(encode_net, _coef)() { return &decnet::kPatterns[kEncodePid].coef[0][0]; }

// p: the encode's table-GF launch (in place: base == out_base, in_off = the
// data shards, out_off = the parity shards); h: key, out (digests).
hipError_t RSG_NET_NAME(launch_encode_hash_net, )(GfApplyParams p, HashParams h, uint64_t shard_len,
                                                  uint64_t n_stripes, hipStream_t stream) {
    using L = NetShape<kNetC, 4>;
    if (p.C != (uint32_t)kNetC || p.R != 4 || n_stripes == 0 || shard_len == 0 || p.base != p.out_base ||
        p.stripe_stride != p.out_stripe_stride || 5 * p.stripe_stride >= (1ull << 32) ||
        (n_stripes + L::SPW - 1) / L::SPW > 0x7fffffffull || (shard_len + dma::CH - 1) / dma::CH > 0xffffffffull)
        return hipErrorInvalidValue;
    p.n_store = 4;
    p.copy_mask = 0;
    const Tuning& t = tuning();  // one snapshot for the whole launch
    p.cached_stores = t.get_cached ? 1u : 0u;
    p.wave_prio = (uint32_t)t.get_prio;
    p.units = (uint32_t)((shard_len + dma::CH - 1) / dma::CH);
    p.byte_end = shard_len;
    h.len = shard_len;
    h.n = n_stripes;
    h.shards = kNetC + 4;
    h.stripe_stride = p.stripe_stride;
    h.nbases = kNetC;
    for (int c = 0; c < kNetC; ++c) h.base[c] = p.base + p.in_off[c];
    hipLaunchKernelGGL((RSG_NET_NAME(k_decode_records_net, )<kEncodePid, kNetC, 4, true>),
                       dim3((uint32_t)((n_stripes + L::SPW - 1) / L::SPW)), dim3(64 * L::WAVES), 0, stream, p, h);
    return hipGetLastError();
}

// The pattern whose coefficient rows equal the launch's (R x K, row-major),
// or -1: matched byte for byte, so a network is only ever run on exactly the
// matrix it was generated for.
int RSG_NET_NAME(records_net, _pattern)(int heal, int nf, int R, int n_store, const uint8_t* coef) {
    for (int i = 0; i < decnet::kCount; ++i) {
        const decnet::Pattern& pt = decnet::kPatterns[i];
        if (pt.heal != heal || pt.nf != nf || pt.R != R || pt.n_store != n_store) continue;
        bool eq = true;
        for (int r = 0; r < R && eq; ++r)
            for (int c = 0; c < kNetC && eq; ++c) eq = pt.coef[r][c] == coef[r * kNetC + c];
        if (eq) return i;
    }
    return -1;
}
#endif

}  // namespace rsg
