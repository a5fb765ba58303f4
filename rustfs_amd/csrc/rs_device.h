// rs_device.h — device helpers shared by the kernel translation units of
// librsgpu (rs_kernels.hip, rs_decode.hip): GF(2^8) table multiply (v_perm)
// and 16-byte access helpers, lane-parallel HighwayHash-256 (HHQuad), the
// raw LDS barrier and the LDS-DMA ring constants of the one-pass kernels.
// Internal; included once per translation unit.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "rs_kernels.h"

namespace rsg {

// ---------------------------------------------------------------------------
// GF(2^8) matrix apply, vector path: 16-byte units, every shard 16-B aligned.
// Block = 256 threads = 4 waves; thread t of block (stripe, chunk) handles unit
// chunk*256 + t, so each wave's loads/stores are contiguous 1 KiB per shard
// (global_load_dwordx4 / global_store_dwordx4).

__device__ __forceinline__ uint32_t gf_mul_word(const uint32_t* t, uint32_t s0, uint32_t s1, uint32_t s2) {
    return __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
           __builtin_amdgcn_perm(t[4], t[4], s2);
}

// acc ^= a ^ b ^ c for the three lookups of one word x coefficient, with the
// gfx950 three-input XOR (v_bitop3_b32, truth table 0x96), which issues at the
// full v_xor rate (2.3 SIMD cycles per wave64 op, tools/kbench/op_rates.hip).
// Taking inputs in pairs folds the six lookups into the accumulator with three
// ops instead of six v_xor: even input: acc = x3(acc, a, b), pend = c; odd
// input: acc = x3(acc, pend, a), acc = x3(acc, b, c).
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc | (a ^ b) in one v_bitop3_b32 (truth table over (S0, S1, S2) =
// (a, b, acc), index S0*4 + S1*2 + S2): the surplus-parity compares OR
// their differences into one word per stripe, tested once at the end.
__device__ __forceinline__ uint32_t or_diff(uint32_t acc, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(a, b, acc, 0xBE);
}

// odd: input index parity (a compile-time constant in the unrolled loops)
__device__ __forceinline__ void gf_fold(bool odd, uint32_t& acc, uint32_t& pend, uint32_t a, uint32_t b, uint32_t c) {
    if (odd) {
        acc = x3(acc, pend, a);
        acc = x3(acc, b, c);
    } else {
        acc = x3(acc, a, b);
        pend = c;
    }
}

// One 16-byte unit per thread and no loop (126 VGPRs for RS(8,4): 4 waves per
// SIMD).  A per-thread unit loop pushed it to 130 VGPRs (3 waves per SIMD) and
// ran ~8 % slower; 2 or 4 units with all loads issued first ran 12-60 % slower
// (tools/kbench/encode_variants.hip).
//
// acc[r] ^= sum over inputs c in [C0, C0+CN) of tab[r][c] * x[c - C0]  (4 words)
template <int C0, int CN, int R>
__device__ __forceinline__ void gf_accumulate(const GfApplyParams& p, const uint4* x, uint32_t (&acc)[R][4]) {
#pragma unroll
    for (int i = 0; i < CN; ++i) {
        const int c = C0 + i;
        const uint32_t w[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t s0 = w[q] & 0x07070707u;
            const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
            const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(p.tab[r][c], s0, s1, s2);
        }
    }
}

// 16-byte accesses with no alignment promise: gfx950 runs HSA code in
// unaligned-access mode, so these stay single global_load/store_dwordx4 and let
// shards of any length (S = ceil(1 MiB / 6) = 174763, ceil(1 MiB / 12) = 87382)
// take the vector path; only the S % 16 tail goes to the byte kernel.
__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st16(uint8_t* p, const uint4& v) { __builtin_memcpy(p, &v, 16); }
// Non-temporal 16-byte store at any alignment (unaligned-access mode): for
// output that this pass never reads back (GET's gathered data).
typedef uint32_t v4u_any __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ void st16_nt_half(uint8_t* p, const uint2& v) {  // 8 bytes, non-temporal
    typedef uint32_t v2u_any __attribute__((ext_vector_type(2), aligned(1)));
    const v2u_any w = {v.x, v.y};
    __builtin_nontemporal_store(w, (v2u_any*)p);
}
__device__ __forceinline__ void st16_nt(uint8_t* p, const uint4& v) {
    const v4u_any w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (v4u_any*)p);
}

// Output row r of a launch: its effective mode and address.
__device__ __forceinline__ uint8_t* gf_dst(const GfApplyParams& p, uint8_t* obase, uint64_t off, int r, uint32_t stripe,
                                          uint32_t& mode) {
    mode = p.mode;
    if (mode == GF_MODE_STORE_COMPARE) {
        mode = (uint32_t)r < p.n_store ? GF_MODE_STORE : GF_MODE_COMPARE;
        if (mode == GF_MODE_COMPARE) return p.out_base + (uint64_t)stripe * p.cmp_stripe_stride + p.out_off[r] + off;
    }
    return obase + p.out_off[r] + off;
}

// The bytes an XOR / COMPARE row reads back, loaded together with the inputs
// so their latency overlaps the arithmetic (STORE rows load nothing).
template <int R>
__device__ __forceinline__ void gf_preload(const GfApplyParams& p, uint8_t* obase, uint64_t off, uint32_t stripe,
                                           uint4 (&old)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t mode;
        const uint8_t* dst = gf_dst(p, obase, off, r, stripe, mode);
        if (mode != GF_MODE_STORE) old[r] = ld16(dst);
    }
}

template <int R>
__device__ __forceinline__ void gf_store(const GfApplyParams& p, uint8_t* obase, uint64_t off,
                                         const uint32_t (&acc)[R][4], uint32_t stripe, const uint4 (&old)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t mode;
        uint8_t* dst = gf_dst(p, obase, off, r, stripe, mode);
        const uint4 v = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        const uint4 o = old[r];
        if (mode == GF_MODE_STORE) {
            st16(dst, v);
        } else if (mode == GF_MODE_XOR) {
            st16(dst, make_uint4(o.x ^ v.x, o.y ^ v.y, o.z ^ v.z, o.w ^ v.w));
        } else {  // GF_MODE_COMPARE: clear the stripe's ok flag on mismatch
            if ((o.x ^ v.x) | (o.y ^ v.y) | (o.z ^ v.z) | (o.w ^ v.w)) p.ok_flags[stripe] = 0;
        }
    }
}

// B threads per workgroup.  One-wave workgroups (B = 64) are the default:
// consecutive workgroups still sweep one stripe's columns in order, but waves
// are replaced one at a time instead of four together; RS(8,4) n = 4096 runs
// 1.06 ms against 1.09-1.15 ms at B = 256 (tools/kbench/block_probe.hip,
// profiles/r02/experiments/blk1_block_probe.txt).  RSG_VEC_BLOCK=256 selects
// the 256-thread form for A/B runs.
// The !PRE kernels' store: each row loads what it reads back (XOR /
// COMPARE) only at its store.  The launcher uses them for plain STORE
// launches, where this form compiles to the fastest measured encode (RS(8,4)
// n = 4096: 1.065 ms; a store-only body with fewer registers ran 1.10-1.13 ms
// at every occupancy, profiles/r02/ab_occ/).
template <int R>
__device__ __forceinline__ void gf_store_late(const GfApplyParams& p, uint8_t* obase, uint64_t off,
                                              const uint32_t (&acc)[R][4], uint32_t stripe) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t mode = p.mode;
        uint8_t* dst = obase + p.out_off[r] + off;
        if (mode == GF_MODE_STORE_COMPARE) {
            mode = (uint32_t)r < p.n_store ? GF_MODE_STORE : GF_MODE_COMPARE;
            if (mode == GF_MODE_COMPARE) dst = p.out_base + (uint64_t)stripe * p.cmp_stripe_stride + p.out_off[r] + off;
        }
        const uint4 v = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        if (mode == GF_MODE_STORE) {
            // non-temporal: the parity / rebuilt rows are not read back by this
            // pass (RS(8,4) encode 1.074 -> 1.043-1.056 ms, profiles/r05/ab_nt/)
            st16_nt(dst, v);
        } else if (mode == GF_MODE_XOR) {
            const uint4 o = ld16(dst);
            st16(dst, make_uint4(o.x ^ v.x, o.y ^ v.y, o.z ^ v.z, o.w ^ v.w));
        } else {  // GF_MODE_COMPARE: clear the stripe's ok flag on mismatch
            const uint4 o = ld16(dst);
            if ((o.x ^ v.x) | (o.y ^ v.y) | (o.z ^ v.z) | (o.w ^ v.w)) p.ok_flags[stripe] = 0;
        }
    }
}

template <int R>
__device__ __forceinline__ void gf_store(const GfApplyParams& p, uint8_t* obase, uint64_t off,
                                         const uint32_t (&acc)[R][4], uint32_t stripe) {
    uint4 old[R];
    gf_preload<R>(p, obase, off, stripe, old);
    gf_store<R>(p, obase, off, acc, stripe, old);
}

// ---------------------------------------------------------------------------
// HighwayHash-256 (public spec; the `highway` crate 1.3.0 behind
// crates/utils/src/hash.rs:123-127).

// 8-byte little-endian load at any alignment: one global_load_dwordx2 in
// gfx950's unaligned-access mode (as ld16 below).
__device__ __forceinline__ uint64_t ld64_any(const uint8_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}


// ---------------------------------------------------------------------------
// HighwayHash-256, lane-parallel: one message per 4-lane quad, lane q holds
// u64 lane q of v0/v1/mul0/mul1 (8 VGPRs).  The mul/add half of Update is
// lane-local; ZipperMergeAndAdd mixes lanes (0,1) and (2,3): it needs only the
// partner's high dword (one DPP quad_perm move) and is three v_perm_b32 with
// per-lane-parity selectors (derived in DESIGN.md §HighwayHash):
//   low  dword = (own.b3, other.b4, own.b2, own.b5)                 both parities
//   high dword = (other.b6, own.b1, other.b7, own.b0)  even lane  (add0)
//              = (own.b1, other.b6, own.b0, other.b7)  odd lane   (add1)

struct HHQuad {
    uint64_t v0, v1, mul0, mul1;
    uint32_t sel_hi;  // per-lane high-dword selector
};

__device__ __forceinline__ uint32_t quad_swap_pairs(uint32_t x) {  // lane q <- lane q^1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__device__ __forceinline__ uint32_t quad_swap_halves(uint32_t x) {  // lane q <- lane q^2
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
}

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Built as a 2-dword vector so the two v_perm results land in one register
// pair and the following 64-bit add is a single v_lshl_add_u64 (building it
// with shifts/ors cost an extra v_mov and add per zipper).
__device__ __forceinline__ uint64_t hh_zip(uint64_t x, uint32_t sel_hi) {
    const u32x2 xv = __builtin_bit_cast(u32x2, x);
    const uint32_t other_hi = quad_swap_pairs(xv.y);
    const uint32_t t = __builtin_amdgcn_perm(xv.y, xv.x, 0x05020C03u);  // own.b3, 0, own.b2, own.b5
    u32x2 z;
    z.x = __builtin_amdgcn_perm(other_hi, t, 0x03020400u);  // t.b0, other.b4, t.b2, t.b3
    z.y = __builtin_amdgcn_perm(other_hi, xv.x, sel_hi);
    return __builtin_bit_cast(uint64_t, z);
}

__device__ __forceinline__ void hhq_init(HHQuad& s, const uint64_t* key, uint32_t q) {
    const uint64_t i0[4] = {0xdbe6d5d5fe4cce2full, 0xa4093822299f31d0ull, 0x13198a2e03707344ull,
                            0x243f6a8885a308d3ull};
    const uint64_t i1[4] = {0x3bd39e10cb0ef593ull, 0xc0acf169b5f18a8cull, 0xbe5466cf34e90c6cull,
                            0x452821e638d01377ull};
    uint64_t kq = key[0], m0 = i0[0], m1 = i1[0];
    if (q == 1) { kq = key[1]; m0 = i0[1]; m1 = i1[1]; }
    if (q == 2) { kq = key[2]; m0 = i0[2]; m1 = i1[2]; }
    if (q == 3) { kq = key[3]; m0 = i0[3]; m1 = i1[3]; }
    s.mul0 = m0;
    s.mul1 = m1;
    s.v0 = m0 ^ kq;
    s.v1 = m1 ^ ((kq >> 32) | (kq << 32));
    s.sel_hi = (q & 1) ? 0x07000601u : 0x00070106u;
}

__device__ __forceinline__ void hhq_update(HHQuad& s, uint64_t a) {
    s.v1 += s.mul0 + a;
    s.mul0 ^= (uint64_t)(uint32_t)s.v1 * (s.v0 >> 32);
    s.v0 += s.mul1;
    s.mul1 ^= (uint64_t)(uint32_t)s.v0 * (s.v1 >> 32);
    s.v0 += hh_zip(s.v1, s.sel_hi);
    s.v1 += hh_zip(s.v0, s.sel_hi);
}

// Remainder packet word q built from the message tail (size_mod32 = len % 32 > 0).
__device__ __forceinline__ void hhq_remainder(HHQuad& s, const uint8_t* tail, uint32_t size_mod32, uint32_t q) {
    s.v0 += ((uint64_t)size_mod32 << 32) + size_mod32;
    uint32_t h0 = (uint32_t)s.v1, h1 = (uint32_t)(s.v1 >> 32);
    h0 = (h0 << size_mod32) | (h0 >> (32u - size_mod32));
    h1 = (h1 << size_mod32) | (h1 >> (32u - size_mod32));
    s.v1 = (uint64_t)h0 | ((uint64_t)h1 << 32);
    const uint32_t copy = size_mod32 & ~3u, mod4 = size_mod32 & 3u;
    uint64_t w = 0;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
        const uint32_t pos = 8 * q + b;
        uint32_t v = 0;
        if (pos < copy) v = tail[pos];
        else if (size_mod32 & 16u) { if (pos >= 28) v = tail[size_mod32 - 32 + pos]; }
        else if (mod4) {
            if (pos == 16) v = tail[copy];
            else if (pos == 17) v = tail[copy + (mod4 >> 1)];
            else if (pos == 18) v = tail[copy + mod4 - 1];
        }
        w |= (uint64_t)v << (8 * b);
    }
    hhq_update(s, w);
}

// 10 x PermuteAndUpdate, ModularReduction; lane q writes digest bytes [8q, 8q+8).
// Finalize; returns lane q's digest word (bytes [8q, 8q+8) little-endian).
__device__ __forceinline__ uint64_t hhq_digest(HHQuad& s, uint32_t q) {
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        const uint32_t lo = quad_swap_halves((uint32_t)s.v0), hi = quad_swap_halves((uint32_t)(s.v0 >> 32));
        hhq_update(s, (uint64_t)hi | ((uint64_t)lo << 32));  // rot32 of v0[q^2]
    }
    const uint64_t a_v1 = s.v1 + s.mul1, a_v0 = s.v0 + s.mul0;
    const uint32_t p_lo = quad_swap_pairs((uint32_t)a_v1), p_hi = quad_swap_pairs((uint32_t)(a_v1 >> 32));
    const uint64_t partner_v1 = (uint64_t)p_lo | ((uint64_t)p_hi << 32);
    uint64_t h;
    if (q & 1) {  // h[odd] from a3 = own v1+mul1, a2 = partner's, a1 = own v0+mul0
        const uint64_t a3 = a_v1 & 0x3FFFFFFFFFFFFFFFull, a2 = partner_v1;
        h = a_v0 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
    } else {      // h[even] = a0 ^ (a2 << 1) ^ (a2 << 2), a2 = own v1+mul1
        h = a_v0 ^ (a_v1 << 1) ^ (a_v1 << 2);
    }
    return h;
}

__device__ __forceinline__ void hhq_finish(HHQuad& s, uint8_t* out, uint32_t q) {
    const uint64_t h = hhq_digest(s, q);
#pragma unroll
    for (int b = 0; b < 8; ++b) out[8 * q + b] = (uint8_t)(h >> (8 * b));  // any alignment
}

__device__ __forceinline__ void st64_any(uint8_t* p, uint64_t v) { __builtin_memcpy(p, &v, 8); }

__device__ __forceinline__ uint64_t u64_of(const uint2& v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }

// The 8 bytes at p = shard + off of a shard of `len` bytes, those at or past
// len read as zero (the partial last chunk of a shard of any length).
__device__ __forceinline__ uint64_t ld64_part(const uint8_t* p, uint64_t off, uint64_t len) {
    if (off + 8 <= len) return ld64_any(p);
    uint64_t v = 0;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b)
        if (off + b < len) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

// Store the bytes of v that fall before len (see ld64_part).
__device__ __forceinline__ void st64_part(uint8_t* p, uint64_t v, uint64_t off, uint64_t len) {
    if (off + 8 <= len) {
        st64_any(p, v);
        return;
    }
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b)
        if (off + b < len) p[b] = (uint8_t)(v >> (8 * b));
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// A constant in a VGPR: VOP2 v_and with two VGPR operands issues at full rate
// on gfx950, with a literal (constant bus) at half rate (tools/kbench/op_rates.hip).
__device__ __forceinline__ uint32_t vgpr_const(uint32_t v) {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "i"(v));
    return r;
}

namespace dma {
constexpr uint32_t CH = 512;          // bytes per shard per step
constexpr uint32_t IP = 2 * CH + 32;  // LDS pitch of one DMA instruction (rows of stripes i and i+4)
constexpr uint32_t PP = CH + 32;      // parity row pitch
constexpr int SPW = 8, HS = 4, D = 3, NP = 2, EW = 4;

// s_waitcnt vmcnt(n) only (gfx9 encoding; n <= 63)
constexpr uint32_t vmcnt_imm(int n) {
    return 0x0F70u | ((uint32_t)(n > 63 ? 63 : n) & 15u) | (((uint32_t)(n > 63 ? 63 : n) >> 4) & 3u) << 14;
}

// 16 packets of one stream (8 B per lane, 32 B apart) from LDS, one asm.
// zeros over the 16 8-byte words read16 reads at LDS address a
__device__ __forceinline__ void zero16(uint32_t a) {
    const uint64_t z = 0;
    asm volatile(
        "ds_write_b64 %0, %1 offset:0\n\t"
        "ds_write_b64 %0, %1 offset:32\n\t"
        "ds_write_b64 %0, %1 offset:64\n\t"
        "ds_write_b64 %0, %1 offset:96\n\t"
        "ds_write_b64 %0, %1 offset:128\n\t"
        "ds_write_b64 %0, %1 offset:160\n\t"
        "ds_write_b64 %0, %1 offset:192\n\t"
        "ds_write_b64 %0, %1 offset:224\n\t"
        "ds_write_b64 %0, %1 offset:256\n\t"
        "ds_write_b64 %0, %1 offset:288\n\t"
        "ds_write_b64 %0, %1 offset:320\n\t"
        "ds_write_b64 %0, %1 offset:352\n\t"
        "ds_write_b64 %0, %1 offset:384\n\t"
        "ds_write_b64 %0, %1 offset:416\n\t"
        "ds_write_b64 %0, %1 offset:448\n\t"
        "ds_write_b64 %0, %1 offset:480"
        :
        : "v"(a), "v"(z)
        : "memory");
}

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


__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// 8x8 bit transpose of 8 dwords (bs::transpose) with two shifts and two
// v_bfi_b32 per masked swap; its own inverse
__device__ __forceinline__ void swap_bfi(uint32_t& lo, uint32_t& hi, int s, uint32_t mask) {
    const uint32_t a = lo, b = hi;
    lo = bfi(mask, a, b << s);
    hi = bfi(mask, a >> s, b);
}
__device__ __forceinline__ void transpose(uint32_t (&w)[8], uint32_t m4, uint32_t m2, uint32_t m1) {
#pragma unroll
    for (int d = 0; d < 4; ++d) swap_bfi(w[d], w[d + 4], 4, m4);
    swap_bfi(w[0], w[2], 2, m2);
    swap_bfi(w[1], w[3], 2, m2);
    swap_bfi(w[4], w[6], 2, m2);
    swap_bfi(w[5], w[7], 2, m2);
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap_bfi(w[d], w[d + 1], 1, m1);
}

}  // namespace dma

}  // namespace rsg
