// rs_kernels.hip — CDNA4 (gfx950) kernels of the Reed–Solomon erasure engine.
//
// Hot path: parity[r][b] = XOR_c G[r][c] * data[c][b] over GF(2^8)/0x11D for
// every byte b of every stripe (ReedSolomon::encode behind
// ReedSolomonEncoder::encode, crates/ecstore/src/erasure/coding/erasure.rs:396),
// and the same product with an inverted sub-matrix for reconstruct
// (erasure.rs:411-428, bridge.rs:274-307).  Byte-field work: no MFMA.
//
// GF multiply by a per-launch constant c is done 4 bytes at a time with
// v_perm_b32 byte lookups.  A byte x splits into 3-bit, 3-bit and 2-bit fields
// and, because multiplication by c is GF(2)-linear,
//     c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// with T0[i] = c*i, T1[i] = c*(i<<3), T2[i] = c*(i<<6).  T0/T1 are 8-byte tables
// (two dwords, one v_perm_b32 source pair), T2 a 4-byte table (one dword).  The
// field selectors are computed once per data word and shared by every output
// row, so one word-coefficient multiply-accumulate is 3 v_perm_b32 + 3 v_xor.
// The 5 table dwords per coefficient are computed on the host
// (rsgpu.cpp: coef_tables) and arrive in the kernel-argument segment, i.e. in
// SGPRs — wave-uniform, no per-byte LDS log/antilog lookups (those cannot meet
// the HBM op budget).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rs_kernels.h"

namespace rsg {

// ---------------------------------------------------------------------------
// GF(2^8) matrix apply, vector path: 16-byte units, every shard 16-B aligned.
// Block = 256 threads = 4 waves; thread t of block b handles unit
// (chunk*UNITS_PER_THREAD + j)*256 + t, j < UNITS_PER_THREAD, so each wave's
// loads/stores are contiguous 1 KiB per shard (global_load_dwordx4).

__device__ __forceinline__ uint32_t gf_mul_word(const uint32_t* t, uint32_t s0, uint32_t s1, uint32_t s2) {
    return __builtin_amdgcn_perm(t[1], t[0], s0) ^ __builtin_amdgcn_perm(t[3], t[2], s1) ^
           __builtin_amdgcn_perm(t[4], t[4], s2);
}

template <int C, int R>
__global__ __launch_bounds__(256) void k_gf_apply_vec(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;

#pragma unroll 1
    for (uint32_t j = 0; j < p.units_per_thread; ++j) {
        const uint32_t u = (chunk * p.units_per_thread + j) * 256u + threadIdx.x;
        if (u >= p.units) return;
        const uint64_t off = (uint64_t)u * 16u;

        uint4 x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = *(const uint4*)(sbase + p.in_off[c] + off);

        uint32_t acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;

#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint32_t w[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u;
                const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
                const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r][q] ^= gf_mul_word(p.tab[r][c], s0, s1, s2);
            }
        }

#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint4* dst = (uint4*)(obase + p.out_off[r] + off);
            uint4 v = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
            if (p.mode == GF_MODE_STORE) {
                *dst = v;
            } else if (p.mode == GF_MODE_XOR) {
                uint4 o = *dst;
                *dst = make_uint4(o.x ^ v.x, o.y ^ v.y, o.z ^ v.z, o.w ^ v.w);
            } else {  // GF_MODE_COMPARE: clear the stripe's ok flag on mismatch
                uint4 o = *dst;
                if ((o.x ^ v.x) | (o.y ^ v.y) | (o.z ^ v.z) | (o.w ^ v.w)) p.ok_flags[stripe] = 0;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Byte path: any alignment, any length.  One thread per byte column.  Used for
// unaligned shards (e.g. S = ceil(1 MiB / 6)) and the S % 16 tail.
template <int R>
__global__ __launch_bounds__(256) void k_gf_apply_byte(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint64_t b = (uint64_t)p.byte_begin + (uint64_t)chunk * 256u + threadIdx.x;
    if (b >= p.byte_end) return;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;

    uint32_t acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
    for (uint32_t c = 0; c < p.C; ++c) {
        const uint32_t x = sbase[p.in_off[c] + b];
        const uint32_t s0 = x & 7u, s1 = (x >> 3) & 7u, s2 = x >> 6;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] ^= gf_mul_word(p.tab[r][c], s0, s1, s2);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* dst = obase + p.out_off[r] + b;
        const uint8_t v = (uint8_t)acc[r];
        if (p.mode == GF_MODE_STORE) *dst = v;
        else if (p.mode == GF_MODE_XOR) *dst ^= v;
        else if (*dst != v) p.ok_flags[stripe] = 0;
    }
}

// ---------------------------------------------------------------------------
// HighwayHash-256 (public spec; the `highway` crate 1.3.0 used by
// crates/utils/src/hash.rs:123-127).  One thread per message (first slice).

struct HHState {
    uint64_t v0[4], v1[4], mul0[4], mul1[4];
};

__device__ __forceinline__ void hh_reset(const uint64_t* key, HHState& s) {
    const uint64_t i0[4] = {0xdbe6d5d5fe4cce2full, 0xa4093822299f31d0ull, 0x13198a2e03707344ull,
                            0x243f6a8885a308d3ull};
    const uint64_t i1[4] = {0x3bd39e10cb0ef593ull, 0xc0acf169b5f18a8cull, 0xbe5466cf34e90c6cull,
                            0x452821e638d01377ull};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.mul0[i] = i0[i];
        s.mul1[i] = i1[i];
        s.v0[i] = i0[i] ^ key[i];
        s.v1[i] = i1[i] ^ ((key[i] >> 32) | (key[i] << 32));
    }
}

__device__ __forceinline__ void hh_zipper(uint64_t v1, uint64_t v0, uint64_t& add1, uint64_t& add0) {
    add0 += (((v0 & 0xff000000ull) | (v1 & 0xff00000000ull)) >> 24) |
            (((v0 & 0xff0000000000ull) | (v1 & 0xff000000000000ull)) >> 16) | (v0 & 0xff0000ull) |
            ((v0 & 0xff00ull) << 32) | ((v1 & 0xff00000000000000ull) >> 8) | (v0 << 56);
    add1 += (((v1 & 0xff000000ull) | (v0 & 0xff00000000ull)) >> 24) | (v1 & 0xff0000ull) |
            ((v1 & 0xff0000000000ull) >> 16) | ((v1 & 0xff00ull) << 24) |
            ((v0 & 0xff000000000000ull) >> 8) | ((v1 & 0xffull) << 48) | (v0 & 0xff00000000000000ull);
}

__device__ __forceinline__ uint64_t mul32x32(uint64_t a, uint64_t b) {
    return (uint64_t)(uint32_t)a * (uint64_t)(uint32_t)b;
}

__device__ __forceinline__ void hh_update(const uint64_t* lanes, HHState& s) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.v1[i] += s.mul0[i] + lanes[i];
        s.mul0[i] ^= mul32x32(s.v1[i], s.v0[i] >> 32);
        s.v0[i] += s.mul1[i];
        s.mul1[i] ^= mul32x32(s.v0[i], s.v1[i] >> 32);
    }
    hh_zipper(s.v1[1], s.v1[0], s.v0[1], s.v0[0]);
    hh_zipper(s.v1[3], s.v1[2], s.v0[3], s.v0[2]);
    hh_zipper(s.v0[1], s.v0[0], s.v1[1], s.v1[0]);
    hh_zipper(s.v0[3], s.v0[2], s.v1[3], s.v1[2]);
}

__device__ __forceinline__ uint64_t ld64_any(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

__device__ void hh_finish(const uint8_t* tail, uint32_t size_mod32, HHState& s, uint8_t* out) {
    if (size_mod32) {
        const uint32_t size_mod4 = size_mod32 & 3u;
        const uint8_t* rem = tail + (size_mod32 & ~3u);
        uint8_t packet[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) packet[i] = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s.v0[i] += ((uint64_t)size_mod32 << 32) + size_mod32;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t h0 = (uint32_t)s.v1[i], h1 = (uint32_t)(s.v1[i] >> 32);
            h0 = (h0 << size_mod32) | (h0 >> (32u - size_mod32));
            h1 = (h1 << size_mod32) | (h1 >> (32u - size_mod32));
            s.v1[i] = (uint64_t)h0 | ((uint64_t)h1 << 32);
        }
        for (uint32_t i = 0; i < (size_mod32 & ~3u); ++i) packet[i] = tail[i];
        if (size_mod32 & 16u) {
            // last 4 bytes of the message (size_mod32 >= 16: no underflow)
            for (uint32_t i = 0; i < 4; ++i) packet[28 + i] = tail[size_mod32 - 4 + i];
        } else if (size_mod4) {
            packet[16] = rem[0];
            packet[17] = rem[size_mod4 >> 1];
            packet[18] = rem[size_mod4 - 1];
        }
        uint64_t lanes[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) lanes[i] = ld64_any(packet + 8 * i);
        hh_update(lanes, s);
    }
#pragma unroll 1
    for (int it = 0; it < 10; ++it) {
        uint64_t pm[4];
        pm[0] = (s.v0[2] >> 32) | (s.v0[2] << 32);
        pm[1] = (s.v0[3] >> 32) | (s.v0[3] << 32);
        pm[2] = (s.v0[0] >> 32) | (s.v0[0] << 32);
        pm[3] = (s.v0[1] >> 32) | (s.v0[1] << 32);
        hh_update(pm, s);
    }
    uint64_t h[4];
    for (int half = 0; half < 2; ++half) {
        const int a = 2 * half;
        const uint64_t a3 = (s.v1[a + 1] + s.mul1[a + 1]) & 0x3FFFFFFFFFFFFFFFull;
        const uint64_t a2 = s.v1[a] + s.mul1[a];
        const uint64_t a1 = s.v0[a + 1] + s.mul0[a + 1];
        const uint64_t a0 = s.v0[a] + s.mul0[a];
        h[a + 1] = a1 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
        h[a] = a0 ^ (a2 << 1) ^ (a2 << 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int b = 0; b < 8; ++b) out[i * 8 + b] = (uint8_t)(h[i] >> (8 * b));
}

// Message j of n: bytes [msg_base(j), msg_base(j) + len).  Messages are
// addressed either as data + j*stride (plain batch) or, for the per-shard
// digests of encoded stripes, as data + (j / shards)*stripe_stride +
// (j % shards)*shard_pitch.
__global__ __launch_bounds__(64) void k_hh256_thread(const HashParams p) {
    const uint64_t j = (uint64_t)blockIdx.x * 64u + threadIdx.x;
    if (j >= p.n) return;
    const uint64_t stripe = j / p.shards, shard = j - stripe * p.shards;
    const uint8_t* msg = p.data + stripe * p.stripe_stride + shard * p.shard_pitch;
    HHState s;
    hh_reset(p.key, s);
    const uint64_t full = p.len & ~(uint64_t)31;
    if (p.aligned16) {
#pragma unroll 1
        for (uint64_t i = 0; i < full; i += 32) {
            const uint4 a = *(const uint4*)(msg + i);
            const uint4 b = *(const uint4*)(msg + i + 16);
            const uint64_t lanes[4] = {(uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32),
                                       (uint64_t)b.x | ((uint64_t)b.y << 32), (uint64_t)b.z | ((uint64_t)b.w << 32)};
            hh_update(lanes, s);
        }
    } else {
#pragma unroll 1
        for (uint64_t i = 0; i < full; i += 32) {
            const uint64_t lanes[4] = {ld64_any(msg + i), ld64_any(msg + i + 8), ld64_any(msg + i + 16),
                                       ld64_any(msg + i + 24)};
            hh_update(lanes, s);
        }
    }
    uint8_t digest[32];
    hh_finish(msg + full, (uint32_t)(p.len & 31), s, digest);
    uint8_t* o = p.out + j * 32u;
#pragma unroll
    for (int i = 0; i < 32; ++i) o[i] = digest[i];
}

// ---------------------------------------------------------------------------
// Launchers.

using GfKernel = void (*)(const GfApplyParams);

template <int C>
static GfKernel pick_vec_r(int R) {
    switch (R) {
        case 1: return k_gf_apply_vec<C, 1>;
        case 2: return k_gf_apply_vec<C, 2>;
        case 3: return k_gf_apply_vec<C, 3>;
        case 4: return k_gf_apply_vec<C, 4>;
    }
    return nullptr;
}

static GfKernel pick_vec(int C, int R) {
    switch (C) {
        case 1: return pick_vec_r<1>(R);
        case 2: return pick_vec_r<2>(R);
        case 3: return pick_vec_r<3>(R);
        case 4: return pick_vec_r<4>(R);
        case 5: return pick_vec_r<5>(R);
        case 6: return pick_vec_r<6>(R);
        case 7: return pick_vec_r<7>(R);
        case 8: return pick_vec_r<8>(R);
        case 9: return pick_vec_r<9>(R);
        case 10: return pick_vec_r<10>(R);
        case 11: return pick_vec_r<11>(R);
        case 12: return pick_vec_r<12>(R);
        case 13: return pick_vec_r<13>(R);
        case 14: return pick_vec_r<14>(R);
        case 15: return pick_vec_r<15>(R);
        case 16: return pick_vec_r<16>(R);
    }
    return nullptr;
}

static GfKernel pick_byte(int R) {
    switch (R) {
        case 1: return k_gf_apply_byte<1>;
        case 2: return k_gf_apply_byte<2>;
        case 3: return k_gf_apply_byte<3>;
        case 4: return k_gf_apply_byte<4>;
    }
    return nullptr;
}

hipError_t launch_gf_apply_vec(GfApplyParams p, uint64_t n_stripes, hipStream_t stream) {
    GfKernel k = pick_vec((int)p.C, (int)p.R);
    if (!k || p.units == 0 || n_stripes == 0) return hipErrorInvalidValue;
    if (p.units_per_thread == 0) p.units_per_thread = 1;
    const uint32_t per_block = 256u * p.units_per_thread;
    p.chunks_per_stripe = (p.units + per_block - 1) / per_block;
    const uint64_t blocks = (uint64_t)p.chunks_per_stripe * n_stripes;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_gf_apply_byte(GfApplyParams p, uint64_t n_stripes, hipStream_t stream) {
    GfKernel k = pick_byte((int)p.R);
    if (!k || p.byte_end <= p.byte_begin || n_stripes == 0) return hipErrorInvalidValue;
    const uint64_t span = p.byte_end - p.byte_begin;
    p.chunks_per_stripe = (uint32_t)((span + 255u) / 256u);
    const uint64_t blocks = (uint64_t)p.chunks_per_stripe * n_stripes;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_hh256(const HashParams& p, hipStream_t stream) {
    if (p.n == 0) return hipSuccess;
    const uint64_t blocks = (p.n + 63u) / 64u;
    hipLaunchKernelGGL(k_hh256_thread, dim3((uint32_t)blocks), dim3(64), 0, stream, p);
    return hipGetLastError();
}

}  // namespace rsg
