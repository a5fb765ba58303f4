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

#include <array>
#include <atomic>
#include <deque>
#include <mutex>
#include <string>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_device.h"
#include "gf_bitslice.h"

namespace rsg {

#include "rs84_xornet.h"  // generated (tools/gen_xornet.py); uses x3

// PRE: the launch has XOR / COMPARE rows, whose read-back operands are loaded
// with the inputs, or copy-through inputs (a separate instantiation: the
// plain STORE encode and reconstruct kernels keep their register budget).
template <int C, int R, int B, bool PRE>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(2))) void k_gf_apply_vec(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * (uint32_t)B + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint4 old[R];
    if constexpr (PRE) gf_preload<R>(p, obase, off, stripe, old);
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    gf_accumulate<0, C, R>(p, x, acc);
    if constexpr (PRE) gf_store<R>(p, obase, off, acc, stripe, old);
    else gf_store_late<R>(p, obase, off, acc, stripe);
    // Copy-through last, with non-temporal stores (written once, never read
    // back by this pass): GET with 2 data shards lost (6 copies, 2 rebuilt, 2
    // compared) 1.85 ms with the copies among the input loads, 1.61 ms here,
    // 1.58 ms non-temporal (tools/kbench/get_probe.hip).
    if (PRE && p.copy_mask) {  // wave-uniform
#pragma unroll
        for (int c = 0; c < C; ++c)
            if ((p.copy_mask >> c) & 1u) st16_nt(obase + p.copy_off[c] + off, x[c]);
    }
}

// Rolled over the inputs in groups of G=8 (any C <= 16, R <= 8): the next
// group's 8 loads are issued before the current group's arithmetic, and the
// tables are indexed by the scalar loop counter (scalar loads, one group's
// worth in SGPRs).  The unrolled kernel above keeps all C inputs and, for
// C > 8, parks all C*R coefficient tables in VGPRs (~250 VGPRs at C=16, R=4:
// 2 waves per SIMD); rolled in groups of 4, RS(16,4) ran at 65-66 % of HBM
// peak, in groups of 8 (128 B in flight per lane, 105 VGPRs) at 72-73 %
// (tools/kbench/xor3_variants.hip).  For C <= 8, R <= 4 the unrolled kernel is
// faster and stays the default there.  G = 12 for 9-12 inputs (RS(12,4), the
// 16-drive default; RS(10,4)): one group, every input's load in flight at
// once instead of 8 then 4.
template <int R, int B, bool PRE, int G = 8>
__global__ __launch_bounds__(B) void k_gf_apply_loop(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * (uint32_t)B + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    const uint32_t C = p.C;
    uint32_t acc[R][4], pend[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[r][q] = pend[r][q] = 0u;
    uint4 x[G], y[G];
#pragma unroll
    for (int g = 0; g < G; ++g)
        if ((uint32_t)g < C) x[g] = ld16(sbase + p.in_off[g] + off);
    uint4 old[R];
    if constexpr (PRE) gf_preload<R>(p, obase, off, stripe, old);
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < C; c0 += G) {
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (c0 + G + g < C) y[g] = ld16(sbase + p.in_off[c0 + G + g] + off);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t c = c0 + g;
            if (c >= C) break;  // wave-uniform
            if (PRE && ((p.copy_mask >> c) & 1u)) st16(obase + p.copy_off[c] + off, x[g]);
            const uint32_t w[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t s0 = w[q] & 0x07070707u;
                const uint32_t s1 = (w[q] >> 3) & 0x07070707u;
                const uint32_t s2 = (w[q] >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t* t = p.tab[r][c];
                    gf_fold(g & 1, acc[r][q], pend[r][q], __builtin_amdgcn_perm(t[1], t[0], s0),
                            __builtin_amdgcn_perm(t[3], t[2], s1), __builtin_amdgcn_perm(t[4], t[4], s2));
                }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) x[g] = y[g];
    }
    if (C & 1u) {  // an odd C leaves the last input's third lookup pending
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] ^= pend[r][q];
    }
    if constexpr (PRE) gf_store<R>(p, obase, off, acc, stripe, old);
    else gf_store_late<R>(p, obase, off, acc, stripe);
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
        if ((p.copy_mask >> c) & 1u) obase[p.copy_off[c] + b] = (uint8_t)x;
        const uint32_t s0 = x & 7u, s1 = (x >> 3) & 7u, s2 = x >> 6;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] ^= gf_mul_word(p.tab[r][c], s0, s1, s2);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint32_t mode = p.mode;
        uint8_t* dst = obase + p.out_off[r] + b;
        if (mode == GF_MODE_STORE_COMPARE) {
            mode = (uint32_t)r < p.n_store ? GF_MODE_STORE : GF_MODE_COMPARE;
            if (mode == GF_MODE_COMPARE) dst = p.out_base + (uint64_t)stripe * p.cmp_stripe_stride + p.out_off[r] + b;
        }
        const uint8_t v = (uint8_t)acc[r];
        if (mode == GF_MODE_STORE) *dst = v;
        else if (mode == GF_MODE_XOR) *dst ^= v;
        else if (*dst != v) p.ok_flags[stripe] = 0;
    }
}

// Plain / per-shard batch hash: quad j hashes message j (16 messages per wave).
// Every lane issues its own 8-byte loads.  DEPTH = 1: one batch of 8 packets
// fetched, then hashed; DEPTH = 2 (default): two batches (16 packets, 128 B per
// lane) in flight, the next batch's loads issued before the current batch is
// hashed; DEPTH = 3: three.  A launch of few messages (the GET engine's 8 data records per
// stripe: 2 waves per SIMD at 4096 stripes) needs the deeper pipeline to keep
// enough bytes in flight per CU.  COPY: also store the message bytes to
// copy_base[b] + r*copy_stride (multi-file).
//
// COPY = 2 (staged copy, multi-file mode): each wave passes its 16 messages'
// 8-packet batches (16 x 256 B) through a wave-private LDS tile and stores them
// 16 B per lane, 256 contiguous bytes per message (four whole messages' pieces
// per instruction) instead of 16 scattered 32-byte pieces of 8 B per lane.
// The whole wave stays in the loop (a quad past n hashes message 0 and stores
// nothing) because its lanes store other quads' bytes.
//
// UNAL (verify / digest launches with messages at odd offsets: BitrotWriter
// records of RS(6,4) at 1 MiB blocks, 32 + 174763 bytes): each lane loads
// the aligned 8-byte word of its packet piece and the quad rebuilds the
// message bytes with a funnel shift across neighbouring lanes (one DPP quad
// rotation per word and v_alignbyte_b32), instead of 8-byte loads at odd
// addresses — which ran the all-present RS(6,4) GET at 0.53 of HBM against
// 0.78 for aligned RS(8,4) records (profiles/r04/n/).  Lane 3's last word of a batch starts the next
// packet: the quad loads that aligned word too (it holds a message byte, so
// the load stays inside the caller's buffer).
template <int COPY, int DEPTH, bool UNAL = false>
__global__ __launch_bounds__(256) void k_hh256_quad(const HashParams p) {
    const uint64_t j0 = ((uint64_t)blockIdx.x * 256u + threadIdx.x) >> 2;
    const uint32_t q = threadIdx.x & 3u;
    const bool alive = j0 < p.n;
    if (COPY != 2 && !alive) return;  // whole quads exit together
    const uint64_t j = alive ? j0 : 0;
    const uint8_t* msg;
    uint8_t* dst = nullptr;
    uint8_t* flag = p.flags ? p.flags + j : nullptr;
    if (p.nbases) {
        const uint64_t b = j / p.per_base, r = j - b * p.per_base;
        msg = p.base[b] + r * p.stripe_stride;
        if (p.flag_base[b]) flag = p.flag_base[b] + r;
        // copy mode: files without a copy_base (parity records verified in
        // the same launch as the data records they back up) are only hashed
        if constexpr (COPY != 0) dst = p.copy_base[b] ? p.copy_base[b] + r * p.copy_stride : nullptr;
    } else {
        const uint64_t stripe = j / p.shards, shard = j - stripe * p.shards;
        msg = p.data + stripe * p.stripe_stride + shard * p.shard_pitch;
    }
    // staged copy: this lane stores bytes [16 (lane & 15), +16) of every
    // 256-byte batch of wave messages 4 kk + (lane >> 4), kk = 0..3
    __shared__ __attribute__((aligned(16))) uint8_t stage[COPY == 2 ? 4 * 4096 : 16];
    uint8_t* sdst[4] = {nullptr, nullptr, nullptr, nullptr};
    uint8_t* const stg = stage + (COPY == 2 ? (threadIdx.x >> 6) * 4096u : 0u);
    const uint32_t lane = threadIdx.x & 63u;
    if constexpr (COPY == 2) {
        const uint64_t wj = ((uint64_t)blockIdx.x * 256u + (threadIdx.x & ~63u)) >> 2;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const uint64_t jj = wj + 4 * kk + (lane >> 4);
            if (jj < p.n) {
                const uint64_t b = jj / p.per_base, r = jj - b * p.per_base;
                if (p.copy_base[b]) sdst[kk] = p.copy_base[b] + r * p.copy_stride + (lane & 15u) * 16u;
            }
        }
    }
    HHQuad s;
    hhq_init(s, p.key, q);
    const uint64_t packets = p.len >> 5;
    uint64_t t = 0;
    const uint32_t mis = UNAL ? (uint32_t)((uintptr_t)msg & 7u) : 0u;  // the message's byte offset in its word
    const uint8_t* const am = msg - mis;
    // 8-byte loads at any alignment (records put data 32 B after the digest,
    // shards of unaligned length are common); UNAL: aligned words, w[8] = the
    // word that starts the next packet
    auto fetch = [&](uint64_t (&w)[9], uint64_t t0) {
        if constexpr (UNAL) {
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = *(const uint64_t*)(am + (t0 + i) * 32 + 8 * q);
            w[8] = mis ? *(const uint64_t*)(am + (t0 + 8) * 32) : 0ull;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = ld64_any(msg + (t0 + i) * 32 + 8 * q);
        }
    };
    // UNAL: lane q's message word = its aligned word >> 8 mis, filled from the
    // next lane's (lane 3: the next packet's first word)
    auto realign = [&](uint64_t (&w)[9]) {
        uint64_t nx[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const u32x2 v = __builtin_bit_cast(u32x2, w[i]);
            u32x2 r;
            r.x = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.x, 0x39, 0xF, 0xF, false);  // quad_perm [1,2,3,0]
            r.y = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.y, 0x39, 0xF, 0xF, false);
            nx[i] = __builtin_bit_cast(uint64_t, r);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t hi = q == 3 ? (i < 7 ? nx[i + 1] : w[8]) : nx[i];
            const uint32_t l0 = (uint32_t)w[i], l1 = (uint32_t)(w[i] >> 32), h0 = (uint32_t)hi,
                           h1 = (uint32_t)(hi >> 32);
            const uint32_t a0 = __builtin_amdgcn_alignbyte(l1, l0, mis), a1 = __builtin_amdgcn_alignbyte(h0, l1, mis);
            const uint32_t b1 = __builtin_amdgcn_alignbyte(h1, h0, mis);
            w[i] = mis < 4 ? ((uint64_t)a1 << 32 | a0) : ((uint64_t)b1 << 32 | a1);
        }
    };
    auto consume = [&](uint64_t (&w)[9], uint64_t t0) {
        if constexpr (UNAL) realign(w);
#pragma unroll
        for (int i = 0; i < 8; ++i) hhq_update(s, w[i]);
        if constexpr (COPY == 1) {
            if (dst) {
#pragma unroll
                for (int i = 0; i < 8; ++i) st64_any(dst + (t0 + i) * 32 + 8 * q, w[i]);
            }
        } else if constexpr (COPY == 2) {
            // one wave's LDS instructions execute in order: the reads below see
            // these writes, and the next batch's writes follow these reads
#pragma unroll
            for (int i = 0; i < 8; ++i) *(uint64_t*)(stg + (lane >> 2) * 256u + i * 32 + 8 * q) = w[i];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const uint4 v = *(const uint4*)(stg + (4 * kk + (lane >> 4)) * 256u + (lane & 15u) * 16u);
                if (sdst[kk]) st16_nt(sdst[kk] + t0 * 32, v);
            }
        }
    };
    const uint64_t nb = packets / 8;  // whole 8-packet batches
    if constexpr (DEPTH >= 2) {
        // DEPTH register batches: batch x lives in w[x % DEPTH]; the loads of
        // batch x + DEPTH - 1 are issued before batch x is hashed.  Loads past
        // the last batch are clamped to it (inside the message) and unused.
        if (nb) {
            uint64_t w[DEPTH][9];
#pragma unroll
            for (int d = 0; d < DEPTH - 1; ++d) fetch(w[d], ((uint64_t)d < nb ? (uint64_t)d : nb - 1) * 8);
            uint64_t b = 0;
            for (; b + DEPTH <= nb; b += DEPTH) {
#pragma unroll
                for (int d = 0; d < DEPTH; ++d) {
                    const uint64_t nxt = b + d + DEPTH - 1;
                    fetch(w[(d + DEPTH - 1) % DEPTH], (nxt < nb ? nxt : nb - 1) * 8);
                    consume(w[d], (b + d) * 8);
                }
            }
#pragma unroll
            for (int d = 0; d < DEPTH - 1; ++d)  // fewer than DEPTH batches left, all fetched
                if (b + d < nb) consume(w[d], (b + d) * 8);
            t = nb * 8;
        }
    } else {
        for (; t + 8 <= packets; t += 8) {
            uint64_t w[9];
            fetch(w, t);
            consume(w, t);
        }
    }
    if (!alive) return;  // (COPY == 2) the wave-wide staged batches are done
    for (; t < packets; ++t) {
        const uint64_t w = ld64_any(msg + t * 32 + 8 * q);
        hhq_update(s, w);
        if (COPY && dst) st64_any(dst + t * 32 + 8 * q, w);
    }
    const uint32_t rem = (uint32_t)(p.len & 31);
    if (rem) {
        hhq_remainder(s, msg + packets * 32, rem, q);
        if (COPY && dst)
            for (uint32_t b = 8 * q; b < rem && b < 8 * q + 8; ++b) dst[packets * 32 + b] = msg[packets * 32 + b];
    }
    if (flag) {  // verify before use (split_and_verify, bitrot.rs:227-247)
        const uint8_t* want = p.nbases ? msg + p.digest_off : p.expect + j * p.expect_stride;
        const uint64_t h = hhq_digest(s, q);
        if (h != ld64_any(want + 8 * q)) *flag = 0;
    } else {
        hhq_finish(s, p.nbases ? const_cast<uint8_t*>(msg) + p.digest_off : p.out + j * (p.out_stride ? p.out_stride : 32u),
                   q);
    }
}

// ---------------------------------------------------------------------------
// Fused RS encode + per-shard HighwayHash-256 (BitrotWriter digests,
// bitrot.rs:496-502) in one pass over HBM.  One workgroup owns SPW stripes and
// walks them in 512-byte column chunks with fixed wave roles:
//   waves 0..SPW-1 (encoders, one per stripe): load the k data chunks (8 B per
//     lane per shard), compute and store the m parity chunks, and stage all
//     k+m chunks in LDS; the next chunk's loads are issued before the barrier.
//   waves SPW.. (hashers): the SPW*(k+m) HighwayHash streams of the workgroup,
//     one 4-lane quad per stream, 16 streams per wave, each advanced by 16
//     packets per chunk.  HighwayHash is sequential per shard, so a stripe has
//     only (k+m) x 4 lanes of hash parallelism; packing the streams of several
//     stripes into full hasher waves (SPW = 4 for RS(8,4): 48 streams = 3 waves)
//     keeps every hasher lane busy.
// Per chunk:  encoders compute(i) | bar A | write rows(i) | bar B | loads(i+2)..
//             hashers             | bar A |               | bar B | hash(i) ..
// so the encoders' arithmetic for chunk i+1 overlaps the hashing of chunk i.
// Barriers are raw s_barrier with an explicit lgkmcnt wait: __syncthreads()
// would also drain the in-flight global loads (vmcnt(0)).  Stripes past the end
// of the batch keep their waves in the barrier sequence with memory ops masked.
constexpr uint32_t kFusedChunk = 512;                 // bytes per shard per step
constexpr uint32_t kFusedPitch = kFusedChunk + 32;    // LDS row pitch: conflict-free ds_read_b64

constexpr int fused_spw_for(int T) {  // stripes per workgroup: fill hasher waves, cap LDS
    return (T % 16 == 0) ? 1 : (T % 8 == 0) ? 2 : (T % 4 == 0 || T <= 6) ? 4 : 2;
}
template <int T>
constexpr int fused_spw() {
    return fused_spw_for(T);
}

// ABLATE_ (measurement builds only: tools/kbench/fused_variants.hip defines
// RSG_MEASUREMENT_BUILD before including this file): bit 0 skips the GF
// arithmetic, bit 1 the hash updates, bit 3 records each wave's HW_ID in its
// stripe's first digest words, bit 4 raises the hasher waves' issue priority
// (s_setprio 1), bit 5 the encoder waves'.  In the shipped library every
// ablation bit compiles to 0.
template <int C, int R, int SPW, int ABLATE_ = 0>
__global__ __launch_bounds__(64 * (SPW + (SPW * (C + R) + 15) / 16))
__attribute__((amdgpu_waves_per_eu(R == 1 ? 4 : C <= 8 ? 7 : C <= 12 ? 5 : 4)))
void k_encode_hash_fused(const GfApplyParams p,
                                                                                              const HashParams h) {
    static_assert(ABLATE_ == 0 || RSG_MEASUREMENT_BUILD, "ablation variants exist in measurement builds only");
    constexpr int ABLATE = RSG_MEASUREMENT_BUILD ? ABLATE_ : 0;
    // LDS: [C][R] coefficient tables (32 B each: T0 T0' T1 T1' | T2), then
    // SPW x (C+R) chunk rows.  Tables are read from LDS (broadcast) at their
    // use: held in registers across the chunk loop they cost 64+ VGPRs.
    extern __shared__ uint8_t lds_all[];
    constexpr int T = C + R;
    constexpr uint32_t kTabBytes = C * R * 32;
    constexpr uint32_t kStripeRows = T * kFusedPitch;
    uint8_t* rows = lds_all + kTabBytes;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t chunks = p.units;  // ceil(S / kFusedChunk)

    for (uint32_t i = threadIdx.x; i < (uint32_t)(C * R); i += blockDim.x) {
        const int c = i / R, r = i % R;
        uint8_t* d = lds_all + i * 32;
        *(uint4*)d = make_uint4(p.tab[r][c][0], p.tab[r][c][1], p.tab[r][c][2], p.tab[r][c][3]);
        *(uint32_t*)(d + 16) = p.tab[r][c][4];
    }
    __syncthreads();
    if constexpr (ABLATE & 8) {
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + (wave < SPW ? wave : 0);
        if (lane == 0 && stripe < n) ((uint32_t*)(h.out + stripe * T * 32u))[wave < SPW ? 0 : 1 + (wave - SPW)] =
            __builtin_amdgcn_s_getreg(0xF804);
        return;
    }

    // Shards of any length (p.byte_end = S): chunks = ceil(S / 512); the
    // last one holds `tail` bytes (1..512).  Its loads read nothing past the
    // shard (zeros instead, so the parity bytes past S are zero too), its
    // stores write nothing past it, and the hashers run its whole packets and
    // then HighwayHash's remainder packet — RS(12,4) at 1 MiB blocks has
    // S = 87382 (170 chunks + 342 bytes), and its shards sit at every
    // alignment (8-byte accesses at any address: gfx950's unaligned mode).
    const uint64_t S = p.byte_end;
    const uint32_t tail = (uint32_t)(S - (uint64_t)(chunks - 1) * kFusedChunk);
    if (wave < (uint32_t)SPW) {
        // ------------------------------ encoder ------------------------------
        if constexpr (ABLATE & 32) __builtin_amdgcn_s_setprio(1);
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + wave;
        const bool live = stripe < n;  // a dead stripe re-reads stripe 0 and stores nothing
        uint8_t* sb = p.out_base + (live ? stripe : 0) * p.stripe_stride;
        uint8_t* my_rows = rows + wave * kStripeRows;
        const uint32_t m7 = vgpr_const(0x07070707u), m3 = vgpr_const(0x03030303u);
        // the GF rows of one chunk (x: 8 bytes of every data shard per lane)
        auto rows_of = [&](const uint2 (&x)[C], uint32_t (&acc)[R][2]) {
            // opaque per-iteration zero: keeps the table reads at their use
            // instead of hoisted out of the loop into (spilled) registers
            uint32_t tz;
            asm volatile("s_mov_b32 %0, 0" : "=s"(tz));
            const uint8_t* tabs = lds_all + tz;
            uint32_t pend[R][2];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = pend[r][0] = pend[r][1] = 0u;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if constexpr (ABLATE & 1) {
                    acc[c % R][0] ^= x[c].x;
                    acc[c % R][1] ^= x[c].y;
                    continue;
                }
                const uint32_t s0a = x[c].x & m7, s0b = x[c].y & m7;
                const uint32_t s1a = (x[c].x >> 3) & m7, s1b = (x[c].y >> 3) & m7;
                const uint32_t s2a = (x[c].x >> 6) & m3, s2b = (x[c].y >> 6) & m3;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint8_t* tp = tabs + (c * R + r) * 32;  // wave-uniform: broadcast read
                    const uint4 t4 = *(const uint4*)tp;
                    const uint32_t t2 = *(const uint32_t*)(tp + 16);
                    gf_fold(c & 1, acc[r][0], pend[r][0], __builtin_amdgcn_perm(t4.y, t4.x, s0a),
                            __builtin_amdgcn_perm(t4.w, t4.z, s1a), __builtin_amdgcn_perm(t2, t2, s2a));
                    gf_fold(c & 1, acc[r][1], pend[r][1], __builtin_amdgcn_perm(t4.y, t4.x, s0b),
                            __builtin_amdgcn_perm(t4.w, t4.z, s1b), __builtin_amdgcn_perm(t2, t2, s2b));
                }
            }
            if constexpr (C % 2 == 1 && !(ABLATE & 1)) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    acc[r][0] ^= pend[r][0];
                    acc[r][1] ^= pend[r][1];
                }
            }
        };
        // a chunk's data and parity rows into this stripe's LDS rows, between
        // barrier A (the hashers are done with the previous chunk's rows) and
        // B (this chunk's rows are ready)
        auto publish = [&](const uint2 (&x)[C], const uint32_t (&acc)[R][2]) {
            lds_barrier();  // A
#pragma unroll
            for (int c = 0; c < C; ++c) *(uint2*)(my_rows + c * kFusedPitch + lane * 8u) = x[c];
#pragma unroll
            for (int r = 0; r < R; ++r)
                *(uint2*)(my_rows + (C + r) * kFusedPitch + lane * 8u) = make_uint2(acc[r][0], acc[r][1]);
            lds_barrier();  // B
        };
        const uint32_t whole = tail == kFusedChunk ? chunks : chunks - 1;  // chunks of 512 bytes
        uint2 x[C];
        if (whole) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __builtin_bit_cast(uint2, ld64_any(sb + p.in_off[c] + lane * 8u));
        }
#pragma unroll 1
        for (uint32_t ch = 0; ch < whole; ++ch) {
            const uint64_t off = (uint64_t)ch * kFusedChunk + lane * 8u;
            uint32_t acc[R][2];
            rows_of(x, acc);
            if (live) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    st64_any(sb + p.out_off[r] + off, (uint64_t)acc[r][0] | ((uint64_t)acc[r][1] << 32));
            }
            uint2 y[C];
            if (ch + 1 < whole) {
#pragma unroll
                for (int c = 0; c < C; ++c)
                    y[c] = __builtin_bit_cast(uint2, ld64_any(sb + p.in_off[c] + off + kFusedChunk));
            }
            publish(x, acc);
            if (ch + 1 < whole) {
#pragma unroll
                for (int c = 0; c < C; ++c) x[c] = y[c];
            }
        }
        if (whole < chunks) {  // the partial last chunk: nothing read or written at or past S
            const uint64_t off = (uint64_t)whole * kFusedChunk + lane * 8u;
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = __builtin_bit_cast(uint2, ld64_part(sb + p.in_off[c] + off, off, S));
            uint32_t acc[R][2];
            rows_of(x, acc);
            if (live) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    st64_part(sb + p.out_off[r] + off, (uint64_t)acc[r][0] | ((uint64_t)acc[r][1] << 32), off, S);
            }
            publish(x, acc);
        }
    } else {
        // ------------------------------ hasher -------------------------------
        if constexpr (ABLATE & 16) __builtin_amdgcn_s_setprio(1);
        const uint32_t g = (wave - SPW) * 16u + (lane >> 2);  // stream of this quad
        const uint32_t ls = g / T, shard = g - ls * T;        // local stripe, shard
        const uint64_t stripe = (uint64_t)blockIdx.x * SPW + ls;
        const bool live = g < (uint32_t)(SPW * T) && stripe < n;
        const uint8_t* row0 = rows + (live ? ls * kStripeRows + shard * kFusedPitch : 0);
        const uint8_t* row = row0 + 8 * q;
        HHQuad st;
        hhq_init(st, h.key, q);
#pragma unroll 1
        for (uint32_t ch = 0; ch + 1 < chunks; ++ch) {
            lds_barrier();  // A
            lds_barrier();  // B
            if (live) {
#pragma unroll 4
                for (int t = 0; t < (int)(kFusedChunk / 32); ++t) {
                    const u32x2 v = *(const u32x2*)(row + t * 32);
                    if constexpr (ABLATE & 2) {
                        st.v0 ^= __builtin_bit_cast(uint64_t, v);
                    } else {
                        hhq_update(st, __builtin_bit_cast(uint64_t, v));
                    }
                }
            }
        }
        lds_barrier();  // A (last chunk)
        lds_barrier();  // B
        if (live) {  // the last chunk's whole packets, then the remainder packet
            const uint32_t full = tail / 32;
#pragma unroll 1
            for (uint32_t t = 0; t < full; ++t) hhq_update(st, __builtin_bit_cast(uint64_t, *(const u32x2*)(row + t * 32)));
            if (tail % 32) hhq_remainder(st, row0 + full * 32, tail % 32, q);
            hhq_finish(st, h.out + (stripe * T + shard) * 32u, q);
        }
    }
}

// ---------------------------------------------------------------------------
// Fused RS encode + HighwayHash-256 with LDS-DMA data and bit-sliced
// encoders, for a compile-time encode matrix (RS(8,4)).  Same output as
// k_encode_hash_fused; 1.48-1.50 ms against 1.55-1.62 ms for RS(8,4),
// n = 4096, 1 MiB stripes (tools/kbench/fused_r2.hip "v8 bar D3").
//
// One workgroup of 10 waves owns 8 stripes and walks them in 512-byte steps:
//   data-hasher waves (K/2): each brings 8 of the step's K x 4 data-row DMA
//     instructions (global_load_lds, 16 B per lane; an instruction carries one
//     shard of stripes i and i + 4) into a 3-slot LDS ring two steps ahead,
//     then hashes 16 data streams of the current step straight out of the ring;
//   encoder waves (4): stripe group g = stripes {2g, 2g+1, 2g+4, 2g+5}, 8 B
//     per lane of each, read from the ring, bit-transposed into planes, every
//     parity row one compile-time XOR network (v_bitop3) over the planes,
//     transposed back, stored to HBM and to a double-buffered parity-row area;
//   parity-hasher waves (M/2): the parity streams one step behind.
// One barrier per step.  The DMA writes LDS behind the compiler's back, so
// its completion is awaited with counted vmcnt waits and the data rows are
// read with asm ds_read_b64 (the compiler adds no vmcnt(0) for them).  Dead
// stripes (past n) re-read stripe 0 and store nothing.
namespace dma {
template <int K, int M, int NE = EW, int SP = SPW>
struct Shape {
    static constexpr int SPW = SP, HS = SP / 2;       // stripes per workgroup, per DMA half
    static constexpr int NI = HS * K;                 // DMA instructions per step (1 KiB each)
    static constexpr uint32_t DSLOT = NI * IP;        // one step of all data rows
    static constexpr uint32_t PSLOT = SPW * M * PP;   // one step of all parity rows
    static constexpr int DATA = (SPW * K) / 16;       // data-hasher waves
    static constexpr int PAR = (SPW * M + 15) / 16;   // parity-hasher waves
    static constexpr int ENC = NE;                    // encoder waves: 1 per stripe group, or 2 (split, alternate steps)
    static constexpr int WAVES = NE + DATA + PAR;
};

// One encoder wave per stripe group computing all four RS(8,4) parity rows:
// the 64 input planes go through the generated common-subexpression XOR
// network (rs84_xornet.h: 239 three-input XORs instead of 504), and each data
// shard is bit-transposed once per group instead of once per row pair
// (per group and step: 8 + 4 transposes + 239 XORs, against 2 x (8 + 2)
// transposes + 504 XORs for two encoder() waves).
template <int K, int M, int NT, int SP, bool SPLIT>
__device__ __forceinline__ void encoder_net(const GfApplyParams& p, uint64_t n, uint32_t steps, uint64_t s0,
                                            uint32_t g, uint32_t ph, const uint8_t* ring, uint8_t* prow) {
    static_assert(K == 8 && M == 4, "the XOR network is RS(8,4)'s");
    using L = Shape<K, M, SPLIT ? SP / 2 : SP / 4, SP>;
    constexpr int SPW = L::SPW, HS = L::HS;
    constexpr uint32_t LAG = SPLIT ? 2 : 1;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
    const uint32_t mys[4] = {2 * g, 2 * g + 1, 2 * g + HS, 2 * g + HS + 1};
    uint8_t* const base = p.out_base;
    uint64_t pdst[4];
    bool live[4];  // wave-uniform: a dead stripe (past n) computes stripe 0's rows and stores nothing
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        live[j] = s0 + mys[j] < n;
        pdst[j] = (live[j] ? s0 + mys[j] : 0) * p.stripe_stride + lane * 8u;
    }
    uint32_t P[64];
    // step s's data rows, bit-transposed into the 64 planes
    auto load = [&](uint32_t s) {
        const uint8_t* slot = ring + (s % D) * L::DSLOT + 2 * g * IP + lane * 8u;
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const uint8_t* row = slot + HS * c * IP;
            const uint2 a0 = *(const uint2*)row, a1 = *(const uint2*)(row + IP);
            const uint2 a2 = *(const uint2*)(row + CH), a3 = *(const uint2*)(row + IP + CH);
            uint32_t w[8] = {a0.x, a0.y, a1.x, a1.y, a2.x, a2.y, a3.x, a3.y};
            transpose(w, m4, m2, m1);
#pragma unroll
            for (int j = 0; j < 8; ++j) P[8 * c + j] = w[j];
        }
    };
    // step s's parity: network, planes back to bytes, HBM + parity-row area
    auto emit = [&](uint32_t s) {
        uint32_t O[32];
        xn::rs84_encode_planes(P, O);
#pragma unroll
        for (int r = 0; r < M; ++r) {
            uint32_t w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = O[8 * r + i];
            transpose(w, m4, m2, m1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint2 v = make_uint2(w[2 * j], w[2 * j + 1]);
                if (live[j]) {
                    if constexpr (NT & 2) st16_nt_half(base + pdst[j] + p.out_off[r] + (uint64_t)s * CH, v);
                    else *(uint2*)(base + pdst[j] + p.out_off[r] + (uint64_t)s * CH) = v;
                }
                *(uint2*)(prow + (s % NP) * L::PSLOT + (r * SPW + mys[j]) * PP + lane * 8u) = v;
            }
        }
    };
    const uint32_t intervals = steps + LAG;  // interval t: between B(t) and B(t+1)
    lds_barrier();  // B(0): slot 0 landed
#pragma unroll 1
    for (uint32_t t = 0; t < intervals; ++t) {
        if constexpr (SPLIT) {
            // two waves per group on alternate steps; a step straddles one
            // barrier: its rows are read while in the ring (interval s), its
            // parity emitted in interval s+1 (published by B(s+2))
            if (t < steps && t % 2 == ph) load(t);
            else if (t >= 1 && t - 1 < steps && (t - 1) % 2 == ph) emit(t - 1);
        } else if (t < steps) {
            load(t);
            emit(t);  // published by B(t+1)
        }
        if (t + 1 < intervals) lds_barrier();  // B(t+1)
    }
}
}  // namespace dma

template <int K, int M, int NE = dma::EW, int NT = 0, int SP = dma::SPW>
__global__ __launch_bounds__((64 * dma::Shape<K, M, NE, SP>::WAVES)) void k_encode_hash_dma(const GfApplyParams p,
                                                                                          const HashParams h) {
    using namespace dma;
    static_assert(K == 8 && M == 4, "the XOR network is RS(8,4)'s");
    static_assert(NE == SP / 4 || NE == SP / 2, "one encoder wave per stripe group, or two (split)");
    constexpr bool SPLIT = NE == SP / 2;
    constexpr uint32_t LAG = SPLIT ? 2 : 1;  // steps the parity hashers trail the DMA'd data
    using L = Shape<K, M, NE, SP>;
    constexpr int SPW = L::SPW, HS = L::HS;
    __shared__ __attribute__((aligned(16))) uint8_t ring[D * L::DSLOT];
    __shared__ __attribute__((aligned(16))) uint8_t prow[NP * L::PSLOT];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t steps = p.units;  // S / CH
    const uint64_t s0 = (uint64_t)blockIdx.x * SPW;
    const uint32_t ring_base = (uint32_t)(uintptr_t)ring;

    const uint32_t intervals = steps + LAG;  // interval t: between B(t) and B(t+1)
    if (wave < (uint32_t)NE) {
        if (p.wave_prio & kPrioGf) __builtin_amdgcn_s_setprio(2);
        const uint32_t g = SPLIT ? wave / 2 : wave, ph = SPLIT ? wave % 2 : 0;
        encoder_net<K, M, NT, SP, SPLIT>(p, n, steps, s0, g, ph, ring, prow);
        return;
    }
    // ---------------------------------- hashers ----------------------------------
    if (p.wave_prio & kPrioHash) __builtin_amdgcn_s_setprio(2);
    const uint32_t hw = wave - NE, j = lane >> 2;
    const bool is_data = hw < (uint32_t)L::DATA;
    constexpr int NDI = 8;  // DMA instructions a data-hasher wave owns
    uint32_t stripe_l, shard, roff;
    if (is_data) {
        // data hasher hw owns DMA instructions [8 hw, 8 hw + 8): it brings them
        // into the ring D-1 steps ahead and hashes both halves of each: quad j
        // takes instruction 8 hw + (j & 7), half j >> 3 (conflict-free
        // ds_read_b64: the 8 quads of a 32-lane group read rows 32 B apart mod 256)
        const uint32_t idx = NDI * hw + (j & 7u), half = j >> 3;
        shard = idx / HS;
        stripe_l = idx % HS + HS * half;
        roff = idx * IP + half * CH + 8 * q;
    } else {
        uint32_t pi = 16 * (hw - L::DATA) + j;  // parity row index r * SPW + stripe
        if (pi >= (uint32_t)(SPW * M)) pi = 0;  // idle quad
        shard = K + pi / SPW;
        stripe_l = pi % SPW;
        roff = pi * PP + 8 * q;
    }
    const bool live = s0 + stripe_l < n && (is_data || 16 * (hw - L::DATA) + j < (uint32_t)(SPW * M));
    HHQuad st;
    hhq_init(st, h.key, q);
    auto hash16 = [&](uint32_t a) {
        uint64_t w[16];
        read16(a, w);
#pragma unroll
        for (int t = 0; t < 16; ++t) hhq_update(st, w[t]);
    };
    if (is_data) {
        // DMA instruction 8 hw + k: shard c = (8 hw + k) / 4, stripe pair
        // i = k % 4: lanes 0-31 stripe i, lanes 32-63 stripe i + 4
        // Sources as a wave-uniform base (the lower half's stripe, SGPRs) +
        // a 32-bit per-lane offset (the upper half's stripe HS stripes on,
        // or the lower one again when that is past n), so every
        // global_load_lds takes the saddr form and a step costs HS VALU adds
        const uint8_t* base = p.out_base;
        const uint8_t* ub[HS];
        uint32_t vlane[HS];
#pragma unroll
        for (int i = 0; i < HS; ++i) {
            const uint64_t lo = s0 + i, hi = lo + HS;
            ub[i] = base + (lo < n ? lo : 0) * p.stripe_stride;
            vlane[i] = (lane & 31u) * 16u + ((lane >> 5) && hi < n ? (uint32_t)(HS * p.stripe_stride) : 0u);
        }
        auto dma = [&](uint32_t step) {
            uint32_t voff[HS];
#pragma unroll
            for (int i = 0; i < HS; ++i) voff[i] = vlane[i] + step * CH;
#pragma unroll
            for (int k = 0; k < NDI; ++k) {
                const uint32_t c = (NDI * hw + k) / HS;  // wave-uniform
                const uint8_t* src = ub[k % HS] + p.in_off[c] + (uint64_t)voff[k % HS];
                __builtin_amdgcn_global_load_lds(
                    (const void*)src,
                    (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT + (NDI * hw + k) * IP),
                    16, 0, (NT & 1) ? 2 : 0);  // NT bit 0: non-temporal data loads
            }
        };
#pragma unroll
        for (int d = 0; d < D - 1; ++d) dma(d < (int)steps ? d : steps - 1);
        __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * NDI));  // DMA(0) landed
        lds_barrier();  // B(0)
#pragma unroll 1
        for (uint32_t t = 0; t < intervals; ++t) {
            if (t < steps) {
                dma(t + D - 1 < steps ? t + D - 1 : steps - 1);  // into the slot step t-1 used
                hash16(ring_base + (t % D) * L::DSLOT + roff);
                __builtin_amdgcn_s_waitcnt(vmcnt_imm((D - 2) * NDI));  // DMA(t+1) landed
            }
            if (t + 1 < intervals) lds_barrier();  // B(t+1)
        }
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));  // the clamped tail DMA has landed
    } else {
        lds_barrier();  // B(0)
#pragma unroll 1
        for (uint32_t t = 0; t < intervals; ++t) {
            if (t >= LAG) hash16((uint32_t)(uintptr_t)prow + ((t - LAG) % NP) * L::PSLOT + roff);  // published by B(t)
            if (t + 1 < intervals) lds_barrier();  // B(t+1)
        }
    }
    if (live) hhq_finish(st, h.out + ((s0 + stripe_l) * (K + M) + shard) * 32u, q);
}

// ---------------------------------------------------------------------------
// Fused RS(8,4) encode + HighwayHash-256 for batches of FEW LARGE stripes
// (config 4's 4-8 MiB stripes at 4 GiB per launch: 512-1024 stripes), where
// k_encode_hash_dma's 8-stripe workgroups leave CUs idle and the ring
// kernel's table-GF encoder wave is the pace.  One
// workgroup owns SPW (2 or 4) stripes and walks them in 1 KiB steps:
//   data-hasher waves (SPW/2): each brings 16 of the step's SPW x 8 data
//     rows into a 3-slot LDS ring by LDS-DMA (one 1 KiB row = one
//     global_load_lds of 16 B per lane) two steps ahead, then hashes those 16
//     streams straight out of the ring (32 packets per stream per step);
//   encoder waves: stripe pair e, 16 B of each stripe per lane (8 dwords),
//     bit-transposed into planes, all four parity rows from the generated XOR
//     network (rs84_xornet.h), transposed back, stored to HBM and into a
//     double-buffered parity-row area;
//   one parity-hasher wave: the SPW x 4 parity streams.
// One barrier per step.  A lone encoder wave issues its ~830 dependent
// instructions per step at ~5 cycles each, more than a step's memory time
// (4 MiB stripes, SPW = 4: the encoder SIMD sets the pace), so with SPLIT
// each stripe pair has TWO encoder waves taking alternate steps, and each
// step's work straddles one barrier: in the interval a step's data is in the
// ring the wave reads and bit-transposes it (the planes stay in registers),
// in the next it runs the network, transposes back and stores; the parity
// hasher is then two steps behind.  Per stripe-KiB this issues ~408 encoder
// and ~456 hash instructions against ~768 + 456 for the ring kernel's table GF.
namespace wide {
constexpr uint32_t CH = 1024;       // bytes per shard per step
constexpr uint32_t RP = CH + 32;    // LDS row pitch: the 8 quads of a half-wave hit distinct banks
constexpr int D = 3, NP = 2;
template <int SPW, bool SPLIT>
struct Shape {
    static constexpr int ENC = SPLIT ? SPW : SPW / 2, DH = SPW / 2, PH = 1;
    static constexpr int WAVES = ENC + DH + PH;
    static constexpr uint32_t DSLOT = SPW * 8 * RP;  // one step of data rows
    static constexpr uint32_t PSLOT = SPW * 4 * RP;  // one step of parity rows
    static constexpr uint32_t LDS = D * DSLOT + NP * PSLOT;
    static constexpr int LAG = SPLIT ? 2 : 1;        // steps the parity hasher trails the DMA
};
// 32 packets of one stream (8 B per lane, 32 B apart) from LDS
__device__ __forceinline__ void read32(uint32_t a, uint64_t (&w)[32]) {
    uint64_t (&lo)[16] = *reinterpret_cast<uint64_t(*)[16]>(&w[0]);
    uint64_t (&hi)[16] = *reinterpret_cast<uint64_t(*)[16]>(&w[16]);
    dma::read16(a, lo);
    dma::read16(a + 512, hi);
}
// Planes of stripe pair e (16 B of each per lane) from a ring slot.
__device__ __forceinline__ void load_planes(const uint8_t* slot, uint32_t e, uint32_t (&P)[64], uint32_t m4,
                                            uint32_t m2, uint32_t m1) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const uint4 a = *(const uint4*)(slot + ((2 * e) * 8 + c) * RP);
        const uint4 b = *(const uint4*)(slot + ((2 * e + 1) * 8 + c) * RP);
        uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        dma::transpose(w, m4, m2, m1);
#pragma unroll
        for (int j = 0; j < 8; ++j) P[8 * c + j] = w[j];
    }
}
// Network + back-transposes + stores of one step of stripe pair e.
template <int SPW, bool SPLIT>
__device__ __forceinline__ void emit_parity(const GfApplyParams& p, const uint32_t (&P)[64], uint32_t e, uint32_t s,
                                            bool liveA, bool liveB, uint64_t dA, uint64_t dB, uint8_t* prow_slot,
                                            uint32_t m4, uint32_t m2, uint32_t m1) {
    uint32_t O[32];
    xn::rs84_encode_planes(P, O);
    uint8_t* pr = prow_slot + (threadIdx.x & 63u) * 16u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = O[8 * r + i];
        dma::transpose(w, m4, m2, m1);
        const uint4 va = make_uint4(w[0], w[1], w[2], w[3]), vb = make_uint4(w[4], w[5], w[6], w[7]);
        const uint64_t off = p.out_off[r] + (uint64_t)s * CH;
        if (liveA) st16_nt(p.out_base + dA + off, va);
        if (liveB) st16_nt(p.out_base + dB + off, vb);
        *(uint4*)(pr + ((2 * e) * 4 + r) * RP) = va;
        *(uint4*)(pr + ((2 * e + 1) * 4 + r) * RP) = vb;
    }
}
}  // namespace wide

template <int SPW, bool SPLIT>
__global__ __launch_bounds__((64 * wide::Shape<SPW, SPLIT>::WAVES)) void k_encode_hash_wide(const GfApplyParams p,
                                                                                          const HashParams h) {
    using namespace wide;
    using L = Shape<SPW, SPLIT>;
    static_assert(SPW == 2 || SPW == 4, "stripe pairs per encoder wave");
    __shared__ __attribute__((aligned(16))) uint8_t lds[L::LDS];
    uint8_t* const ring = lds;
    uint8_t* const prow = lds + D * L::DSLOT;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t n = h.n;
    const uint32_t steps = p.units;  // S / CH
    const uint64_t s0 = (uint64_t)blockIdx.x * SPW;
    uint8_t* const base = p.out_base;
    // Intervals: interval t runs between barriers B(t) and B(t+1); there are
    // steps + LAG of them (the last ends without a barrier), so every wave
    // passes B(0) .. B(steps + LAG - 1).
    const uint32_t intervals = steps + L::LAG;

    if (wave < (uint32_t)L::ENC) {
        // ------------------------------ encoder ------------------------------
        const uint32_t e = SPLIT ? wave / 2 : wave;  // stripes 2e, 2e+1 of the workgroup
        const uint32_t ph = SPLIT ? wave % 2 : 0;    // SPLIT: this wave's steps are s % 2 == ph
        const bool liveA = s0 + 2 * e < n, liveB = s0 + 2 * e + 1 < n;
        const uint64_t dA = (liveA ? s0 + 2 * e : 0) * p.stripe_stride + lane * 16u;
        const uint64_t dB = (liveB ? s0 + 2 * e + 1 : 0) * p.stripe_stride + lane * 16u;
        const uint32_t m4 = vgpr_const(0x0f0f0f0fu), m2 = vgpr_const(0x33333333u), m1 = vgpr_const(0x55555555u);
        uint32_t P[64];
        lds_barrier();  // B(0): slot 0 landed
#pragma unroll 1
        for (uint32_t t = 0; t < intervals; ++t) {
            if constexpr (SPLIT) {
                if (t < steps && t % 2 == ph) {  // first half of step t: its data is in the ring now
                    load_planes(ring + (t % D) * L::DSLOT + lane * 16u, e, P, m4, m2, m1);
                } else if (t >= 1 && t - 1 < steps && (t - 1) % 2 == ph) {  // second half of step t-1
                    emit_parity<SPW, SPLIT>(p, P, e, t - 1, liveA, liveB, dA, dB, prow + ((t - 1) % NP) * L::PSLOT,
                                            m4, m2, m1);
                }
            } else if (t < steps) {
                load_planes(ring + (t % D) * L::DSLOT + lane * 16u, e, P, m4, m2, m1);
                emit_parity<SPW, SPLIT>(p, P, e, t, liveA, liveB, dA, dB, prow + (t % NP) * L::PSLOT, m4, m2, m1);
            }
            if (t + 1 < intervals) lds_barrier();  // B(t+1)
        }
        return;
    }
    HHQuad st;
    hhq_init(st, h.key, q);
    const uint32_t j = lane >> 2;  // stream (quad) of this wave
    if (wave < (uint32_t)(L::ENC + L::DH)) {
        // ------------- data hasher + DMA: stripes 2w, 2w+1, all 8 data shards -------------
        const uint32_t w = wave - L::ENC;
        const uint32_t stripe_l = 2 * w + j / 8, shard = j % 8;
        const bool live = s0 + stripe_l < n;
        // row sources as a wave-uniform base (SGPRs) + a 32-bit per-lane
        // offset, so each global_load_lds takes the saddr form and a step
        // costs one VALU add for all 16 rows (the hash chain's wave issues it)
        const uint8_t* ub[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint64_t sg = s0 + 2 * w + i;
            ub[i] = base + (sg < n ? sg : 0) * p.stripe_stride;
        }
        const uint32_t row_of = (stripe_l * 8 + shard) * RP + 8 * q;
        auto dma = [&](uint32_t step) {
            const uint32_t voff = lane * 16u + step * CH;
#pragma unroll
            for (int k = 0; k < 16; ++k) {  // row k: stripe 2w + k/8, shard k%8 (wave-uniform)
                const uint8_t* g = ub[k / 8] + p.in_off[k % 8] + (uint64_t)voff;
                __builtin_amdgcn_global_load_lds(
                    (const void*)g,
                    (__attribute__((address_space(3))) void*)(ring + (step % D) * L::DSLOT +
                                                              ((2 * w + k / 8) * 8 + k % 8) * RP),
                    16, 0, 2);  // non-temporal: read once
            }
        };
#pragma unroll
        for (int d = 0; d < D - 1; ++d) dma(d < (int)steps ? d : steps - 1);
        __builtin_amdgcn_s_waitcnt(dma::vmcnt_imm((D - 2) * 16));  // DMA(0) landed
        lds_barrier();  // B(0)
        const uint32_t ring_base = (uint32_t)(uintptr_t)ring;
#pragma unroll 1
        for (uint32_t t = 0; t < intervals; ++t) {
            if (t < steps) {
                dma(t + D - 1 < steps ? t + D - 1 : steps - 1);  // into the slot step t-1 used
                uint64_t wv[32];
                read32(ring_base + (t % D) * L::DSLOT + row_of, wv);
#pragma unroll
                for (int k = 0; k < 32; ++k) hhq_update(st, wv[k]);
                __builtin_amdgcn_s_waitcnt(dma::vmcnt_imm((D - 2) * 16));  // DMA(t+1) landed
            }
            if (t + 1 < intervals) lds_barrier();  // B(t+1)
        }
        __builtin_amdgcn_s_waitcnt(dma::vmcnt_imm(0));  // the clamped tail DMA has landed
        if (live) hhq_finish(st, h.out + ((s0 + stripe_l) * 12 + shard) * 32u, q);
        return;
    }
    // -------------- parity hasher: SPW x 4 streams, LAG steps behind the DMA --------------
    const bool on = j < (uint32_t)(SPW * 4);
    const uint32_t pj = on ? j : 0, stripe_l = pj / 4, r = pj % 4;
    const bool live = on && s0 + stripe_l < n;
    const uint32_t row_of = (stripe_l * 4 + r) * RP + 8 * q;
    const uint32_t prow_base = (uint32_t)(uintptr_t)prow;
    lds_barrier();  // B(0)
#pragma unroll 1
    for (uint32_t t = 0; t < intervals; ++t) {
        if (t >= (uint32_t)L::LAG) {  // parity rows of step t-LAG, published by B(t)
            uint64_t wv[32];
            read32(prow_base + ((t - L::LAG) % NP) * L::PSLOT + row_of, wv);
#pragma unroll
            for (int k = 0; k < 32; ++k) hhq_update(st, wv[k]);
        }
        if (t + 1 < intervals) lds_barrier();  // B(t+1)
    }
    if (live) hhq_finish(st, h.out + ((s0 + stripe_l) * 12 + 8 + r) * 32u, q);
}

// ---------------------------------------------------------------------------
// Fused RS encode + HighwayHash-256, ring variant for batches of few large
// stripes (config 4's 4-16 MiB stripes at 4 GiB per launch: 256-1024 stripes).
// There the packed kernel above has too few bytes in flight (one 512-B chunk
// per stripe) and at most n/4 workgroups: it waits on HBM latency, not on the
// SIMDs.  Here one workgroup owns ONE stripe:
//   waves 0..E-1 (encoders): each owns a 1 KiB column of every E KiB chunk
//     (16 B per lane per shard), keeps the loads of the next chunk in flight
//     (D = 2 register sets, rotated by unrolling, never copied: a copy of a
//     register with a load pending would wait for it; D = 3 measured no
//     faster), computes and stores parity, and writes all k+m rows of the
//     chunk into LDS slot ch & 1;
//   waves E.. (hashers): one 4-lane quad per shard stream; after the barrier
//     that publishes slot ch & 1 they hash it while the encoders fill the other.
// One barrier per chunk (double-buffered rows): the encoders write slot ch & 1
// only after the barrier that ended the hashers' pass over chunk ch - 2.  Per
// stripe the hash is sequential (HighwayHash), so the floor is the issue time
// of the quad's update chain (~19 instructions per 32-byte packet, one wave
// alone on its SIMD: ~95 cycles); everything else hides under it.  E = 2 for
// up to ~3 stripes per CU, E = 1 above; E = 4 puts the hasher on a SIMD with
// an encoder and runs 20 % slower.
constexpr uint32_t kRingCol = 1024;  // bytes per encoder wave per shard per chunk

constexpr int kRingMaxC = 8;  // C > 8 takes the packed kernel

template <int C, int R, int D = 2>
__global__ __launch_bounds__(64 * (2 + (C + R + 15) / 16))
void k_encode_hash_ring(const GfApplyParams p, const HashParams h, const uint32_t E) {
    extern __shared__ uint8_t lds_all[];
    constexpr int T = C + R;
    constexpr uint32_t kTabBytes = C * R * 32;
    const uint32_t CW = kRingCol * E, pitch = CW + 32, slot = T * pitch;
    uint8_t* rows = lds_all + kTabBytes;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u, q = lane & 3u;
    const uint64_t stripe = blockIdx.x;
    const uint32_t nch = p.units;  // S / CW

    for (uint32_t i = threadIdx.x; i < (uint32_t)(C * R); i += blockDim.x) {
        const int c = i / R, r = i % R;
        uint8_t* d = lds_all + i * 32;
        *(uint4*)d = make_uint4(p.tab[r][c][0], p.tab[r][c][1], p.tab[r][c][2], p.tab[r][c][3]);
        *(uint32_t*)(d + 16) = p.tab[r][c][4];
    }
    __syncthreads();

    if (wave < E) {
        // ------------------------------ encoder ------------------------------
        uint8_t* sb = p.out_base + stripe * p.stripe_stride;
        const uint32_t col = wave * kRingCol + lane * 16u;
        const uint32_t m7 = vgpr_const(0x07070707u), m3 = vgpr_const(0x03030303u);
        uint4 b[D][C];
        auto load = [&](uint4 (&x)[C], uint32_t ch) {
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = ld16(sb + p.in_off[c] + (uint64_t)ch * CW + col);
        };
        auto step = [&](uint4 (&x)[C], uint4 (&nxt)[C], uint32_t ch) {
            if (ch + (D - 1) < nch) load(nxt, ch + (D - 1));
            uint32_t tz;  // opaque zero: table reads stay at their use
            asm volatile("s_mov_b32 %0, 0" : "=s"(tz));
            const uint8_t* tabs = lds_all + tz;
            uint32_t acc[R][4], pend[R][4];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
            // tables of input c+1 are read (LDS broadcast) while input c is
            // multiplied.  Their address carries an opaque zero computed from
            // the accumulator after input c-1, so the compiler cannot hoist
            // all C*R tables (160 VGPRs at RS(8,4)) to the top of the chunk.
            uint4 ta[R], na[R];
            uint32_t tb[R], nb[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                ta[r] = *(const uint4*)(tabs + r * 32);
                tb[r] = *(const uint32_t*)(tabs + r * 32 + 16);
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (c + 1 < C) {
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        asm volatile("" : "+v"(acc[r][0]), "+v"(acc[r][1]), "+v"(acc[r][2]), "+v"(acc[r][3]));
                    // likewise input c+1's field selectors stay after this point
                    asm volatile("" : "+v"(x[c + 1].x), "+v"(x[c + 1].y), "+v"(x[c + 1].z), "+v"(x[c + 1].w));
                    uint32_t z;
                    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                    const uint8_t* tn = tabs + z + (c + 1) * R * 32;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        na[r] = *(const uint4*)(tn + r * 32);
                        nb[r] = *(const uint32_t*)(tn + r * 32 + 16);
                    }
                }
                const uint32_t w[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t s0 = w[k] & m7, s1 = (w[k] >> 3) & m7, s2 = (w[k] >> 6) & m3;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        gf_fold(c & 1, acc[r][k], pend[r][k], __builtin_amdgcn_perm(ta[r].y, ta[r].x, s0),
                                __builtin_amdgcn_perm(ta[r].w, ta[r].z, s1), __builtin_amdgcn_perm(tb[r], tb[r], s2));
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    ta[r] = na[r];
                    tb[r] = nb[r];
                }
            }
            if constexpr (C % 2 == 1) {
#pragma unroll
                for (int r = 0; r < R; ++r)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[r][k] ^= pend[r][k];
            }
            const uint64_t off = (uint64_t)ch * CW + col;
#pragma unroll
            for (int r = 0; r < R; ++r) st16(sb + p.out_off[r] + off, make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]));
            uint8_t* buf = rows + (ch & 1u) * slot + col;
#pragma unroll
            for (int c = 0; c < C; ++c) *(uint4*)(buf + c * pitch) = x[c];
#pragma unroll
            for (int r = 0; r < R; ++r)
                *(uint4*)(buf + (C + r) * pitch) = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
            lds_barrier();  // rows of chunk ch published in slot ch & 1
        };
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if ((uint32_t)d < nch) load(b[d], d);
#pragma unroll 1
        for (uint32_t ch = 0; ch < nch; ch += D) {
            step(b[0], b[D - 1], ch);
            if (ch + 1 >= nch) break;
            step(b[1], b[0], ch + 1);
            if constexpr (D == 3) {
                if (ch + 2 >= nch) break;
                step(b[2], b[1], ch + 2);
            }
        }
    } else {
        // ------------------------------ hasher -------------------------------
        const uint32_t g = (wave - E) * 16u + (lane >> 2);  // shard stream of this quad
        const bool live = g < (uint32_t)T;
        const uint32_t roff = (live ? g * pitch : 0) + 8 * q;
        const uint32_t packets = CW / 32;
        HHQuad st;
        hhq_init(st, h.key, q);
#pragma unroll 1
        for (uint32_t ch = 0; ch < nch; ++ch) {
            lds_barrier();
            if (live) {
                const uint8_t* row = rows + (ch & 1u) * slot + roff;
#pragma unroll 1
                for (uint32_t t = 0; t < packets; t += 8) {
                    u32x2 v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = *(const u32x2*)(row + (t + i) * 32);
#pragma unroll
                    for (int i = 0; i < 8; ++i) hhq_update(st, __builtin_bit_cast(uint64_t, v[i]));
                }
            }
        }
        if (live) hhq_finish(st, h.out + (stripe * T + g) * 32u, q);
    }
}

// ---------------------------------------------------------------------------
// Launchers.

// Kernel-choice knobs (Tuning, rs_kernels.h).  The library runs the
// defaults; a knob changes only through rsg_set_tuning (tests and A/B runs,
// set_tuning below) or — in measurement builds only (RSG_MEASUREMENT_BUILD) —
// from its RSG_* environment variable, read once.  A production process's
// environment cannot change which kernels run.  Every setting is published as
// a new immutable snapshot (launches in flight keep reading the one they
// loaded); snapshots live for the process.
namespace {

// name -> the knob's field; false for an unknown name or a value out of range
bool set_knob(Tuning& v, const std::string& name, const char* value) {
    if (!value || !*value) return false;
    const std::string s(value);
    char* endp = nullptr;
    const long x = strtol(value, &endp, 10);
    const bool is_num = endp && *endp == '\0';
    auto flag = [&](bool& f) {
        if (s != "0" && s != "1") return false;
        f = s == "1";
        return true;
    };
    auto num = [&](int& f, int lo, int hi) {
        if (!is_num || x < lo || x > hi) return false;
        f = (int)x;
        return true;
    };
    auto one_of = [&](int& f, int a, int b, int c = -1000, int d = -1000, int e = -1000) {
        if (!is_num || (x != a && x != b && x != c && x != d && x != e)) return false;
        f = (int)x;
        return true;
    };
    if (name == "RSG_FUSED") return flag(v.fused);
    if (name == "RSG_LOST_DISK_FAST") return flag(v.lost_disk_fast);
    if (name == "RSG_ZERO_COPY") return flag(v.zero_copy);
    if (name == "RSG_VEC_BLOCK") return one_of(v.vec_block, 0, 64, 256);
    if (name == "RSG_VEC_OCC") return num(v.vec_occ, -1, 8);
    if (name == "RSG_ROLLED") return flag(v.rolled);
    if (name == "RSG_HASH_COPY") return flag(v.hash_direct_copy);
    if (name == "RSG_HASH_DEPTH") return num(v.hash_depth, 1, 3);
    if (name == "RSG_FUSED_KIND") {
        static const char* const kinds[] = {"auto",   "packed", "ring", "dma",  "wide2",
                                            "wide4",  "split2", "split4", "net", "table"};
        for (int i = 0; i < 10; ++i)
            if (s == kinds[i]) {
                v.fused_kind = i;
                return true;
            }
        return false;
    }
    if (name == "RSG_FUSED_SPW1") return flag(v.fused_spw1);
    if (name == "RSG_ENC_PRIO") return num(v.enc_prio, 0, 3);
    if (name == "RSG_DMA_EW") return one_of(v.dma_ew, 2, 4);
    if (name == "RSG_DMA_NT") return num(v.dma_nt, 0, 3);
    if (name == "RSG_DMA_SPW") return one_of(v.dma_spw, 4, 8);
    if (name == "RSG_DMA_PRIO") return num(v.get_prio, 0, 3);
    if (name == "RSG_DECODE_NET") return flag(v.decode_net);
    if (name == "RSG_NET12_RD") return RSG_MEASUREMENT_BUILD ? one_of(v.net12_rd, 2, 4) : one_of(v.net12_rd, 2, 2);
    if (name == "RSG_HASH_UNAL") return flag(v.hash_unal);
    if (name == "RSG_GET_CACHED") return flag(v.get_cached);
    return false;
}

// the knob's current setting in set_knob's syntax; false for an unknown name
bool knob_value(const Tuning& v, const std::string& name, std::string& out) {
    auto b = [&](bool f) { out = f ? "1" : "0"; return true; };
    auto i = [&](int x) { out = std::to_string(x); return true; };
    if (name == "RSG_FUSED") return b(v.fused);
    if (name == "RSG_LOST_DISK_FAST") return b(v.lost_disk_fast);
    if (name == "RSG_ZERO_COPY") return b(v.zero_copy);
    if (name == "RSG_VEC_BLOCK") return i(v.vec_block);
    if (name == "RSG_VEC_OCC") return i(v.vec_occ);
    if (name == "RSG_ROLLED") return b(v.rolled);
    if (name == "RSG_HASH_COPY") return b(v.hash_direct_copy);
    if (name == "RSG_HASH_DEPTH") return i(v.hash_depth);
    if (name == "RSG_FUSED_KIND") {
        static const char* const kinds[] = {"auto",   "packed", "ring", "dma",  "wide2",
                                            "wide4",  "split2", "split4", "net", "table"};
        out = kinds[v.fused_kind >= 0 && v.fused_kind < 10 ? v.fused_kind : 0];
        return true;
    }
    if (name == "RSG_FUSED_SPW1") return b(v.fused_spw1);
    if (name == "RSG_ENC_PRIO") return i(v.enc_prio);
    if (name == "RSG_DMA_EW") return i(v.dma_ew);
    if (name == "RSG_DMA_NT") return i(v.dma_nt);
    if (name == "RSG_DMA_SPW") return i(v.dma_spw);
    if (name == "RSG_DMA_PRIO") return i(v.get_prio);
    if (name == "RSG_DECODE_NET") return b(v.decode_net);
    if (name == "RSG_NET12_RD") return i(v.net12_rd);
    if (name == "RSG_HASH_UNAL") return b(v.hash_unal);
    if (name == "RSG_GET_CACHED") return b(v.get_cached);
    return false;
}

#if RSG_MEASUREMENT_BUILD
const char* const kKnobs[] = {"RSG_FUSED", "RSG_LOST_DISK_FAST", "RSG_ZERO_COPY", "RSG_VEC_BLOCK", "RSG_VEC_OCC",
                              "RSG_ROLLED", "RSG_HASH_COPY", "RSG_HASH_DEPTH", "RSG_FUSED_KIND", "RSG_FUSED_SPW1",
                              "RSG_ENC_PRIO", "RSG_DMA_EW", "RSG_DMA_NT", "RSG_DMA_SPW", "RSG_DMA_PRIO",
                              "RSG_DECODE_NET", "RSG_NET12_RD", "RSG_HASH_UNAL", "RSG_GET_CACHED"};
#endif

std::mutex g_tuning_mu;
std::atomic<const Tuning*> g_tuning{nullptr};
std::deque<Tuning>& tuning_store() {
    static std::deque<Tuning> d;  // every published snapshot (a deque never moves its elements)
    return d;
}

bool same_tuning(const Tuning& a, const Tuning& b) {
    // every Tuning field (rs_kernels.h): a new knob must be added here too
    return a.fused == b.fused && a.lost_disk_fast == b.lost_disk_fast && a.zero_copy == b.zero_copy &&
           a.vec_block == b.vec_block && a.vec_occ == b.vec_occ && a.rolled == b.rolled &&
           a.hash_direct_copy == b.hash_direct_copy && a.hash_depth == b.hash_depth &&
           a.fused_kind == b.fused_kind && a.fused_spw1 == b.fused_spw1 && a.enc_prio == b.enc_prio &&
           a.dma_ew == b.dma_ew && a.dma_nt == b.dma_nt && a.dma_spw == b.dma_spw && a.get_prio == b.get_prio &&
           a.decode_net == b.decode_net && a.net12_rd == b.net12_rd && a.hash_unal == b.hash_unal &&
           a.get_cached == b.get_cached;
}

// Snapshots are immutable and never freed (a launch on another thread may
// still be reading the one it took), so an equal snapshot already published is
// reused: the store holds at most one per distinct setting, however many
// rsg_set_tuning calls a long A/B or test process makes.
const Tuning* publish(const Tuning& v) {  // under g_tuning_mu
    const Tuning* t = nullptr;
    for (const Tuning& s : tuning_store())
        if (same_tuning(s, v)) t = &s;
    if (!t) {
        tuning_store().push_back(v);
        t = &tuning_store().back();
    }
    g_tuning.store(t, std::memory_order_release);
    return t;
}

Tuning initial_tuning() {
    Tuning v;  // the defaults (rs_kernels.h)
#if RSG_MEASUREMENT_BUILD
    for (const char* name : kKnobs)
        if (const char* e = getenv(name)) (void)set_knob(v, name, e);  // an invalid value keeps the default
#endif
    return v;
}

}  // namespace

const Tuning& tuning() {
    if (const Tuning* t = g_tuning.load(std::memory_order_acquire)) return *t;
    std::lock_guard<std::mutex> lk(g_tuning_mu);
    if (const Tuning* t = g_tuning.load(std::memory_order_acquire)) return *t;
    return *publish(initial_tuning());
}

// rsg_set_tuning: name NULL = every knob back to its default; value NULL =
// this knob back to its default.  RSG_ERR_INVALID_ARG (1) for an unknown
// name or a value the knob does not take; nothing changes then.
int set_tuning(const char* name, const char* value) {
    (void)tuning();
    std::lock_guard<std::mutex> lk(g_tuning_mu);
    if (!name) {
        publish(Tuning{});
        return 0;
    }
    const std::string nm(name);
    Tuning v = *g_tuning.load(std::memory_order_acquire);
    if (!value) {  // this knob's default
        std::string d;
        if (!knob_value(Tuning{}, nm, d) || !set_knob(v, nm, d.c_str())) return 1;
        publish(v);
        return 0;
    }
    if (!set_knob(v, nm, value)) return 1;
    publish(v);
    return 0;
}

// rsg_get_tuning: the knob's current setting (NUL-terminated in out[cap]).
int get_tuning(const char* name, char* out, size_t cap) {
    std::string v;
    if (!name || !out || !knob_value(tuning(), name, v) || v.size() + 1 > cap) return 1;
    memcpy(out, v.c_str(), v.size() + 1);
    return 0;
}

using GfKernel = void (*)(const GfApplyParams);

template <int C, int B, bool PRE>
static GfKernel pick_vec_r(int R) {
    switch (R) {
        case 1: return k_gf_apply_vec<C, 1, B, PRE>;
        case 2: return k_gf_apply_vec<C, 2, B, PRE>;
        case 3: return k_gf_apply_vec<C, 3, B, PRE>;
        case 4: return k_gf_apply_vec<C, 4, B, PRE>;
    }
    return nullptr;
}

// Unrolled kernel for C <= 8 inputs and R <= 4 outputs, the rolled one above
// (k_gf_apply_loop); RSG_ROLLED=1 forces the rolled kernel for A/B runs.
template <int B, bool PRE>
static GfKernel pick_vec_b(const Tuning& t, int C, int R) {
    if (C <= 8 && R <= 4 && !t.rolled) {
        switch (C) {
            case 1: return pick_vec_r<1, B, PRE>(R);
            case 2: return pick_vec_r<2, B, PRE>(R);
            case 3: return pick_vec_r<3, B, PRE>(R);
            case 4: return pick_vec_r<4, B, PRE>(R);
            case 5: return pick_vec_r<5, B, PRE>(R);
            case 6: return pick_vec_r<6, B, PRE>(R);
            case 7: return pick_vec_r<7, B, PRE>(R);
            case 8: return pick_vec_r<8, B, PRE>(R);
        }
        return nullptr;
    }
    if (C < 1 || C > kMaxC) return nullptr;
    if (C > 8 && C <= 12 && R <= 4 && !t.rolled) {
        switch (R) {
            case 1: return k_gf_apply_loop<1, B, PRE, 12>;
            case 2: return k_gf_apply_loop<2, B, PRE, 12>;
            case 3: return k_gf_apply_loop<3, B, PRE, 12>;
            case 4: return k_gf_apply_loop<4, B, PRE, 12>;
        }
    }
    switch (R) {
        case 1: return k_gf_apply_loop<1, B, PRE>;
        case 2: return k_gf_apply_loop<2, B, PRE>;
        case 3: return k_gf_apply_loop<3, B, PRE>;
        case 4: return k_gf_apply_loop<4, B, PRE>;
        case 5: return k_gf_apply_loop<5, B, PRE>;
        case 6: return k_gf_apply_loop<6, B, PRE>;
        case 7: return k_gf_apply_loop<7, B, PRE>;
        case 8: return k_gf_apply_loop<8, B, PRE>;
    }
    return nullptr;
}

// Workgroup size of a vector GF launch.  One-wave workgroups (the
// dispatcher refills a SIMD wave by wave; RS(8,4) encode 1.090 -> 1.066 ms,
// RS(16,4) 0.959 -> 0.934 ms, profiles/r02/ab_block/) where every shard row
// starts on a 128-byte line; four-wave workgroups where any does not — each
// workgroup's 16-byte loads of a shard span one contiguous run, and a run
// that starts mid-line touches one line more than its length needs: 9 lines
// per KiB for one wave, 33 per 4 KiB for four (RS(12,4) at 1 MiB blocks, S =
// 87382: encode 1.274 -> 1.112 ms, 0.562 -> 0.644 of HBM,
// profiles/r04/c/enc12_ab.txt).  Tuning::vec_block forces one for A/B runs.
// (Eight- and sixteen-wave workgroups for the rolled kernel measured slower
// again in round 6: RS(12,4) 1.066 -> 1.214 / 1.501 ms, profiles/r06/enc12/.)
static int vec_block_for(const Tuning& t, const GfApplyParams& p) {
    if (t.vec_block) return t.vec_block;
    bool lines = (uintptr_t)p.base % 128 == 0 && (uintptr_t)p.out_base % 128 == 0 && p.stripe_stride % 128 == 0 &&
                 p.out_stripe_stride % 128 == 0;
    for (uint32_t c = 0; c < p.C && lines; ++c) lines = p.in_off[c] % 128 == 0;
    for (uint32_t r = 0; r < p.R && lines; ++r) lines = p.out_off[r] % 128 == 0;
    return lines ? 64 : 256;
}

// Resident waves per SIMD for a vector GF launch, imposed through padding LDS
// (0 = as many as the registers allow; enforced with an otherwise unused
// dynamic LDS allocation per one-wave workgroup: 160 KiB / (4 SIMDs x occ)
// each).  Default: 2 for the read-heavy rebuilds of one or two shards from 8
// inputs, where fewer waves in flight stream better (RS(8,4) n = 4096: 1 lost
// 0.846 -> 0.814 ms, 2 lost 0.905 -> 0.888 ms; profiles/r02/ab_occ2/), else
// no cap.  RSG_VEC_OCC forces one value for A/B runs (tools/enc_ab.py).
static int vec_occupancy(const Tuning& t, int C, int R, bool pre) {
    if (t.vec_occ >= 0) return t.vec_occ;
    return (!pre && C == 8 && R <= 2) ? 2 : 0;
}

static GfKernel pick_vec(const Tuning& t, int C, int R, bool pre, int B) {
    if (B == 256) return pre ? pick_vec_b<256, true>(t, C, R) : pick_vec_b<256, false>(t, C, R);
    return pre ? pick_vec_b<64, true>(t, C, R) : pick_vec_b<64, false>(t, C, R);
}

static GfKernel pick_byte(int R) {
    switch (R) {
        case 1: return k_gf_apply_byte<1>;
        case 2: return k_gf_apply_byte<2>;
        case 3: return k_gf_apply_byte<3>;
        case 4: return k_gf_apply_byte<4>;
        case 5: return k_gf_apply_byte<5>;
        case 6: return k_gf_apply_byte<6>;
        case 7: return k_gf_apply_byte<7>;
        case 8: return k_gf_apply_byte<8>;
    }
    return nullptr;
}

hipError_t launch_gf_apply_vec(GfApplyParams p, uint64_t n_stripes, hipStream_t stream) {
    const Tuning& t = tuning();  // one snapshot for the whole launch (rsg_set_tuning may publish another)
    const bool pre = p.mode != GF_MODE_STORE || p.copy_mask != 0;
    const uint32_t B = (uint32_t)vec_block_for(t, p);
    GfKernel k = pick_vec(t, (int)p.C, (int)p.R, pre, (int)B);
    if (!k || p.units == 0 || n_stripes == 0) return hipErrorInvalidValue;
    p.chunks_per_stripe = (p.units + B - 1) / B;
    const uint64_t blocks = (uint64_t)p.chunks_per_stripe * n_stripes;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const int occ = vec_occupancy(t, (int)p.C, (int)p.R, pre);
    const size_t lds = occ ? (size_t)(160 * 1024) / (size_t)(4 * occ * (B / 64)) / 16 * 16 : 0;
    hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(B), lds, stream, p);
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

// Bytes [0, n) of device memory src to dst, the device view of page-locked
// host memory: the record engines' verdicts (a few KiB of flags) copied back
// by a kernel on the call's stream.  A copy-engine transfer there made the
// next call's kernels wait for the handoff to the copy engine and back.
__global__ __launch_bounds__(256) void k_copy_to_host(uint8_t* dst, const uint8_t* src, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x, w = n / 16;
    if (i < w) ((uint4*)dst)[i] = ((const uint4*)src)[i];
    else if (i == w)
        for (uint64_t b = w * 16; b < n; ++b) dst[b] = src[b];
}

hipError_t launch_copy_to_host(uint8_t* dst, const uint8_t* src, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (((uintptr_t)dst | (uintptr_t)src) % 16 || n / 16 / 256 + 1 > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_copy_to_host, dim3((uint32_t)(n / 16 / 256 + 1)), dim3(256), 0, stream, dst, src, n);
    return hipGetLastError();
}

hipError_t launch_hh256(const HashParams& p, hipStream_t stream) {
    if (p.n == 0) return hipSuccess;
    const uint64_t blocks = (p.n * 4u + 255u) / 256u;  // one quad per message
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    bool copy = false;  // copy mode when any file of the launch has a copy target
    for (uint32_t b = 0; b < p.nbases; ++b) copy = copy || p.copy_base[b];
    if (!copy && launch_verify_records_dma(p, stream)) return hipGetLastError();
    // copy mode: staged 16-byte stores (COPY = 2) by default (Tuning:
    // direct 8-byte stores for A/B runs); 8-packet batches in flight per
    // lane: 2 by default
    const Tuning& t = tuning();  // one snapshot for the whole launch
    const bool direct_copy = t.hash_direct_copy;
    const int depth = t.hash_depth;
    using HashKernel = void (*)(const HashParams);
    HashKernel k;
    // messages at odd offsets (record pitch 174795 of RS(6,4) at 1 MiB
    // blocks): aligned loads and a funnel shift, 1.005 -> 0.899 ms for the
    // all-present GET; at even offsets (RS(10,4), RS(12,4): 2 mod 8) the
    // hardware's unaligned loads are 4-5 % faster than the funnel
    // (profiles/r04/o/).  Tuning::hash_unal, RSG_HASH_UNAL=0: always the loads.
    bool even = true;
    if (p.nbases) {
        even = p.stripe_stride % 2 == 0;
        for (uint32_t b = 0; b < p.nbases; ++b) even = even && (uintptr_t)p.base[b] % 2 == 0;
    } else {
        even = (uintptr_t)p.data % 2 == 0 && p.stripe_stride % 2 == 0 && p.shard_pitch % 2 == 0;
    }
    if (!copy && depth == 2 && !even && t.hash_unal) k = k_hh256_quad<0, 2, true>;
    else if (!copy) k = depth == 1 ? k_hh256_quad<0, 1> : depth == 2 ? k_hh256_quad<0, 2> : k_hh256_quad<0, 3>;
    else if (direct_copy) k = depth == 1 ? k_hh256_quad<1, 1> : depth == 2 ? k_hh256_quad<1, 2> : k_hh256_quad<1, 3>;
    else k = depth == 1 ? k_hh256_quad<2, 1> : depth == 2 ? k_hh256_quad<2, 2> : k_hh256_quad<2, 3>;
    hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

using FusedKernel = void (*)(const GfApplyParams, const HashParams);

struct FusedPick {
    FusedKernel k;
    int spw, waves;
};

// packed: SPW = fused_spw (full hasher waves); !packed: one stripe per
// workgroup (A/B only, measurement builds).
template <int C, int R>
static FusedPick fused_entry(bool packed) {
    constexpr int spw = fused_spw<C + R>();
    if constexpr (spw == 1) {
        (void)packed;
        return {k_encode_hash_fused<C, R, 1>, 1, 1 + (C + R + 15) / 16};
    } else {
#if RSG_MEASUREMENT_BUILD  // the unpacked A/B variants (~60 kernels) stay out of the product library
        if (!packed) return {k_encode_hash_fused<C, R, 1>, 1, 1 + (C + R + 15) / 16};
#endif
        (void)packed;
        return {k_encode_hash_fused<C, R, spw>, spw, spw + (spw * (C + R) + 15) / 16};
    }
}

template <int C>
static FusedPick pick_fused_r(int R, bool packed) {
    switch (R) {
        case 1: return fused_entry<C, 1>(packed);
        case 2: return fused_entry<C, 2>(packed);
        case 3: return fused_entry<C, 3>(packed);
        case 4: return fused_entry<C, 4>(packed);
    }
    return {nullptr, 0, 0};
}

static FusedPick pick_fused(int C, int R, bool packed) {
    switch (C) {
        case 1: return pick_fused_r<1>(R, packed);
        case 2: return pick_fused_r<2>(R, packed);
        case 3: return pick_fused_r<3>(R, packed);
        case 4: return pick_fused_r<4>(R, packed);
        case 5: return pick_fused_r<5>(R, packed);
        case 6: return pick_fused_r<6>(R, packed);
        case 7: return pick_fused_r<7>(R, packed);
        case 8: return pick_fused_r<8>(R, packed);
        case 9: return pick_fused_r<9>(R, packed);
        case 10: return pick_fused_r<10>(R, packed);
        case 11: return pick_fused_r<11>(R, packed);
        case 12: return pick_fused_r<12>(R, packed);
        case 13: return pick_fused_r<13>(R, packed);
        case 14: return pick_fused_r<14>(R, packed);
        case 15: return pick_fused_r<15>(R, packed);
        case 16: return pick_fused_r<16>(R, packed);
    }
    return {nullptr, 0, 0};
}

// The packed table kernel takes shards of any length at any alignment (a
// partial last chunk); the ring, wide and DMA kernels need whole 16-byte
// aligned steps (checked where they are picked).
bool fused_supported(int C, int R, uint64_t shard_len) {
    return C >= 1 && C <= kMaxC && R >= 1 && R <= 4 && shard_len >= 1 &&
           (shard_len + kFusedChunk - 1) / kFusedChunk <= 0xffffffffull;
}

// 16-byte aligned shards and stripes (the ring kernel's 16-byte accesses)
static bool aligned16(const GfApplyParams& p) {
    if ((uintptr_t)p.base % 16 || p.stripe_stride % 16) return false;
    for (uint32_t c = 0; c < p.C; ++c)
        if (p.in_off[c] % 16) return false;
    for (uint32_t r = 0; r < p.R; ++r)
        if (p.out_off[r] % 16) return false;
    return true;
}

// The DMA kernel bakes the RS(8,4) encode matrix in at compile time: it is
// selected only when the launch's coefficient tables are exactly that
// matrix's (an encode launch, in place, a3-style layout), 16-byte aligned
// (LDS-DMA moves 16 B per lane) and whole 512-byte steps.
static bool dma_tables_match(const GfApplyParams& p) {
    static const auto want = [] {
        constexpr bs::EncodeRows<8, 4> E{};
        std::array<uint32_t, 4 * 8 * 5> t{};
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 8; ++c) {
                const uint8_t co = E.g[r][c];
                auto pack = [&](int sh, int f) {
                    uint32_t v = 0;
                    for (int i = 0; i < 4; ++i) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + i) << sh)) << (8 * i);
                    return v;
                };
                uint32_t* d = &t[(r * 8 + c) * 5];
                d[0] = pack(0, 0); d[1] = pack(0, 4); d[2] = pack(3, 0); d[3] = pack(3, 4); d[4] = pack(6, 0);
            }
        return t;
    }();
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c)
            for (int q = 0; q < 5; ++q)
                if (p.tab[r][c][q] != want[(r * 8 + c) * 5 + q]) return false;
    return true;
}

// The launch's tables are exactly those of the R x C rows `coef` (row-major).
static bool tables_match(const GfApplyParams& p, const uint8_t* coef, int C, int R) {
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < C; ++c) {
            const uint8_t co = coef[r * C + c];
            auto pack = [&](int sh, int f) {
                uint32_t v = 0;
                for (int i = 0; i < 4; ++i) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + i) << sh)) << (8 * i);
                return v;
            };
            const uint32_t want[5] = {pack(0, 0), pack(0, 4), pack(3, 0), pack(3, 4), pack(6, 0)};
            for (int q = 0; q < 5; ++q)
                if (p.tab[r][c][q] != want[q]) return false;
        }
    return true;
}

// RS(12,4) / RS(10,4) encode in place over 1024+ stripes (256+ workgroups of
// 4): the fused network kernel (rs_decode_netq.hip, k_decode_records_net12 /
// _net10 with ENC).
// RS(8,4) / RS(6,4) encode in place: the 8-stripe network kernel with ENC
// (rs_decode_net.hip) — from 2048 stripes (256+ workgroups).
static bool net_enc_supported(const GfApplyParams& p, uint64_t n_stripes) {
    if ((p.C != 8 && p.C != 6) || p.R != 4 || p.mode != GF_MODE_STORE || p.copy_mask ||
        p.base != p.out_base || p.stripe_stride != p.out_stripe_stride || n_stripes < 2048 ||
        5 * p.stripe_stride >= (1ull << 32))
        return false;
    const uint8_t* coef = p.C == 8 ? encode_net_coef() : encode_net6_coef();
    return tables_match(p, coef, (int)p.C, 4);
}

static hipError_t launch_encode_hash_net_c(const GfApplyParams& p, const HashParams& h, uint64_t shard_len,
                                           uint64_t n_stripes, hipStream_t stream) {
    if (p.C == 8) return launch_encode_hash_net(p, h, shard_len, n_stripes, stream);
    return launch_encode_hash_net6(p, h, shard_len, n_stripes, stream);
}

// Encode in place on the run-time-table one-pass kernel with ENC, for the
// geometries rs_decode.hip builds it for (table_enc_geometry).
static bool table_enc_supported(const GfApplyParams& p, uint64_t n_stripes) {
    return table_enc_geometry((int)p.C, (int)p.R) &&
           p.mode == GF_MODE_STORE && !p.copy_mask &&
           p.base == p.out_base && p.stripe_stride == p.out_stripe_stride && n_stripes >= 1 &&
           5 * p.stripe_stride < (1ull << 32);
}

static bool netq_enc_supported(const GfApplyParams& p, uint64_t n_stripes) {
    if ((p.C != 12 && p.C != 10) || p.R != 4 || p.mode != GF_MODE_STORE || p.copy_mask || p.base != p.out_base ||
        p.stripe_stride != p.out_stripe_stride || n_stripes < 1024 || 5 * p.stripe_stride >= (1ull << 32))
        return false;
    return p.C == 12 ? tables_match(p, encode_net12_coef(), 12, 4) : tables_match(p, encode_net10_coef(), 10, 4);
}

static bool dma_supported(const GfApplyParams& p, uint64_t shard_len, uint64_t n_stripes) {
    if (p.C != 8 || p.R != 4 || p.mode != GF_MODE_STORE || p.copy_mask || p.base != p.out_base ||
        p.stripe_stride != p.out_stripe_stride || n_stripes == 0 || n_stripes > 0x7fffffffull * dma::SPW)
        return false;
    if (shard_len < dma::CH || shard_len % dma::CH || shard_len / dma::CH > 0xffffffffull) return false;
    if ((uintptr_t)p.base % 16 || p.stripe_stride % 16) return false;
    if (dma::SPW / 2 * p.stripe_stride + shard_len >= (1ull << 32)) return false;  // 32-bit per-lane DMA offsets
    for (int c = 0; c < 8; ++c)
        if (p.in_off[c] % 16) return false;
    for (int r = 0; r < 4; ++r)
        if (p.out_off[r] % 8) return false;
    return dma_tables_match(p);
}

static hipError_t launch_encode_hash_dma(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                         hipStream_t stream) {
    // Tuning (A/B runs only): enc_prio = wave priorities (default none);
    // dma_ew = 4: two encoder waves per stripe group taking alternate steps
    // (split, as the wide kernel) instead of one; dma_nt: non-temporal
    // data loads (bit 0) and parity stores (bit 1), default both: 1.30 ->
    // 1.28 ms at n = 4096 (profiles/r02/ab_nt/); dma_spw = 4: four stripes
    // per workgroup, two workgroups per CU — measured slower (n = 4096: 1.39
    // vs 1.25 ms; profiles/r02/ab_spw/)
    const Tuning& t = tuning();  // one snapshot for the whole launch
    const int ew = t.dma_ew, nt = t.dma_nt, spw = t.dma_spw;
    p.wave_prio = (uint32_t)t.enc_prio;
    p.units = (uint32_t)(shard_len / dma::CH);
    h.n = n_stripes;
    const uint64_t blocks = (n_stripes + dma::SPW - 1) / dma::SPW;
    const dim3 grid((uint32_t)blocks), blk2(64 * dma::Shape<8, 4, 2>::WAVES);
    if (spw == 4 && ew != 4 && (n_stripes + 3) / 4 <= 0x7fffffffull) {
        const dim3 g4((uint32_t)((n_stripes + 3) / 4)), b4(64 * dma::Shape<8, 4, 1, 4>::WAVES);
        hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 1, 3, 4>), g4, b4, 0, stream, p, h);
        return hipGetLastError();
    }
    if (ew == 4)  // split encoders: two waves per stripe group on alternate steps
        hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 4, 3>), grid, dim3(64 * dma::Shape<8, 4, 4>::WAVES), 0, stream, p,
                           h);
    else if (nt == 1) hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 2, 1>), grid, blk2, 0, stream, p, h);
    else if (nt == 2) hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 2, 2>), grid, blk2, 0, stream, p, h);
    else if (nt == 3) hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 2, 3>), grid, blk2, 0, stream, p, h);
    else hipLaunchKernelGGL((k_encode_hash_dma<8, 4, 2>), grid, blk2, 0, stream, p, h);
    return hipGetLastError();
}

// Few large RS(8,4) stripes: k_encode_hash_wide with SPW stripes per
// workgroup (same preconditions as the DMA kernel, plus whole 1 KiB steps).
static bool wide_supported(const GfApplyParams& p, uint64_t shard_len, uint64_t n_stripes) {
    return dma_supported(p, shard_len, n_stripes) && shard_len % wide::CH == 0 && p.out_off[0] % 16 == 0 &&
           p.out_off[1] % 16 == 0 && p.out_off[2] % 16 == 0 && p.out_off[3] % 16 == 0;
}

static hipError_t launch_encode_hash_wide(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                          int spw, bool split, hipStream_t stream) {
    p.units = (uint32_t)(shard_len / wide::CH);
    h.n = n_stripes;
    const uint64_t blocks = (n_stripes + spw - 1) / spw;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)blocks);
    if (spw == 4 && split)
        hipLaunchKernelGGL((k_encode_hash_wide<4, true>), grid, dim3(64 * wide::Shape<4, true>::WAVES), 0, stream, p, h);
    else if (spw == 4)
        hipLaunchKernelGGL((k_encode_hash_wide<4, false>), grid, dim3(64 * wide::Shape<4, false>::WAVES), 0, stream, p,
                           h);
    else if (split)
        hipLaunchKernelGGL((k_encode_hash_wide<2, true>), grid, dim3(64 * wide::Shape<2, true>::WAVES), 0, stream, p, h);
    else
        hipLaunchKernelGGL((k_encode_hash_wide<2, false>), grid, dim3(64 * wide::Shape<2, false>::WAVES), 0, stream, p,
                           h);
    return hipGetLastError();
}

hipError_t launch_encode_hash_fused(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                    hipStream_t stream) {
    // Packed workgroups measured as fast or faster than one stripe per
    // workgroup at every batch size tried (n = 256..65536; profiles/r01/README.md);
    // Tuning::fused_spw1 selects the unpacked variant for A/B runs.
    const Tuning& t = tuning();  // one snapshot for the whole launch
    const bool unpacked = t.fused_spw1;
    // Few stripes (below ~8 per CU): the ring kernel (one stripe per
    // workgroup, E KiB chunks, next chunk in flight) beats the packed one
    // 1.1-3.2x (tools/kbench/ring_variants.hip);
    // Tuning::fused_kind (packed|ring|dma) forces one for A/B runs.
    const int kind = t.fused_kind;
    if (kind >= 4 && kind <= 7 && wide_supported(p, shard_len, n_stripes))
        return launch_encode_hash_wide(p, h, shard_len, n_stripes, (kind == 5 || kind == 7) ? 4 : 2, kind >= 6,
                                       stream);
    // RS(8,4), 512-2047 stripes (config 4's 4 and 8 MiB stripes at 4 GiB per
    // launch): the wide kernel with split encoders, 4 stripes per workgroup
    // from 1024 stripes (256+ workgroups), else 2; 4 MiB stripes, n = 1024:
    // 1.27 ms against 1.77 ms for the ring kernel, 8 MiB, n = 512: 1.51 ms
    // against 2.04 ms (profiles/r03/kind/).
    if (kind == 0 && n_stripes >= 512 && n_stripes < 2048 && wide_supported(p, shard_len, n_stripes))
        return launch_encode_hash_wide(p, h, shard_len, n_stripes, n_stripes >= 1024 ? 4 : 2, true, stream);
    if (kind != 1 && kind != 3 && (kind == 2 || n_stripes < 2048)) {
        uint32_t E = n_stripes <= 768 ? 2u : 1u;
        if (E == 2 && !ring_supported((int)p.C, (int)p.R, shard_len, E)) E = 1;
        if (ring_supported((int)p.C, (int)p.R, shard_len, E) && aligned16(p))
            return launch_encode_hash_ring(p, h, shard_len, n_stripes, E, stream);
    }
    // RSG_FUSED_KIND=table: the run-time-table one-pass kernel (A/B)
    if (kind == 9 && table_enc_supported(p, n_stripes))
        return launch_encode_hash_table(p, h, shard_len, n_stripes, stream);
    // RSG_FUSED_KIND=net: the 8-stripe network kernel for RS(8,4) too (A/B)
    if (kind == 8 && net_enc_supported(p, n_stripes)) return launch_encode_hash_net_c(p, h, shard_len, n_stripes, stream);
    // RS(8,4), 2048+ stripes: the LDS-DMA bit-sliced kernel (RSG_FUSED_KIND=
    // packed keeps the table kernel for A/B runs)
    if (kind != 1 && (kind == 3 || n_stripes >= 2048) && dma_supported(p, shard_len, n_stripes))
        return launch_encode_hash_dma(p, h, shard_len, n_stripes, stream);
    // RS(12,4) / RS(10,4), 1024+ stripes: the network kernel (LDS-DMA ring, 4
    // network waves, any shard length and alignment); RSG_FUSED_KIND=packed
    // keeps the table kernel for A/B runs
    if (kind != 1 && netq_enc_supported(p, n_stripes))
        return p.C == 12 ? launch_encode_hash_net12(p, h, shard_len, n_stripes, stream)
                         : launch_encode_hash_net10(p, h, shard_len, n_stripes, stream);
    // RS(6,4), 2048+ stripes: the 8-stripe network kernel (n = 4096 at 1 MiB
    // blocks: 2.11 -> 1.62 ms; RS(4,4) measured 1.5 % slower than the packed
    // table kernel and keeps it, profiles/r05/ab_fused_net/)
    if (kind != 1 && p.C == 6 && net_enc_supported(p, n_stripes))
        return launch_encode_hash_net_c(p, h, shard_len, n_stripes, stream);
    // Geometries without a network, 1024+ stripes: the run-time-table
    // one-pass kernel with ENC where it measured faster than the packed
    // kernel (table_enc_geometry: k >= 9, and most of k = 3..8 since round 6)
    if (kind != 1 && n_stripes >= 1024 && table_enc_supported(p, n_stripes))
        return launch_encode_hash_table(p, h, shard_len, n_stripes, stream);
    const FusedPick f = pick_fused((int)p.C, (int)p.R, !unpacked);
    if (!f.k || !fused_supported((int)p.C, (int)p.R, shard_len) || n_stripes == 0 || n_stripes > 0x7fffffffull)
        return hipErrorInvalidValue;
    p.units = (uint32_t)((shard_len + kFusedChunk - 1) / kFusedChunk);
    p.byte_end = shard_len;
    h.n = n_stripes;
    const size_t lds = (size_t)p.C * p.R * 32 + (size_t)f.spw * (p.C + p.R) * kFusedPitch;
    const uint64_t blocks = (n_stripes + f.spw - 1) / f.spw;
    hipLaunchKernelGGL(f.k, dim3((uint32_t)blocks), dim3(64 * f.waves), lds, stream, p, h);
    return hipGetLastError();
}

using RingKernel = void (*)(const GfApplyParams, const HashParams, const uint32_t);

template <int C>
static RingKernel pick_ring_r(int R) {
    switch (R) {
        case 1: return k_encode_hash_ring<C, 1>;
        case 2: return k_encode_hash_ring<C, 2>;
        case 3: return k_encode_hash_ring<C, 3>;
        case 4: return k_encode_hash_ring<C, 4>;
    }
    return nullptr;
}

static RingKernel pick_ring(int C, int R) {
    switch (C) {
        case 1: return pick_ring_r<1>(R);
        case 2: return pick_ring_r<2>(R);
        case 3: return pick_ring_r<3>(R);
        case 4: return pick_ring_r<4>(R);
        case 5: return pick_ring_r<5>(R);
        case 6: return pick_ring_r<6>(R);
        case 7: return pick_ring_r<7>(R);
        case 8: return pick_ring_r<8>(R);
    }
    return nullptr;
}

size_t ring_lds_bytes(int C, int R, uint32_t E) {
    return (size_t)C * R * 32 + 2ull * (C + R) * (kRingCol * E + 32);
}

bool ring_supported(int C, int R, uint64_t shard_len, uint32_t E) {
    return C >= 1 && C <= kRingMaxC && R >= 1 && R <= 4 && (E == 1 || E == 2) &&
           shard_len >= kRingCol * E && shard_len % (kRingCol * E) == 0 &&
           shard_len / (kRingCol * E) <= 0xffffffffull && ring_lds_bytes(C, R, E) <= 160 * 1024;
}

hipError_t launch_encode_hash_ring(GfApplyParams p, HashParams h, uint64_t shard_len, uint64_t n_stripes,
                                   uint32_t E, hipStream_t stream) {
    RingKernel k = pick_ring((int)p.C, (int)p.R);
    if (!k || !ring_supported((int)p.C, (int)p.R, shard_len, E) || n_stripes == 0 || n_stripes > 0x7fffffffull)
        return hipErrorInvalidValue;
    p.units = (uint32_t)(shard_len / (kRingCol * E));
    h.n = n_stripes;
    const uint32_t waves = E + (p.C + p.R + 15) / 16;
    const size_t lds = ring_lds_bytes((int)p.C, (int)p.R, E);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k, dim3((uint32_t)n_stripes), dim3(64 * waves), lds, stream, p, h, E);
    return hipGetLastError();
}

}  // namespace rsg
