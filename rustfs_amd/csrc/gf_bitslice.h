// gf_bitslice.h — bit-sliced GF(2^8) matrix apply for compile-time matrices
// (the encode matrix of a fixed (k, m) geometry).  Used by the LDS-DMA fused
// encode + HighwayHash kernel (rs_kernels.hip k_encode_hash_dma, RS(8,4)),
// whose launcher checks at run time that the codec's encode rows equal
// EncodeRows<K, M> before selecting it; tools/kbench/ (bs_variants.hip,
// fused_bs.hip, fused_r2.hip) compare it with the table kernels.
//
// Multiplication by a constant c is GF(2)-linear on the 8 bits of a byte: an
// 8x8 bit matrix B_c with column j = c * 2^j.  If 32 bytes are held as 8 bit
// planes (plane j = bit j of each byte, one 32-bit register), then c * x for
// all 32 bytes is plane-wise XOR: out plane i = XOR over j with B_c[i][j] of
// in plane j, and a whole parity row
//     parity_r = XOR_c G[r][c] * data_c
// is, per output plane, one XOR chain over the (c, j) terms where
// B_{G[r][c]}[i][j] = 1.  With G known at compile time those chains are
// straight-line code: ~16 terms per input dword for RS(8,4) (1040 terms per
// 32-byte column over 8 inputs), folded 2 at a time by the gfx950 three-input
// XOR (v_bitop3_b32), against 3 v_perm_b32 + 1.5 XOR per word x coefficient
// for the table kernels (rs_kernels.hip header).  v_perm issues at ~half the
// rate of v_xor/v_bitop3 on gfx950 (tools/kbench/op_rates.hip), so the XOR
// network costs about half the SIMD cycles of the table lookups.
//
// Planes come from an 8x8 bit transpose of the 8 dwords a lane holds (byte q of
// dwords 0..7 is one 8x8 bit matrix; three rounds of masked swaps between
// dword pairs, v_bfi_b32 per half): plane j byte q bit d = bit j of byte q of
// dword d.  The transpose is its own inverse, so the same network turns output
// planes back into bytes.  Any byte order inside a plane works as long as input
// and output use the same one, which lets a lane's 32 bytes be two 16-byte
// pieces 1 KiB apart (fully coalesced dwordx4 loads/stores per wave).
//
// The matrix follows the reference construction (reed-solomon-erasure's
// Vandermonde build; rsgpu.cpp:build_matrix, erasure.rs:448-470): G = V *
// inv(V[0..k)), V[r][c] = r^c over GF(2^8)/0x11D; the microbenchmarks compare
// its parity byte for byte with the production kernels fed rsgpu.cpp's rows.
#pragma once

#include <stdint.h>

namespace rsg {
namespace bs {

constexpr uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1d : 0));
    }
    return r;
}

constexpr uint8_t gpow(uint8_t a, int n) {
    uint8_t r = 1;
    for (int i = 0; i < n; ++i) r = gmul(r, a);
    return r;
}

constexpr uint8_t ginv(uint8_t a) { return gpow(a, 254); }

// Parity rows (m x k) of the (k+m) x k systematic encode matrix.
template <int K, int M>
struct EncodeRows {
    uint8_t g[M][K];
    constexpr EncodeRows() : g() {
        uint8_t w[K][2 * K] = {};
        for (int r = 0; r < K; ++r) {
            for (int c = 0; c < K; ++c) w[r][c] = gpow((uint8_t)r, c);
            w[r][K + r] = 1;
        }
        for (int c = 0; c < K; ++c) {
            int p = c;
            while (p < K && w[p][c] == 0) ++p;
            for (int j = 0; j < 2 * K; ++j) {
                const uint8_t t = w[p][j];
                w[p][j] = w[c][j];
                w[c][j] = t;
            }
            const uint8_t iv = ginv(w[c][c]);
            for (int j = 0; j < 2 * K; ++j) w[c][j] = gmul(w[c][j], iv);
            for (int r = 0; r < K; ++r) {
                if (r == c || w[r][c] == 0) continue;
                const uint8_t f = w[r][c];
                for (int j = 0; j < 2 * K; ++j) w[r][j] ^= gmul(f, w[c][j]);
            }
        }
        for (int r = 0; r < M; ++r)
            for (int c = 0; c < K; ++c) {
                uint8_t a = 0;
                for (int i = 0; i < K; ++i) a ^= gmul(gpow((uint8_t)(K + r), i), w[i][K + c]);
                g[r][c] = a;
            }
    }
};

// Bit (i, j) of B_c: bit i of c * 2^j.
constexpr bool bm(uint8_t c, int i, int j) { return (gmul(c, (uint8_t)(1u << j)) >> i) & 1u; }

// Row masks: bit j of mask[r][c][i] = B_{G[r][c]}[i][j].
template <int K, int M>
struct PlaneMasks {
    uint8_t mask[M][K][8];
    constexpr PlaneMasks() : mask() {
        const EncodeRows<K, M> e;
        for (int r = 0; r < M; ++r)
            for (int c = 0; c < K; ++c)
                for (int i = 0; i < 8; ++i) {
                    uint8_t v = 0;
                    for (int j = 0; j < 8; ++j) v |= (uint8_t)(bm(e.g[r][c], i, j) << j);
                    mask[r][c][i] = v;
                }
    }
};

// Term lists: for output plane (r, i), the input planes c*8+j to XOR.
template <int K, int M>
struct Terms {
    uint16_t n[M][8];
    uint8_t idx[M][8][K * 8];
    constexpr Terms() : n(), idx() {
        const EncodeRows<K, M> e;
        for (int r = 0; r < M; ++r)
            for (int i = 0; i < 8; ++i) {
                int t = 0;
                for (int c = 0; c < K; ++c)
                    for (int j = 0; j < 8; ++j)
                        if (bm(e.g[r][c], i, j)) idx[r][i][t++] = (uint8_t)(c * 8 + j);
                n[r][i] = (uint16_t)t;
            }
    }
};

// One round of the 8x8 bit transpose: swap the bits of `lo` outside `mask`
// with the bits of `hi` inside it, shifted by s (two v_bfi_b32 + two shifts).
__device__ __forceinline__ void swap_bits(uint32_t& lo, uint32_t& hi, int s, uint32_t mask) {
    const uint32_t a = lo, b = hi;
    lo = (a & mask) | ((b << s) & ~mask);
    hi = ((a >> s) & mask) | (b & ~mask);
}

// Bytes <-> bit planes for 8 dwords (its own inverse).  The masks come in
// VGPRs: a VOP3 with an SGPR or literal operand issues at half rate.
__device__ __forceinline__ void transpose(uint32_t (&w)[8], uint32_t m4, uint32_t m2, uint32_t m1) {
#pragma unroll
    for (int d = 0; d < 4; ++d) swap_bits(w[d], w[d + 4], 4, m4);
    swap_bits(w[0], w[2], 2, m2);
    swap_bits(w[1], w[3], 2, m2);
    swap_bits(w[4], w[6], 2, m2);
    swap_bits(w[5], w[7], 2, m2);
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap_bits(w[d], w[d + 1], 1, m1);
}

}  // namespace bs
}  // namespace rsg
