/*
 * rs_oracle.c — scalar CPU restatement of the reference erasure hot path.
 * TEST INFRASTRUCTURE ONLY (see rs_oracle.h header comment).
 *
 * Reference anchors (all paths under /root/reference):
 *   docs/architecture/erasure-coding.md:41-50   GF(2^8) Vandermonde "rs-vandermonde"
 *   crates/ecstore/src/erasure/coding/erasure.rs:396-441  ReedSolomonEncoder
 *       encode / reconstruct_data / reconstruct / verify -> reed_solomon_erasure
 *   crates/ecstore/src/erasure/codec/bridge.rs:274-307     reconstruct_opt path
 *   crates/utils/src/hash.rs:22-47, 95-141                 HighwayHash256S keying
 */
#include "rs_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* GF(2^8): reed_solomon_erasure::galois_8 uses the generating polynomial 29
 * (x^8 + x^4 + x^3 + x^2 + 1 = 0x11D) and generator 2. */

static uint8_t g_log[256];
static uint8_t g_exp[510];
static int g_init = 0;

static void gf_init(void) {
    if (g_init) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_log[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 510; i++) g_exp[i] = g_exp[i - 255];
    g_log[0] = 0;
    g_init = 1;
}

uint8_t ro_gf_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

uint8_t ro_gf_div(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0) return 0;
    int l = (int)g_log[a] - (int)g_log[b];
    if (l < 0) l += 255;
    return g_exp[l];
}

/* galois_8::exp: exp(a, 0) = 1 for every a (including 0); exp(0, n>0) = 0. */
uint8_t ro_gf_exp(uint8_t a, int n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    int l = ((int)g_log[a] * n) % 255;
    return g_exp[l];
}

/* ------------------------------------------------------------------------- */
/* Matrices. */

int ro_invert(int n, uint8_t *mat) {
    gf_init();
    /* Augment [mat | I] and run Gauss-Jordan (the inverse is unique, so the
     * pivoting order does not affect the result). */
    uint8_t *w = (uint8_t *)malloc((size_t)n * 2 * n);
    if (!w) return -1;
    for (int r = 0; r < n; r++) {
        memcpy(w + (size_t)r * 2 * n, mat + (size_t)r * n, n);
        memset(w + (size_t)r * 2 * n + n, 0, n);
        w[(size_t)r * 2 * n + n + r] = 1;
    }
    for (int c = 0; c < n; c++) {
        int p = c;
        while (p < n && w[(size_t)p * 2 * n + c] == 0) p++;
        if (p == n) { free(w); return -1; }
        if (p != c) {
            for (int j = 0; j < 2 * n; j++) {
                uint8_t t = w[(size_t)p * 2 * n + j];
                w[(size_t)p * 2 * n + j] = w[(size_t)c * 2 * n + j];
                w[(size_t)c * 2 * n + j] = t;
            }
        }
        uint8_t *row = w + (size_t)c * 2 * n;
        uint8_t piv = row[c];
        if (piv != 1) {
            for (int j = 0; j < 2 * n; j++) row[j] = ro_gf_div(row[j], piv);
        }
        for (int r = 0; r < n; r++) {
            if (r == c) continue;
            uint8_t *o = w + (size_t)r * 2 * n;
            uint8_t f = o[c];
            if (!f) continue;
            for (int j = 0; j < 2 * n; j++) o[j] ^= ro_gf_mul(f, row[j]);
        }
    }
    for (int r = 0; r < n; r++) memcpy(mat + (size_t)r * n, w + (size_t)r * 2 * n + n, n);
    free(w);
    return 0;
}

/* reed_solomon_erasure::ReedSolomon::build_matrix:
 *   vandermonde(total, k)[r][c] = exp(r, c);  top = rows 0..k;  M = V * inv(top). */
int ro_build_matrix(int k, int m, uint8_t *out) {
    gf_init();
    if (k <= 0 || m <= 0 || k + m > 256) return -1;
    int t = k + m;
    uint8_t *v = (uint8_t *)malloc((size_t)t * k);
    uint8_t *top = (uint8_t *)malloc((size_t)k * k);
    if (!v || !top) { free(v); free(top); return -1; }
    for (int r = 0; r < t; r++)
        for (int c = 0; c < k; c++) v[(size_t)r * k + c] = ro_gf_exp((uint8_t)r, c);
    memcpy(top, v, (size_t)k * k);
    if (ro_invert(k, top) != 0) { free(v); free(top); return -1; }
    for (int r = 0; r < t; r++)
        for (int c = 0; c < k; c++) {
            uint8_t acc = 0;
            for (int i = 0; i < k; i++) acc ^= ro_gf_mul(v[(size_t)r * k + i], top[(size_t)i * k + c]);
            out[(size_t)r * k + c] = acc;
        }
    free(v);
    free(top);
    return 0;
}

/* code_some_slices: out[r] = XOR_c rows[r][c] * in[c]  (byte-wise, scalar). */
void ro_matrix_apply(int R, int C, const uint8_t *rows, const uint8_t *const *in,
                     uint8_t *const *out, size_t len) {
    gf_init();
    for (int r = 0; r < R; r++) {
        uint8_t *o = out[r];
        memset(o, 0, len);
        for (int c = 0; c < C; c++) {
            uint8_t f = rows[(size_t)r * C + c];
            if (!f) continue;
            const uint8_t *src = in[c];
            unsigned lf = g_log[f];
            for (size_t b = 0; b < len; b++) {
                uint8_t x = src[b];
                if (x) o[b] ^= g_exp[lf + g_log[x]];
            }
        }
    }
}

int ro_encode(int k, int m, uint8_t *const *shards, size_t len) {
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    if (!mat || ro_build_matrix(k, m, mat) != 0) { free(mat); return -1; }
    ro_matrix_apply(m, k, mat + (size_t)k * k, (const uint8_t *const *)shards, shards + k, len);
    free(mat);
    return 0;
}

/* reed_solomon_erasure reconstruct_internal: the sub-matrix is built from the
 * first k present shards in ascending index order; missing data shards are
 * rebuilt with rows of its inverse; missing parity (when !data_only) is then
 * re-encoded from the complete data shards. */
int ro_reconstruct(int k, int m, uint8_t *const *shards, const uint8_t *present,
                   size_t len, int data_only) {
    int t = k + m;
    int nvalid = 0;
    for (int i = 0; i < t; i++) nvalid += present[i] ? 1 : 0;
    if (nvalid < k) return -2;
    if (nvalid == t) return 0;

    uint8_t *mat = (uint8_t *)malloc((size_t)t * k);
    uint8_t *sub = (uint8_t *)malloc((size_t)k * k);
    const uint8_t **sub_in = (const uint8_t **)malloc(sizeof(uint8_t *) * (size_t)k);
    if (!mat || !sub || !sub_in || ro_build_matrix(k, m, mat) != 0) {
        free(mat); free(sub); free(sub_in); return -1;
    }
    int s = 0;
    for (int i = 0; i < t && s < k; i++) {
        if (!present[i]) continue;
        memcpy(sub + (size_t)s * k, mat + (size_t)i * k, k);
        sub_in[s] = shards[i];
        s++;
    }
    if (ro_invert(k, sub) != 0) { free(mat); free(sub); free(sub_in); return -1; }

    for (int i = 0; i < k; i++) {
        if (present[i]) continue;
        uint8_t *o = shards[i];
        ro_matrix_apply(1, k, sub + (size_t)i * k, sub_in, &o, len);
    }
    if (!data_only) {
        for (int p = 0; p < m; p++) {
            if (present[k + p]) continue;
            uint8_t *o = shards[k + p];
            ro_matrix_apply(1, k, mat + (size_t)(k + p) * k, (const uint8_t *const *)shards, &o, len);
        }
    }
    free(mat);
    free(sub);
    free(sub_in);
    return 0;
}

int ro_verify(int k, int m, const uint8_t *const *shards, size_t len) {
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    uint8_t *buf = (uint8_t *)malloc(len ? len : 1);
    if (!mat || !buf || ro_build_matrix(k, m, mat) != 0) { free(mat); free(buf); return -1; }
    int ok = 1;
    for (int p = 0; p < m && ok; p++) {
        uint8_t *o = buf;
        ro_matrix_apply(1, k, mat + (size_t)(k + p) * k, shards, &o, len);
        if (memcmp(buf, shards[k + p], len) != 0) ok = 0;
    }
    free(mat);
    free(buf);
    return ok;
}

/* ------------------------------------------------------------------------- */
/* HighwayHash-256 (public spec; the algorithm of the `highway` crate 1.3.0).
 * State: v0, v1, mul0, mul1 — four 64-bit lanes each. */

typedef struct {
    uint64_t v0[4], v1[4], mul0[4], mul1[4];
} hh_state;

static void hh_reset(const uint64_t key[4], hh_state *s) {
    static const uint64_t init0[4] = {0xdbe6d5d5fe4cce2full, 0xa4093822299f31d0ull,
                                      0x13198a2e03707344ull, 0x243f6a8885a308d3ull};
    static const uint64_t init1[4] = {0x3bd39e10cb0ef593ull, 0xc0acf169b5f18a8cull,
                                      0xbe5466cf34e90c6cull, 0x452821e638d01377ull};
    for (int i = 0; i < 4; i++) {
        s->mul0[i] = init0[i];
        s->mul1[i] = init1[i];
        s->v0[i] = init0[i] ^ key[i];
        s->v1[i] = init1[i] ^ ((key[i] >> 32) | (key[i] << 32));
    }
}

static void hh_zipper_add(uint64_t v1, uint64_t v0, uint64_t *add1, uint64_t *add0) {
    *add0 += (((v0 & 0xff000000ull) | (v1 & 0xff00000000ull)) >> 24) |
             (((v0 & 0xff0000000000ull) | (v1 & 0xff000000000000ull)) >> 16) |
             (v0 & 0xff0000ull) | ((v0 & 0xff00ull) << 32) |
             ((v1 & 0xff00000000000000ull) >> 8) | (v0 << 56);
    *add1 += (((v1 & 0xff000000ull) | (v0 & 0xff00000000ull)) >> 24) |
             (v1 & 0xff0000ull) | ((v1 & 0xff0000000000ull) >> 16) |
             ((v1 & 0xff00ull) << 24) | ((v0 & 0xff000000000000ull) >> 8) |
             ((v1 & 0xffull) << 48) | (v0 & 0xff00000000000000ull);
}

static void hh_update(const uint64_t lanes[4], hh_state *s) {
    for (int i = 0; i < 4; i++) {
        s->v1[i] += s->mul0[i] + lanes[i];
        s->mul0[i] ^= (s->v1[i] & 0xffffffffull) * (s->v0[i] >> 32);
        s->v0[i] += s->mul1[i];
        s->mul1[i] ^= (s->v0[i] & 0xffffffffull) * (s->v1[i] >> 32);
    }
    hh_zipper_add(s->v1[1], s->v1[0], &s->v0[1], &s->v0[0]);
    hh_zipper_add(s->v1[3], s->v1[2], &s->v0[3], &s->v0[2]);
    hh_zipper_add(s->v0[1], s->v0[0], &s->v1[1], &s->v1[0]);
    hh_zipper_add(s->v0[3], s->v0[2], &s->v1[3], &s->v1[2]);
}

static uint64_t rd64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

static void hh_packet(const uint8_t *p, hh_state *s) {
    uint64_t lanes[4] = {rd64(p), rd64(p + 8), rd64(p + 16), rd64(p + 24)};
    hh_update(lanes, s);
}

static void hh_rotate32(unsigned count, uint64_t lanes[4]) {
    for (int i = 0; i < 4; i++) {
        uint32_t h0 = (uint32_t)lanes[i];
        uint32_t h1 = (uint32_t)(lanes[i] >> 32);
        h0 = (h0 << count) | (h0 >> (32 - count));
        h1 = (h1 << count) | (h1 >> (32 - count));
        lanes[i] = (uint64_t)h0 | ((uint64_t)h1 << 32);
    }
}

static void hh_remainder(const uint8_t *bytes, size_t size_mod32, hh_state *s) {
    size_t size_mod4 = size_mod32 & 3;
    const uint8_t *rem = bytes + (size_mod32 & ~(size_t)3);
    uint8_t packet[32] = {0};
    for (int i = 0; i < 4; i++) s->v0[i] += ((uint64_t)size_mod32 << 32) + size_mod32;
    hh_rotate32((unsigned)size_mod32, s->v1);
    for (size_t i = 0; i < (size_t)(rem - bytes); i++) packet[i] = bytes[i];
    if (size_mod32 & 16) {
        for (int i = 0; i < 4; i++) packet[28 + i] = rem[i + size_mod4 - 4];
    } else if (size_mod4) {
        packet[16 + 0] = rem[0];
        packet[16 + 1] = rem[size_mod4 >> 1];
        packet[16 + 2] = rem[size_mod4 - 1];
    }
    hh_packet(packet, s);
}

static void hh_permute_update(hh_state *s) {
    uint64_t p[4];
    p[0] = (s->v0[2] >> 32) | (s->v0[2] << 32);
    p[1] = (s->v0[3] >> 32) | (s->v0[3] << 32);
    p[2] = (s->v0[0] >> 32) | (s->v0[0] << 32);
    p[3] = (s->v0[1] >> 32) | (s->v0[1] << 32);
    hh_update(p, s);
}

static void hh_modred(uint64_t a3u, uint64_t a2, uint64_t a1, uint64_t a0, uint64_t *m1, uint64_t *m0) {
    uint64_t a3 = a3u & 0x3FFFFFFFFFFFFFFFull;
    *m1 = a1 ^ ((a3 << 1) | (a2 >> 63)) ^ ((a3 << 2) | (a2 >> 62));
    *m0 = a0 ^ (a2 << 1) ^ (a2 << 2);
}

void ro_hh256(const uint64_t key[4], const uint8_t *data, size_t len, uint8_t out[32]) {
    hh_state s;
    hh_reset(key, &s);
    size_t full = len & ~(size_t)31;
    for (size_t i = 0; i < full; i += 32) hh_packet(data + i, &s);
    if (len & 31) hh_remainder(data + full, len & 31, &s);
    for (int i = 0; i < 10; i++) hh_permute_update(&s);
    uint64_t h[4];
    hh_modred(s.v1[1] + s.mul1[1], s.v1[0] + s.mul1[0], s.v0[1] + s.mul0[1], s.v0[0] + s.mul0[0], &h[1], &h[0]);
    hh_modred(s.v1[3] + s.mul1[3], s.v1[2] + s.mul1[2], s.v0[3] + s.mul0[3], s.v0[2] + s.mul0[2], &h[3], &h[2]);
    /* u8x32_from_u64x4: little-endian per lane (hash.rs:95-102). */
    for (int i = 0; i < 4; i++)
        for (int b = 0; b < 8; b++) out[i * 8 + b] = (uint8_t)(h[i] >> (8 * b));
}

/* MAGIC_HIGHWAY_HASH256_KEY (hash.rs:22-25) parsed as 4 LE u64 (hash.rs:32-47). */
static const uint8_t k_magic[32] = {
    0x4b, 0xe7, 0x34, 0xfa, 0x8e, 0x23, 0x8a, 0xcd, 0x26, 0x3e, 0x83, 0xe6, 0xbb, 0x96, 0x85, 0x52,
    0x04, 0x0f, 0x93, 0x5d, 0xa3, 0x9f, 0x44, 0x14, 0x97, 0xe0, 0x9d, 0x13, 0x22, 0xde, 0x36, 0xa0};

void ro_hh256s(const uint8_t *data, size_t len, uint8_t out[32]) {
    uint64_t key[4] = {rd64(k_magic), rd64(k_magic + 8), rd64(k_magic + 16), rd64(k_magic + 24)};
    ro_hh256(key, data, len, out);
}

void ro_hh256s_legacy(const uint8_t *data, size_t len, uint8_t out[32]) {
    static const uint64_t key[4] = {3, 4, 2, 1};
    ro_hh256(key, data, len, out);
}
