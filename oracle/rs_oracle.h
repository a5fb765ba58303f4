/*
 * rs_oracle.h — CPU restatement of the reference's erasure hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by,
 * or called from the product library (librsgpu.so) or its Python mirror.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU baseline.
 *
 * What it restates (the reference's arithmetic lives in third-party crates that
 * are not vendored under /root/reference; see DESIGN.md "Oracle"):
 *   - rustfs-erasure-codec 8.0.2 (fork of reed-solomon-erasure v8, imported as
 *     reed_solomon_erasure::galois_8; Cargo.toml:285, Cargo.lock:9514-9527):
 *     GF(2^8) / 0x11D, generator 2, systematic matrix V * inv(V[0..k]) with
 *     V[r][c] = r^c; encode, reconstruct (first k present shards, ascending),
 *     reconstruct_data, verify.
 *   - highway 1.3.0 (Cargo.toml:260, Cargo.lock:5007): HighwayHash-256, keyed
 *     as crates/utils/src/hash.rs:22-47, serialised LE as hash.rs:95-102.
 *
 * Pinned against the reference's own golden vectors (tests/golden/
 * reference_vectors.json).
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GF(2^8), polynomial 0x11D, generator 2 ---- */
uint8_t ro_gf_mul(uint8_t a, uint8_t b);
uint8_t ro_gf_div(uint8_t a, uint8_t b);   /* b != 0 */
uint8_t ro_gf_exp(uint8_t a, int n);       /* a^n, exp(0,0) = 1 */

/* Systematic encoding matrix, (k+m) x k row-major, written to out.
 * Returns 0, or -1 on bad geometry (k == 0, m == 0, k+m > 256). */
int ro_build_matrix(int k, int m, uint8_t *out);

/* Gauss-Jordan inverse of an n x n matrix in place.  Returns 0 or -1 (singular). */
int ro_invert(int n, uint8_t *mat);

/* out[r][b] = XOR_c rows[r][c] * in[c][b]  (rows: R x C row-major). */
void ro_matrix_apply(int R, int C, const uint8_t *rows, const uint8_t *const *in,
                     uint8_t *const *out, size_t len);

/* ReedSolomon::encode — shards[0..k) data, shards[k..k+m) overwritten. */
int ro_encode(int k, int m, uint8_t *const *shards, size_t len);

/* ReedSolomon::reconstruct / reconstruct_data.  present[i] != 0 marks a valid
 * shard; missing shards are written in place (caller-provided buffers).
 * data_only != 0: parity shards that are missing are left untouched.
 * Returns 0, -2 if fewer than k shards are present. */
int ro_reconstruct(int k, int m, uint8_t *const *shards, const uint8_t *present,
                   size_t len, int data_only);

/* ReedSolomon::verify — 1 if parity matches data, 0 otherwise. */
int ro_verify(int k, int m, const uint8_t *const *shards, size_t len);

/* ---- HighwayHash-256 ---- */
void ro_hh256(const uint64_t key[4], const uint8_t *data, size_t len, uint8_t out[32]);
/* HashAlgorithm::HighwayHash256S (hash.rs:123-127) with the pi-derived key. */
void ro_hh256s(const uint8_t *data, size_t len, uint8_t out[32]);
/* HashAlgorithm::HighwayHash256SLegacy (key [3,4,2,1], hash.rs:28-30). */
void ro_hh256s_legacy(const uint8_t *data, size_t len, uint8_t out[32]);

/* ---- CPU baseline (restated reference algorithm: split-nibble pshufb MAC) ---- */
/* Encode n stripes in the a3 layout (n x (k+m) x S bytes, stride = (k+m)*S),
 * optionally writing (k+m) HH256S digests per stripe.  threads <= 0: all cores.
 * Returns 0, or -1 on bad geometry. */
int ro_encode_batch_mt(int k, int m, size_t S, size_t n, uint8_t *stripes,
                       uint8_t *digests, int threads);
/* Non-zero when the vector (AVX2) split-nibble path is in use. */
int ro_simd_level(void);

#ifdef __cplusplus
}
#endif
#endif
