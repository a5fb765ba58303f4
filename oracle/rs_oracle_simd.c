/*
 * rs_oracle_simd.c — the CPU baseline: the reference's own SIMD algorithm,
 * restated.  TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline leg + tests).
 *
 * rustfs-erasure-codec is built with feature `simd-accel`
 * (crates/ecstore/Cargo.toml:178), whose C code multiplies a shard by a GF(2^8)
 * constant with split-nibble tables and `pshufb` (low nibble table, high nibble
 * table, XOR).  This file restates that loop with AVX2 (`vpshufb`, 32 bytes per
 * step) and falls back to the scalar oracle when AVX2 is absent.  Work is split
 * one stripe per thread, as rustfs runs one encode per tokio worker
 * (crates/ecstore/src/erasure/coding/encode.rs:504-530).
 */
#include "rs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#if defined(__x86_64__)
#include <immintrin.h>
#define RO_HAVE_X86 1
#else
#define RO_HAVE_X86 0
#endif

int ro_simd_level(void) {
#if RO_HAVE_X86
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") ? 2 : 0;
#else
    return 0;
#endif
}

#if RO_HAVE_X86
/* dst (^)= c * src over len bytes; first != 0 writes instead of accumulating. */
__attribute__((target("avx2"))) static void mul_slice_avx2(const uint8_t lo[16], const uint8_t hi[16],
                                                           const uint8_t *src, uint8_t *dst, size_t len,
                                                           int first) {
    const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    const __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(src + i));
        __m256i l = _mm256_and_si256(x, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        if (!first) p = _mm256_xor_si256(p, _mm256_loadu_si256((const __m256i *)(dst + i)));
        _mm256_storeu_si256((__m256i *)(dst + i), p);
    }
    for (; i < len; i++) {
        uint8_t x = src[i];
        uint8_t p = lo[x & 15] ^ hi[x >> 4];
        dst[i] = first ? p : (uint8_t)(dst[i] ^ p);
    }
}
#endif

typedef struct {
    int k, m;
    size_t S, n;
    uint8_t *stripes;
    uint8_t *digests;
    const uint8_t *lo; /* m*k*16 */
    const uint8_t *hi;
    const uint8_t *rows; /* m*k coefficients */
    int simd;
    size_t next; /* atomic work counter */
} batch_job;

static void encode_one(const batch_job *J, size_t s) {
    int k = J->k, m = J->m;
    size_t S = J->S;
    uint8_t *base = J->stripes + s * (size_t)(k + m) * S;
    for (int p = 0; p < m; p++) {
        uint8_t *dst = base + (size_t)(k + p) * S;
        if (J->simd) {
#if RO_HAVE_X86
            for (int c = 0; c < k; c++) {
                size_t t = (size_t)p * k + c;
                mul_slice_avx2(J->lo + t * 16, J->hi + t * 16, base + (size_t)c * S, dst, S, c == 0);
            }
#endif
        } else {
            const uint8_t *in[256];
            for (int c = 0; c < k; c++) in[c] = base + (size_t)c * S;
            ro_matrix_apply(1, k, J->rows + (size_t)p * k, in, &dst, S);
        }
    }
    if (J->digests) {
        for (int i = 0; i < k + m; i++)
            ro_hh256s(base + (size_t)i * S, S, J->digests + (s * (size_t)(k + m) + i) * 32);
    }
}

static void *worker(void *arg) {
    batch_job *J = (batch_job *)arg;
    for (;;) {
        size_t s = __atomic_fetch_add(&J->next, 1, __ATOMIC_RELAXED);
        if (s >= J->n) break;
        encode_one(J, s);
    }
    return NULL;
}

int ro_encode_batch_mt(int k, int m, size_t S, size_t n, uint8_t *stripes, uint8_t *digests, int threads) {
    if (k <= 0 || m <= 0 || k + m > 256) return -1;
    uint8_t *mat = (uint8_t *)malloc((size_t)(k + m) * k);
    uint8_t *lo = (uint8_t *)malloc((size_t)m * k * 16);
    uint8_t *hi = (uint8_t *)malloc((size_t)m * k * 16);
    if (!mat || !lo || !hi || ro_build_matrix(k, m, mat) != 0) {
        free(mat); free(lo); free(hi);
        return -1;
    }
    const uint8_t *rows = mat + (size_t)k * k;
    for (int t = 0; t < m * k; t++)
        for (int x = 0; x < 16; x++) {
            lo[t * 16 + x] = ro_gf_mul(rows[t], (uint8_t)x);
            hi[t * 16 + x] = ro_gf_mul(rows[t], (uint8_t)(x << 4));
        }
    batch_job J = {k, m, S, n, stripes, digests, lo, hi, rows, ro_simd_level() >= 2, 0};
    if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = (int)(n ? n : 1);
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    int started = 0;
    for (int i = 1; i < threads; i++)
        if (pthread_create(&tid[i], NULL, worker, &J) == 0) started = i;
        else break;
    worker(&J);
    for (int i = 1; i <= started; i++) pthread_join(tid[i], NULL);
    free(tid);
    free(mat); free(lo); free(hi);
    return 0;
}
