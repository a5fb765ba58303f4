// get_probe.hip — the degraded GET's GF pass (rsg_decode_records_dev fast
// path, RS(8,4), data shards 0 and 1 lost): survivors 2..7 + parity 8, 9 read
// in place from 12 record files, data 0 and 1 rebuilt into the output, data
// 2..7 copied through, parity 10 and 11 re-derived and compared.  The
// production PRE kernel against register-capped and reordered variants.
// Measurement code.  Usage: get_probe [n] [separate files 0|1] [verify launch before each GF launch 0|1] [round file allocations to this many bytes] [compare rows match 0|1] [no copy-through 0|1]
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

// ORDER 0: production order (preload, copy, accumulate, store)
// ORDER 1: copies after the rebuilt rows' stores
// ORDER 2: compare operands loaded late (at the compare), copies first
// ORDER 3: as 1 with non-temporal copy stores
template <int C, int R, int WPE, int ORDER>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_get(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * 64u + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint4 old[R];
    if (ORDER != 2) gf_preload<R>(p, obase, off, stripe, old);
    if (ORDER != 1 && ORDER != 3 && p.copy_mask) {
#pragma unroll
        for (int c = 0; c < C; ++c)
            if ((p.copy_mask >> c) & 1u) st16(obase + p.copy_off[c] + off, x[c]);
    }
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    gf_accumulate<0, C, R>(p, x, acc);
    if (ORDER == 2) gf_store_late<R>(p, obase, off, acc, stripe);
    else gf_store<R>(p, obase, off, acc, stripe, old);
    if (ORDER == 1 && p.copy_mask) {
#pragma unroll
        for (int c = 0; c < C; ++c)
            if ((p.copy_mask >> c) & 1u) st16(obase + p.copy_off[c] + off, x[c]);
    }
    if (ORDER == 3 && p.copy_mask) {  // at the end, non-temporal
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int c = 0; c < C; ++c)
            if ((p.copy_mask >> c) & 1u) {
                v4u w = {x[c].x, x[c].y, x[c].z, x[c].w};
                __builtin_nontemporal_store(w, (v4u*)(obase + p.copy_off[c] + off));
            }
    }
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x)
    {
        uint64_t z = (i + seed * 0x1000000000ull) * 0x9E3779B97F4A7C15ull;  // splitmix64: uniform random bytes
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    constexpr int K = 8, M = 4;
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    const uint64_t S = 131072, rec = 32 + S;
    const bool separate = argc > 2 && atoi(argv[2]);  // one allocation per shard file (as the engine's callers)
    uint8_t *files = nullptr, *out;
    uint8_t* fsep[K + M];
    uint8_t* ok;
    if (separate) {
        for (int i = 0; i < K + M; ++i) {
            const uint64_t round = argc > 4 ? strtoull(argv[4], nullptr, 0) : 0;  // allocation size rounding
            const uint64_t bytes = round ? ((uint64_t)n * rec + round - 1) / round * round : (uint64_t)n * rec;
            CK(hipMalloc(&fsep[i], bytes));
            k_fill<<<4096, 256>>>(fsep[i], (uint64_t)n * rec, 5 + i);
        }
    } else {
        CK(hipMalloc(&files, (uint64_t)(K + M) * n * rec));
        k_fill<<<4096, 256>>>(files, (uint64_t)(K + M) * n * rec, 5);
    }
    CK(hipMalloc(&out, (uint64_t)n * K * S));
    CK(hipMalloc(&ok, n * 4));
    auto file = [&](int i) {  // body of record 0 of file i
        return separate ? fsep[i] + 32 : files + (uint64_t)i * n * rec + 32;
    };
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    const int surv[8] = {2, 3, 4, 5, 6, 7, 8, 9};
    p.base = file(surv[0]);
    p.stripe_stride = rec;
    for (int c = 0; c < 8; ++c) p.in_off[c] = (uint64_t)(file(surv[c]) - p.base);
    p.out_base = out;
    p.out_stripe_stride = K * S;
    p.out_off[0] = 0;      // data 0
    p.out_off[1] = S;      // data 1
    p.out_off[2] = (uint64_t)(file(10) - out);  // compare rows: parity 10, 11 in their files
    p.out_off[3] = (uint64_t)(file(11) - out);
    p.cmp_stripe_stride = rec;
    p.mode = GF_MODE_STORE_COMPARE;
    p.n_store = 2;
    p.ok_flags = ok;
    const bool nocopy = argc > 6 && atoi(argv[6]);  // heal shape: no copy-through
    for (int c = 0; c < 6 && !nocopy; ++c) {
        p.copy_mask |= 1u << c;
        p.copy_off[c] = (uint64_t)(2 + c) * S;
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 8; ++c)
            for (int q = 0; q < 5; ++q) p.tab[r][c][q] = 0x01020304u * (r + 1) + c * 0x10101010u + q;
    const bool match = argc > 5 && atoi(argv[5]);  // compare rows = identity of inputs 0 / 1, targets = those files
    if (match) {
        auto gm = [](uint8_t a, uint8_t b) { uint8_t r = 0; while (b) { if (b & 1) r ^= a; a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1D : 0)); b >>= 1; } return r; };
        for (int r = 2; r < 4; ++r) {
            for (int c = 0; c < 8; ++c) {
                const uint8_t co = c == r - 2 ? 1 : 0;
                auto pack = [&](int sh, int f) { uint32_t v = 0; for (int q = 0; q < 4; ++q) v |= (uint32_t)gm(co, (uint8_t)((f + q) << sh)) << (8 * q); return v; };
                p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
            }
            // the target: a copy of input r-2's file in parity file 8+r (distinct memory, equal bytes)
            CK(hipMemcpy(file(8 + r) - 32, file(surv[r - 2]) - 32, (uint64_t)n * rec, hipMemcpyDeviceToDevice));
            p.out_off[r] = (uint64_t)(file(8 + r) - out);
        }
    }
    p.C = 8; p.R = 4; p.units = S / 16; p.chunks_per_stripe = (p.units + 63) / 64;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct V { const char* name; void (*f)(const GfApplyParams); };
    std::vector<V> vs = {
        {"prod (launcher)", nullptr},
        {"wpe2 order0", k_get<8, 4, 2, 0>}, {"wpe3 order0", k_get<8, 4, 3, 0>}, {"wpe4 order0", k_get<8, 4, 4, 0>},
        {"wpe2 order1", k_get<8, 4, 2, 1>}, {"wpe3 order1", k_get<8, 4, 3, 1>}, {"wpe4 order1", k_get<8, 4, 4, 1>},
        {"wpe2 order2", k_get<8, 4, 2, 2>}, {"wpe3 order2", k_get<8, 4, 3, 2>}, {"wpe4 order2", k_get<8, 4, 4, 2>},
        {"wpe2 order3", k_get<8, 4, 2, 3>}, {"wpe3 order3", k_get<8, 4, 3, 3>},
    };
    // interleave: the engine's verify launch (10 present record files) before every GF launch
    const bool inter = argc > 3 && atoi(argv[3]);
    uint8_t* vflags;
    CK(hipMalloc(&vflags, (uint64_t)(K + M) * n));
    HashParams h;
    memset(&h, 0, sizeof(h));
    h.len = S;
    h.per_base = n;
    h.stripe_stride = rec;
    for (int q = 0; q < 4; ++q) h.key[q] = 0x0123456789abcdefull * (q + 1);
    h.digest_off = -32;
    const int present[10] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
    h.nbases = 10;
    h.n = 10ull * n;
    for (int b2 = 0; b2 < 10; ++b2) {
        h.base[b2] = file(present[b2]);
        h.flag_base[b2] = vflags + (uint64_t)present[b2] * n;
    }
    std::vector<std::vector<float>> t(vs.size());
    float hash_ms = 0;
    for (int it = 0; it < 10; ++it)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipMemset(ok, 1, n * 4));
            if (inter) {
                CK(hipMemset(vflags, 1, (uint64_t)(K + M) * n));
                CK(hipEventRecord(a));
                CK(launch_hh256(h, 0));
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&hash_ms, a, b));
            }
            CK(hipEventRecord(a));
            if (!vs[v].f) CK(launch_gf_apply_vec(p, n, 0));
            else hipLaunchKernelGGL(vs[v].f, dim3(p.chunks_per_stripe * n), dim3(64), 0, 0, p);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t[v].push_back(ms);
        }
    if (inter) printf("verify launch (10 files): %.4f ms\n", hash_ms);
    if (separate)
        for (int i = 0; i < K + M; ++i) printf("file %d at %p (mod 2 MiB %llu)\n", i, (void*)fsep[i], (unsigned long long)((uintptr_t)fsep[i] % (2u << 20)));
    std::vector<uint8_t> okh(n);
    CK(hipMemcpy(okh.data(), ok, n, hipMemcpyDeviceToHost));
    printf("ok flags of the last launch: %d of %u stripes consistent\n", (int)std::count(okh.begin(), okh.end(), 1), n);
    const double alg = (double)n * S * (8 + 2 + 2 + (nocopy ? 0 : 6));  // reads 8 + 2 compared, writes 2 rebuilt (+ 6 copied)
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("%-16s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", vs[v].name, x[x.size() / 2], x[0],
               alg / (x[x.size() / 2] * 1e-3) / 1e9, 100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
