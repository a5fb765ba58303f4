// ring_variants.hip — fused encode + HH256S for few large stripes: the packed
// production kernel against the ring kernel at E = 1, 2 encoder waves (D = 2, 3), plus
// the unfused pair, RS(8,4), interleaved timing in one process.  Checks every
// variant's digests and parity against the packed kernel.  Not part of the
// product.  Usage: ring_variants S n [iters]
#include "../../rustfs_amd/csrc/rs_kernels.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;
#ifndef KK
#define KK 8
#endif
#ifndef MM
#define MM 4
#endif
constexpr int K = KK, M = MM;

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) { if (b & 1) r ^= a; b >>= 1; a = (a << 1) ^ ((a & 0x80) ? 0x1d : 0); }
    return r;
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

// the ring kernel with three register sets (next two chunks in flight)
static hipError_t ring_d3(GfApplyParams p, HashParams h, uint64_t S, uint64_t n, uint32_t E) {
    if (!ring_supported(K, M, S, E)) return hipErrorInvalidValue;
    auto k = k_encode_hash_ring<K, M, 3>;
    p.units = (uint32_t)(S / (kRingCol * E));
    h.n = n;
    const size_t lds = ring_lds_bytes(K, M, E);
    if (lds > 65536) CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k, dim3((uint32_t)n), dim3(64 * (E + (K + M + 15) / 16)), lds, 0, p, h, E);
    return hipGetLastError();
}

int main(int argc, char** argv) {
    const uint64_t S = argc > 1 ? strtoull(argv[1], 0, 10) : 2097152;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 10) : 256;
    const int iters = argc > 3 ? atoi(argv[3]) : 6;
    const uint64_t STRIDE = (K + M) * S;
    uint8_t *d, *dig;
    CK(hipMalloc(&d, n * STRIDE));
    CK(hipMalloc(&dig, n * (K + M) * 32));
    k_fill<<<4096, 256>>>(d, n * STRIDE, 3);
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    // any fixed invertible-looking coefficients do for timing; parity is checked between variants
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            const uint8_t co = (uint8_t)(0x1d * (r + 1) + 7 * c + 3);
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE;
    HashParams h;
    memset(&h, 0, sizeof(h));
    const uint64_t key[4] = {0xcd8a238efa34e74bull, 0x528596bbe6833e26ull, 0x14449fa35d930f04ull, 0xa036de22139de097ull};
    memcpy(h.key, key, sizeof(key));
    h.out = dig;
    h.n = n;
    HashParams hq;
    memset(&hq, 0, sizeof(hq));
    hq.data = d; hq.len = S; hq.n = n * (K + M); hq.shards = K + M; hq.shard_pitch = S; hq.stripe_stride = STRIDE;
    memcpy(hq.key, key, sizeof(key));
    hq.out = dig;
    GfApplyParams pe = p;
    pe.units = (uint32_t)(S / 16);
    struct V { const char* name; std::function<hipError_t()> f; };
    std::vector<V> vs = {
        {"packed (prod)", [&] { return launch_encode_hash_fused(p, h, S, n, 0); }},
        {"ring E=1", [&] { return launch_encode_hash_ring(p, h, S, n, 1, 0); }},
        {"ring E=2", [&] { return launch_encode_hash_ring(p, h, S, n, 2, 0); }},
        {"ring D=3 E=2", [&] { return ring_d3(p, h, S, n, 2); }},
        {"encode+quad hash", [&] { hipError_t e = launch_gf_apply_vec(pe, n, 0); return e ? e : launch_hh256(hq, 0); }},
        {"encode only", [&] { return launch_gf_apply_vec(pe, n, 0); }},
    };
    {
        const size_t nd = n * (K + M) * 32;
        std::vector<uint8_t> ref(nd), got(nd), pref(M * S), pgot(M * S);
        CK(vs[0].f());
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ref.data(), dig, nd, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pref.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
        for (size_t v = 1; v < vs.size() - 1; ++v) {
            CK(hipMemset(dig, 0, nd));
            CK(hipMemset(d + (n - 1) * STRIDE + K * S, 0, M * S));
            const hipError_t e = vs[v].f();
            if (e != hipSuccess) { printf("%s: launch %s\n", vs[v].name, hipGetErrorString(e)); continue; }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), dig, nd, hipMemcpyDeviceToHost));
            CK(hipMemcpy(pgot.data(), d + (n - 1) * STRIDE + K * S, M * S, hipMemcpyDeviceToHost));
            printf("%s: digests %s, parity %s\n", vs[v].name, memcmp(ref.data(), got.data(), nd) ? "MISMATCH" : "ok",
                   memcmp(pref.data(), pgot.data(), M * S) ? "MISMATCH" : "ok");
        }
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> t(vs.size());
    for (int it = 0; it < iters; ++it)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(a));
            if (vs[v].f() != hipSuccess) continue;
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it) t[v].push_back(ms);
        }
    const double pay = (double)n * K * S, alg = (double)n * STRIDE;
    printf("S=%llu n=%llu RS(%d,%d)\n", (unsigned long long)S, (unsigned long long)n, K, M);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        if (x.empty()) continue;
        std::sort(x.begin(), x.end());
        const double med = x[x.size() / 2];
        printf("  %-18s med %8.4f ms min %8.4f -> %7.1f GiB/s payload, %5.1f%% HBM\n", vs[v].name, med, x[0],
               pay / (med * 1e-3) / 1073741824.0, 100 * alg / (med * 1e-3) / 8e12);
    }
    return 0;
}
