// block_probe.hip — the production encode kernel's body (k_gf_apply_vec) at
// workgroup sizes 64 / 128 / 256 threads, same block -> (stripe, column)
// order.  Measurement code.  Usage: block_probe [n] [k] [m]
#include "../../rustfs_amd/csrc/rs_kernels.hip"
#include "../../rustfs_amd/csrc/gf_bitslice.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace rsg;

template <int C, int R, int B, int WPE>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_vec_b(const GfApplyParams p) {
    const uint32_t stripe = blockIdx.x / p.chunks_per_stripe;
    const uint32_t chunk = blockIdx.x - stripe * p.chunks_per_stripe;
    const uint8_t* sbase = p.base + (uint64_t)stripe * p.stripe_stride;
    uint8_t* obase = p.out_base + (uint64_t)stripe * p.out_stripe_stride;
    const uint32_t u = chunk * B + threadIdx.x;
    if (u >= p.units) return;
    const uint64_t off = (uint64_t)u * 16u;
    uint4 x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = ld16(sbase + p.in_off[c] + off);
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0u;
    gf_accumulate<0, C, R>(p, x, acc);
    gf_store<R>(p, obase, off, acc, stripe);
}

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x)
        ((uint64_t*)p)[i] = (i + seed) * 0x9E3779B97F4A7C15ull;
}

template <int K, int M>
int run(uint32_t n, uint64_t S) {
    const uint64_t STRIDE = (K + M) * S;
    uint8_t* d;
    CK(hipMalloc(&d, (uint64_t)n * STRIDE));
    k_fill<<<4096, 256>>>(d, (uint64_t)n * STRIDE, 3);
    constexpr bs::EncodeRows<K, M> E{};
    GfApplyParams p;
    memset(&p, 0, sizeof(p));
    p.base = d; p.out_base = d; p.stripe_stride = STRIDE; p.out_stripe_stride = STRIDE;
    for (int c = 0; c < K; ++c) p.in_off[c] = c * S;
    for (int r = 0; r < M; ++r) p.out_off[r] = (K + r) * S;
    for (int r = 0; r < M; ++r)
        for (int c = 0; c < K; ++c) {
            const uint8_t co = E.g[r][c];
            auto pack = [&](int sh, int f) { uint32_t v = 0; for (int i = 0; i < 4; ++i) v |= (uint32_t)bs::gmul(co, (uint8_t)((f + i) << sh)) << (8 * i); return v; };
            p.tab[r][c][0] = pack(0, 0); p.tab[r][c][1] = pack(0, 4); p.tab[r][c][2] = pack(3, 0); p.tab[r][c][3] = pack(3, 4); p.tab[r][c][4] = pack(6, 0);
        }
    p.C = K; p.R = M; p.mode = GF_MODE_STORE; p.units = S / 16;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct V { const char* name; int B; void (*f)(const GfApplyParams); };
    std::vector<V> vs = {
        {"prod 256", 256, nullptr},
        {"B64 w4", 64, k_vec_b<K, M, 64, 4>},
        {"B64 w8", 64, k_vec_b<K, M, 64, 8>},
        {"B128 w4", 128, k_vec_b<K, M, 128, 4>},
        {"B256 w4", 256, k_vec_b<K, M, 256, 4>},
        {"B64 w2", 64, k_vec_b<K, M, 64, 2>},
        {"B512 w4", 512, k_vec_b<K, M, 512, 4>},
    };
    std::vector<std::vector<float>> t(vs.size());
    std::vector<uint8_t> ref(M * S), got(M * S);
    for (int it = 0; it < 12; ++it)
        for (size_t v = 0; v < vs.size(); ++v) {
            GfApplyParams q = p;
            q.chunks_per_stripe = (q.units + vs[v].B - 1) / vs[v].B;
            CK(hipEventRecord(a));
            if (!vs[v].f) CK(launch_gf_apply_vec(p, n, 0));
            else hipLaunchKernelGGL(vs[v].f, dim3(q.chunks_per_stripe * n), dim3(vs[v].B), 0, 0, q);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t[v].push_back(ms);
            if (it == 0) {
                CK(hipMemcpy(v == 0 ? ref.data() : got.data(), d + (uint64_t)(n - 1) * STRIDE + K * S, M * S,
                             hipMemcpyDeviceToHost));
                if (v > 0 && memcmp(ref.data(), got.data(), M * S)) printf("%s: PARITY MISMATCH\n", vs[v].name);
            }
        }
    const double alg = (double)n * STRIDE;
    for (size_t v = 0; v < vs.size(); ++v) {
        auto& x = t[v];
        std::sort(x.begin(), x.end());
        printf("RS(%d,%d) S=%llu n=%u %-10s med %.4f ms min %.4f -> %.1f GB/s (%.1f%%)\n", K, M, (unsigned long long)S,
               n, vs[v].name, x[x.size() / 2], x[0], alg / (x[x.size() / 2] * 1e-3) / 1e9,
               100 * alg / (x[x.size() / 2] * 1e-3) / 8e12);
    }
    CK(hipFree(d));
    return 0;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 4096;
    run<8, 4>(n, 131072);
    run<4, 2>(n, 262144);
    run<8, 1>(n, 131072);
    return 0;
}
