// lib_encode.cpp — rsg_encode_batch_dev from plain C++ (no torch): RS(8,4),
// 1 MiB stripes, n stripes in one hipMalloc buffer, 20 back-to-back calls with
// events between, on the null stream and on a created stream.  Separates the
// library kernel's speed from the Python/torch process around it.  Not part of
// the product.  Build: hipcc -O2 lib_encode.cpp -I../../include -L../../rustfs_amd -lrsgpu
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "rsgpu.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 4096, S = 131072, stride = 12 * S;
    uint8_t* d;
    CK(hipMalloc(&d, n * stride));
    k_fill<<<4096, 256>>>(d, n * stride, 9);
    CK(hipDeviceSynchronize());
    rsg_ctx* ctx;
    if (rsg_create(0, &ctx)) { printf("rsg_create failed\n"); return 1; }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (hipStream_t s : {st, (hipStream_t)0, st, (hipStream_t)0}) {
        for (int i = 0; i < 3; ++i) rsg_encode_batch_dev(ctx, 8, 4, S, n, d, S, stride, nullptr, 0, s);
        std::vector<hipEvent_t> ev(21);
        for (auto& e : ev) CK(hipEventCreate(&e));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(ev[0], s));
        for (int i = 0; i < 20; ++i) {
            if (rsg_encode_batch_dev(ctx, 8, 4, S, n, d, S, stride, nullptr, 0, s)) { printf("encode failed\n"); return 1; }
            CK(hipEventRecord(ev[i + 1], s));
        }
        CK(hipEventSynchronize(ev[20]));
        float tot = 0;
        for (int i = 0; i < 20; ++i) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            tot += ms;
        }
        printf("%s stream: avg %.4f ms per encode of %zu stripes -> %.1f GB/s\n", s ? "created" : "null", tot / 20, n,
               n * stride / (tot / 20 * 1e-3) / 1e9);
    }
    rsg_destroy(ctx);
    return 0;
}
