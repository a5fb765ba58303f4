// get_engine_probe.cpp — the GET engine (rsg_decode_records_dev) driven
// straight through the C ABI from C++ (no Python, no torch): RS(8,4), n
// records of 1 MiB blocks per shard file, shard files as separate hipMallocs,
// data shards `lost` absent.  Times whole calls with host clocks; run under
// rocprofv3 --kernel-trace for per-kernel times.  Measurement code.
// Usage: get_engine_probe [n] [lost mask] [reps] [corrupt mask]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#include "../../include/rsgpu.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define RS(x) do { int r_ = (x); if (r_ != 0) { printf("rsg error %d at %d\n", r_, __LINE__); exit(1); } } while (0)

__global__ void k_fill(uint8_t* p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed * 0x1000000000ull) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        ((uint64_t*)p)[i] = z ^ (z >> 31);
    }
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? atoi(argv[1]) : 4096;
    const unsigned lost = argc > 2 ? strtoul(argv[2], nullptr, 0) : 0x3;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const unsigned corrupt = argc > 4 ? strtoul(argv[4], nullptr, 0) : 0;  // shard files whose bodies are inverted
    const int k = 8, m = 4, t = k + m;
    const size_t S = 131072, rec = 32 + S;
    rsg_ctx* ctx;
    RS(rsg_create(0, &ctx));
    // encode n stripes in a3 layout with digests, then frame them as records
    uint8_t *st, *dig;
    CK(hipMalloc(&st, n * t * S));
    CK(hipMalloc(&dig, n * t * 32));
    k_fill<<<4096, 256>>>(st, n * t * S, 7);
    RS(rsg_encode_batch_dev(ctx, k, m, S, n, st, S, t * S, dig, RSG_HASH_HIGHWAY256S, nullptr));
    std::vector<uint8_t*> files(t);
    for (int i = 0; i < t; ++i) {
        CK(hipMalloc(&files[i], n * rec));
        CK(hipMemcpy2D(files[i], rec, dig + i * 32, t * 32, 32, n, hipMemcpyDeviceToDevice));
        CK(hipMemcpy2D(files[i] + 32, rec, st + i * S, t * S, S, n, hipMemcpyDeviceToDevice));
    }
    for (int i = 0; i < t; ++i)
        if ((corrupt >> i) & 1) k_fill<<<4096, 256>>>(files[i] + 32, n * rec - 64, 99 + i);  // rotten records
    CK(hipFree(st));
    CK(hipFree(dig));
    uint8_t* out;
    CK(hipMalloc(&out, n * k * S));
    std::vector<const uint8_t*> in(t);
    for (int i = 0; i < t; ++i) in[i] = (lost >> i) & 1 ? nullptr : files[i];
    std::vector<int> status(n);
    CK(hipDeviceSynchronize());
    for (int r = 0; r < reps; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        RS(rsg_decode_records_dev(ctx, k, m, S, n, in.data(), RSG_HASH_HIGHWAY256S, 1, out, status.data(), nullptr));
        auto t1 = std::chrono::steady_clock::now();
        int bad = 0;
        for (size_t s = 0; s < n; ++s) bad += status[s] != 0;
        printf("call %d: %.3f ms, %d stripes not ok\n", r, std::chrono::duration<double, std::milli>(t1 - t0).count(), bad);
    }
    rsg_destroy(ctx);
    return 0;
}
