// copy_probe.hip — PCIe rates of the host-batch PUT pipeline's copy shapes
// (rsg_encode_batch_host_submit) between page-locked host memory and HBM:
// 1-D vs 2-D (pitched rows) H2D of the data shards, D2H of the parity shards
// as one 2-D copy or m narrow ones, and both directions at once.
// Measurement code.  Usage: copy_probe [blocks] [k] [m]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? atoi(argv[1]) : 64;
    const int k = argc > 2 ? atoi(argv[2]) : 8, m = argc > 3 ? atoi(argv[3]) : 4;
    const size_t S = (1 << 20) / k, stride = (k + m) * S, total = n * stride;
    uint8_t *h, *h2, *d, *d2;
    CK(hipHostMalloc((void**)&h, total, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h2, total, hipHostMallocDefault));
    CK(hipMalloc((void**)&d, total));
    CK(hipMalloc((void**)&d2, total));
    for (size_t i = 0; i < total; i += 4096) h[i] = (uint8_t)i, h2[i] = (uint8_t)(i >> 12);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Case { const char* name; double bytes; std::function<void()> run; };
    std::vector<Case> cases = {
        {"H2D 1-D whole stripes (k+m)", (double)total, [&] { CK(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s1)); }},
        {"H2D 1-D data bytes only", (double)n * k * S, [&] { CK(hipMemcpyAsync(d, h, n * k * S, hipMemcpyHostToDevice, s1)); }},
        {"H2D 2-D data rows (prod)", (double)n * k * S,
         [&] { CK(hipMemcpy2DAsync(d, stride, h, stride, k * S, n, hipMemcpyHostToDevice, s1)); }},
        {"D2H 1-D parity bytes", (double)n * m * S, [&] { CK(hipMemcpyAsync(h, d, n * m * S, hipMemcpyDeviceToHost, s1)); }},
        {"D2H 2-D parity rows (1 copy)", (double)n * m * S,
         [&] { CK(hipMemcpy2DAsync(h + k * S, stride, d + k * S, stride, m * S, n, hipMemcpyDeviceToHost, s1)); }},
        {"D2H 2-D per parity shard (prod)", (double)n * m * S,
         [&] {
             for (int p = 0; p < m; ++p)
                 CK(hipMemcpy2DAsync(h + (k + p) * S, stride, d + (k + p) * S, stride, S, n, hipMemcpyDeviceToHost, s1));
         }},
        {"D2H per-stripe 1-D parity", (double)n * m * S,
         [&] {
             for (size_t i = 0; i < n; ++i)
                 CK(hipMemcpyAsync(h + i * stride + k * S, d + i * stride + k * S, m * S, hipMemcpyDeviceToHost, s1));
         }},
        {"H2D 2-D data + D2H 2-D parity, 2 streams", (double)n * (k + m) * S,
         [&] {
             CK(hipMemcpy2DAsync(d, stride, h, stride, k * S, n, hipMemcpyHostToDevice, s1));
             CK(hipMemcpy2DAsync(h2 + k * S, stride, d2 + k * S, stride, m * S, n, hipMemcpyDeviceToHost, s2));
         }},
        {"H2D 1-D + D2H 1-D same size, 2 streams", (double)2 * n * k * S,
         [&] {
             CK(hipMemcpyAsync(d, h, n * k * S, hipMemcpyHostToDevice, s1));
             CK(hipMemcpyAsync(h2, d2, n * k * S, hipMemcpyDeviceToHost, s2));
         }},
    };
    for (auto& c : cases) {
        std::vector<float> t;
        for (int it = 0; it < 8; ++it) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a, s1));
            CK(hipStreamWaitEvent(s2, a, 0));
            c.run();
            CK(hipEventRecord(b, s2));
            CK(hipStreamWaitEvent(s1, b, 0));
            CK(hipEventRecord(b, s1));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (it > 1) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-42s %7.1f MiB  med %.3f ms -> %.1f GB/s\n", c.name, c.bytes / (1 << 20), t[t.size() / 2],
               c.bytes / (t[t.size() / 2] * 1e-3) / 1e9);
    }
    return 0;
}
