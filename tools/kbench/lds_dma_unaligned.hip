// lds_dma_unaligned.hip — can global_load_lds_dwordx4 take a source address
// that is not 16-byte aligned (RS(12,4) records: 32 + 87382 = 87414 bytes,
// so record bodies sit at every alignment mod 16)?  Checks the bytes that
// land in LDS against the source for offsets 0..15, then times a streaming
// read through an LDS ring at offset 0 and 6.  Measurement code.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_probe(const uint8_t* src, uint8_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    const uint32_t lane = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src + i * 1024 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(lds + i * 1024), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    for (int i = lane; i < 4096; i += 64) out[i] = lds[i];
}

// streaming read: each workgroup walks `per` KiB rows through a 4-slot ring
__global__ void k_stream(const uint8_t* src, uint64_t per, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 1024 * 4];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint8_t* base = src + (uint64_t)blockIdx.x * per * 1024 * 4 + w * 1024;
    uint32_t acc = 0;
    for (uint64_t r = 0; r < per; ++r) {
        __builtin_amdgcn_global_load_lds((const void*)(base + r * 4096 + lane * 16),
                                         (__attribute__((address_space(3))) void*)(lds + (r & 3) * 4096 + w * 1024),
                                         16, 0, 0);
        if (r >= 2) {
            __builtin_amdgcn_s_waitcnt(0x0F72);  // vmcnt(2)
            acc ^= *(const uint32_t*)(lds + ((r - 2) & 3) * 4096 + w * 1024 + lane * 16);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const size_t N = 1 << 20;
    uint8_t *h = (uint8_t*)malloc(N), *d, *o;
    uint8_t got[4096];
    for (size_t i = 0; i < N; ++i) h[i] = (uint8_t)(i * 131 + (i >> 8) * 7 + 3);
    CK(hipMalloc((void**)&d, N));
    CK(hipMalloc((void**)&o, 4096));
    CK(hipMemcpy(d, h, N, hipMemcpyHostToDevice));
    for (int off = 0; off < 16; ++off) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d + 64 + off, o);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got, o, 4096, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < 4096; ++i) bad += got[i] != h[64 + off + i];
        printf("offset %2d: %s (%d bytes differ)\n", off, bad ? "WRONG" : "exact", bad);
    }
    const size_t big = (size_t)4 << 30;
    uint8_t* b;
    uint32_t* sink;
    CK(hipMalloc((void**)&b, big + 64));
    CK(hipMalloc((void**)&sink, 64));
    CK(hipMemset(b, 1, big + 64));
    const uint64_t per = 1024;  // rows of 4 KiB per workgroup
    const uint32_t blocks = (uint32_t)(big / (per * 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int off : {0, 6, 0, 6}) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, b + off, per, sink);
        CK(hipEventRecord(e0));
        for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(256), 0, 0, b + off, per, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("stream offset %d: %.3f ms per 4 GiB read = %.1f GB/s\n", off, ms / 10, big / (ms / 10 * 1e-3) / 1e9);
    }
    return 0;
}
