// Which SIMD each wave of a workgroup lands on (HW_REG_HW_ID simd_id bits),
// for workgroups of W waves holding most of the LDS (one per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
template <int W>
__global__ __launch_bounds__(64 * W) void probe(uint32_t* out) {
    __shared__ uint8_t pad[120 * 1024];
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t wave = threadIdx.x >> 6;
    pad[threadIdx.x] = (uint8_t)hw;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * W + wave] = hw + pad[(threadIdx.x + 64) % (64 * W)] * 0;
}
template <int W>
void run() {
    const int blocks = 512;
    uint32_t* d; hipMalloc(&d, blocks * W * 4);
    hipLaunchKernelGGL(probe<W>, dim3(blocks), dim3(64 * W), 0, 0, d);
    uint32_t h[blocks * W];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int hist[16][4] = {};
    for (int b = 0; b < blocks; ++b)
        for (int w = 0; w < W; ++w) hist[w][(h[b * W + w] >> 4) & 3]++;
    printf("W=%d  per wave: SIMD histogram over %d workgroups; first wg hw=0x%x\n", W, blocks, h[0]);
    for (int w = 0; w < W; ++w) printf("  wave %2d: %4d %4d %4d %4d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    // relative placement: simd(w) - simd(0) mod 4
    int rel[16][4] = {};
    for (int b = 0; b < blocks; ++b)
        for (int w = 0; w < W; ++w) rel[w][(((h[b * W + w] >> 4) & 3) - ((h[b * W] >> 4) & 3) + 4) & 3]++;
    for (int w = 0; w < W; ++w) printf("  wave %2d rel: %4d %4d %4d %4d\n", w, rel[w][0], rel[w][1], rel[w][2], rel[w][3]);
    hipFree(d);
}
int main() { run<8>(); run<12>(); run<10>(); run<13>(); return 0; }
