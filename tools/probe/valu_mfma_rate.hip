// Probe: VALU issue throughput per SIMD and its overlap with i8 MFMAs on gfx950.
// Each wave runs ITER iterations of: M independent v_mfma_i32_32x32x32_i8 (M=0..1)
// plus K independent v_add_u32 (8 chains).  Grid = 256 CUs x WPS waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int M, int K>
__global__ __launch_bounds__(256) void k(int *out, int iters) {
    v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
    v16i c0 = {0}, c1 = {0};
    uint32_t x[8];
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    for (int it = 0; it < iters; it++) {
        if (M >= 1) c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        if (M >= 2) c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < K; q++) {
            asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[q & 7]) : "v"(x[(q + 3) & 7]));
        }
    }
    int s = c0[0] + c1[3];
    for (int j = 0; j < 8; j++) s += x[j];
    if (s == 0x12345) out[0] = s;
}

template <int M, int K>
float run(int wps, int iters) {
    int *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    dim3 grid(256 * wps);  // 256-thread blocks: one wave per SIMD per block
    hipLaunchKernelGGL((k<M, K>), grid, dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<M, K>), grid, dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(d);
    return ms;
}

int main() {
    const int iters = 20000;
    const double clk = 2.4e6;  // cycles per ms at 2.4 GHz
    for (int wps : {1, 2, 4}) {
        float t;
        t = run<0, 32>(wps, iters);
        printf("wps=%d  VALU only   : %.2f cycles per v_add per SIMD\n", wps, t * clk / (iters * 32.0 * wps));
        t = run<1, 0>(wps, iters);
        printf("wps=%d  MFMA only   : %.2f cycles per MFMA per SIMD\n", wps, t * clk / (iters * 1.0 * wps));
        t = run<1, 4>(wps, iters);
        printf("wps=%d  MFMA+4 VALU : %.2f cycles per iteration per SIMD\n", wps, t * clk / (iters * 1.0 * wps));
        t = run<1, 8>(wps, iters);
        printf("wps=%d  MFMA+8 VALU : %.2f cycles per iteration per SIMD\n", wps, t * clk / (iters * 1.0 * wps));
        t = run<1, 16>(wps, iters);
        printf("wps=%d  MFMA+16 VALU: %.2f cycles per iteration per SIMD\n", wps, t * clk / (iters * 1.0 * wps));
        t = run<2, 16>(wps, iters);
        printf("wps=%d  2MFMA+16 VALU: %.2f cycles per iteration per SIMD\n", wps, t * clk / (iters * 1.0 * wps));
    }
    return 0;
}
