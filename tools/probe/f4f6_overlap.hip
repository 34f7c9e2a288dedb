// Probe: how much VALU issue the FP4 x FP6 v_mfma_scale_f32_32x32x64_f8f6f4
// leaves to the SIMD on gfx950 -- within one wave and across the waves of a
// SIMD.  Each wave runs ITER iterations of M independent scaled MFMAs and K
// independent v_or3_b32 (8 chains); "split" runs MFMA-only and VALU-only waves
// side by side on every SIMD.  Grid = 256 CUs x WPS waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 f4f6_overlap.hip -o f4f6_overlap
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int M, int K, bool SPLIT>
__global__ __launch_bounds__(256) void k(int *out, int iters) {
    v8i a = {(int)threadIdx.x, 1, 2, 3, 0, 0, 0, 0}, b = {3, 2, 1, (int)threadIdx.x, 5, 6, 0, 0};
    v16f c[4];
    for (int m = 0; m < 4; m++)
        for (int r = 0; r < 16; r++) c[m][r] = 8388608.0f + r;
    uint32_t x[8];
    for (int j = 0; j < 8; j++) x[j] = threadIdx.x + j;
    // SPLIT: even waves of a block do the MFMAs, odd waves the VALU
    const bool do_m = !SPLIT || ((threadIdx.x >> 6) & 1) == 0, do_v = !SPLIT || ((threadIdx.x >> 6) & 1) == 1;
    const int sa = (threadIdx.x & 32) ? 138 : 127;
    for (int it = 0; it < iters; it++) {
        if (do_m) {
#pragma unroll
            for (int m = 0; m < M; m++) c[m] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c[m], 4, 2, 0, sa, 0, 130);
        }
        if (do_v) {
#pragma unroll
            for (int q = 0; q < K; q++)
                asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[q & 7]) : "v"(x[(q + 3) & 7]), "v"(x[(q + 5) & 7]));
        }
    }
    float s = 0;
    for (int m = 0; m < M; m++) s += c[m][0] + c[m][15];
    for (int j = 0; j < 8; j++) s += (float)x[j];
    if (s == 1.2345f) out[0] = (int)s;
}

template <int M, int K, bool SPLIT>
float run(int wps, int iters) {
    int *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    dim3 grid(256 * wps);  // 256-thread blocks: one wave per SIMD per block
    hipLaunchKernelGGL((k<M, K, SPLIT>), grid, dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<M, K, SPLIT>), grid, dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(d);
    return ms;
}

int main() {
    const int iters = 20000;
    const double clk = 2.4e6;  // cycles per ms at 2.4 GHz (nominal; DVFS lowers it)
    for (int wps : {1, 2, 4}) {
        float t;
        t = run<0, 32, false>(wps, iters);
        printf("wps=%d  VALU only        : %.2f cycles per v_or3 per SIMD\n", wps, t * clk / (iters * 32.0 * wps));
        t = run<2, 0, false>(wps, iters);
        printf("wps=%d  MFMA only        : %.2f cycles per MFMA per SIMD\n", wps, t * clk / (iters * 2.0 * wps));
        for (int kk : {4, 8, 12, 16, 24}) {
            switch (kk) {
            case 4: t = run<2, 8, false>(wps, iters); break;
            case 8: t = run<2, 16, false>(wps, iters); break;
            case 12: t = run<2, 24, false>(wps, iters); break;
            case 16: t = run<2, 32, false>(wps, iters); break;
            default: t = run<2, 48, false>(wps, iters); break;
            }
            printf("wps=%d  2 MFMA + %2d VALU : %.2f cycles per MFMA per SIMD (same wave)\n", wps, 2 * kk,
                   t * clk / (iters * 2.0 * wps));
        }
        if (wps >= 2) {
            t = run<2, 16, true>(wps, iters);
            printf("wps=%d  split 2 MFMA | 16 VALU: %.2f cycles per iteration-pair per SIMD\n", wps,
                   t * clk / (iters * wps / 2.0));
            t = run<2, 32, true>(wps, iters);
            printf("wps=%d  split 2 MFMA | 32 VALU: %.2f cycles per iteration-pair per SIMD\n", wps,
                   t * clk / (iters * wps / 2.0));
        }
    }
    return 0;
}
