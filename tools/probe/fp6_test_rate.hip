// Probe: throughput of the scan's inner pattern on one SIMD -- two FP4 x FP6
// MFMAs (32x32x64) and the max3 threshold tests of their results -- as
// (a) dependent: tests read this round's results (the scan's structure),
// (b) pipelined: tests read the previous round's results,
// (c) MFMA only, (d) tests only; 1-8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -ffinite-math-only -mllvm -amdgpu-mfma-vgpr-form fp6_test_rate.hip -o fp6rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float max16(const v16f &a) {
    const float t0 = fmaxf(fmaxf(a[0], a[1]), a[2]), t1 = fmaxf(fmaxf(a[3], a[4]), a[5]);
    const float t2 = fmaxf(fmaxf(a[6], a[7]), a[8]), t3 = fmaxf(fmaxf(a[9], a[10]), a[11]);
    const float t4 = fmaxf(fmaxf(a[12], a[13]), a[14]);
    return fmaxf(fmaxf(fmaxf(t0, t1), t2), fmaxf(fmaxf(t3, t4), a[15]));
}

__device__ __forceinline__ v16f mm(const v8i &a, const v8i &b, const v16f &c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 2, 0, 127, 0, 127);
}

template <int MODE>
__global__ __launch_bounds__(256) void k(int *out, int iters, float thr) {
    v8i a0 = {(int)threadIdx.x, 1, 2, 3, 0, 0, 0, 0}, a1 = {3, (int)threadIdx.x, 1, 2, 0, 0, 0, 0};
    v8i b = {5, 6, (int)threadIdx.x, 7, 8, 9, 0, 0};
    v16f z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    v16f p0 = z, p1 = z, c0 = z, c1 = z;
    for (int j = 0; j < 16; j++) { p0[j] = threadIdx.x * 0.5f + j; p1[j] = j - threadIdx.x * 0.25f; }
    int hits = 0;
    for (int it = 0; it < iters; it++) {
        b[0] += it;  // a new B every round (as a new strand tile)
        if (MODE == 0) {  // dependent
            c0 = mm(a0, b, z), c1 = mm(a1, b, z);
            hits += __ballot(max16(c0) > thr) != 0;
            hits += __ballot(max16(c1) > thr) != 0;
        } else if (MODE == 1) {  // pipelined
            c0 = mm(a0, b, z), c1 = mm(a1, b, z);
            hits += __ballot(max16(p0) > thr) != 0;
            hits += __ballot(max16(p1) > thr) != 0;
            p0 = c0;
            p1 = c1;
        } else if (MODE == 4) {  // pipelined, unrolled x2, interleaved: MFMA, 9 VALU, MFMA, 9 VALU
            b[1] += it;
            c0 = mm(a0, b, z);
            c1 = mm(a1, b, z);
            hits += __ballot(max16(p0) > thr) != 0;
            hits += __ballot(max16(p1) > thr) != 0;
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 9, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 9, 0);
            b[2] += it;
            p0 = mm(a0, b, z);
            p1 = mm(a1, b, z);
            hits += __ballot(max16(c0) > thr) != 0;
            hits += __ballot(max16(c1) > thr) != 0;
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x002, 9, 1);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
            __builtin_amdgcn_sched_group_barrier(0x002, 9, 1);
            it++;
        } else if (MODE == 2) {  // MFMA only
            p0 = mm(a0, b, p0);
            p1 = mm(a1, b, p1);
        } else {  // tests only
            hits += __ballot(max16(p0) > thr) != 0;
            hits += __ballot(max16(p1) > thr) != 0;
#pragma unroll
            for (int j = 0; j < 16; j++) asm volatile("" : "+v"(p0[j]), "+v"(p1[j]));  // no hoisting, no code
        }
    }
    if (hits == 12345 || p0[3] + p1[7] + c0[1] + c1[2] == -1.0f) out[0] = hits;
}

template <int MODE>
float run(int wps, int iters) {
    int *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    dim3 grid(256 * wps);
    hipLaunchKernelGGL((k<MODE>), grid, dim3(256), 0, 0, d, iters, 1e9f);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<MODE>), grid, dim3(256), 0, 0, d, iters, 1e9f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(d);
    return ms;
}

int main() {
    const int iters = 20000;
    const char *names[5] = {"dependent", "pipelined", "mfma_only", "tests_only", "interleave"};
    for (int wps = 1; wps <= 8; wps *= 2) {
        float t[5] = {run<0>(wps, iters), run<1>(wps, iters), run<2>(wps, iters), run<3>(wps, iters),
                      run<4>(wps, iters)};
        for (int m = 0; m < 5; m++) {
            // per SIMD: wps waves x iters rounds x 2 MFMAs (32 cycles each at 2.4 GHz nominal)
            const double mfma_ms = (double)wps * iters * 2 * 32 / 2.4e9 * 1e3;
            printf("waves/SIMD %d %-10s %8.3f ms  (MFMA-bound %.3f ms -> %.0f%%)\n", wps, names[m], t[m], mfma_ms,
                   100.0 * mfma_ms / t[m]);
        }
    }
    return 0;
}
