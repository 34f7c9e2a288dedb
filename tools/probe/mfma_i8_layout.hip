// Probe: operand/result lane maps of v_mfma_i32_32x32x32_i8 on gfx950.
// A[32][32], B[32][32] int8; lane l supplies 16 bytes of A and of B under the
// hypothesis  A: row l&31, k = 16*(l>>5)+j ;  B: col l&31, k = 16*(l>>5)+j ;
// C: col l&31, row (r&3)+8*(r>>2)+4*(l>>5).  Prints mismatches vs the CPU product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
__global__ void k(const int8_t *A, const int8_t *B, int32_t *C) {
    int l = threadIdx.x;
    int r = l & 31, h = l >> 5;
    v4i a, b;
    int8_t *pa = (int8_t *)&a, *pb = (int8_t *)&b;
    for (int j = 0; j < 16; j++) {
        pa[j] = A[r * 32 + 16 * h + j];
        pb[j] = B[(16 * h + j) * 32 + r];
    }
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int q = 0; q < 16; q++) C[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = c[q];
}
int main() {
    int8_t A[1024], B[1024];
    int32_t C[1024], R[1024];
    unsigned s = 1;
    for (int i = 0; i < 1024; i++) { s = s * 1103515245 + 12345; A[i] = (int8_t)(s >> 16); s = s * 1103515245 + 12345; B[i] = (int8_t)(s >> 16); }
    for (int i = 0; i < 32; i++) for (int j = 0; j < 32; j++) { int t = 0; for (int q = 0; q < 32; q++) t += A[i * 32 + q] * B[q * 32 + j]; R[i * 32 + j] = t; }
    int8_t *dA, *dB; int32_t *dC;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
    hipMemcpy(dA, A, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, B, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; i++) bad += C[i] != R[i];
    printf("mfma_i32_32x32x32_i8 layout hypothesis: %d of 1024 mismatches\n", bad);
    return bad != 0;
}
