// Probe: operand/result layout and scale semantics of
// v_mfma_scale_f32_32x32x64_f8f6f4 with an FP4 (e2m1) A and an FP6 (e2m3) B.
// Each lane feeds raw dwords; the host checks the outputs against layout
// hypotheses.  Build: hipcc --offload-arch=gfx950 -O2 f4f6_layout.hip -o f4f6
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int SA, int SB>
__global__ void k(const uint32_t *a, const uint32_t *b, float *out) {
    const int l = threadIdx.x;
    v8i va = {0, 0, 0, 0, 0, 0, 0, 0}, vb = va;
    for (int i = 0; i < 4; i++) va[i] = a[l * 4 + i];
    for (int i = 0; i < 6; i++) vb[i] = b[l * 6 + i];
    v16f c = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(va, vb, c, 4, 2, 0, SA, 0, SB);
    for (int r = 0; r < 16; r++) out[l * 16 + r] = c[r];
}

static float fp4(uint32_t x) {
    const float mag[8] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6};
    return (x & 8 ? -1.f : 1.f) * mag[x & 7];
}
static float fp6(uint32_t x) {  // e2m3, bias 1
    const uint32_t e = (x >> 3) & 3, m = x & 7;
    const float v = e == 0 ? m / 8.f : (1 + m / 8.f) * std::ldexp(1.f, (int)e - 1);
    return (x & 32 ? -1.f : 1.f) * v;
}
static uint32_t bits(const uint32_t *w, int pos, int n) {
    uint64_t x = w[pos / 32] | ((uint64_t)w[pos / 32 + 1] << 32);
    return (uint32_t)(x >> (pos % 32)) & ((1u << n) - 1);
}

int main() {
    std::mt19937 rng(1);
    std::vector<uint32_t> a(64 * 4 + 1), b(64 * 6 + 1);
    for (auto &x : a) x = rng();
    for (auto &x : b) x = rng();
    uint32_t *da, *db;
    float *dout;
    hipMalloc(&da, a.size() * 4);
    hipMalloc(&db, b.size() * 4);
    hipMalloc(&dout, 64 * 16 * 4);
    hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
    // A[i][k], B[k][j] under the hypothesis: lane l holds row/col l & 31, k = 32 (l >> 5) + e,
    // element e at bits [4e, 4e+4) (A) / [6e, 6e+6) (B) of the lane's dwords
    std::vector<double> A(32 * 64), B(64 * 32);
    for (int l = 0; l < 64; l++)
        for (int e = 0; e < 32; e++) {
            const int k = 32 * (l >> 5) + e;
            A[(l & 31) * 64 + k] = fp4(bits(&a[l * 4], 4 * e, 4));
            B[k * 32 + (l & 31)] = fp6(bits(&b[l * 6], 6 * e, 6));
        }
    const int scales[3][2] = {{0, 0}, {127, 127}, {128, 127}};
    for (int si = 0; si < 3; si++) {
        if (si == 0) hipLaunchKernelGGL((k<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dout);
        if (si == 1) hipLaunchKernelGGL((k<127, 127>), dim3(1), dim3(64), 0, 0, da, db, dout);
        if (si == 2) hipLaunchKernelGGL((k<128, 127>), dim3(1), dim3(64), 0, 0, da, db, dout);
        std::vector<float> out(64 * 16);
        hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
        int ok = 0;
        double ratio = 0;
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < 16; r++) {
                const int i = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), j = l & 31;
                double c = 0;
                for (int kk = 0; kk < 64; kk++) c += A[i * 64 + kk] * B[kk * 32 + j];
                if (c == out[l * 16 + r]) ok++;
                if (c != 0 && ratio == 0) ratio = out[l * 16 + r] / c;
            }
        printf("scale a=%d b=%d: %d/1024 outputs match the hypothesis (first ratio %g); out[0]=%g\n", scales[si][0],
               scales[si][1], ok, ratio, out[0]);
    }
    return 0;
}
