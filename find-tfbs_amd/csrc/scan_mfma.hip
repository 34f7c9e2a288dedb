// Matrix-core scan (gfx950 v_mfma_i32_32x32x32_i8) for strands with L <= 32
// whose weights split into two int8 digits (mfma.cpp).
//
// matches (pattern.rs:141-171) scores every window i of a haplotype with
// sum_j w[j][nuc(i + j)] (N = 0, pattern.rs:119-135).  For 32 consecutive
// windows x 32 strands that is one int8 GEMM: A[window][4 j + c] = one-hot of
// the window's bases (all zero for N and past the haplotype end), B[4 j + c]
// [strand] = the strand's weight digits.  Each K chunk (8 columns) is two
// MFMAs into the same int32 accumulator: A (entries 1) x B_lo and A (entries
// 64) x B_hi, so acc = sum_j (64 a + b) = the exact score.
//
//  * A workgroup (4 waves) stages one super tile (tiles of 32 strands of equal
//    K depth: B fragments + strand metadata) in LDS; every B fragment is read
//    with one conflict-free ds_read_b128 per lane.
//  * Each wave takes haplotypes; per 32-window tile it builds the one-hot A
//    fragments once (from the packed 2-bit words and the N mask) and reuses
//    them for every strand tile of the super tile.  The strand-tile loop is
//    software-pipelined over two accumulators: the MFMAs of tile t + 1 are
//    issued before the threshold test of tile t reads its accumulator.
//  * C layout: lane l holds strand column l & 31 and windows (r & 3) + 8 (r >> 2)
//    + 4 (l >> 5), r < 16.  A max-reduce of the 16 scores against the lane's
//    min_score and one ballot gate the (rare) hit handling, which applies the
//    inner-range overlap test (range.rs:18-21 as main.rs:503 uses it) and adds
//    to the count of the strand's pattern_id slot atomically (counts are zeroed
//    before the scan), so a tile may mix slots freely.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "scan.hpp"

namespace tfbs {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kMBlock = 256;  // 4 waves, one per SIMD

// The packed words (and N-mask words) a lane needs for its window of the
// 32-window tile at i0: lane l covers window i0 + (l & 31).  Issued one tile
// ahead of use so the global-load latency overlaps the previous tile's MFMAs.
struct WinWords {
    uint32_t w[3], m[2];
};

__device__ __forceinline__ void load_window(const ScanArgs &A, const DevHap &hm, uint32_t i0, uint32_t lane,
                                            WinWords &ww) {
    const uint32_t ic = min(i0 + (lane & 31), hm.len);  // reads stay inside the +3 word pad
    const uint32_t *w = A.words + hm.word_off + (ic >> 4);
    ww.w[0] = w[0];
    ww.w[1] = w[1];
    ww.w[2] = w[2];
    if (hm.flags & HAP_HAS_N) {
        const uint32_t *m = A.nmask + hm.nmask_off + (ic >> 5);
        ww.m[0] = m[0];
        ww.m[1] = m[1];
    } else {
        ww.m[0] = ww.m[1] = 0;
    }
}

// One-hot A fragments (entries 1 and 64) of the 32-window tile at i0: in chunk
// kc, lane l covers columns 8 kc + 4 (l >> 5) + t of its window.
template <int NK>
__device__ __forceinline__ void build_onehot(const DevHap &hm, uint32_t i0, uint32_t lane, const WinWords &ww,
                                             v4i (&alo)[NK], v4i (&ahi)[NK]) {
    const uint32_t i = i0 + (lane & 31);
    const uint32_t h = lane >> 5;
    const uint32_t ic = min(i, hm.len);
    const uint32_t sh = 2 * (ic & 15);
    const uint32_t img_lo = __builtin_amdgcn_alignbit(ww.w[1], ww.w[0], sh);  // bases i .. i+15
    const uint32_t img_hi = __builtin_amdgcn_alignbit(ww.w[2], ww.w[1], sh);  // bases i+16 .. i+31
    // bases that exist and are not N
    const int32_t rem = (int32_t)hm.len - (int32_t)i;
    uint32_t vm = rem >= 32 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
    vm &= ~__builtin_amdgcn_alignbit(ww.m[1], ww.m[0], ic & 31);
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        const uint32_t img = kc < 2 ? img_lo : img_hi;
        const uint32_t code = (img >> (16 * (kc & 1) + 8 * h)) & 0xFFu;  // bases 8 kc + 4 h .. + 3
        const uint32_t vb = vm >> (8 * kc + 4 * h);
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint32_t c = (code >> (2 * t)) & 3u;
            const uint32_t d = ((vb >> t) & 1u) << (8 * c);
            alo[kc][t] = (int)d;
            ahi[kc][t] = (int)(d << 6);
        }
    }
}

template <int NK>
struct BFrag {
    v4i lo[NK], hi[NK];
    int32_t thr;
};

template <int NK>
__device__ __forceinline__ void load_tile(const char *s_img, const DevMSuper &S, uint32_t ti, uint32_t lane,
                                          BFrag<NK> &f) {
    const char *b = s_img + ti * (NK * 2 * kMFragBytes) + lane * 16;
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        f.lo[kc] = *reinterpret_cast<const v4i *>(b + (2 * kc) * kMFragBytes);
        f.hi[kc] = *reinterpret_cast<const v4i *>(b + (2 * kc + 1) * kMFragBytes);
    }
    f.thr = reinterpret_cast<const int32_t *>(s_img + S.meta_off + ti * kMMetaBytes)[lane & 31];
}

template <int NK>
__device__ __forceinline__ v16i tile_scores(const v4i (&alo)[NK], const v4i (&ahi)[NK], const BFrag<NK> &f) {
    v16i acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(alo[kc], f.lo[kc], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(ahi[kc], f.hi[kc], acc, 0, 0, 0);
    }
    return acc;
}

struct HapCtx {
    DevHap hm;
    uint32_t hap, n_inner;
    const int32_t *inner;
};

// The rare path of check_tile, out of line so that its registers do not
// constrain the hot loop; everything by value (an address-taken argument would
// route the caller's haplotype state through scratch).  One ballot per score
// register finds the registers holding hits; only those windows run the
// validity test (i + L <= len), the inner-range overlap test (range.rs:18-21 as
// main.rs:503 uses it) and the atomic count of the strand's pattern_id slot.
__device__ __noinline__ void tile_hits(v16i acc, int32_t thr, const int32_t *meta, uint32_t len, uint32_t flags,
                                       uint32_t pos_off, uint64_t count_off, uint32_t hap, uint32_t i0, uint32_t lane,
                                       const int32_t *inner, uint32_t n_inner, uint32_t *counts, const int32_t *posrel,
                                       unsigned long long *hits, uint32_t hits_wpp, uint32_t n_pat) {
    const uint32_t n = lane & 31, h = lane >> 5;
    const uint32_t L = (uint32_t)meta[32 + n];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const uint32_t i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const bool hit = acc[r] > thr && i + L <= len;
        if (__ballot(hit) == 0) continue;
        if (hit) {
            const uint32_t slot = (uint32_t)meta[64 + n];
            const int32_t p = (flags & HAP_HAS_POS) ? posrel[pos_off + i] : (int32_t)i;
            for (uint32_t k = 0; k < n_inner; k++) {
                const int32_t s = inner[2 * k];
                const uint32_t span = (uint32_t)(inner[2 * k + 1] - s);
                if ((uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span)
                    atomicAdd(counts + count_off + (uint64_t)slot * n_inner + k, 1u);
            }
            if (hits && i / 64 < hits_wpp)
                atomicOr(hits + ((size_t)hap * n_pat + (uint32_t)meta[96 + n]) * hits_wpp + i / 64, 1ull << (i & 63));
        }
    }
}

// Threshold test of one strand tile: the max of the lane's 16 scores against its
// strand's min_score, one ballot; hits go to tile_hits.
template <int NK>
__device__ __forceinline__ void check_tile(const ScanArgs &A, const DevMSuper &S, const char *s_img, uint32_t ti,
                                           const v16i &acc, int32_t thr, const HapCtx &H, uint32_t i0, uint32_t lane) {
    int32_t m = max(max(max(acc[0], acc[1]), max(acc[2], acc[3])), max(max(acc[4], acc[5]), max(acc[6], acc[7])));
    m = max(m, max(max(max(acc[8], acc[9]), max(acc[10], acc[11])), max(max(acc[12], acc[13]), max(acc[14], acc[15]))));
    if (__builtin_expect(__ballot(m > thr) == 0, 1)) return;
    tile_hits(acc, thr, reinterpret_cast<const int32_t *>(s_img + S.meta_off + ti * kMMetaBytes), H.hm.len, H.hm.flags,
              H.hm.pos_off, H.hm.count_off, H.hap, i0, lane, H.inner, H.n_inner, A.counts, A.posrel, A.hits,
              A.hits_wpp, A.n_patterns_total);
}
template <int NK, bool PIPE>
__device__ __forceinline__ void scan_super(const ScanArgs &A, const DevMSuper &S, const char *s_img, uint32_t hg,
                                           uint32_t lane, uint32_t wave) {
    constexpr uint32_t kWaves = kMBlock / 64;
    const uint32_t nt = S.tile_count;
    for (uint32_t hh = wave; hh < A.haps_per_block; hh += kWaves) {
        HapCtx H;
        H.hap = hg * A.haps_per_block + hh;
        if (H.hap >= A.n_haps) break;
        H.hm = A.haps[H.hap];
        if (H.hm.len < S.lmin) continue;
        const DevRegion rg = A.regions[H.hm.region];
        H.inner = A.inner + 2 * (size_t)rg.inner_off;
        H.n_inner = rg.n_inner;
        const uint32_t nwin = H.hm.len - S.lmin + 1;
        WinWords ww;
        load_window(A, H.hm, 0, lane, ww);
        for (uint32_t i0 = 0; i0 < nwin; i0 += kMWindows) {
            v4i alo[NK], ahi[NK];
            build_onehot<NK>(H.hm, i0, lane, ww, alo, ahi);
            if (i0 + kMWindows < nwin) load_window(A, H.hm, i0 + kMWindows, lane, ww);  // next tile's words
            if (!PIPE) {  // one tile at a time; the other waves of the SIMD hide the latencies
                for (uint32_t ti = 0; ti < nt; ti++) {
                    BFrag<NK> f;
                    load_tile<NK>(s_img, S, ti, lane, f);
                    __builtin_amdgcn_sched_barrier(0);  // every B read of the tile issues before its MFMAs
                    const v16i acc = tile_scores<NK>(alo, ahi, f);
                    check_tile<NK>(A, S, s_img, ti, acc, f.thr, H, i0, lane);
                }
                continue;
            }
            // two-stage pipeline over the strand tiles: scores of tile t + 1 are
            // in flight on the matrix core while tile t is tested
            BFrag<NK> fa, fb;
            load_tile<NK>(s_img, S, 0, lane, fa);
            v16i acc0 = tile_scores<NK>(alo, ahi, fa);
            int32_t thr0 = fa.thr;
            for (uint32_t ti = 0; ti < nt; ti += 2) {
                v16i acc1;
                int32_t thr1 = 0;
                const bool has1 = ti + 1 < nt;
                if (has1) {
                    load_tile<NK>(s_img, S, ti + 1, lane, fb);
                    acc1 = tile_scores<NK>(alo, ahi, fb);
                    thr1 = fb.thr;
                }
                check_tile<NK>(A, S, s_img, ti, acc0, thr0, H, i0, lane);
                if (!has1) break;
                if (ti + 2 < nt) {
                    load_tile<NK>(s_img, S, ti + 2, lane, fa);
                    acc0 = tile_scores<NK>(alo, ahi, fa);
                    thr0 = fa.thr;
                }
                check_tile<NK>(A, S, s_img, ti + 1, acc1, thr1, H, i0, lane);
            }
        }
    }
}

// Grid: n_msupers x ceil(n_haps / haps_per_block); dynamic LDS = the largest image.
// PIPE: software-pipelined tile loop, two workgroups (waves) per SIMD;
// otherwise a plain loop under a 4-waves-per-SIMD register budget.
template <bool PIPE>
__global__ __launch_bounds__(kMBlock, PIPE ? 2 : 4) void scan_mfma_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) int32_t smem[];
    const uint32_t sidx = blockIdx.x % A.n_msupers;
    const uint32_t hg = blockIdx.x / A.n_msupers;
    const DevMSuper S = A.msupers[sidx];
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.mimage + S.img_off / 4);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        for (uint32_t i = threadIdx.x; i < S.img_bytes / 16; i += kMBlock) dst[i] = src[i];
    }
    __syncthreads();
    const char *s_img = reinterpret_cast<const char *>(smem);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    switch (S.nk) {
    case 1: scan_super<1, PIPE>(A, S, s_img, hg, lane, wave); break;
    case 2: scan_super<2, PIPE>(A, S, s_img, hg, lane, wave); break;
    case 3: scan_super<3, PIPE>(A, S, s_img, hg, lane, wave); break;
    default: scan_super<4, PIPE>(A, S, s_img, hg, lane, wave); break;
    }
}

typedef void (*MfmaKernel)(ScanArgs);
MfmaKernel mfma_variant(int pipe) { return pipe ? scan_mfma_kernel<true> : scan_mfma_kernel<false>; }

}  // namespace

int mfma_kernel_set_lds(size_t lds_bytes, int pipe) {
    if (lds_bytes <= 64 * 1024) return TFBS_OK;
    hipError_t e = hipFuncSetAttribute((const void *)mfma_variant(pipe), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_bytes);
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("MFMA LDS attribute: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_mfma(const ScanArgs &a0, size_t lds_bytes, int pipe, uint32_t n_haps, hipStream_t stream) {
    if (n_haps == 0 || a0.n_msupers == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / a0.n_msupers - 1);
    int launches = 0;
    for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
        const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
        const uint32_t h0 = (uint32_t)(g0 * hpb);
        ScanArgs a = a0;
        a.haps = a0.haps + h0;
        a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
        a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
        hipLaunchKernelGGL(mfma_variant(pipe), dim3(a0.n_msupers * ng), dim3(kMBlock), lds_bytes, stream, a);
        launches++;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_mfma_kernel launch: ") + hipGetErrorString(e));
    return launches;
}

}  // namespace tfbs
