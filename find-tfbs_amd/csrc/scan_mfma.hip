// Matrix-core scan (gfx950 v_mfma_i32_32x32x32_i8) for strands with L <= 32
// whose weights stay within 127 x 255 (mfma.cpp).
//
// matches (pattern.rs:141-171) scores every window i of a haplotype with
// sum_j w[j][nuc(i + j)] (N = 0, pattern.rs:119-135).  For 32 consecutive
// windows x 32 strands that is one int8 GEMM: A[window][k] = one-hot of the
// window's bases (all zero for N), B[k][strand] = the strand's weights.  The
// weights split as w = s q + r (per-strand scale s, int8 q and r): a K chunk
// of 32 covers 8 columns of the coarse digits q, so one MFMA per 8 columns
// gives Q; Q > thr_q is necessary for a hit (mfma.cpp), and the rare tiles
// that pass it are rescored exactly as s Q + one-hot x r.
//
//  * A workgroup (4 waves, 4 workgroups per CU) stages one super tile (tiles of
//    32 strands of equal K depth: coarse and residual B fragments + strand
//    metadata), the one-hot table and the packed words of its haplotypes in
//    LDS.  Every B fragment is one conflict-free ds_read_b128 per lane.
//  * Each wave takes haplotypes; per 32-window tile it builds the A fragments
//    once (one table read per chunk) and reuses them for every strand tile of
//    the super tile, two window tiles per B fragment read.
//  * C layout: lane l holds strand column l & 31 and windows (r & 3) + 8 (r >> 2)
//    + 4 (l >> 5), r < 16.  A max-reduce of the 16 coarse sums against the
//    lane's thr_q and one ballot gate the exact rescore; its max against
//    min_score and a second ballot gate the (rare, ~1e-4 per window and
//    strand) hit handling, which applies the inner-range overlap test
//    (range.rs:18-21 as main.rs:503 uses it) and adds to the count of the
//    strand's pattern_id slot atomically (counts are zeroed before the scan),
//    so a tile may mix slots.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "scan.hpp"

namespace tfbs {
namespace {

// Bottleneck probes (tools/probe_build.sh, never in the product build):
// TFBS_MFMA_PROBE=1 skips the threshold test (scores kept live), =2 reads every
// B fragment from tile 0, =3 skips the hit handling (results wrong; timing only),
// =4 counts hit-path entries, hits and invalid-window hits (printed per launch),
// =5 enters the hit path and returns at once, =6 keeps one B fragment set in
// registers instead of reading each tile's from LDS.
#ifndef TFBS_MFMA_PROBE
#define TFBS_MFMA_PROBE 0
#endif
// TFBS_MFMA_PIPE=1: software-pipelined strand loop (tests of tile t-1 after the
// MFMAs of tile t)
#ifndef TFBS_MFMA_PIPE
#define TFBS_MFMA_PIPE 0
#endif

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kMBlock = 256;          // 4 waves
constexpr int kMOnehotBytes = 4096;   // LDS: one-hot table, image, words
constexpr uint32_t kMStagedMax = 40 * 1024;  // LDS per workgroup at 4 workgroups per CU (160 KiB)
// per K depth (chunks of 8 columns): window tiles per step and the waves per
// SIMD the kernel is compiled for (the registers of two A sets + two
// accumulators)
constexpr uint32_t kMfmaWindowTiles[kMMaxChunks + 1] = {1, 2, 2, 2, 2};
// waves per SIMD the depth kernels' registers allow (see mfma_depth_budgets)
constexpr uint32_t kMfmaRegWaves[kMMaxChunks + 1] = {4, 6, 5, 4, 4};
constexpr int kMfmaMinWaves[kMMaxChunks + 1] = {4, 4 - TFBS_MFMA_PIPE, 4 - TFBS_MFMA_PIPE, 4 - TFBS_MFMA_PIPE, 4 - TFBS_MFMA_PIPE};

// The packed words (and N-mask words) a lane needs for its window of the
// 32-window tile at i0 (lane l covers window i0 + (l & 31)), read one tile
// ahead of use.
struct WinWords {
    uint32_t w[3], m[2];
};

__device__ __forceinline__ void load_window(const ScanArgs &A, const uint32_t *words, const DevHap &hm, uint32_t i0,
                                            uint32_t lane, WinWords &ww) {
    const uint32_t ic = min(i0 + (lane & 31), hm.len);  // reads stay inside the +3 word pad
    const uint32_t *w = words + hm.word_off + (ic >> 4);
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

// A fragments of the 32-window tile at i0: chunk kc, lane half h = lane >> 5:
// columns 8 kc + 4 h .. + 3 of the lane's window as one-hot bytes, read from
// the LDS table by the 4-mer code; N bases zeroed in haplotypes that have them.
template <int NK>
__device__ __forceinline__ void build_onehot(const DevHap &hm, uint32_t i0, uint32_t lane, const WinWords &ww,
                                             const char *s_onehot, v4i (&a)[NK]) {
    const uint32_t i = i0 + (lane & 31);
    const uint32_t ic = min(i, hm.len);
    const uint32_t sh = 2 * (ic & 15);
    const uint32_t img_lo = __builtin_amdgcn_alignbit(ww.w[1], ww.w[0], sh);  // bases i .. i+15
    const uint32_t img_hi = __builtin_amdgcn_alignbit(ww.w[2], ww.w[1], sh);  // bases i+16 .. i+31
    const uint32_t hb = 8 * (lane >> 5);
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        const uint32_t code = __builtin_amdgcn_ubfe(kc < 2 ? img_lo : img_hi, 16 * (kc & 1) + hb, 8);
        a[kc] = *reinterpret_cast<const v4i *>(s_onehot + code * 16);
    }
    // Bases past the haplotype end need no mask: they only reach windows with
    // i + L > len (rejected in tile_hits) or columns >= L (zero weights).
    if (hm.flags & HAP_HAS_N) {  // N scores 0 (pattern.rs:119-135): clear its one-hot
        const uint32_t vm = ~__builtin_amdgcn_alignbit(ww.m[1], ww.m[0], ic & 31) >> (hb / 2);
#pragma unroll
        for (int kc = 0; kc < NK; kc++)
#pragma unroll
            for (int t = 0; t < 4; t++) a[kc][t] = ((vm >> (8 * kc + t)) & 1u) ? a[kc][t] : 0;
    }
}

template <int NK>
struct BFrag {
    v4i b[NK];
    int32_t thr;
};

template <int NK>
__device__ __forceinline__ void load_tile(const char *s_img, const DevMSuper &S, uint32_t ti, uint32_t lane,
                                          BFrag<NK> &f) {
#if TFBS_MFMA_PROBE == 6
    (void)s_img;
    (void)S;
    (void)ti;
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        f.b[kc] = v4i{(int)lane, (int)kc, 1, 2};
        asm volatile("" : "+v"(f.b[kc]));
    }
    f.thr = 1 << 30;
    return;
#endif
    const char *p = s_img + (TFBS_MFMA_PROBE == 2 ? 0 : ti) * (2 * NK * kMFragBytes) + lane * 16;
#pragma unroll
    for (int kc = 0; kc < NK; kc++) f.b[kc] = *reinterpret_cast<const v4i *>(p + kc * kMFragBytes);
    f.thr = reinterpret_cast<const int32_t *>(s_img + S.meta_off + ti * kMMetaBytes)[kMetaThrQ + (lane & 31)];
}

template <int NK>
__device__ __forceinline__ v16i tile_scores(const v4i (&a)[NK], const BFrag<NK> &f) {
    v16i acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kc = 0; kc < NK; kc++) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kc], f.b[kc], acc, 0, 0, 0);
    return acc;
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// haplotype / region descriptors as wave-uniform (SGPR) values
__device__ __forceinline__ DevHap load_hap(const DevHap *p) {
    DevHap h = *p;
    h.word_off = uni(h.word_off);
    h.len = uni(h.len);
    h.region = uni(h.region);
    h.flags = uni(h.flags);
    h.nmask_off = uni(h.nmask_off);
    h.pos_off = uni(h.pos_off);
    h.count_off = ((uint64_t)uni((uint32_t)(h.count_off >> 32)) << 32) | uni((uint32_t)h.count_off);
    return h;
}

// Hit-handling context in LDS, so that the out-of-line rare path takes only
// the scores and a few scalars as arguments (all in registers, no scratch).
struct KernelHitCtx {
    uint32_t *counts;
    const int32_t *posrel;
    unsigned long long *hits;
    uint32_t hits_wpp, n_pat;
};
struct WaveHitCtx {  // written by the wave at each haplotype
    const int32_t *inner;  // global inner ranges of the haplotype's region
    uint64_t count_off;
    uint32_t len, flags, pos_off, hap, n_inner;
    int32_t inner_lds;     // the same ranges at s_inner[inner_lds], or -1
};
constexpr int kMMaxWaves = 8;
constexpr uint32_t kMInnerMax = 64;  // inner ranges of a workgroup's regions kept in LDS
__shared__ KernelHitCtx s_kctx;
__shared__ WaveHitCtx s_wctx[kMMaxWaves];
__shared__ int32_t s_inner[2 * kMInnerMax];
__shared__ uint32_t s_inner_base;    // inner_off of s_inner[0], or UINT32_MAX when not staged
// Per-wave log of the counts a haplotype's hits add to (offsets from its
// count_off), flushed as one batch of global atomics after the haplotype, so
// that the hit path issues no global memory operation.
constexpr uint32_t kMLog = 64;
__shared__ uint32_t s_log[kMMaxWaves][kMLog];
__shared__ uint32_t s_log_n[kMMaxWaves];
extern __shared__ __attribute__((aligned(16))) int32_t s_mdyn[];  // one-hot tables | image | words

#if TFBS_MFMA_PROBE == 4
__device__ unsigned long long g_probe[5];
#endif

// The rare path of check_tile (about one tile in ten), out of line and compact
// so that neither its registers nor its code crowd the hot loop.  Each lane
// collects a 16-bit mask of its registers above its strand's threshold (bit
// 15 - r for register r = window i0 + (r & 3) + 8 (r >> 2) + 4 (lane >> 5)),
// then walks the set bits: the window validity test (i + L <= len), the
// inner-range overlap test (range.rs:18-21 as main.rs:503 uses it) and the
// atomic count of the strand's slot.  meta_off: LDS byte offset of the tile's
// strand metadata (MMeta fields, 32 each); acc: exact scores, thr: min_score.
__device__ __noinline__ void tile_hits(v16i acc, int32_t thr, uint32_t meta_off, uint32_t i0) {
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) m = __builtin_amdgcn_alignbit(m, (uint32_t)(thr - acc[r]), 31);
    m &= 0xFFFFu;
#if TFBS_MFMA_PROBE == 5
    asm volatile("" ::"v"(m));
    return;
#endif
    const uint32_t lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
    const WaveHitCtx &W = s_wctx[uni(threadIdx.x >> 6)];
    const int32_t *meta = reinterpret_cast<const int32_t *>(reinterpret_cast<const char *>(s_mdyn) + meta_off);
    const uint32_t L = (uint32_t)meta[kMetaLen + n];
#if TFBS_MFMA_PROBE == 4
    if (lane == 0) atomicAdd(&g_probe[0], 1ull);
    for (uint32_t q = m; q; q &= q - 1) {
        const uint32_t r = 15 - (31 - __builtin_clz(q & -q));
        const uint32_t i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        atomicAdd(&g_probe[i + L <= W.len ? 1 : 2], 1ull);
    }
#endif
    if (m == 0) return;
    const uint32_t len = W.len, flags = W.flags, pos_off = W.pos_off, n_inner = W.n_inner;
    const int32_t il = W.inner_lds;
    const uint32_t slot = (uint32_t)meta[kMetaSlot + n];
    const uint32_t wave = uni(threadIdx.x >> 6);
    const uint32_t off0 = slot * n_inner;
#pragma unroll 1
    do {
        const uint32_t b = 31 - __builtin_clz(m & -m);  // lowest set bit
        m &= m - 1;
        const uint32_t r = 15 - b;
        const uint32_t i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i + L > len) continue;
        const int32_t p = (flags & HAP_HAS_POS) ? s_kctx.posrel[pos_off + i] : (int32_t)i;
#pragma unroll 1
        for (uint32_t k = 0; k < n_inner; k++) {
            const int32_t s = il >= 0 ? s_inner[il + 2 * k] : W.inner[2 * k];
            const int32_t e = il >= 0 ? s_inner[il + 2 * k + 1] : W.inner[2 * k + 1];
            const uint32_t span = (uint32_t)(e - s);
            if ((uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span) {
                const uint32_t at = atomicAdd(&s_log_n[wave], 1u);
                if (at < kMLog) s_log[wave][at] = off0 + k;
                else atomicAdd(s_kctx.counts + W.count_off + off0 + k, 1u);  // log full
            }
        }
        unsigned long long *hits = s_kctx.hits;
        const uint32_t wpp = s_kctx.hits_wpp;
        if (hits && i / 64 < wpp)
            atomicOr(hits + ((size_t)W.hap * s_kctx.n_pat + (uint32_t)meta[kMetaOrig + n]) * wpp + i / 64, 1ull << (i & 63));
    } while (m);
}

__device__ __forceinline__ int32_t max16(const v16i &acc) {
    int32_t m = max(max(max(acc[0], acc[1]), max(acc[2], acc[3])), max(max(acc[4], acc[5]), max(acc[6], acc[7])));
    return max(m, max(max(max(acc[8], acc[9]), max(acc[10], acc[11])), max(max(acc[12], acc[13]), max(acc[14], acc[15]))));
}

// Threshold test of one strand tile: the max of the lane's 16 coarse sums
// against its strand's thr_q, one ballot.  The tiles that pass (about one in
// eight) are rescored exactly, s Q + one-hot x r with the residual fragments,
// and their scores above min_score go to tile_hits.
template <int NK>
__device__ __forceinline__ void check_tile(const char *s_img, const DevMSuper &S, uint32_t ti, const v16i &acc,
                                           int32_t thr, const v4i (&a)[NK], uint32_t i0, uint32_t lane) {
    if (TFBS_MFMA_PROBE == 1) {
        asm volatile("" ::"v"(acc[0]), "v"(acc[5]), "v"(acc[10]), "v"(acc[15]));
        return;
    }
#if TFBS_MFMA_PROBE == 4
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_probe[3], 1ull);
#endif
    if (__builtin_expect(__ballot(max16(acc) > thr) == 0, 1)) return;
    if (TFBS_MFMA_PROBE == 3) return;
#if TFBS_MFMA_PROBE == 4
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_probe[4], 1ull);
#endif
    const uint32_t meta_off = S.meta_off + ti * kMMetaBytes;
    const int32_t *meta = reinterpret_cast<const int32_t *>(s_img + meta_off);
    const int32_t sc = meta[kMetaScale + (lane & 31)], mn = meta[kMetaMin + (lane & 31)];
    const char *p = s_img + ti * (2 * NK * kMFragBytes) + NK * kMFragBytes + lane * 16;
    v4i br[NK];
#pragma unroll
    for (int kc = 0; kc < NK; kc++) br[kc] = *reinterpret_cast<const v4i *>(p + kc * kMFragBytes);
    v16i ex;
#pragma unroll
    for (int r = 0; r < 16; r++) ex[r] = __mul24(acc[r], sc);  // |Q| <= 127 x 32, s <= 255
#pragma unroll
    for (int kc = 0; kc < NK; kc++) ex = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[kc], br[kc], ex, 0, 0, 0);
    if (__ballot(max16(ex) > mn) == 0) return;
    tile_hits(ex, mn, kMOnehotBytes + meta_off, i0);
}

// Coarse sums of strand tile ti for two window tiles (one B fragment read
// feeds both MFMAs).
template <int NK>
__device__ __forceinline__ void pair_scores(const char *s_img, const DevMSuper &S, uint32_t ti, uint32_t lane,
                                            const v4i (&a0)[NK], const v4i (&a1)[NK], v16i &c0, v16i &c1,
                                            int32_t &thr) {
    BFrag<NK> f;
    load_tile<NK>(s_img, S, ti, lane, f);
    __builtin_amdgcn_sched_barrier(0);  // every B read of the tile issues before its MFMAs
    c0 = v16i{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    c1 = c0;
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[kc], f.b[kc], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[kc], f.b[kc], c1, 0, 0, 0);
    }
    thr = f.thr;
}

// words: the packed haplotype words, indexed by DevHap::word_off (an LDS copy
// of this workgroup's haplotypes, biased by their first word, or global memory).
template <int NK>
__device__ __forceinline__ void scan_super(const ScanArgs &A, const DevMSuper &S, const char *s_img,
                                           const uint32_t *words, uint32_t hg, uint32_t lane, uint32_t wave) {
    constexpr uint32_t kWaves = kMBlock / 64;
    const uint32_t nt = S.tile_count;
    for (uint32_t hh = wave; hh < A.haps_per_block; hh += kWaves) {
        const uint32_t hap = hg * A.haps_per_block + hh;
        if (hap >= A.n_haps) break;
        const DevHap hm = load_hap(A.haps + hap);
        if (hm.len < S.lmin) continue;
        const DevRegion rg = A.regions[hm.region];
        {  // every lane stores the same (uniform) values
            WaveHitCtx &W = s_wctx[wave];
            const uint32_t io = uni(rg.inner_off), ib = s_inner_base;
            W.inner = A.inner + 2 * (size_t)io;
            W.inner_lds = ib == UINT32_MAX ? -1 : (int32_t)(2 * (io - ib));
            W.count_off = hm.count_off;
            W.len = hm.len;
            W.flags = hm.flags;
            W.pos_off = hm.pos_off;
            W.hap = hap;
            W.n_inner = uni(rg.n_inner);
        }
        const uint32_t nwin = hm.len - S.lmin + 1;
        const char *tab = s_img - kMOnehotBytes;
        // window tiles two at a time, so that each B fragment read from LDS
        // feeds two MFMAs (the LDS read rate, not the matrix core, bounds one
        // read per MFMA)
        constexpr uint32_t kStep = kMfmaWindowTiles[NK] * kMWindows;
        WinWords ww0, ww1;
        load_window(A, words, hm, 0, lane, ww0);
        if (kStep > kMWindows && kMWindows < nwin) load_window(A, words, hm, kMWindows, lane, ww1);
        for (uint32_t i0 = 0; i0 < nwin; i0 += kStep) {
            const bool two = kStep > kMWindows && i0 + kMWindows < nwin;
            v4i a0[NK], a1[NK];
            build_onehot<NK>(hm, i0, lane, ww0, tab, a0);
            if (two) build_onehot<NK>(hm, i0 + kMWindows, lane, ww1, tab, a1);
            if (i0 + kStep < nwin) load_window(A, words, hm, i0 + kStep, lane, ww0);  // next step's words
            if (kStep > kMWindows && i0 + kStep + kMWindows < nwin)
                load_window(A, words, hm, i0 + kStep + kMWindows, lane, ww1);
            // the other waves of the SIMD hide the latencies
            if (two) {
#if TFBS_MFMA_PIPE
                // software pipeline: tile t's MFMAs issue before tile t-1's
                // threshold tests, so the tests overlap the matrix pipe
                v16i c0, c1, d0, d1;
                int32_t tc, td;
                pair_scores<NK>(s_img, S, 0, lane, a0, a1, c0, c1, tc);
                uint32_t ti = 1;
                for (; ti + 1 < nt; ti += 2) {
                    pair_scores<NK>(s_img, S, ti, lane, a0, a1, d0, d1, td);
                    check_tile<NK>(s_img, S, ti - 1, c0, tc, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti - 1, c1, tc, a1, i0 + kMWindows, lane);
                    pair_scores<NK>(s_img, S, ti + 1, lane, a0, a1, c0, c1, tc);
                    check_tile<NK>(s_img, S, ti, d0, td, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti, d1, td, a1, i0 + kMWindows, lane);
                }
                if (ti < nt) {
                    pair_scores<NK>(s_img, S, ti, lane, a0, a1, d0, d1, td);
                    check_tile<NK>(s_img, S, ti - 1, c0, tc, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti - 1, c1, tc, a1, i0 + kMWindows, lane);
                    check_tile<NK>(s_img, S, ti, d0, td, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti, d1, td, a1, i0 + kMWindows, lane);
                } else {
                    check_tile<NK>(s_img, S, ti - 1, c0, tc, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti - 1, c1, tc, a1, i0 + kMWindows, lane);
                }
#else
                for (uint32_t ti = 0; ti < nt; ti++) {
                    v16i c0, c1;
                    int32_t tc;
                    pair_scores<NK>(s_img, S, ti, lane, a0, a1, c0, c1, tc);
                    check_tile<NK>(s_img, S, ti, c0, tc, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti, c1, tc, a1, i0 + kMWindows, lane);
                }
#endif
                continue;
            }
            uint32_t ti = 0;
            if (NK <= 4) {  // two strand tiles at a time: tile 0's test overlaps tile 1's MFMAs
                for (; ti + 1 < nt; ti += 2) {
                    BFrag<NK> f0, f1;
                    load_tile<NK>(s_img, S, ti, lane, f0);
                    load_tile<NK>(s_img, S, ti + 1, lane, f1);
                    __builtin_amdgcn_sched_barrier(0);
                    const v16i acc0 = tile_scores<NK>(a0, f0);
                    const v16i acc1 = tile_scores<NK>(a0, f1);
                    check_tile<NK>(s_img, S, ti, acc0, f0.thr, a0, i0, lane);
                    check_tile<NK>(s_img, S, ti + 1, acc1, f1.thr, a0, i0, lane);
                }
            }
            for (; ti < nt; ti++) {
                BFrag<NK> f;
                load_tile<NK>(s_img, S, ti, lane, f);
                __builtin_amdgcn_sched_barrier(0);
                const v16i acc = tile_scores<NK>(a0, f);
                check_tile<NK>(s_img, S, ti, acc, f.thr, a0, i0, lane);
            }
        }
        // the haplotype's logged hits: one batch of global atomics
        const uint32_t nl = min(s_log_n[wave], kMLog);
        for (uint32_t j = lane; j < nl; j += 64) atomicAdd(A.counts + hm.count_off + s_log[wave][j], 1u);
        s_log_n[wave] = 0;
    }
}

// Grid: n_msupers x ceil(n_haps / haps_per_block), 4 waves per SIMD.
// LDS: one-hot tables | super tile image | (STAGED) the packed words of the
// workgroup's haplotypes, copied once so that every window read is an LDS read.
template <bool STAGED, int NK>
__global__ __launch_bounds__(kMBlock, kMfmaMinWaves[NK]) void scan_mfma_kernel(ScanArgs A) {
    static_assert(kMBlock / 64 <= kMMaxWaves, "one hit context per wave");
    int32_t *smem = s_mdyn;
    if (threadIdx.x == 0) s_kctx = KernelHitCtx{A.counts, A.posrel, A.hits, A.hits_wpp, A.n_patterns_total};
    if (threadIdx.x < kMMaxWaves) s_log_n[threadIdx.x] = 0;
    const uint32_t sidx = blockIdx.x % A.n_msupers;
    const uint32_t hg = blockIdx.x / A.n_msupers;
    const DevMSuper S = A.msupers[sidx];
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.mimage + S.img_off / 4);
        for (uint32_t i = threadIdx.x; i < S.img_bytes / 16; i += kMBlock) dst[kMOnehotBytes / 16 + i] = src[i];
        // one-hot table: 4-mer code -> 4 dwords, base t of the code sets byte
        // (base value) of dword t to 1
        for (uint32_t k = threadIdx.x; k < 256; k += kMBlock)
            dst[k] = make_uint4(1u << (8 * (k & 3)), 1u << (8 * ((k >> 2) & 3)), 1u << (8 * ((k >> 4) & 3)),
                                1u << (8 * (k >> 6)));
    }
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t hl = min(h0 + A.haps_per_block, A.n_haps) - 1;
    {  // inner ranges of the group's regions (consecutive in A.inner), for the hit path
        const DevRegion r0 = A.regions[A.haps[h0].region], r1 = A.regions[A.haps[hl].region];
        const uint32_t n = r1.inner_off + r1.n_inner - r0.inner_off;
        if (n <= kMInnerMax)
            for (uint32_t i = threadIdx.x; i < 2 * n; i += kMBlock) s_inner[i] = A.inner[2 * (size_t)r0.inner_off + i];
        if (threadIdx.x == 0) s_inner_base = n <= kMInnerMax ? r0.inner_off : UINT32_MAX;
    }
    const uint32_t *words = A.words;
    if (STAGED) {
        const uint32_t wbeg = A.haps[h0].word_off;
        const uint32_t wend = A.haps[hl].word_off + (A.haps[hl].len + 15) / 16 + 3;
        uint32_t *s_words = reinterpret_cast<uint32_t *>(smem) + (kMOnehotBytes + A.mimg_max) / 4;
        for (uint32_t i = threadIdx.x; i < wend - wbeg; i += kMBlock) s_words[i] = A.words[wbeg + i];
        words = s_words - wbeg;
    }
    __syncthreads();
    const char *s_img = reinterpret_cast<const char *>(smem) + kMOnehotBytes;
    // the wave index is uniform: keep every haplotype-level value in SGPRs
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    scan_super<NK>(A, S, s_img, words, hg, lane, wave);
}

typedef void (*MfmaKernel)(ScanArgs);
template <int NK> MfmaKernel mfma_nk(bool staged) {
    return staged ? scan_mfma_kernel<true, NK> : scan_mfma_kernel<false, NK>;
}
MfmaKernel mfma_variant(bool staged, uint32_t nk) {
    switch (nk) {
    case 1: return mfma_nk<1>(staged);
    case 2: return mfma_nk<2>(staged);
    case 3: return mfma_nk<3>(staged);
    default: return mfma_nk<4>(staged);
    }
}

}  // namespace

uint32_t mfma_group_words(const DevHap *haps, uint32_t n_haps, uint32_t hpb) {
    uint32_t mx = 0;
    for (uint32_t h0 = 0; h0 < n_haps; h0 += hpb) {
        const uint32_t hl = std::min(h0 + hpb, n_haps) - 1;
        mx = std::max(mx, haps[hl].word_off + (haps[hl].len + 15) / 16 + 3 - haps[h0].word_off);
    }
    return mx;
}

size_t mfma_lds_fixed() { return kMOnehotBytes; }

void mfma_depth_budgets(uint32_t out[9]) {
    const uint32_t *waves = kMfmaRegWaves;
    const uint32_t reserve = kMOnehotBytes + 4096 + 2048;  // tables, staged words, hit contexts
    for (int nk = 1; nk <= kMMaxChunks; nk++) out[nk] = (160 * 1024) / waves[nk] - reserve;
}

int launch_mfma(const ScanArgs &a0, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words,
                uint32_t n_haps, const hipStream_t *streams, uint32_t n_streams) {
    if (n_haps == 0 || n_supers == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const size_t static_lds =
        sizeof(KernelHitCtx) + sizeof(s_wctx) + sizeof(s_inner) + sizeof(s_log) + sizeof(s_log_n) + 16;  // hit contexts
    int launches = 0;
    // one launch per K depth (super tiles come sorted by depth): each kernel is
    // compiled for its depth's registers and LDS; the deepest (longest) first
    std::vector<std::pair<uint32_t, uint32_t>> groups;  // [s0, s1) per depth
    for (uint32_t s0 = 0; s0 < n_supers;) {
        uint32_t s1 = s0;
        while (s1 < n_supers && supers[s1].nk == supers[s0].nk) s1++;
        groups.push_back({s0, s1});
        s0 = s1;
    }
    for (size_t gi = 0; gi < groups.size(); gi++) {
        const uint32_t s0 = groups[groups.size() - 1 - gi].first, s1 = groups[groups.size() - 1 - gi].second;
        const hipStream_t stream = streams[gi % n_streams];
        const uint32_t nk = supers[s0].nk;
        size_t img_bytes = 0;
        for (uint32_t k = s0; k < s1; k++) img_bytes = std::max<size_t>(img_bytes, supers[k].img_bytes);
        const uint32_t ns = s1 - s0;
        // stage the group's words in LDS when they fit beside the image at 4 workgroups per CU
        const size_t base = kMOnehotBytes + img_bytes;
        const size_t staged_bytes = base + ((size_t)group_words * 4 + 15) / 16 * 16;
        const bool staged = staged_bytes + static_lds <= std::max<size_t>(kMStagedMax, (160 * 1024) / kMfmaRegWaves[nk]);
        const size_t lds = staged ? staged_bytes : base;
        const MfmaKernel kern = mfma_variant(staged, nk);
        hipError_t e = hipSuccess;
        if (lds > 64 * 1024)
            e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("MFMA LDS attribute: ") + hipGetErrorString(e));
        const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / ns - 1);
        for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
            const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
            const uint32_t h0 = (uint32_t)(g0 * hpb);
            ScanArgs a = a0;
            a.msupers = a0.msupers + s0;
            a.n_msupers = ns;
            a.haps = a0.haps + h0;
            a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
            a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
            a.mimg_max = (uint32_t)img_bytes;
            hipLaunchKernelGGL(kern, dim3(ns * ng), dim3(kMBlock), lds, stream, a);
            launches++;
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_mfma_kernel launch: ") + hipGetErrorString(e));
#if TFBS_MFMA_PROBE == 4
    unsigned long long pr[5] = {0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < n_streams; i++) (void)hipStreamSynchronize(streams[i]);
    (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof pr);
    fprintf(stderr, "probe4 tiles %llu rescored %llu entries %llu hits %llu invalid_hits %llu\n", pr[3], pr[4], pr[0],
            pr[1], pr[2]);
    const unsigned long long z[5] = {0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof z);
#endif
    return launches;
}

}  // namespace tfbs
