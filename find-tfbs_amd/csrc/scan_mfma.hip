// Matrix-core scan (gfx950 v_mfma_scale_f32_32x32x64_f8f6f4, FP4 x FP6) for
// strands with L <= 32 (mfma.cpp).
//
// matches (pattern.rs:141-171) scores every window i of a haplotype with
// sum_j w[j][nuc(i + j)] (N = 0, pattern.rs:119-135).  For 32 consecutive
// windows x 32 strands that is a GEMM: A[window][k] = one-hot of the window's
// bases (all zero for N), B[k][strand] = the strand's weights.  The kernel
// runs it on FP6 digits q of an upper bound (score <= C + s Q, mfma.cpp) with
// the one-hot in FP4, at the matrix cores' FP4/FP6 rate: one MFMA per 16
// columns, exact f32 sums.  Q > thr is necessary for a hit; those candidate
// windows are rescored exactly from the strand's integer weights.
//
//  * A workgroup (4 waves) stages one super tile (tiles of 32 strands of equal
//    K depth: B fragments + strand metadata), the one-hot table and the packed
//    words of its haplotypes in LDS.  Every B fragment is one conflict-free
//    ds_read_b128 + ds_read_b64 per lane.
//  * Each wave takes haplotypes; per 32-window tile it builds the A fragments
//    once (two table reads per chunk) and reuses them for every strand tile of
//    the super tile, two window tiles per B fragment read.
//  * C layout: lane l holds strand column l & 31 and windows (r & 3) + 8 (r >> 2)
//    + 4 (l >> 5), r < 16.  A max-reduce of the 16 coarse sums against the
//    lane's thr and one ballot gate the (rare) candidate handling: each firing
//    lane queues its candidate mask in LDS; drain_queue rescores the queued
//    windows exactly (pattern.rs:125-151), applies the inner-range overlap test
//    (range.rs:18-21 as main.rs:503 uses it) and adds to the count of the
//    strand's pattern_id slot atomically (counts are zeroed before the scan).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "scan.hpp"

namespace tfbs {
namespace {

// Bottleneck probes (tools/probe_build.sh, never in the product build):
// TFBS_MFMA_PROBE=1 skips the threshold test (scores kept live; timing only),
// =2 reads every B fragment from tile 0 (results wrong; timing only), =4 counts
// tiles, firing tiles, candidate lanes, exact hits and rejected candidates
// (printed per launch), =11 never queues candidates, =12 never drains the
// queue (11, 12: results wrong; timing only).
#ifndef TFBS_MFMA_PROBE
#define TFBS_MFMA_PROBE 0
#endif
#ifndef TFBS_MFMA_QUAD  // 2 strand tiles x 2 window tiles per round at K depth 1 (0: pairs only)
#define TFBS_MFMA_QUAD 1
#endif
#ifndef TFBS_MFMA_W4  // 1 strand tile x 4 window tiles per round (steps of 128 windows): bit d-1 = K depth d
#define TFBS_MFMA_W4 0
#endif
#ifndef TFBS_MFMA_W4_PF  // ... with the next round's B fragment read ahead: bit d-1 = K depth d
#define TFBS_MFMA_W4_PF 1
#endif


typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int kMBlock = 256;          // 4 waves
constexpr int kMOnehotBytes = 2048;   // LDS: one-hot table (4-mer -> 4 x 16 bits of FP4), image, words
constexpr uint32_t kMStagedMax = 40 * 1024;  // LDS per workgroup at 4 workgroups per CU (160 KiB)
// per K depth (chunks of 16 columns): window tiles per step and the waves per
// SIMD the kernel is compiled for (the registers of two A sets + two
// accumulators)
constexpr uint32_t kMfmaWindowTiles[kMMaxChunks + 1] = {1, 2, 2};
// waves per SIMD the depth kernels' registers allow (see mfma_depth_budgets)
constexpr uint32_t kMfmaRegWaves[kMMaxChunks + 1] = {4, 6, 5};
#ifndef TFBS_MFMA_D2_WAVES
#define TFBS_MFMA_D2_WAVES 4
#endif
constexpr int kMfmaMinWaves[kMMaxChunks + 1] = {4, 4, TFBS_MFMA_D2_WAVES};

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
// columns 16 kc + 8 h .. + 7 of the lane's window as FP4 one-hot nibbles (1.0
// at the base's position, 16 bits per column), two 4-mer table reads; N
// bases zeroed in haplotypes that have them.
template <int NK>
__device__ __forceinline__ void build_onehot(const DevHap &hm, uint32_t i0, uint32_t lane, const WinWords &ww,
                                             const char *s_onehot, v4i (&a)[NK]) {
    const uint32_t i = i0 + (lane & 31);
    const uint32_t ic = min(i, hm.len);
    const uint32_t sh = 2 * (ic & 15);
    const uint32_t img_lo = __builtin_amdgcn_alignbit(ww.w[1], ww.w[0], sh);  // bases i .. i+15
    const uint32_t img_hi = __builtin_amdgcn_alignbit(ww.w[2], ww.w[1], sh);  // bases i+16 .. i+31
    const uint32_t hb = 16 * (lane >> 5);
    const uint2 *tab = reinterpret_cast<const uint2 *>(s_onehot);
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        const uint32_t img = kc == 0 ? img_lo : img_hi;
        const uint2 x = tab[__builtin_amdgcn_ubfe(img, hb, 8)], y = tab[__builtin_amdgcn_ubfe(img, hb + 8, 8)];
        a[kc] = v4i{(int)x.x, (int)x.y, (int)y.x, (int)y.y};
    }
    // Bases past the haplotype end need no mask: they only reach windows with
    // i + L > len (rejected when the candidate is rescored) or columns >= L
    // (zero weights).
    if (hm.flags & HAP_HAS_N) {  // N scores 0 (pattern.rs:119-135): clear its one-hot
        const uint32_t vm = ~__builtin_amdgcn_alignbit(ww.m[1], ww.m[0], ic & 31) >> (hb / 2);
#pragma unroll
        for (int kc = 0; kc < NK; kc++)
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t keep = ((vm >> (16 * kc + 2 * d)) & 1u ? 0xFFFFu : 0u) |
                                      ((vm >> (16 * kc + 2 * d + 1)) & 1u ? 0xFFFF0000u : 0u);
                a[kc][d] &= keep;
            }
    }
}

// B fragments of one strand tile: per chunk, the lane's 32 FP6 coarse digits
// (192 bits) as dwords 0-3 (at lane * 16) and 4-5 (at 1024 + lane * 8).
template <int NK>
struct BFrag {
    v4i b[NK];
    int2 c[NK];
    float thr;
};

template <int NK>
__device__ __forceinline__ void load_tile(const char *s_img, const DevMSuper &S, uint32_t ti, uint32_t lane,
                                          BFrag<NK> &f) {
    const char *p = s_img + (TFBS_MFMA_PROBE == 2 ? 0 : ti) * (NK * kMFragBytes);
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        if (kc) asm volatile("" ::: "memory");  // no ds_read2 merging across chunks (see the quad loop)
        f.b[kc] = *reinterpret_cast<const v4i *>(p + kc * kMFragBytes + lane * 16);
        f.c[kc] = *reinterpret_cast<const int2 *>(p + kc * kMFragBytes + 1024 + lane * 8);
    }
    f.thr = reinterpret_cast<const float *>(s_img + S.meta_off + ti * kMMetaBytes)[lane & 31];
}

// One coarse chunk: FP4 one-hot (A) x FP6 digits (B), f32 accumulate, unit scales
__device__ __forceinline__ v16f mfma_chunk(const v4i &a, const v4i &b, const int2 &c, const v16f &acc) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{a[0], a[1], a[2], a[3], 0, 0, 0, 0},
                                                           v8i{b[0], b[1], b[2], b[3], c.x, c.y, 0, 0}, acc,
                                                           4 /* A: FP4 e2m1 */, 2 /* B: FP6 e2m3 */, 0, 127, 0, 127);
}

template <int NK>
__device__ __forceinline__ v16f tile_scores(const v4i (&a)[NK], const BFrag<NK> &f) {
    v16f acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kc = 0; kc < NK; kc++) acc = mfma_chunk(a[kc], f.b[kc], f.c[kc], acc);
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

// Candidate handling.  A tile whose coarse test fires (about one in nine)
// appends one entry per lane with a candidate to the wave's queue in LDS.  The
// strand loop stops before a tile pair whose entries might not fit; the queue
// (and the wave's last one) is then drained 64 entries at a time, one per
// lane, by drain_queue, which rescores each candidate window exactly from the
// strand's weights (pattern.rs:125-135) and counts the hits, and the loop
// resumes.  Inlined there, where few registers are live, it adds none.  Entry:
// bits 0-15 the lane's candidate mask (bit 15 - r <-> register r), 16-21 the
// lane, 22-27 the strand tile, 32-39 the haplotype in the workgroup's group,
// 40-63 the window tile start / 32.
constexpr uint32_t kMQueue = 384;  // entries per wave (a round of four tile tests adds at most 256)
__shared__ uint64_t s_queue[kMBlock / 64][kMQueue];
extern __shared__ __attribute__((aligned(16))) int32_t s_mdyn[];  // one-hot table | image | words

#if TFBS_MFMA_PROBE == 13
__device__ unsigned long long g_sink;  // probe 13: the fired-lane count, so the tests stay live
#endif
#if TFBS_MFMA_PROBE == 4
__device__ unsigned long long g_probe[5];
#endif
#if TFBS_MFMA_PROBE == 8
__device__ unsigned int g_trace_n;
__device__ uint4 g_trace[8192];  // (kind << 24 | lane, i or m, L or at, score or i0)
__device__ __forceinline__ void trace(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t k = atomicAdd(&g_trace_n, 1u);
    if (k < 8192) g_trace[k] = make_uint4(a, b, c, d);
}
#endif

// Exact score of window i of haplotype hp for a strand of length L (i + L <= len):
// whole blocks of 8 columns (the weights are zero-padded to them), one load per
// column, N columns masked out.
__device__ __forceinline__ int32_t exact_score(const ScanArgs &A, const uint32_t *words, const DevHap &hp, uint32_t i,
                                               uint32_t L, uint32_t woff) {
    const uint32_t *w = words + hp.word_off + (i >> 4);
    const uint32_t sh = 2 * (i & 15);
    const uint32_t img[2] = {__builtin_amdgcn_alignbit(w[1], w[0], sh), __builtin_amdgcn_alignbit(w[2], w[1], sh)};
    uint32_t live = 0xFFFFFFFFu;  // bit j: base i + j is not N
    if (hp.flags & HAP_HAS_N) {
        const uint32_t *m = A.nmask + hp.nmask_off + (i >> 5);
        live = ~__builtin_amdgcn_alignbit(m[1], m[0], i & 31);
    }
    const int32_t *wt = A.mweights + woff;
    int32_t s = 0;
#pragma unroll 1
    for (uint32_t jb = 0; jb < L; jb += 8) {
        int32_t v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t j = jb + u;
            v[u] = wt[4 * j + ((img[j >> 4] >> (2 * (j & 15))) & 3u)];
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) s += v[u] & -(int32_t)((live >> (jb + u)) & 1u);  // N scores 0
    }
    return s;
}

// One queue entry: each candidate window of the lane's mask is rescored
// exactly; hits add to their slot's count for every inner range they overlap.
__device__ __forceinline__ void drain_entry(const ScanArgs &A, const uint32_t *words, uint32_t tile0,
                                            uint32_t h0, uint64_t q) {
    uint32_t m = (uint32_t)q & 0xFFFFu;
    const uint32_t src = ((uint32_t)q >> 16) & 63u, ti = ((uint32_t)q >> 22) & 63u;
    const uint32_t hap = h0 + ((uint32_t)(q >> 32) & 255u), i0 = (uint32_t)(q >> 40) << 5;
    const uint32_t col = src & 31u, h = src >> 5;
    const int32_t *meta = A.mmeta + (size_t)(tile0 + ti) * kGMetaInts;
    const uint32_t L = (uint32_t)meta[kGLen + col], woff = (uint32_t)meta[kGWoff + col];
    const int32_t mn = meta[kGMin + col];
    const DevHap hp = A.haps[hap];
    const DevRegion rg = A.regions[hp.region];
    const uint32_t off0 = (uint32_t)meta[kGSlot + col] * rg.n_inner;
    const int32_t *inner = A.inner + 2 * (size_t)rg.inner_off;
    while (m) {
        const uint32_t b = 31 - __builtin_clz(m & -m);  // lowest set bit
        m &= m - 1;
        const uint32_t r = 15 - b;
        const uint32_t i = i0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (i + L > hp.len) continue;                   // past the end (pattern.rs:147-150)
        const int32_t sc = exact_score(A, words, hp, i, L, woff);
#if TFBS_MFMA_PROBE == 4
        atomicAdd(&g_probe[sc > mn ? 1 : 2], 1ull);
#endif
#if TFBS_MFMA_PROBE == 8
        trace((2u << 24) | src, i, 0, (uint32_t)sc);
#endif
        if (!(sc > mn)) continue;                       // strict (pattern.rs:151)
        const int32_t p = (hp.flags & HAP_HAS_POS) ? A.posrel[hp.pos_off + i] : (int32_t)i;
        for (uint32_t k = 0; k < rg.n_inner; k++) {     // range.rs:18-21 as main.rs:503 uses it
            const int32_t s = inner[2 * k], en = inner[2 * k + 1];
            const uint32_t span = (uint32_t)(en - s);
            if ((uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span)
                atomicAdd(A.counts + hp.count_off + off0 + k, 1u);
        }
        if (A.hits && i / 64 < A.hits_wpp)
            atomicOr(A.hits + ((size_t)hap * A.n_patterns_total + (uint32_t)meta[kGOrig + col]) * A.hits_wpp +
                         i / 64,
                     1ull << (i & 63));
    }
}

// Drains the wave's first n queue entries (one entry per lane per round).
// h0: the workgroup's first haplotype; tile0: the super tile's first global tile.
__device__ __forceinline__ void drain_queue(const ScanArgs &A, const uint32_t *words, uint32_t tile0,
                                            uint32_t h0, uint32_t n, uint32_t wave) {
#if TFBS_MFMA_PROBE == 12 || TFBS_MFMA_PROBE == 13
    return;  // timing only: queued candidates are dropped
#endif
    for (uint32_t e = threadIdx.x & 63; e < n; e += 64) drain_entry(A, words, tile0, h0, s_queue[wave][e]);
}

__shared__ uint32_t s_qn[kMBlock / 64];

// Drains every wave's queue (entries s_queue[w][0, s_qn[w])) with the whole
// workgroup, one entry per thread per round.
__device__ __forceinline__ void drain_pooled(const ScanArgs &A, const uint32_t *words, uint32_t tile0,
                                             uint32_t h0) {
#if TFBS_MFMA_PROBE == 12
    return;
#endif
    constexpr uint32_t kWaves = kMBlock / 64;
    uint32_t off[kWaves + 1];
    off[0] = 0;
#pragma unroll
    for (uint32_t w = 0; w < kWaves; w++) off[w + 1] = off[w] + s_qn[w];
    for (uint32_t g = threadIdx.x; g < off[kWaves]; g += kMBlock) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t k = 1; k < kWaves; k++) w += g >= off[k];
        drain_entry(A, words, tile0, h0, s_queue[w][g - off[w]]);
    }
}

// The max of a lane's 16 sums: 7 v_max3 + 1 v_max (a balanced pairwise tree
// takes 10)
__device__ __forceinline__ float max16(const v16f &a) {
    const float t0 = fmaxf(fmaxf(a[0], a[1]), a[2]), t1 = fmaxf(fmaxf(a[3], a[4]), a[5]);
    const float t2 = fmaxf(fmaxf(a[6], a[7]), a[8]), t3 = fmaxf(fmaxf(a[9], a[10]), a[11]);
    const float t4 = fmaxf(fmaxf(a[12], a[13]), a[14]);
    return fmaxf(fmaxf(fmaxf(t0, t1), t2), fmaxf(fmaxf(t3, t4), a[15]));
}

// Coarse test of one strand tile: the max of each lane's 16 coarse sums
// against its strand's thr, one ballot.  Both tiles of a pair are tested
// before either branches, so every read of the MFMA results sits in the
// MFMAs' basic block, where the compiler's wait-state accounting holds (a read
// placed after the branch of the first tile's test got too few wait states
// and saw stale sums).
__device__ __forceinline__ uint64_t coarse_test(const v16f &acc, float thr) {
#if TFBS_MFMA_PROBE == 4
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_probe[3], 1ull);
#endif
    if (TFBS_MFMA_PROBE == 1) {
        asm volatile("" ::"v"(acc[0]), "v"(acc[5]), "v"(acc[10]), "v"(acc[15]));
        return 0;
    }
    return __ballot(max16(acc) > thr);
}

// A firing tile (fired = its coarse ballot, about one tile in nine): each
// firing lane queues its candidate mask; qn (wave-uniform) counts the wave's
// queued entries.
__device__ __forceinline__ void queue_tile(const v16f &acc, float thr, uint64_t fired, uint32_t ti, uint32_t hh,
                                           uint32_t i0, uint32_t lane, uint32_t wave, uint32_t &qn) {
    if (__builtin_expect(fired == 0, 1)) return;
#if TFBS_MFMA_PROBE == 13
    qn += (uint32_t)__popcll(fired) & 1u;  // timing only: the tests' cost without the candidate handling
    return;
#endif
#if TFBS_MFMA_PROBE == 4
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_probe[4], 1ull);
    if (fired & (1ull << lane)) atomicAdd(&g_probe[0], 1ull);
#endif
    uint32_t m = 0;  // sign of thr - acc (both multiples of 1/8 below 2^12: exact), packed subtracts
    const v2f t2 = {thr, thr};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        const v2f d = t2 - v2f{acc[r], acc[r + 1]};
        m = __builtin_amdgcn_alignbit(m, __float_as_uint(d[0]), 31);
        m = __builtin_amdgcn_alignbit(m, __float_as_uint(d[1]), 31);
    }
#if TFBS_MFMA_PROBE == 11
    return;  // timing only: no candidate is queued
#endif
    const uint32_t at = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(fired >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fired, 0));
#if TFBS_MFMA_PROBE == 8
    if (fired & (1ull << lane)) trace((1u << 24) | lane, m, at, i0);
#endif
    if (fired & (1ull << lane))  // every firing lane (m != 0) fills its slot
        s_queue[wave][at] = (uint64_t)(m | (lane << 16) | (ti << 22)) | ((uint64_t)(hh | ((i0 >> 5) << 8)) << 32);
    qn += (uint32_t)__popcll(fired);
}

// Coarse sums of strand tile ti for two window tiles (one B fragment read
// feeds both MFMAs).
template <int NK>
__device__ __forceinline__ void pair_scores(const char *s_img, const DevMSuper &S, uint32_t ti, uint32_t lane,
                                            const v4i (&a0)[NK], const v4i (&a1)[NK], v16f &c0, v16f &c1,
                                            float &thr) {
    BFrag<NK> f;
    load_tile<NK>(s_img, S, ti, lane, f);
    __builtin_amdgcn_sched_barrier(0);  // every B read of the tile issues before its MFMAs
    c0 = v16f{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    c1 = c0;
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        c0 = mfma_chunk(a0[kc], f.b[kc], f.c[kc], c0);
        c1 = mfma_chunk(a1[kc], f.b[kc], f.c[kc], c1);
    }
    // both tiles' MFMAs issue before either test reads a result (the first
    // test then runs under the second tile's MFMA)
    __builtin_amdgcn_sched_barrier(0);
    thr = f.thr;
}

// Four window tiles x one strand tile per round (TFBS_MFMA_W4): one B fragment
// read (prefetched a round ahead) feeds four MFMA chains, whose tests share the
// strand tile's thresholds.  Steps of 128 windows while at least three of their
// window tiles hold windows; returns the first window the pair loop still has
// to score.
template <int NK>
__device__ __forceinline__ uint32_t scan_hap_w4(const ScanArgs &A, const DevMSuper &S, const char *s_img,
                                                const uint32_t *words, const DevHap &hm, uint32_t nwin, uint32_t hh,
                                                uint32_t lane, uint32_t wave, uint32_t tile0, uint32_t h0,
                                                uint32_t &qn) {
    const uint32_t nt = S.tile_count;
    const char *tab = s_img - kMOnehotBytes;
    uint32_t i0 = 0;
    for (; i0 + 2 * kMWindows < nwin; i0 += 4 * kMWindows) {
        v4i a[4][NK];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            WinWords ww;
            load_window(A, words, hm, i0 + t * kMWindows, lane, ww);
            build_onehot<NK>(hm, i0 + t * kMWindows, lane, ww, tab, a[t]);
        }
        BFrag<NK> f;
        load_tile<NK>(s_img, S, 0, lane, f);
        constexpr bool kPf = (TFBS_MFMA_W4_PF >> (NK - 1)) & 1;
        for (uint32_t ti = 0; ti < nt; ti++) {
            BFrag<NK> g;
            if (!kPf) {
                if (ti) load_tile<NK>(s_img, S, ti, lane, f);
            } else if (ti + 1 < nt) {
                load_tile<NK>(s_img, S, ti + 1, lane, g);  // next round's fragment
            }
            __builtin_amdgcn_sched_barrier(0);
            v16f c[4];
#pragma unroll
            for (int t = 0; t < 4; t++) c[t] = v16f{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int kc = 0; kc < NK; kc++)
#pragma unroll
                for (int t = 0; t < 4; t++) c[t] = mfma_chunk(a[t][kc], f.b[kc], f.c[kc], c[t]);
            __builtin_amdgcn_sched_barrier(0);
            const float thr = f.thr;
            uint64_t q[4];
#pragma unroll
            for (int t = 0; t < 4; t++) q[t] = coarse_test(c[t], thr);
            if (kPf) f = g;
            if (__builtin_expect((q[0] | q[1] | q[2] | q[3]) == 0, 1)) continue;  // one branch for four tests
#pragma unroll
            for (int t = 0; t < 4; t++) queue_tile(c[t], thr, q[t], ti, hh, i0 + t * kMWindows, lane, wave, qn);
            if (qn > kMQueue - 256) {
                drain_queue(A, words, tile0, h0, qn, wave);
                qn = 0;
            }
        }
    }
    return i0;
}

// words: the packed haplotype words, indexed by DevHap::word_off (an LDS copy
// of this workgroup's haplotypes, biased by their first word, or global memory).
template <int NK>
__device__ __forceinline__ void scan_super(const ScanArgs &A, const DevMSuper &S, const char *s_img,
                                           const uint32_t *words, uint32_t hg, uint32_t lane, uint32_t wave) {
    constexpr uint32_t kWaves = kMBlock / 64;
    const uint32_t nt = S.tile_count;
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t tile0 = S.tile0;
    uint32_t qn = 0;
    for (uint32_t hh = wave; hh < A.haps_per_block; hh += kWaves) {
        const uint32_t hap = hg * A.haps_per_block + hh;
        if (hap >= A.n_haps) break;
        const DevHap hm = load_hap(A.haps + hap);
        if (hm.len < S.lmin) continue;
        const uint32_t nwin = hm.len - S.lmin + 1;
        const char *tab = s_img - kMOnehotBytes;
        // window tiles two at a time, so that each B fragment read from LDS
        // feeds two MFMAs (the LDS read rate, not the matrix core, bounds one
        // read per MFMA)
        constexpr uint32_t kStep = kMfmaWindowTiles[NK] * kMWindows;
        const uint32_t ibeg = ((TFBS_MFMA_W4 >> (NK - 1)) & 1) ? scan_hap_w4<NK>(A, S, s_img, words, hm, nwin, hh, lane, wave, tile0, h0, qn)
                                           : 0;
        if (ibeg >= nwin) continue;
        WinWords ww0, ww1;
        load_window(A, words, hm, ibeg, lane, ww0);
        if (kStep > kMWindows && ibeg + kMWindows < nwin) load_window(A, words, hm, ibeg + kMWindows, lane, ww1);
        for (uint32_t i0 = ibeg; i0 < nwin; i0 += kStep) {
            const bool two = kStep > kMWindows && i0 + kMWindows < nwin;
            v4i a0[NK], a1[NK];
            build_onehot<NK>(hm, i0, lane, ww0, tab, a0);
            if (two) build_onehot<NK>(hm, i0 + kMWindows, lane, ww1, tab, a1);
            if (i0 + kStep < nwin) load_window(A, words, hm, i0 + kStep, lane, ww0);  // next step's words
            if (kStep > kMWindows && i0 + kStep + kMWindows < nwin)
                load_window(A, words, hm, i0 + kStep + kMWindows, lane, ww1);
            // the other waves of the SIMD hide the latencies
            // The loops test the queue's room only after a round that queued
            // something (rare): a round adds at most 64 entries per tile test,
            // so draining above kMQueue - 256 keeps the next round's entries
            // in bounds.  Inlined in that cold branch, the drain adds no
            // registers to the loop.
            uint32_t ti = 0;
            if (two) {
#if TFBS_MFMA_QUAD
                // two strand tiles x two window tiles per round: four
                // independent MFMAs before the first test (3 % faster than
                // pairs at K depth 1; at depth 2 the registers would spill)
                for (; NK == 1 && ti + 1 < nt; ti += 2) {
                    v16f c0, c1, d0, d1;
                    float tc, td;
                    BFrag<NK> f, g;
                    load_tile<NK>(s_img, S, ti, lane, f);
                    // keeps the two tiles' dword 4-5 reads apart: merged into one
                    // ds_read2st64 they need 4 v_mov into the MFMA operand tuples
                    asm volatile("" ::: "memory");
                    load_tile<NK>(s_img, S, ti + 1, lane, g);
                    __builtin_amdgcn_sched_barrier(0);
                    c0 = v16f{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
                    c1 = c0;
                    d0 = c0;
                    d1 = c0;
#pragma unroll
                    for (int kc = 0; kc < NK; kc++) {
                        c0 = mfma_chunk(a0[kc], f.b[kc], f.c[kc], c0);
                        c1 = mfma_chunk(a1[kc], f.b[kc], f.c[kc], c1);
                        d0 = mfma_chunk(a0[kc], g.b[kc], g.c[kc], d0);
                        d1 = mfma_chunk(a1[kc], g.b[kc], g.c[kc], d1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    tc = f.thr;
                    td = g.thr;
                    const uint64_t f0 = coarse_test(c0, tc), f1 = coarse_test(c1, tc);
                    const uint64_t g0 = coarse_test(d0, td), g1 = coarse_test(d1, td);
                    if (__builtin_expect((f0 | f1 | g0 | g1) == 0, 1)) continue;  // one branch for four tests
                    queue_tile(c0, tc, f0, ti, hh, i0, lane, wave, qn);
                    queue_tile(c1, tc, f1, ti, hh, i0 + kMWindows, lane, wave, qn);
                    queue_tile(d0, td, g0, ti + 1, hh, i0, lane, wave, qn);
                    queue_tile(d1, td, g1, ti + 1, hh, i0 + kMWindows, lane, wave, qn);
                    if (qn > kMQueue - 256) {
                        drain_queue(A, words, tile0, h0, qn, wave);
                        qn = 0;
                    }
                }
#endif
                for (; ti < nt; ti++) {
                    v16f c0, c1;
                    float tc;
                    pair_scores<NK>(s_img, S, ti, lane, a0, a1, c0, c1, tc);
#if TFBS_MFMA_PROBE == 20
                    // round 1's failing placement, for the ISA lint (tools/isa_lint.py):
                    // the second tile's test reads its MFMA results after the first tile's branch
                    const uint64_t f0 = coarse_test(c0, tc);
                    queue_tile(c0, tc, f0, ti, hh, i0, lane, wave, qn);
                    const uint64_t f1 = coarse_test(c1, tc);
                    queue_tile(c1, tc, f1, ti, hh, i0 + kMWindows, lane, wave, qn);
#else
                    const uint64_t f0 = coarse_test(c0, tc), f1 = coarse_test(c1, tc);
                    if (__builtin_expect((f0 | f1) == 0, 1)) continue;
                    queue_tile(c0, tc, f0, ti, hh, i0, lane, wave, qn);
                    queue_tile(c1, tc, f1, ti, hh, i0 + kMWindows, lane, wave, qn);
#endif
                    if (qn > kMQueue - 256) {
                        drain_queue(A, words, tile0, h0, qn, wave);
                        qn = 0;
                    }
                }
            } else {
                // two strand tiles at a time: tile 0's test overlaps tile 1's MFMAs
                for (; ti + 1 < nt; ti += 2) {
                    BFrag<NK> f0, f1;
                    load_tile<NK>(s_img, S, ti, lane, f0);
                    load_tile<NK>(s_img, S, ti + 1, lane, f1);
                    __builtin_amdgcn_sched_barrier(0);
                    const v16f acc0 = tile_scores<NK>(a0, f0);
                    const v16f acc1 = tile_scores<NK>(a0, f1);
                    const uint64_t g0 = coarse_test(acc0, f0.thr), g1 = coarse_test(acc1, f1.thr);
                    if (__builtin_expect((g0 | g1) == 0, 1)) continue;
                    queue_tile(acc0, f0.thr, g0, ti, hh, i0, lane, wave, qn);
                    queue_tile(acc1, f1.thr, g1, ti + 1, hh, i0, lane, wave, qn);
                    if (qn > kMQueue - 256) {
                        drain_queue(A, words, tile0, h0, qn, wave);
                        qn = 0;
                    }
                }
                if (ti < nt) {
                    BFrag<NK> f;
                    load_tile<NK>(s_img, S, ti, lane, f);
                    __builtin_amdgcn_sched_barrier(0);
                    const v16f acc = tile_scores<NK>(a0, f);
                    queue_tile(acc, f.thr, coarse_test(acc, f.thr), ti, hh, i0, lane, wave, qn);
                    if (qn > kMQueue - 256) {
                        drain_queue(A, words, tile0, h0, qn, wave);
                        qn = 0;
                    }
                }
            }
        }
    }
    // the waves' last entries, pooled: every wave drains a share of the sum
#if TFBS_MFMA_PROBE == 13
    if (lane == 0) atomicAdd(&g_sink, (unsigned long long)qn);
    return;
#endif
    if (lane == 0) s_qn[wave] = qn;
    __syncthreads();
    drain_pooled(A, words, tile0, h0);
}

// Grid: n_msupers x ceil(n_haps / haps_per_block), 4 waves per SIMD.
// LDS: one-hot table | super tile image | (STAGED) the packed words of the
// workgroup's haplotypes, copied once so that every window read is an LDS read.
template <bool STAGED, int NK>
__global__ __launch_bounds__(kMBlock, kMfmaMinWaves[NK]) void scan_mfma_kernel(ScanArgs A) {
    int32_t *smem = s_mdyn;
    const uint32_t sidx = blockIdx.x % A.n_msupers;
    const uint32_t hg = blockIdx.x / A.n_msupers;
    const DevMSuper S = A.msupers[sidx];
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.mimage + S.img_off / 4);
        for (uint32_t i = threadIdx.x; i < S.img_bytes / 16; i += kMBlock) dst[kMOnehotBytes / 16 + i] = src[i];
        // one-hot table: 4-mer code -> 64 bits, column t (16 bits) holds FP4
        // 1.0 (0x2) in the nibble of its base
        uint2 *tab = reinterpret_cast<uint2 *>(smem);
        for (uint32_t k = threadIdx.x; k < 256; k += kMBlock) {
            uint32_t h[4];
            for (int t = 0; t < 4; t++) h[t] = 2u << (4 * ((k >> (2 * t)) & 3));
            tab[k] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
        }
    }
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t hl = min(h0 + A.haps_per_block, A.n_haps) - 1;
    const char *s_img = reinterpret_cast<const char *>(smem) + kMOnehotBytes;
    const uint32_t *words = A.words;
    if (STAGED) {
        const uint32_t wbeg = A.haps[h0].word_off;
        const uint32_t wend = A.haps[hl].word_off + (A.haps[hl].len + 15) / 16 + 3;
        uint32_t *s_words = reinterpret_cast<uint32_t *>(smem) + (kMOnehotBytes + A.mimg_max) / 4;
        for (uint32_t i = threadIdx.x; i < wend - wbeg; i += kMBlock) s_words[i] = A.words[wbeg + i];
        words = s_words - wbeg;
    }
    __syncthreads();
    // the wave index is uniform: keep every haplotype-level value in SGPRs
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    scan_super<NK>(A, S, s_img, words, hg, lane, wave);
}

typedef void (*MfmaKernel)(ScanArgs);
template <int NK> MfmaKernel mfma_nk(bool staged) {
    return staged ? scan_mfma_kernel<true, NK> : scan_mfma_kernel<false, NK>;
}
MfmaKernel mfma_variant(bool staged, uint32_t nk) {
    return nk == 1 ? mfma_nk<1>(staged) : mfma_nk<2>(staged);
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
    const uint32_t reserve = kMOnehotBytes + 4096 + sizeof(s_queue) + 256;  // table, staged words, queues
    for (int nk = 1; nk <= kMMaxChunks; nk++) out[nk] = (160 * 1024) / waves[nk] - reserve;
}

int launch_mfma(const ScanArgs &a0, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words,
                uint32_t n_haps, const hipStream_t *streams, uint32_t n_streams) {
    if (n_haps == 0 || n_supers == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const size_t static_lds = sizeof(s_queue) + 16;  // candidate queues
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
#if TFBS_MFMA_PROBE == 8
    {
        for (uint32_t i = 0; i < n_streams; i++) (void)hipStreamSynchronize(streams[i]);
        unsigned int n = 0;
        (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_trace_n), sizeof n);
        std::vector<uint4> t(std::min(n, 8192u));
        if (!t.empty()) (void)hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_trace), t.size() * sizeof(uint4));
        for (const uint4 &x : t)
            fprintf(stderr, "%s lane %u %s %u %s %u %s %d\n", (x.x >> 24) == 1 ? "Q" : "D", x.x & 0xFFFFFF,
                    (x.x >> 24) == 1 ? "m" : "i", x.y, (x.x >> 24) == 1 ? "at" : "e", x.z,
                    (x.x >> 24) == 1 ? "i0" : "sc", (int)x.w);
        n = 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trace_n), &n, sizeof n);
    }
#endif
#if TFBS_MFMA_PROBE == 4
    unsigned long long pr[5] = {0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < n_streams; i++) (void)hipStreamSynchronize(streams[i]);
    (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof pr);
    fprintf(stderr, "probe4 tiles %llu fired %llu candidate_lanes %llu hits %llu rejected %llu\n", pr[3], pr[4],
            pr[0], pr[1], pr[2]);
    const unsigned long long z[5] = {0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof z);
#endif
    return launches;
}

}  // namespace tfbs
