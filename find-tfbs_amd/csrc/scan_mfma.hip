// Matrix-core scan (gfx950 v_mfma_scale_f32_32x32x64_f8f6f4, FP6 x FP4) for
// strands with L <= 32 (mfma.cpp).
//
// matches (pattern.rs:141-171) scores every window i of a haplotype with
// sum_j w[j][nuc(i + j)] (N = 0, pattern.rs:119-135).  For 32 windows x a set of
// strands that is a GEMM: the strands' weights times the windows' one-hot bases
// (all zero for N).  The kernel runs it on FP6 digits q <= 0 of an upper bound
// (score <= C + s Q, mfma.cpp) with the one-hot in FP4, at the matrix cores'
// FP4/FP6 rate.  U = 8 Q > T0 is necessary for a hit; those candidate windows are
// rescored exactly from the strand's integer weights.
//
//  * Two strands per GEMM row: the K chunk of 64 holds 8 columns of strand 2n (K
//    block 0) and of strand 2n + 1 (K block 1); A = the digits (scale 2^3: digits x 8
//    = integers; block 1 2^14: the field one up), B = the window's one-hot in both
//    blocks, and the accumulator starts at 2^23 + (1023 - T0) (1 + 2^11).  Every
//    output is an integer in [2^23, 2^24) (exact in f32) whose mantissa holds V = U +
//    1023 - T0 of strand 2n in bits 0-10 and of strand 2n + 1 in bits 11-21, each in
//    [0, 2048) (mfma.cpp clips the digits so); U > T0 iff the field's top bit (10 or
//    21) is set.  One OR tree over a lane's 16 outputs (v_or3 + v_bitop3) tests 32
//    (window, strand) pairs.
//  * A workgroup (8 waves) stages one super tile (tiles of 64 strands of equal
//    K depth), the one-hot table, its group's haplotype descriptors and packed
//    words in LDS.  Every digit fragment is one conflict-free ds_read_b128 +
//    ds_read_b64 per lane and feeds two window tiles.
//  * Window tiles come from the group's window list (build_window_lists): 32
//    listed windows of any of the group's haplotypes per tile, lane l & 31 its
//    own (haplotype, window), so reference-window reuse leaves no holes.
//  * C layout: lane l holds column l & 31 -- the window of its own list entry --
//    and strand pairs (r & 3) + 8 (r >> 2) + 4 (l >> 5), r < 16.  A firing lane
//    (a candidate among its 32 strands) queues a self-contained record (its
//    fields' top bits, its window's list entry, the strand tile) in LDS; the wave
//    decodes its records in batches into (haplotype, strand, window) candidates
//    (drain_queue: no global load); when the wave has scanned
//    it rescores those exactly, one per lane (pattern.rs:125-151), applies the
//    inner-range overlap test (range.rs:18-21 as main.rs:503 uses it) and appends
//    one (haplotype, key) pair per hit and overlapped range to its part of the
//    workgroup's hit list (no count matrix, no atomics: the key assembly,
//    key_kernels.hip, counts them per region); a full wave list spills to a
//    launch-wide list rescored after the scan.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "scan.hpp"

namespace tfbs {
namespace {


typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int kMBlock = 512;          // 8 waves (two per SIMD) share one super tile image
static_assert(kMBlock / 64 == kMBlockWaves, "hit list parts per workgroup");
constexpr int kMOnehotBytes = 2048;   // LDS: one-hot table (4-mer -> 4 x 16 bits of FP4), image, words
constexpr uint32_t kMChunkBytes = 1536;  // one K chunk's B fragments of a 64-strand tile (dwords 0-3 | 4-5)
constexpr uint32_t kMStagedMax = 80 * 1024;  // LDS per workgroup at 2 workgroups per CU (160 KiB)
// waves per SIMD the depth kernels' registers allow (see mfma_depth_budgets)
constexpr uint32_t kMfmaRegWaves[kMMaxChunks + 1] = {4, 4, 4, 4, 4};
constexpr int kMfmaMinWaves[kMMaxChunks + 1] = {4, 4, 4, 4, 4};
constexpr uint32_t kTestMask = (1u << (kMFieldBits - 1)) | (1u << (2 * kMFieldBits - 1));  // the fields' top bits
constexpr uint32_t kQueueBits = 0x20200404u;  // those bits after queue_tile's byte permute (outputs 2j, 2j + 1)
// e8m0 scales: the digits x 8 (K block 0), x 2^(3 + 11) (block 1: the field one up); the one-hot x 1
constexpr int kScaleD0 = 130, kScaleD1 = 130 + kMFieldBits, kScaleOnehot = 127;

// A lane's haplotype (the group's descriptors are staged in LDS, s_hd).
struct LaneHap {
    uint32_t word_off, len, flags, nmask_off;
};

// The packed words (and N-mask words) a lane needs for its window i (read one
// pair of tiles ahead of use).
struct WinWords {
    uint32_t w[3], m[2];
};

__device__ __forceinline__ void load_window(const ScanArgs &A, const uint32_t *words, const LaneHap &hm, uint32_t i,
                                            WinWords &ww) {
    const uint32_t ic = min(i, hm.len);  // reads stay inside the +3 word pad
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

// A fragments of the lane's window i: chunk kc = columns 8 kc .. + 7 as FP4
// one-hot nibbles (1.0 at the base's position, 16 bits per column; the same in
// both lane halves, which the A scales tell apart), two 4-mer table reads; N
// bases zeroed in haplotypes that have them.
template <int NK>
__device__ __forceinline__ void build_onehot(const LaneHap &hm, uint32_t i, const WinWords &ww, const char *s_onehot,
                                             v4i (&a)[NK]) {
    const uint32_t ic = min(i, hm.len);
    const uint32_t sh = 2 * (ic & 15);
    const uint32_t img_lo = __builtin_amdgcn_alignbit(ww.w[1], ww.w[0], sh);  // bases i .. i+15
    const uint32_t img_hi = __builtin_amdgcn_alignbit(ww.w[2], ww.w[1], sh);  // bases i+16 .. i+31
    const uint2 *tab = reinterpret_cast<const uint2 *>(s_onehot);
#pragma unroll
    for (int kc = 0; kc < NK; kc++) {
        const uint32_t img = kc < 2 ? img_lo : img_hi;
        const uint32_t b0 = 16 * (kc & 1);
        const uint2 x = tab[__builtin_amdgcn_ubfe(img, b0, 8)], y = tab[__builtin_amdgcn_ubfe(img, b0 + 8, 8)];
        a[kc] = v4i{(int)x.x, (int)x.y, (int)y.x, (int)y.y};
    }
    // Bases past the haplotype end need no mask: they only reach windows with
    // i + L > len (rejected when the candidate is rescored) or columns >= L
    // (zero digits).
    if (hm.flags & HAP_HAS_N) {  // N scores 0 (pattern.rs:119-135): clear its one-hot
        const uint32_t vm = ~__builtin_amdgcn_alignbit(ww.m[1], ww.m[0], ic & 31);
#pragma unroll
        for (int kc = 0; kc < NK; kc++)
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const uint32_t keep = ((vm >> (8 * kc + 2 * d)) & 1u ? 0xFFFFu : 0u) |
                                      ((vm >> (8 * kc + 2 * d + 1)) & 1u ? 0xFFFF0000u : 0u);
                a[kc][d] &= keep;
            }
    }
}

// B fragments of one strand tile: chunk kc's 32 FP6 digits per lane (192
// bits) as dwords 0-3 (at kc * 1536 + lane * 16) and dwords 4-5 (at kc * 1536 +
// 1024 + lane * 8), mfma_tile_bytes per tile: conflict-free reads.
struct BFrag {
    v4i b;
    int2 c;
};

template <int D>
__device__ __forceinline__ void load_frags(const char *tile, uint32_t lane, BFrag (&f)[D]) {
#pragma unroll
    for (int kc = 0; kc < D; kc++) {
        // no ds_read2 merging across chunks: merged pairs need v_mov copies
        // into the MFMA operand tuples
        if (kc) asm volatile("" ::: "memory");
        f[kc].b = *reinterpret_cast<const v4i *>(tile + kc * 1536 + lane * 16);
        f[kc].c = *reinterpret_cast<const int2 *>(tile + kc * 1536 + 1024 + lane * 8);
    }
}

// One chunk: FP6 digits (A: rows = the tile's 32 strand pairs) x FP4 one-hot (B:
// columns = the tile's 32 windows), f32 accumulate; sa: the lane's A scale (digits x 8,
// x 2^14 for the pair's second strand, K block 1), B scale 1.  (A and B have the same
// lane layout -- lane l: row / column l & 31, K block l >> 5 -- so the image and the
// one-hot serve either operand; with the windows as columns a lane's 16 outputs are 16
// strand pairs of ONE window, the window of its own list entry.)
__device__ __forceinline__ v16f mfma_chunk(const v4i &a, const BFrag &f, const v16f &acc, int sa) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(v8i{f.b[0], f.b[1], f.b[2], f.b[3], f.c.x, f.c.y, 0, 0},
                                                           v8i{a[0], a[1], a[2], a[3], 0, 0, 0, 0}, acc,
                                                           2 /* A: FP6 e2m3 */, 4 /* B: FP4 e2m1 */, 0, sa, 0,
                                                           kScaleOnehot);
}

// Candidate handling.  A firing lane (its window passed the coarse test for some
// strand of the tile; ~40 % of the rounds have one) appends one record to its wave's
// LDS queue (queue_tile): the fields' top bits of its 16 outputs (8 v_perm + 4
// v_bitop3, 16 bytes), its own list entry (the window: s_went) and the tile's first
// global strand | the lane.  The wave decodes its records in batches, one record per
// lane (drain_queue, no global load), into (strand | haplotype in group << 24,
// window) candidates: the first kWaveCands in LDS (s_cand), then the wave's region of
// the global list (A.cands), then the launch-wide overflow list (cand_over_kernel /
// post_scan_kernel).  A tile whose records do not fit drains the queue first and its
// round is scored again (no accumulator live across a drain).  The wave rescores its
// candidates after the scan (rescore_list).
constexpr uint32_t kMQueue = 64;      // records per wave (>= one tile's 64 firing lanes)
constexpr uint32_t kWaveCands = kMWaveCands;  // LDS candidates per wave (C3: 66 mean; the rest in the global list)
__shared__ uint4 s_qdata[kMBlock / 64][kMQueue];
__shared__ uint2 s_qmeta[kMBlock / 64][kMQueue];
__shared__ uint2 s_cand[kMBlock / 64][kWaveCands];
__shared__ uint32_t s_went[kMBlock / 64][64];  // per wave: the current pair's list entries (tile a | tile b)
__shared__ uint32_t s_hnext;  // the workgroup's next pair of window tiles (scan_super)
__shared__ uint4 s_hd[kMMaxHapsPerBlock];   // the group's haplotypes: LaneHap
__shared__ uint4 s_hd2[kMMaxHapsPerBlock];  // and (region, pos_off, drun_off, n_druns) for the rescoring
extern __shared__ __attribute__((aligned(16))) int32_t s_mdyn[];  // one-hot table | image | words


// What the firing path of a round needs: the group's window list (wl, nw
// entries) for the drain, the first global tile and haplotype of the workgroup.
struct GroupCtx {
    const uint32_t *wl;
    const uint16_t *wl16;  // a narrow group's list (16-bit entries), else null
    uint32_t nw, tile0, h0, slot;
    __device__ __forceinline__ uint32_t at(uint32_t q) const { return wl16 ? (uint32_t)wl16[q] : wl[q]; }
};

// What the rescoring reads of a haplotype: DevHap's fields, from the scan
// workgroup's LDS descriptors (s_hd, s_hd2) or from a DevHap.
struct CandHap {
    uint32_t word_off, len, flags, nmask_off, region, pos_off, drun_off, n_druns;
    __device__ __forceinline__ static CandHap of(const DevHap &h) {
        return CandHap{h.word_off, h.len, h.flags, h.nmask_off, h.region, h.pos_off, h.drun_off, h.n_druns};
    }
    __device__ __forceinline__ static CandHap of(const uint4 &a, const uint4 &b) {
        return CandHap{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    }
};

// Exact score of window i of haplotype hp for a strand of length L (i + L <= len):
// one load per column of the strand's blocks of 8 (zero-padded), all issued
// before the first is summed (the rescoring runs where no accumulator is
// live), N columns masked out.
__device__ __forceinline__ int32_t exact_score(const uint32_t *words, const CandHap &hp, uint32_t i, uint32_t L,
                                               const int32_t *wt, uint32_t live) {
    const uint32_t *w = words + hp.word_off + (i >> 4);
    const uint32_t sh = 2 * (i & 15);
    const uint32_t img[2] = {__builtin_amdgcn_alignbit(w[1], w[0], sh), __builtin_amdgcn_alignbit(w[2], w[1], sh)};
    const uint32_t keep = live & (L >= 32 ? ~0u : (1u << L) - 1);  // columns < L that are not N
    int32_t v[32];
#pragma unroll
    for (uint32_t jb = 0; jb < 32; jb += 8) {
        if (jb < L) {  // a lane loads only its strand's blocks
#pragma unroll
            for (uint32_t j = jb; j < jb + 8; j++) v[j] = wt[4 * j + ((img[j >> 4] >> (2 * (j & 15))) & 3u)];
        } else {
#pragma unroll
            for (uint32_t j = jb; j < jb + 8; j++) v[j] = 0;
        }
    }
    int32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < 32; j++) s += v[j] & -(int32_t)((keep >> j) & 1u);  // N scores 0
    return s;
}

// Appends a record to the spill list (rare: hits past a wave's list, reference
// hits past a region's list, inner ranges past 32).
__device__ __forceinline__ void spill_record(const ScanArgs &A, uint32_t head, uint32_t x, uint32_t y) {
    const uint32_t o = atomicAdd(A.over, 1u);
    if (o < A.spill_cap) {
        A.spill[3 * (size_t)o] = head;
        A.spill[3 * (size_t)o + 1] = x;
        A.spill[3 * (size_t)o + 2] = y;
    }
}

// Exact rescoring of one candidate: window i of haplotype hp (hits index hap)
// for the strand g = global tile * 64 + strand in tile.  A HAP_DEDUP haplotype's
// window read because it meets a diff run within the class span, but whose strand
// columns [i, i + L) meet none, is the reference's window for that strand: not
// listed (the key assembly adds the reference's hit, tfbs_internal.hpp).  Returns the hit's
// inner ranges k < 32 (bit k; key = *key0 + k) to be listed by the caller;
// ranges past 32 go to the spill list here.  A hit of the region's reference
// haplotype is also listed for the reuse of its window by the HAP_DEDUP
// haplotypes; a helper reference haplotype (past the region's distinct
// haplotypes) has no counts of its own.  The loads are issued in three
// dependent rounds (strand fields | weights, region, position, N mask | inner
// ranges).
__device__ __forceinline__ uint32_t score_candidate(const ScanArgs &A, const uint32_t *words, const CandHap &hp,
                                                    uint32_t hap, uint32_t g, uint32_t i, uint32_t *key0) {
    const int32_t *meta = A.mmeta + (size_t)(g >> 6) * kGMetaInts;
    const uint32_t sn = g & 63u;
    const int4 sf = *reinterpret_cast<const int4 *>(meta + kGStrandInts * sn);  // min, woff, len, slot
    const DevRegion rg = A.regions[hp.region];
    const uint32_t ic = min(i, hp.len - 1);  // i + L > len: no hit (below), reads stay in range
    const int32_t p = (hp.flags & HAP_HAS_POS) ? A.posrel[hp.pos_off + ic] : (int32_t)i;
    uint32_t live = 0xFFFFFFFFu;  // bit j: base i + j is not N
    if (hp.flags & HAP_HAS_N) {
        const uint32_t *m = A.nmask + hp.nmask_off + (ic >> 5);
        live = ~__builtin_amdgcn_alignbit(m[1], m[0], ic & 31);
    }
    const uint32_t L = (uint32_t)sf.z;
    if (i + L > hp.len) return 0;                       // past the end (pattern.rs:147-150)
    const int32_t sc = exact_score(words, hp, i, L, A.mweights + sf.y, live);
    if (!(sc > sf.x)) return 0;                         // strict (pattern.rs:151)
    if ((hp.flags & HAP_DEDUP) && A.dedup) {  // columns [i, i + L) the reference's: its hit (key assembly)
        bool dirty = false;
        for (uint32_t k = hp.drun_off; k < hp.drun_off + hp.n_druns && !dirty; k++)
            dirty = run_meets(A.druns[2 * k], A.druns[2 * k + 1], i, L);
        if (!dirty) return 0;
    }
    if (A.hits && i / 64 < A.hits_wpp)
        atomicOr(A.hits + ((size_t)hap * A.n_patterns_total + (uint32_t)meta[kGOrig + sn]) * A.hits_wpp + i / 64,
                 1ull << (i & 63));
    if ((hp.flags & HAP_REF) && A.dedup) {  // for the HAP_DEDUP haplotypes' unscanned windows
        const uint32_t at = atomicAdd(A.ref_count + hp.region, 1u);
        if (at < kRefPerRegion) {
            A.ref_hits[2 * ((size_t)hp.region * kRefPerRegion + at)] = g;
            A.ref_hits[2 * ((size_t)hp.region * kRefPerRegion + at) + 1] = i;
        } else {
            spill_record(A, hp.region | 0x80000000u, g, i);
        }
    }
    if (hap >= rg.hap_begin + rg.hap_count) return 0;  // a helper reference haplotype: no keys
    const uint32_t off0 = (uint32_t)sf.w * rg.n_inner;
    const int32_t *inner = A.inner + 2 * (size_t)rg.inner_off;
    // range.rs:18-21 as main.rs:503 uses it
    uint32_t mask = 0;
    const uint32_t nk = min(rg.n_inner, 32u);
    for (uint32_t k = 0; k < nk; k++) {
        const int2 r = *reinterpret_cast<const int2 *>(inner + 2 * k);
        const uint32_t span = (uint32_t)(r.y - r.x);
        if ((uint32_t)(p - r.x) <= span || (uint32_t)(p + (int32_t)L - 1 - r.x) <= span) mask |= 1u << k;
    }
    for (uint32_t k = 32; k < rg.n_inner; k++) {        // ranges past 32 (rare)
        const int32_t s = inner[2 * k], en = inner[2 * k + 1];
        const uint32_t span = (uint32_t)(en - s);
        if ((uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span)
            spill_record(A, hp.region, A.hap_base + hap, off0 + k);
    }
    *key0 = off0;
    return mask;
}

// The hit lists' room per wave (A.cand_cap per workgroup), and the candidates': the
// LDS list's (at most kWaveCands) followed by the wave's region of the global list
// (TFBS_CAND_CAP makes all of them small in the spill tests).
__device__ __forceinline__ uint32_t wave_cand_cap(const ScanArgs &A) { return A.cand_cap / (kMBlock / 64); }
__device__ __forceinline__ uint32_t wave_lds_cap(const ScanArgs &A) { return min(wave_cand_cap(A), kWaveCands); }
// slot: the workgroup's place in the per-workgroup lists (region_base + its
// haplotype group in the merged kernel's ordered launch, ScanArgs::gorder; else +
// its index).
__device__ __forceinline__ uint2 *cand_list(const ScanArgs &A, uint32_t slot, uint32_t wave) {
    return reinterpret_cast<uint2 *>(A.cands) + (size_t)slot * A.cand_cap +
           (size_t)wave * wave_cand_cap(A);
}

// The wave's listed candidates, one per lane (after its scan: no accumulator
// is live, and the other waves keep the matrix cores busy); each hit's
// (haplotype, key) pairs are appended to the wave's part of the workgroup's hit
// list in lane order (ballot prefix: no atomics), the excess spilled.
__device__ __forceinline__ void rescore_list(const ScanArgs &A, const uint32_t *words, uint32_t h0, uint32_t slot, uint32_t wave,
                                             uint32_t lane, uint32_t cn) {
    const uint32_t cap = wave_cand_cap(A);
    const size_t part = (size_t)slot * A.cand_cap + (size_t)wave * cap;
    uint2 *out = reinterpret_cast<uint2 *>(A.hitl) + part;
    uint32_t hn = 0;  // wave-uniform
    const uint32_t lcap = wave_lds_cap(A), n = min(cn, lcap + cap);
    const uint2 *glist = cand_list(A, slot, wave);
    for (uint32_t k0 = 0; k0 < n; k0 += 64) {
        const uint32_t k = k0 + lane;
        uint32_t mask = 0, key0 = 0, hap = 0;
        if (k < n) {
            const uint2 c = k < lcap ? s_cand[wave][k] : glist[k - lcap];
            hap = h0 + (c.x >> 24);
            const uint32_t hl = c.x >> 24;  // the haplotype's descriptors, staged in LDS
            mask = score_candidate(A, words, CandHap::of(s_hd[hl], s_hd2[hl]), hap, c.x & 0xFFFFFFu, c.y, &key0);
        }
        uint64_t act;
        while ((act = __ballot(mask != 0)) != 0) {
            if (mask) {
                const uint32_t at = hn + __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0));
                const uint32_t key = key0 + __builtin_ctz(mask);
                mask &= mask - 1;
                if (at < cap) out[at] = make_uint2(A.hap_base + hap, key);
                else spill_record(A, s_hd2[hap - h0].x, A.hap_base + hap, key);
            }
            hn += (uint32_t)__popcll(act);
        }
    }
    if (lane == 0) {
        A.hitn[(size_t)slot * kMBlockWaves + wave] = min(hn, cap);
        // (the list counters: per-wave stores summed on the host -- one atomic per wave on a
        // shared counter serialises at L2, ~10 ns each, and doubled the C3 step)
        A.candn[(size_t)slot * kMBlockWaves + wave] = cn;
    }
}

// Coarse test of one tile: OR of the lane's 16 outputs, the fields' top bits
// (7 v_or3 + v_bitop3); x != 0 iff the lane has a candidate.  Both tiles of a
// pair are tested in the MFMAs' basic block (tools/isa_lint.py checks the wait
// states).
__device__ __forceinline__ uint32_t coarse_test(const v16f &acc) {
    uint32_t u[16];
#pragma unroll
    for (int r = 0; r < 16; r++) u[r] = __float_as_uint(acc[r]);
#ifdef TFBS_OR_TREE  // a tree of depth 3 (the compiler chains the ORs: depth 8); the empty
                     // asm only hides the partial ORs from reassociation (no instruction)
    uint32_t p[5] = {u[0] | u[1] | u[2], u[3] | u[4] | u[5], u[6] | u[7] | u[8], u[9] | u[10] | u[11],
                     u[12] | u[13] | u[14]};
#pragma unroll
    for (int k = 0; k < 5; k++) asm volatile("" : "+v"(p[k]));
    return ((p[0] | p[1] | p[2]) | (p[3] | p[4] | u[15])) & kTestMask;
#endif
#if defined(TFBS_AB_NOTEST) || defined(TFBS_AB_NOFIRE)
    // timing ablations (wrong results): an opaque zero ends the test; NOTEST reads one
    // accumulator (the MFMAs stay live), NOFIRE keeps the whole test and never fires
    uint32_t z;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z));
#ifdef TFBS_AB_NOTEST
    return u[15] & z;
#endif
#endif
    const uint32_t x = (u[0] | u[1] | u[2]) | (u[3] | u[4] | u[5]) | (u[6] | u[7] | u[8]) | (u[9] | u[10] | u[11]) |
                       (u[12] | u[13] | u[14]) | u[15];
#ifdef TFBS_AB_NOFIRE
    return x & kTestMask & z;
#endif
    return x & kTestMask;
}

// The same tile's candidates decoded at once when the queue is full (rare): the
// lane's mask as drain_queue builds it, each candidate listed as drain_queue lists it.
__device__ __forceinline__ uint32_t record_mask(const uint32_t (&dd)[4]) {
    // dword k (queue_tile): the first strand's top bits of outputs 4k, 4k+1, 4k+2,
    // 4k+3 at 2, 10, 3, 11, the second's at 21, 29, 22, 30.  m bit b: strand b >> 4,
    // output 4 (b >> 1 & 3) + 2 (b & 1) + (b >> 3 & 1)
    uint32_t lo = (dd[0] >> 2) & 0x303u, hi = (dd[0] >> 21) & 0x303u;
#pragma unroll
    for (int k = 1; k < 4; k++) {
        lo |= (dd[k] << (2 * k - 2)) & (0x303u << (2 * k));
        hi |= (dd[k] >> (21 - 2 * k)) & (0x303u << (2 * k));
    }
    return lo | (hi << 16);
}
// bytes 1, 1', 2, 2' of outputs 2j, 2j + 1: top bits at 2, 10, 21, 29; dword k keeps
// those of j = 2k and, one bit up, of j = 2k + 1
__device__ __forceinline__ void record_bits(const v16f &acc, uint32_t (&x)[4]) {
    uint32_t d[8];
#pragma unroll
    for (int j = 0; j < 8; j++)
        d[j] = __builtin_amdgcn_perm(__float_as_uint(acc[2 * j + 1]), __float_as_uint(acc[2 * j]), 0x06020501u);
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = __builtin_amdgcn_bitop3_b32(d[2 * k], d[2 * k + 1] << 1, kQueueBits, 0xe4);  // M ? d[2k] : d[2k+1] << 1
}
// Lists the candidates of mask m (bit b: strand b >> 4 of output r(b)) of a record
// whose tile's first global strand | lane is gl and whose window entry is ent; one
// per lane per pass.
__device__ __forceinline__ void list_mask(const ScanArgs &A, const GroupCtx &G, uint32_t wave, uint32_t m, uint32_t gl,
                                          uint32_t ent, uint32_t &cn) {
    const uint32_t lcap = wave_lds_cap(A), cap = lcap + wave_cand_cap(A);
    uint2 *glist = cand_list(A, G.slot, wave);
    const uint32_t hl = ent & (kMMaxHapsPerBlock - 1), i = ent >> 6;
    const uint32_t gbase = (gl & ~63u) + 8 * ((gl >> 5) & 1u);  // the tile's first strand; lanes 32-63: pairs + 4
    uint64_t act;
    while ((act = __ballot(m != 0)) != 0) {
        if (m) {
            const uint32_t b = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t r = 4 * ((b >> 1) & 3u) + 2 * (b & 1u) + ((b >> 3) & 1u);
            const uint32_t g = gbase + 2 * ((r & 3u) + 8 * (r >> 2)) + (b >> 4);
            const uint32_t slot = cn + __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0));
            const uint2 c = make_uint2(g | (hl << 24), i);
            if (slot < lcap) {
                s_cand[wave][slot] = c;
            } else if (slot < cap) {
                glist[slot - lcap] = c;
            } else {  // rescored after the scan (cand_over_kernel / post_scan_kernel)
                const uint32_t o = atomicAdd(A.over + 1, 1u);
                if (o < A.cand_over_cap) {
                    A.cand_over[3 * (size_t)o] = A.hap_base + G.h0 + hl;  // batch index
                    A.cand_over[3 * (size_t)o + 1] = g;
                    A.cand_over[3 * (size_t)o + 2] = i;
                }
            }
        }
        cn += (uint32_t)__popcll(act);
    }
}

// Decodes the wave's first n queue records, one per lane per pass: the record's
// candidate bits (both strands of its 16 outputs) gathered into one mask, each
// candidate listed (one per lane per round; cn: the wave's count, uniform).
__device__ __forceinline__ void drain_queue(const ScanArgs &A, const GroupCtx &G, uint32_t n, uint32_t wave,
                                            uint32_t lane, uint32_t &cn) {
    for (uint32_t e0 = 0; e0 < n; e0 += 64) {
        const uint32_t e = e0 + lane;
        uint32_t m = 0, ent = 0, gl = 0;
        if (e < n) {
            const uint4 d = s_qdata[wave][e];
            const uint2 q = s_qmeta[wave][e];
            ent = q.x;
            gl = q.y;
            const uint32_t dd[4] = {d.x, d.y, d.z, d.w};
            m = record_mask(dd);
        }
        list_mask(A, G, wave, m, gl, ent, cn);
    }
}

// A firing tile (x: the lane's coarse test; q: the lane's list position, rows past
// the list's nw entries being the last tile's padding; the queue has room for the
// tile's records): each firing lane queues one record -- bytes 1-2 of its outputs
// (the fields' top bits), its list entry (window row lane & 31 of window tile
// `which`, s_went) and g0 | lane (g0: the strand tile's first global strand) --;
// qn (uniform) counts the wave's records.
__device__ __forceinline__ void queue_tile(const ScanArgs &A, const GroupCtx &G, const v16f &acc, bool mine, uint64_t f,
                                           uint32_t g0, uint32_t went, uint32_t which, uint32_t lane, uint32_t wave,
                                           uint32_t &qn, uint32_t &cn) {
    const uint32_t nf = (uint32_t)__popcll(f);
    uint32_t ent = 0, x[4] = {0, 0, 0, 0};
    if (mine) {
#ifdef TFBS_WENT_LDS  // (A/B: the round-6 first version's LDS copy of the pair's entries)
        ent = s_went[wave][which * 32 + (lane & 31)];
#else
        ent = went;  // the lane's own entry of tile `which` (lanes l and l + 32 load the same)
#endif
        record_bits(acc, x);
    }
    if (__builtin_expect(qn + nf > kMQueue, 0)) {  // the queue is full (dense hits): decoded first
        drain_queue(A, G, qn, wave, lane, cn);
        qn = 0;
    }
    if (mine) {
        const uint32_t at = __builtin_amdgcn_mbcnt_hi((uint32_t)(f >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)f, qn));
        s_qdata[wave][at] = uint4{x[0], x[1], x[2], x[3]};
        s_qmeta[wave][at] = make_uint2(ent, g0 | lane);
    }
    qn += nf;
}

// One round's chains with chunk 0's B fragment already loaded (f0: read during the
// round before, so the round's first MFMAs do not wait for LDS); chunks 1.. are read
// before the first MFMA is issued.  a1 / c1: the pair's second window tile (TWO).
template <int D, int NK, bool TWO>
__device__ __forceinline__ void round_scores(const char *tile, uint32_t lane, const BFrag &f0, const v4i (&a0)[NK],
                                             const v4i (&a1)[NK], const v16f &cb, int sa, v16f &c0, v16f &c1) {
#ifndef TFBS_B_ALL
    if (D >= 3) {
        // depth 3-4 (the class whose A fragments take 32 VGPRs): chunk kc + 1's
        // fragment read as chunk kc's MFMAs issue, a scheduling barrier between the
        // chunks -- two fragments live instead of D (no scratch spill in the merged
        // kernel)
        BFrag cur = f0;
        c0 = cb;
        if (TWO) c1 = cb;
#pragma unroll
        for (int kc = 0; kc < D; kc++) {
            BFrag nx;
            if (kc + 1 < D) {
                nx.b = *reinterpret_cast<const v4i *>(tile + (kc + 1) * 1536 + lane * 16);
                nx.c = *reinterpret_cast<const int2 *>(tile + (kc + 1) * 1536 + 1024 + lane * 8);
            }
            c0 = mfma_chunk(a0[kc], cur, c0, sa);
            if (TWO) c1 = mfma_chunk(a1[kc], cur, c1, sa);
            __builtin_amdgcn_sched_barrier(0);
            if (kc + 1 < D) cur = nx;
        }
        return;
    }
#endif
    BFrag f[D];
    f[0] = f0;
#pragma unroll
    for (int kc = 1; kc < D; kc++) {
        f[kc].b = *reinterpret_cast<const v4i *>(tile + kc * 1536 + lane * 16);
        f[kc].c = *reinterpret_cast<const int2 *>(tile + kc * 1536 + 1024 + lane * 8);
    }
    c0 = cb;
    if (TWO) c1 = cb;
#pragma unroll
    for (int kc = 0; kc < D; kc++) {
        c0 = mfma_chunk(a0[kc], f[kc], c0, sa);
        if (TWO) c1 = mfma_chunk(a1[kc], f[kc], c1, sa);
    }
}
__device__ __forceinline__ void load_frag0(const char *tile, uint32_t lane, BFrag &f) {
    f.b = *reinterpret_cast<const v4i *>(tile + lane * 16);
    f.c = *reinterpret_cast<const int2 *>(tile + 1024 + lane * 8);
}

#ifdef TFBS_ROUND_PROF
// Per-round clock split (profiling builds only, TFBS_SCAN_PROF words 8-15): per wave,
// shader cycles from a two-tile round's top to its first MFMA's issue (the chunk-0 B
// fragment and the matrix pipe), first to last MFMA issued, last MFMA to the test's
// decision, the firing path; rounds, fired rounds; the super tiles' restaging; the
// pairs' own work (next pair, list entries, A fragments).  s_memtime between
// scheduling barriers: the stamps order the round but add their own latency.
__shared__ unsigned long long s_rprof[kMBlock / 64][8];
#define RPROF_T() ({ __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                     __builtin_amdgcn_sched_barrier(0); t_; })
#define RPROF_ADD(wave, k, v) do { if ((threadIdx.x & 63) == 0) s_rprof[wave][k] += (v); } while (0)
#endif

// The strand tiles of depth D, [tb, te) (images from `img`), x window tiles ta (A
// fragments a0) and, if TWO, ta + 1 (a1) of the group's list: per strand tile one
// round (D chunks x the window tiles), the coarse test of both tiles with one vector
// compare, the firing path (queue_tile) only when some lane fired.  A pointer loop (3
// scalar instructions per round); the next round's chunk-0 B fragment is read
// unconditionally (past the last tile: the image area is padded by kMChunkBytes, the
// value unused).
template <int D, int NK, bool TWO>
__device__ __forceinline__ void scan_segment(const ScanArgs &A, const char *img, uint32_t tb, uint32_t te,
                                             const GroupCtx &G, uint32_t lane, uint32_t wave, const v4i (&a0)[NK],
                                             const v4i (&a1)[NK], uint32_t ta, uint32_t e0, uint32_t e1, const v16f &cb,
                                             int sa, uint32_t &qn, uint32_t &cn) {
    constexpr uint32_t kTB = mfma_tile_bytes(D);
    const char *tile = img;
    const char *const end = img + (te - tb) * kTB;
    uint32_t g0 = (G.tile0 + tb) * kMStrands;  // the tile's first global strand
    const uint32_t q0 = kMWindows * ta + (lane & 31);  // the lane's list positions (tile a; tile b: + 32)
    BFrag pf;
    load_frag0(img, lane, pf);
#ifdef TFBS_ROUND_PROF
    unsigned long long pb = 0, pm = 0, pt = 0, pfi = 0, nr = 0, nf = 0;
#endif
    do {
#ifdef TFBS_ROUND_PROF
        const unsigned long long t0 = RPROF_T();
        BFrag f[D];
        f[0] = pf;
#pragma unroll
        for (int kc = 1; kc < D; kc++) {
            f[kc].b = *reinterpret_cast<const v4i *>(tile + kc * 1536 + lane * 16);
            f[kc].c = *reinterpret_cast<const int2 *>(tile + kc * 1536 + 1024 + lane * 8);
        }
        v16f c0 = mfma_chunk(a0[0], f[0], cb, sa), c1;
        const unsigned long long t1 = RPROF_T();
        if (TWO) c1 = mfma_chunk(a1[0], f[0], cb, sa);
#pragma unroll
        for (int kc = 1; kc < D; kc++) {
            c0 = mfma_chunk(a0[kc], f[kc], c0, sa);
            if (TWO) c1 = mfma_chunk(a1[kc], f[kc], c1, sa);
        }
        const unsigned long long t2 = RPROF_T();
#else
        v16f c0, c1;
        round_scores<D, NK, TWO>(tile, lane, pf, a0, a1, cb, sa, c0, c1);
#endif
#ifdef TFBS_NO_READ2
        asm volatile("" ::: "memory");  // (A/B) no ds_read2 merged with the round's reads: no v_mov copies
#endif
        load_frag0(tile + kTB, lane, pf);
        const uint32_t x0 = coarse_test(c0), x1 = TWO ? coarse_test(c1) : 0u;
        const bool fired = __ballot((x0 | x1) != 0) != 0;
#ifdef TFBS_ROUND_PROF
        const unsigned long long t3 = RPROF_T();
#endif
        if (__builtin_expect(fired, 0)) {
#ifdef TFBS_ROUND_PROF
            nf++;
#endif
            // cold: queue the firing lanes' records (padding rows left out), or list
            // a tile's candidates at once when the queue is full
            const bool m0 = x0 != 0 && q0 < G.nw, m1 = TWO && x1 != 0 && q0 + kMWindows < G.nw;
            const uint64_t f0 = __ballot(m0), f1 = __ballot(m1);
            if (f0) queue_tile(A, G, c0, m0, f0, g0, e0, 0, lane, wave, qn, cn);
            if (TWO && f1) queue_tile(A, G, c1, m1, f1, g0, e1, 1, lane, wave, qn, cn);
        }
#ifdef TFBS_ROUND_PROF
        const unsigned long long t4 = RPROF_T();
        pb += t1 - t0;
        pm += t2 - t1;
        pt += t3 - t2;
        pfi += t4 - t3;
        nr++;
#endif
        tile += kTB;
        g0 += kMStrands;
    } while (tile != end);
#ifdef TFBS_ROUND_PROF
    if (TWO) {
        RPROF_ADD(wave, 0, pb);
        RPROF_ADD(wave, 1, pm);
        RPROF_ADD(wave, 2, pt);
        RPROF_ADD(wave, 3, pfi);
        RPROF_ADD(wave, 4, nr);
        RPROF_ADD(wave, 5, nf);
    }
#endif
}

// One step: every strand tile of the super tile (depth segments 1..NK, byte
// d - 1 of seg = the end of depth d) x the window tiles ta and, if TWO, ta + 1.
template <int NK, bool TWO>
__device__ __forceinline__ void scan_step(const ScanArgs &A, const char *s_img, uint32_t seg, const GroupCtx &G,
                                          uint32_t lane, uint32_t wave, const v4i (&a0)[NK], const v4i (&a1)[NK],
                                          uint32_t ta, uint32_t e0, uint32_t e1, const v16f &cb, int sa, uint32_t &qn,
                                          uint32_t &cn) {
    uint32_t tb = NK > 2 ? (seg >> 8) & 255u : 0;  // class 4 starts at depth 3 (no tile of depth 1-2)
    const char *img = s_img;
#define TFBS_SEGMENT(D)                                                                                          \
    if (D <= NK && D + 1 >= NK) { /* a class holds depths NK - 1 and NK (mfma_depth_class) */                  \
        const uint32_t te = (seg >> (8 * (D - 1))) & 255u;                                                     \
        if (te > tb)                                                                                             \
            scan_segment<(D <= NK ? D : 1), NK, TWO>(A, img, tb, te, G, lane, wave, a0, a1, ta, e0, e1, cb, sa, qn, cn); \
        img += (te - tb) * mfma_tile_bytes(D);                                                                   \
        tb = te;                                                                                                 \
    }
    TFBS_SEGMENT(1)
    TFBS_SEGMENT(2)
    TFBS_SEGMENT(3)
    TFBS_SEGMENT(4)
#undef TFBS_SEGMENT
}

// The A fragments of list entry we (window << 6 | haplotype in the group): the
// lane's haplotype from the LDS descriptors, its window's words, the one-hot.
template <int NK>
__device__ __forceinline__ void entry_onehot(const ScanArgs &A, const uint32_t *words, uint32_t we, const char *tab,
                                             v4i (&a)[NK]) {
    const uint4 d = s_hd[we & (kMMaxHapsPerBlock - 1)];
    const LaneHap hm{d.x, d.y, d.z, d.w};
    const uint32_t i = we >> 6;
    WinWords ww;
    load_window(A, words, hm, i, ww);
    build_onehot<NK>(hm, i, ww, tab, a);
}

// words: the packed haplotype words, indexed by DevHap::word_off (an LDS copy
// of this workgroup's haplotypes, biased by their first word, or global memory).
// The group's window list (the windows of its haplotypes the class reads) is
// cut into tiles of 32 windows (the last one padded with its last window),
// handed to the waves two at a time from an LDS counter -- the waves finish
// together however the windows fall -- and the next pair's list entries are
// loaded while the current pair is scored.
#ifdef TFBS_SCAN_PROF
// per wave: [0] s_memtime at the kernel's start, [1] after the staging barrier, [2]
// after the scan loops, [3] (the same), [4] after the rescoring, [5] / [6]
// s_memrealtime (100 MHz, one clock for the chip) at the start and the end, [7] pairs
// scored | candidates << 32; [8, 16) TFBS_ROUND_PROF's split
#define SCAN_STAMP(k, v) \
    do { if (A.prof && lane == 0) A.prof[((size_t)slot * kMBlockWaves + wave) * kScanProfWords + (k)] = (v); } while (0)
#else
#define SCAN_STAMP(k, v) do { } while (0)
#endif

// One super tile's window pairs over the group's list of its depth class, then the
// wave's last queue records decoded (qn, cn: the wave's queued records and listed
// candidates, carried over super tiles).  Returns the pairs this wave scored.
template <int NK>
__device__ __forceinline__ uint32_t scan_loop(const ScanArgs &A, const DevMSuper &S, const char *s_img,
                                              const uint32_t *words, uint32_t hg, uint32_t slot, uint32_t lane,
                                              uint32_t wave, uint32_t &qn, uint32_t &cn) {
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t h1 = min(h0 + A.haps_per_block, A.n_haps);
    const uint64_t e0 = A.wlist_off[NK > 2][h0];
    GroupCtx G;
    G.wl = A.wlist[NK > 2] + e0;
    G.wl16 = (A.gnarrow && A.gnarrow[hg]) ? A.wlist16[NK > 2] + e0 : nullptr;
    G.nw = (uint32_t)(A.wlist_off[NK > 2][h1] - e0);
    G.tile0 = S.tile0;
    G.h0 = h0;
    G.slot = slot;
    const uint32_t ntile = (G.nw + kMWindows - 1) / kMWindows, npair = (ntile + 1) / 2;
    const float a0f = __uint_as_float(S.acc0);
    v16f cb = {a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f, a0f};
    asm volatile("" : "+v"(cb));  // kept in VGPRs: every round's MFMAs read it (no per-round copies)
    const int sa = lane < 32 ? kScaleD0 : kScaleD1;
    const char *tab = s_img - kMOnehotBytes;
    auto next_pair = [&]() {
        uint32_t p = 0;
        if (lane == 0) p = atomicAdd(&s_hnext, 1u);
        return (uint32_t)__builtin_amdgcn_readfirstlane(p);
    };
    // lane l scores window row l & 31 of each tile
    auto entries = [&](uint32_t p, uint32_t &ea, uint32_t &eb) {
        const uint32_t q = kMWindows * 2 * p + (lane & 31);
        ea = G.at(min(q, G.nw - 1));
        eb = G.at(min(q + kMWindows, G.nw - 1));
    };
    uint32_t p = next_pair(), ea = 0, eb = 0, n_pairs = 0;
    if (p < npair) entries(p, ea, eb);
    while (p < npair) {
        n_pairs++;
#ifdef TFBS_ROUND_PROF
        const unsigned long long tp0 = RPROF_T();
#endif
        const uint32_t pn = next_pair();
        const bool two = 2 * p + 1 < ntile;
        v4i a0[NK], a1[NK];
        entry_onehot<NK>(A, words, ea, tab, a0);
        entry_onehot<NK>(A, words, eb, tab, a1);  // (a copy of the last window when !two: unused)
#ifdef TFBS_WENT_LDS
        s_went[wave][lane] = lane < 32 ? ea : eb;  // the firing path's windows (queue_tile)
#endif
        const uint32_t e0 = ea, e1 = eb;          // (the firing path's entries: the lane's own)
        if (pn < npair) entries(pn, ea, eb);      // in flight while this pair is scored
#ifdef TFBS_ROUND_PROF
        // the A fragments awaited here (their LDS reads), so that the pair's first
        // round does not carry them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long tp1 = RPROF_T();
        RPROF_ADD(wave, 7, tp1 - tp0);
#endif
        if (two) scan_step<NK, true>(A, s_img, S.seg, G, lane, wave, a0, a1, 2 * p, e0, e1, cb, sa, qn, cn);
        else scan_step<NK, false>(A, s_img, S.seg, G, lane, wave, a0, a1, 2 * p, e0, e1, cb, sa, qn, cn);
        p = pn;
    }
    drain_queue(A, G, qn, wave, lane, cn);  // (the records are self-contained: a drain per super tile)
    qn = 0;
    return n_pairs;
}

// LDS staging of a workgroup (a plain copy loop: batching all loads before the
// stores was slower, 2.84 -> 3.10 ms per C3 step).
__device__ __forceinline__ void stage_image(const ScanArgs &A, const DevMSuper &S, uint4 *dst) {
    const uint4 *src = reinterpret_cast<const uint4 *>(A.mimage + S.img_off / 4);
    const uint32_t n16 = S.img_bytes / 16;
    for (uint32_t i = threadIdx.x; i < n16; i += kMBlock) dst[kMOnehotBytes / 16 + i] = src[i];
}

// The one-hot table (4-mer code -> 64 bits, column t (16 bits) holds FP4 1.0 (0x2)
// in the nibble of its base), the group's descriptors and (STAGED) its packed
// words after the image budget; returns the words' base for DevHap::word_off.
template <bool STAGED>
__device__ __forceinline__ const uint32_t *stage_group(const ScanArgs &A, int32_t *smem, uint32_t h0, uint32_t hn) {
    uint2 *tab = reinterpret_cast<uint2 *>(smem);
    for (uint32_t k = threadIdx.x; k < 256; k += kMBlock) {
        uint32_t h[4];
        for (int t = 0; t < 4; t++) h[t] = 2u << (4 * ((k >> (2 * t)) & 3));
        tab[k] = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    }
    if (threadIdx.x < hn) {  // (32 of DevHap's 48 bytes)
        s_hd[threadIdx.x] = A.hd[h0 + threadIdx.x];
        s_hd2[threadIdx.x] = A.hd2[h0 + threadIdx.x];
    }
    if (!STAGED) return A.words;
    const uint4 f = A.hd[h0], l = A.hd[h0 + hn - 1];
    const uint32_t wbeg = f.x;
    const uint32_t wend = l.x + (l.y + 15) / 16 + 3;
    uint32_t *s_words = reinterpret_cast<uint32_t *>(smem) + (kMOnehotBytes + A.mimg_max + kMChunkBytes) / 4;
    for (uint32_t i = threadIdx.x; i < wend - wbeg; i += kMBlock) s_words[i] = A.words[wbeg + i];
    return s_words - wbeg;
}

// Grid: n_msupers x ceil(n_haps / haps_per_block), 4 waves per SIMD (two workgroups per CU).
// LDS: one-hot table | super tile image | (STAGED) the packed words of the
// workgroup's haplotypes, copied once so that every window read is an LDS read.
template <bool STAGED, int NK>
__global__ __launch_bounds__(kMBlock, kMfmaMinWaves[NK]) void scan_mfma_kernel(ScanArgs A) {
#ifdef TFBS_SCAN_PROF
    const unsigned long long t_start = __builtin_amdgcn_s_memtime(), r_start = __builtin_amdgcn_s_memrealtime();
#endif
    int32_t *smem = s_mdyn;
    const uint32_t sidx = blockIdx.x % A.n_msupers;
    const uint32_t hg = blockIdx.x / A.n_msupers;
    const uint32_t slot = A.region_base + blockIdx.x;
    const DevMSuper S = A.msupers[sidx];
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t hn = min(h0 + A.haps_per_block, A.n_haps) - h0;
    stage_image(A, S, reinterpret_cast<uint4 *>(smem));
    if (threadIdx.x == 0) s_hnext = 0;
    const uint32_t *words = stage_group<STAGED>(A, smem, h0, hn);
    __syncthreads();
    const char *s_img = reinterpret_cast<const char *>(smem) + kMOnehotBytes;
    // the wave index is uniform: keep every group-level value in SGPRs
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef TFBS_SCAN_PROF
    SCAN_STAMP(0, t_start);
    SCAN_STAMP(5, r_start);
    SCAN_STAMP(1, __builtin_amdgcn_s_memtime());
#endif
    uint32_t qn = 0, cn = 0;
    const uint32_t n_pairs = scan_loop<NK>(A, S, s_img, words, hg, slot, lane, wave, qn, cn);
    (void)n_pairs;
    SCAN_STAMP(2, __builtin_amdgcn_s_memtime());
    SCAN_STAMP(3, __builtin_amdgcn_s_memtime());
    rescore_list(A, words, h0, slot, wave, lane, cn);
    SCAN_STAMP(4, __builtin_amdgcn_s_memtime());
    SCAN_STAMP(6, __builtin_amdgcn_s_memrealtime());
    SCAN_STAMP(7, (unsigned long long)n_pairs | ((unsigned long long)cn << 32));
}

// One workgroup per haplotype group for EVERY super tile (the depth classes in
// turn): the group's words, descriptors and one-hot table are staged once, each
// super tile's image in turn (a barrier on either side), and the wave rescores its
// candidates of all of them once at the end -- the per-workgroup costs (staging,
// the rescoring's dependent loads) are paid once per group instead of once per
// super tile.  LDS: one-hot table | the largest image | (STAGED) words.
}  // namespace
// post_scan_kernel's work by one workgroup of NT threads (defined below); s_sum: NT + 1
// words of LDS
template <uint32_t NT>
__device__ void post_one_block(const ScanArgs &A, uint32_t tid, uint32_t n_regions, uint32_t *__restrict__ bcnt,
                               uint32_t *__restrict__ boff, uint32_t *__restrict__ sorted,
                               uint32_t *__restrict__ report, uint32_t *__restrict__ need_wide, uint32_t *s_sum);
namespace {

template <bool STAGED>
__global__ __launch_bounds__(kMBlock, 4) void scan_mfma_all_kernel(ScanArgs A) {
#ifdef TFBS_SCAN_PROF
    const unsigned long long t_start = __builtin_amdgcn_s_memtime(), r_start = __builtin_amdgcn_s_memrealtime();
#endif
    int32_t *smem = s_mdyn;
    const uint32_t hg = A.gorder ? A.gorder[blockIdx.x] : blockIdx.x;  // (its lists and stamps at slot hg)
    const uint32_t slot = A.region_base + hg;
    const uint32_t h0 = hg * A.haps_per_block;
    const uint32_t hn = min(h0 + A.haps_per_block, A.n_haps) - h0;
    const uint32_t *words = stage_group<STAGED>(A, smem, h0, hn);
    const char *s_img = reinterpret_cast<const char *>(smem) + kMOnehotBytes;
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifdef TFBS_SETPRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // (A/B) the workgroup's second half wins issue ties
#endif
    uint32_t qn = 0, cn = 0, n_pairs = 0;
#ifdef TFBS_SCAN_PROF
    bool first = true;
#endif
#ifdef TFBS_ROUND_PROF
    if (threadIdx.x < kMBlockWaves * 8) (&s_rprof[0][0])[threadIdx.x] = 0;
#endif
    for (uint32_t si = 0; si < A.n_msupers; si++) {
        const DevMSuper S = A.msupers[si];
#ifdef TFBS_ROUND_PROF
        const unsigned long long ts0 = RPROF_T();
#endif
        __syncthreads();  // the previous image's readers are done
#ifdef TFBS_AB_NORESTAGE  // timing ablation (wrong results): the first image only
        if (si == 0)
#endif
        stage_image(A, S, reinterpret_cast<uint4 *>(smem));
        if (threadIdx.x == 0) s_hnext = 0;
        __syncthreads();
#ifdef TFBS_ROUND_PROF
        if (si) RPROF_ADD(wave, 6, RPROF_T() - ts0);
#endif
#ifdef TFBS_SCAN_PROF
        if (first) {
            SCAN_STAMP(0, t_start);
            SCAN_STAMP(5, r_start);
            SCAN_STAMP(1, __builtin_amdgcn_s_memtime());
            first = false;
        }
#endif
        n_pairs += S.nk > 2 ? scan_loop<4>(A, S, s_img, words, hg, slot, lane, wave, qn, cn)
                            : scan_loop<2>(A, S, s_img, words, hg, slot, lane, wave, qn, cn);
    }
    (void)n_pairs;
    SCAN_STAMP(2, __builtin_amdgcn_s_memtime());
    SCAN_STAMP(3, __builtin_amdgcn_s_memtime());
#ifndef TFBS_AB_NORESCORE  // timing ablation (wrong results): no rescoring
    rescore_list(A, words, h0, slot, wave, lane, cn);
#endif
    SCAN_STAMP(4, __builtin_amdgcn_s_memtime());
    SCAN_STAMP(6, __builtin_amdgcn_s_memrealtime());
    SCAN_STAMP(7, (unsigned long long)n_pairs | ((unsigned long long)cn << 32));
#ifdef TFBS_ROUND_PROF
    for (int k = 0; k < 8; k++) SCAN_STAMP(8 + k, s_rprof[wave][k]);
#endif
    if (A.post_done) {  // fused post-scan: the last workgroup to finish does it
        __syncthreads();  // every wave's lists and spill records are written
        uint32_t *s_t = reinterpret_cast<uint32_t *>(&s_qdata[0][0]);  // (the queues are empty now)
        if (threadIdx.x == 0) {
            __threadfence();  // (release: this workgroup's records)
            s_t[0] = atomicAdd(A.post_done, 1u) == gridDim.x - 1 ? 1u : 0u;
        }
        __syncthreads();
        if (s_t[0]) {
            __threadfence();  // (acquire: every workgroup's records)
            post_one_block<kMBlock>(A, threadIdx.x, A.post_regions, A.post_bcnt, A.post_boff, A.post_sorted,
                                    A.post_report, A.post_need_wide, s_t + 4);
        }
    }
}

// Candidates past the waves' lists (drain_queue), one per thread; their
// hits go to the spill list.
__global__ __launch_bounds__(256) void cand_over_kernel(ScanArgs A) {
    const uint32_t n = min(A.over[1], A.cand_over_cap);
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
        const uint32_t hap = A.cand_over[3 * (size_t)k], g = A.cand_over[3 * (size_t)k + 1];
        const DevHap hp = A.haps[hap];
        uint32_t key0 = 0;
        for (uint32_t m = score_candidate(A, A.words, CandHap::of(hp), hap, g, A.cand_over[3 * (size_t)k + 2], &key0); m;
             m &= m - 1)
            spill_record(A, hp.region, hap, key0 + __builtin_ctz(m));
    }
}

// ---------------------------------------------------------------------------
// Window lists (ScanArgs::wlist): per depth class of span S, the windows [0, len
// - lmin + 1) of every haplotype, only those meeting a diff run for a HAP_DEDUP
// haplotype (tfbs_internal.hpp): f(lo, hi) gets them as ascending intervals.
template <class F>
__device__ __forceinline__ uint32_t for_windows(const DevHap &hm, const uint32_t *druns, uint32_t lmin, uint32_t S,
                                                uint32_t dedup, F &&f) {
    if (hm.len < lmin) return 0;
    const uint32_t nw = hm.len - lmin + 1;
    if (!dedup || !(hm.flags & HAP_DEDUP)) {
        f(0u, nw);
        return nw;
    }
    uint32_t n = 0, next = 0;  // windows below next are listed
    for (uint32_t k = 0; k < hm.n_druns; k++) {
        const uint32_t a = druns[2 * (hm.drun_off + k)], b = druns[2 * (hm.drun_off + k) + 1];
        const uint32_t lo = max(next, a >= S - 1 ? a - (S - 1) : 0u), hi = min(b, nw - 1) + 1;
        if (hi > lo) {
            f(lo, hi);
            n += hi - lo;
            next = hi;
        }
    }
    return n;
}

__global__ __launch_bounds__(256) void wl_count_kernel(const DevHap *__restrict__ haps, uint32_t n,
                                                       const uint32_t *__restrict__ druns, uint32_t lmin, uint32_t S,
                                                       uint32_t dedup, uint64_t *__restrict__ cnt) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h > n) return;
    cnt[h] = h < n ? for_windows(haps[h], druns, lmin, S, dedup, [](uint32_t, uint32_t) {}) : 0u;
}

// one wave per haplotype: its entries written 64 at a time
__global__ __launch_bounds__(256) void wl_fill_kernel(const DevHap *__restrict__ haps, uint32_t n,
                                                      const uint32_t *__restrict__ druns, uint32_t lmin, uint32_t S,
                                                      uint32_t dedup, uint32_t hpb, const uint64_t *__restrict__ off,
                                                      uint32_t *__restrict__ list, uint16_t *__restrict__ list16,
                                                      const uint8_t *__restrict__ gnarrow) {
    const uint32_t h = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (h >= n) return;
    uint64_t at = off[h];
    const uint32_t hl = h % hpb;
    const bool narrow = gnarrow && gnarrow[h / hpb];
    for_windows(haps[h], druns, lmin, S, dedup, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t w = lo + lane; w < hi; w += 64) {
            if (narrow) list16[at + (w - lo)] = (uint16_t)((w << 6) | hl);
            else list[at + (w - lo)] = (w << 6) | hl;
        }
        at += hi - lo;
    });
}

__global__ __launch_bounds__(256) void group_cost_kernel(const uint64_t *__restrict__ off0,
                                                         const uint64_t *__restrict__ off1, uint32_t n_haps, uint32_t hpb,
                                                         uint32_t n_groups, uint32_t w0, uint32_t w1,
                                                         uint32_t *__restrict__ cost) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= n_groups) return;
    const uint32_t h0 = g * hpb, h1 = min(h0 + hpb, n_haps);
    uint64_t c = 0;
    if (off0) c += (off0[h1] - off0[h0] + 2 * kMWindows - 1) / (2 * kMWindows) * w0;
    if (off1) c += (off1[h1] - off1[h0] + 2 * kMWindows - 1) / (2 * kMWindows) * w1;
    cost[g] = (uint32_t)min<uint64_t>(c, 0xFFFFFFFFu);
}

// The scan's compact haplotype descriptors (ScanArgs::hd): word offset, length,
// flags, N-mask offset of every DevHap.
__global__ __launch_bounds__(256) void hd_kernel(const DevHap *__restrict__ haps, uint32_t n, uint4 *__restrict__ hd,
                                                  uint4 *__restrict__ hd2) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h < n) {
        const DevHap x = haps[h];
        hd[h] = make_uint4(x.word_off, x.len, x.flags, x.nmask_off);
        hd2[h] = make_uint4(x.region, x.pos_off, x.drun_off, x.n_druns);
    }
}

// In-place exclusive scan of u64 values, 4096 per workgroup; sums[b] = tile b's total.
constexpr uint32_t kScanThreads = 1024, kScanTile = 4 * kScanThreads;
__global__ __launch_bounds__(kScanThreads) void scan_tile_kernel(uint64_t *__restrict__ x, uint64_t n,
                                                                 uint64_t *__restrict__ sums) {
    __shared__ uint64_t s[2][kScanThreads];
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + 4 * t;
    uint64_t v[4], tot = 0;
    for (int k = 0; k < 4; k++) {
        v[k] = base + k < n ? x[base + k] : 0;
        tot += v[k];
    }
    int cur = 0;
    s[0][t] = tot;
    __syncthreads();
    for (uint32_t o = 1; o < kScanThreads; o <<= 1) {
        s[cur ^ 1][t] = s[cur][t] + (t >= o ? s[cur][t - o] : 0);
        cur ^= 1;
        __syncthreads();
    }
    uint64_t run = s[cur][t] - tot;
    for (int k = 0; k < 4; k++) {
        if (base + k < n) x[base + k] = run;
        run += v[k];
    }
    if (t == kScanThreads - 1) sums[blockIdx.x] = s[cur][t];
}

__global__ __launch_bounds__(256) void scan_add_kernel(uint64_t *__restrict__ x, uint64_t n,
                                                       const uint64_t *__restrict__ sums) {
    const uint64_t add = sums[blockIdx.x];
    for (uint32_t k = threadIdx.x; k < kScanTile; k += 256) {
        const uint64_t i = (uint64_t)blockIdx.x * kScanTile + k;
        if (i < n) x[i] += add;
    }
}

int exclusive_scan(uint64_t *x, uint64_t n, uint64_t *tmp, hipStream_t stream) {
    const uint64_t nt = (n + kScanTile - 1) / kScanTile;
    if (nt == 0) return TFBS_OK;
    hipLaunchKernelGGL(scan_tile_kernel, dim3((uint32_t)nt), dim3(kScanThreads), 0, stream, x, n, tmp);
    if (nt > 1) {
        if (int rc = exclusive_scan(tmp, nt, tmp + nt, stream)) return rc;
        hipLaunchKernelGGL(scan_add_kernel, dim3((uint32_t)nt), dim3(256), 0, stream, x, n, tmp);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan kernels: ") + hipGetErrorString(e));
    return TFBS_OK;
}

typedef void (*MfmaKernel)(ScanArgs);
template <int NK> MfmaKernel mfma_nk(bool staged) {
    return staged ? scan_mfma_kernel<true, NK> : scan_mfma_kernel<false, NK>;
}
MfmaKernel mfma_variant(bool staged, uint32_t nk) {  // depth classes (mfma_depth_class)
    return nk <= 2 ? mfma_nk<2>(staged) : mfma_nk<4>(staged);
}
MfmaKernel mfma_all_variant(bool staged) { return staged ? scan_mfma_all_kernel<true> : scan_mfma_all_kernel<false>; }

}  // namespace

// The scan's post-processing in one launch: every workgroup rescores its share of
// the overflow candidates (cand_over_kernel's work, when `cand`), then the last
// workgroup to finish -- the one whose ticket on *done (zeroed before) is the
// grid's last -- buckets the spill records by region (a histogram, an exclusive
// scan into boff, a scatter into sorted; bcnt n_regions + 1 zeroed before) on its
// own: spills are rare, and no records (the usual case) costs one counter read.
constexpr uint32_t kPostBlock = 256;

// boff[0 .. n_regions]: the exclusive prefix of the bucket counts (one workgroup of
// kPostBlock threads) -- each thread a run of consecutive buckets, one block scan of
// the runs' sums (not one per 256 buckets: 10 000 regions took 40 scans of 16
// barriers); the counts are zeroed for the scatter's fill counters
template <uint32_t NT = kPostBlock>
__device__ void spill_bucket_offsets(uint32_t tid, uint32_t n_regions, uint32_t *__restrict__ bcnt,
                                     uint32_t *__restrict__ boff, uint32_t *s_sum) {
    const uint32_t per = (n_regions + NT) / NT;  // ceil((n_regions + 1) / NT)
    const uint32_t i0 = min(tid * per, n_regions + 1), i1 = min(i0 + per, n_regions + 1);
    uint32_t mine = 0;
    for (uint32_t i = i0; i < i1; i++) mine += i < n_regions ? bcnt[i] : 0u;
    s_sum[tid] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < NT; o <<= 1) {
        const uint32_t t = tid >= o ? s_sum[tid - o] : 0u;
        __syncthreads();
        s_sum[tid] += t;
        __syncthreads();
    }
    uint32_t at = s_sum[tid] - mine;
    for (uint32_t i = i0; i < i1; i++) {
        const uint32_t v = i < n_regions ? bcnt[i] : 0u;
        boff[i] = at;
        at += v;
        if (i < n_regions) bcnt[i] = 0;
    }
}

// report (optional): the final overflow counters copied there by the last workgroup (the
// assembly's check, when its leftover pass -- which copies them otherwise -- is not
// launched); need_wide (optional: the wide kernels are not launched): set when the
// records are too many for the last workgroup, so that the host reruns the assembly
// with them.
// The overflow candidates' rescoring, block blk of nblk (NT threads): the hits' spill
// records get their slots one atomic per wave (C5: ~120 000 records through one
// counter, one atomic each, took ~1 ms); the loop is wave-uniform for the wave sum.
template <uint32_t NT>
__device__ void post_candidates(const ScanArgs &A, uint32_t tid, uint32_t blk, uint32_t nblk) {
    const uint32_t n = min(A.over[1], A.cand_over_cap), lane = tid & 63;
    for (uint32_t k0 = blk * NT; k0 < n; k0 += nblk * NT) {
        const uint32_t k = k0 + tid;
        uint32_t m = 0, key0 = 0, region = 0, hap = 0;
        if (k < n) {
            hap = A.cand_over[3 * (size_t)k];
            const uint32_t g = A.cand_over[3 * (size_t)k + 1];
            const DevHap hp = A.haps[hap];
            region = hp.region;
            m = score_candidate(A, A.words, CandHap::of(hp), hap, g, A.cand_over[3 * (size_t)k + 2], &key0);
        }
        const uint32_t c = (uint32_t)__builtin_popcount(m);
        uint32_t inc = c;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= o) inc += t;
        }
        const uint32_t total = (uint32_t)__shfl((int)inc, 63);
        uint32_t base = 0;
        if (lane == 0 && total) base = atomicAdd(A.over, total);
        uint32_t at = (uint32_t)__shfl((int)base, 0) + inc - c;
        for (; m; m &= m - 1, at++)
            if (at < A.spill_cap) {
                A.spill[3 * (size_t)at] = region;
                A.spill[3 * (size_t)at + 1] = hap;
                A.spill[3 * (size_t)at + 2] = key0 + __builtin_ctz(m);
            }
    }
}

// The last workgroup's part (every workgroup's spill records visible): the overflow
// counters to report, then the records bucketed by region when they are few.
template <uint32_t NT>
__device__ void post_buckets(const ScanArgs &A, uint32_t tid, uint32_t n_regions, uint32_t *__restrict__ bcnt,
                             uint32_t *__restrict__ boff, uint32_t *__restrict__ sorted,
                             uint32_t *__restrict__ report, uint32_t *__restrict__ need_wide, uint32_t *s_sum) {
    if (report && tid < 2) report[tid] = __atomic_load_n(A.over + tid, __ATOMIC_RELAXED);
    const uint32_t n = min(__atomic_load_n(A.over, __ATOMIC_RELAXED), A.spill_cap);
    if (n == 0) return;  // no records: the readers skip the buckets (AsmArgs::spill_count)
    if (n > kPostSerial) {  // spill_hist_wide_kernel + spill_scatter_wide_kernel's
        if (need_wide && tid == 0) *need_wide = 1u;
        return;
    }
    for (uint32_t e = tid; e < n; e += NT) atomicAdd(&bcnt[A.spill[3 * (size_t)e] & 0x7FFFFFFFu], 1u);
    __threadfence();  // (the counters' atomics and boff's stores seen by every thread of the block)
    __syncthreads();
    spill_bucket_offsets<NT>(tid, n_regions, bcnt, boff, s_sum);
    __threadfence();  // (the counters' atomics and boff's stores seen by every thread of the block)
    __syncthreads();
    for (uint32_t e = tid; e < n; e += NT) {
        const uint32_t r = A.spill[3 * (size_t)e] & 0x7FFFFFFFu;
        const uint32_t at = boff[r] + atomicAdd(&bcnt[r], 1u);
        sorted[3 * (size_t)at] = A.spill[3 * (size_t)e];
        sorted[3 * (size_t)at + 1] = A.spill[3 * (size_t)e + 1];
        sorted[3 * (size_t)at + 2] = A.spill[3 * (size_t)e + 2];
    }
}

template <uint32_t NT>
__device__ void post_one_block(const ScanArgs &A, uint32_t tid, uint32_t n_regions, uint32_t *__restrict__ bcnt,
                               uint32_t *__restrict__ boff, uint32_t *__restrict__ sorted,
                               uint32_t *__restrict__ report, uint32_t *__restrict__ need_wide, uint32_t *s_sum) {
    post_candidates<NT>(A, tid, 0, 1);
    __threadfence();  // (its spill records, for the whole block)
    __syncthreads();
    post_buckets<NT>(A, tid, n_regions, bcnt, boff, sorted, report, need_wide, s_sum);
}
// (the merged scan kernel's tail, instantiated above this definition)
template __device__ void post_one_block<kMBlock>(const ScanArgs &, uint32_t, uint32_t, uint32_t *, uint32_t *,
                                                 uint32_t *, uint32_t *, uint32_t *, uint32_t *);

__global__ __launch_bounds__(kPostBlock) void post_scan_kernel(ScanArgs A, uint32_t cand, uint32_t *done,
                                                              uint32_t n_regions, uint32_t *__restrict__ bcnt,
                                                              uint32_t *__restrict__ boff,
                                                              uint32_t *__restrict__ sorted,
                                                              uint32_t *__restrict__ report,
                                                              uint32_t *__restrict__ need_wide) {
    __shared__ uint32_t s_last, s_sum[kPostBlock];
    const uint32_t tid = threadIdx.x;
    if (cand) post_candidates<kPostBlock>(A, tid, blockIdx.x, gridDim.x);
    __syncthreads();
    if (tid == 0) {
        __threadfence();  // (release: this workgroup's spill records)
        s_last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();  // (acquire: every workgroup's records)
    post_buckets<kPostBlock>(A, tid, n_regions, bcnt, boff, sorted, report, need_wide, s_sum);
}

// More than kPostSerial spill records: their bucket counts over the whole grid, then
// the last workgroup (finish ticket) the offsets; the scatter below, also over the
// grid (C5's ~120 000 records took ~1 ms in post_scan_kernel's last workgroup).
__global__ __launch_bounds__(kPostBlock) void spill_hist_wide_kernel(ScanArgs A, uint32_t *done, uint32_t n_regions,
                                                                     uint32_t *__restrict__ bcnt,
                                                                     uint32_t *__restrict__ boff) {
    __shared__ uint32_t s_last, s_sum[kPostBlock];
    const uint32_t tid = threadIdx.x;
    const uint32_t n = min(A.over[0], A.spill_cap);
    if (n <= kPostSerial) return;  // (uniform: post_scan_kernel bucketed them)
    for (uint32_t e = blockIdx.x * kPostBlock + tid; e < n; e += gridDim.x * kPostBlock)
        atomicAdd(&bcnt[A.spill[3 * (size_t)e] & 0x7FFFFFFFu], 1u);
    __syncthreads();
    if (tid == 0) {
        __threadfence();  // (release: this workgroup's counts)
        s_last = atomicAdd(done, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();  // (acquire: every workgroup's counts)
    spill_bucket_offsets(tid, n_regions, bcnt, boff, s_sum);
}

__global__ __launch_bounds__(256) void spill_scatter_wide_kernel(ScanArgs A, const uint32_t *__restrict__ boff,
                                                                 uint32_t *__restrict__ bcnt,
                                                                 uint32_t *__restrict__ sorted) {
    const uint32_t n = min(A.over[0], A.spill_cap);
    if (n <= kPostSerial) return;  // (post_scan_kernel scattered them)
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const uint32_t r = A.spill[3 * (size_t)e] & 0x7FFFFFFFu;
        const uint32_t at = boff[r] + atomicAdd(&bcnt[r], 1u);
        sorted[3 * (size_t)at] = A.spill[3 * (size_t)e];
        sorted[3 * (size_t)at + 1] = A.spill[3 * (size_t)e + 1];
        sorted[3 * (size_t)at + 2] = A.spill[3 * (size_t)e + 2];
    }
}

int launch_post_fused(const ScanArgs &a, bool cand, uint32_t *done, uint32_t n_regions, uint32_t *bcnt, uint32_t *boff,
                      uint32_t *sorted, hipStream_t stream, bool wide, uint32_t *report, uint32_t *need_wide,
                      uint32_t cand_grid) {
    // (256 workgroups: 1 024 cost C2 14 us in dispatch and finish tickets and did not
    // speed up C5's rescoring; the wide scatter's 128 exit at once when there is nothing
    // for them -- and are left out when the batch's last assembly did not need them)
    hipLaunchKernelGGL(post_scan_kernel, dim3(cand ? cand_grid : 1), dim3(kPostBlock), 0, stream, a, cand ? 1u : 0u, done,
                       n_regions, bcnt, boff, sorted, report, wide ? nullptr : need_wide);
    if (wide) {
        hipLaunchKernelGGL(spill_hist_wide_kernel, dim3(128), dim3(kPostBlock), 0, stream, a, done + 1, n_regions, bcnt,
                           boff);
        hipLaunchKernelGGL(spill_scatter_wide_kernel, dim3(128), dim3(256), 0, stream, a, boff, bcnt, sorted);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("post_scan_kernel launch: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_post_scan(const ScanArgs &a, hipStream_t stream) {
    hipLaunchKernelGGL(cand_over_kernel, dim3(256), dim3(256), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("cand_over_kernel launch: ") + hipGetErrorString(e));
    return 1;
}

uint32_t mfma_group_words(const DevHap *haps, uint32_t n_haps, uint32_t hpb) {
    uint32_t mx = 0;
    for (uint32_t h0 = 0; h0 < n_haps; h0 += hpb) {
        const uint32_t hl = std::min(h0 + hpb, n_haps) - 1;
        mx = std::max(mx, haps[hl].word_off + (haps[hl].len + 15) / 16 + 3 - haps[h0].word_off);
    }
    return mx;
}

size_t scan_tmp_words(size_t n) {
    size_t w = 0;
    for (size_t nt = (n + kScanTile - 1) / kScanTile; nt > 0; nt = nt > 1 ? (nt + kScanTile - 1) / kScanTile : 0) w += nt;
    return w + 1;
}

int build_window_lists(const DevHap *haps, uint32_t n_haps, const uint32_t *druns, const uint32_t lmin[2],
                       const uint32_t span[2], uint32_t hpb, uint32_t dedup, WindowListBufs &bufs, uint64_t total[2], hipStream_t stream,
                       int (*ensure_list)(void *ctx, int c, uint64_t n, uint32_t **p, uint16_t **p16),
                       void *ensure_ctx) {
    if (n_haps && bufs.hd) hipLaunchKernelGGL(hd_kernel, dim3((n_haps + 255) / 256), dim3(256), 0, stream, haps, n_haps,
                                             bufs.hd, bufs.hd2);
    for (int c = 0; c < 2; c++) {
        total[c] = 0;
        if (!lmin[c]) continue;
        const uint32_t S = span[c] ? span[c] : kMChunkCols * (c ? 4 : 2);  // the windows dirty for the longest strand
        hipLaunchKernelGGL(wl_count_kernel, dim3(n_haps / 256 + 1), dim3(256), 0, stream, haps, n_haps, druns, lmin[c],
                           S, dedup, bufs.off[c]);
        if (int rc = exclusive_scan(bufs.off[c], (uint64_t)n_haps + 1, bufs.scan_tmp, stream)) return rc;
        hipError_t e = hipMemcpyAsync(&total[c], bufs.off[c] + n_haps, 8, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("window list size: ") + hipGetErrorString(e));
        if (int rc = ensure_list(ensure_ctx, c, std::max<uint64_t>(total[c], 1), &bufs.list[c], &bufs.list16[c]))
            return rc;
        if (n_haps)
            hipLaunchKernelGGL(wl_fill_kernel, dim3((n_haps + 3) / 4), dim3(256), 0, stream, haps, n_haps, druns,
                               lmin[c], S, dedup, hpb, bufs.off[c], bufs.list[c], bufs.list16[c], bufs.gnarrow);
        e = hipGetLastError();
        if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("wl_fill_kernel: ") + hipGetErrorString(e));
    }
    return TFBS_OK;
}

int group_costs(const uint64_t *off0, const uint64_t *off1, uint32_t n_haps, uint32_t hpb, uint32_t w0, uint32_t w1,
                uint32_t *cost, hipStream_t stream) {
    const uint32_t ng = (n_haps + hpb - 1) / hpb;
    if (ng == 0) return TFBS_OK;
    hipLaunchKernelGGL(group_cost_kernel, dim3((ng + 255) / 256), dim3(256), 0, stream, off0, off1, n_haps, hpb, ng, w0,
                       w1, cost);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("group_cost_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

size_t mfma_lds_fixed() { return kMOnehotBytes; }

void mfma_depth_budgets(uint32_t out[9]) {
    const uint32_t *waves = kMfmaRegWaves;
    const uint32_t reserve = kMOnehotBytes + 4096 + sizeof(s_qdata) + sizeof(s_qmeta) + sizeof(s_cand) + sizeof(s_went) + sizeof(s_hd) + sizeof(s_hd2) +
                             256;  // table, staged words, queues
    // workgroups per CU = 4 SIMDs x waves per SIMD / waves per workgroup
    for (int nk = 1; nk <= kMMaxChunks; nk++) out[nk] = (160 * 1024) / (4 * waves[nk] / (kMBlock / 64)) - reserve;
}

int launch_mfma_all(const ScanArgs &a0, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words,
                    uint32_t n_haps, hipStream_t stream, HitSrc *srcs, uint32_t *n_srcs) {
    *n_srcs = 0;
    if (n_haps == 0 || n_supers == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const DevMSuper &last = supers[n_supers - 1];
    if ((uint64_t)(last.tile0 + last.tile_count) * kMStrands > (1u << 24) || hpb > kMMaxHapsPerBlock)
        return fail(TFBS_E_ARG, "matrix-core scan: more than 2^24 strands or 64 haplotypes per workgroup");
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const size_t static_lds = sizeof(s_qdata) + sizeof(s_qmeta) + sizeof(s_cand) + sizeof(s_went) + sizeof(s_hnext) + sizeof(s_hd) + sizeof(s_hd2);
    size_t img_bytes = 0;
    for (uint32_t k = 0; k < n_supers; k++) img_bytes = std::max<size_t>(img_bytes, supers[k].img_bytes);
    const size_t base = kMOnehotBytes + img_bytes + kMChunkBytes;  // (the padding: scan_segment's B prefetch)
    const size_t staged_bytes = base + ((size_t)group_words * 4 + 15) / 16 * 16;
    const bool staged = staged_bytes + static_lds <= kMStagedMax;
    // (TFBS_SCAN_LDS_MIN: an occupancy A/B -- more LDS per workgroup, fewer per CU)
    static const size_t lds_min = getenv("TFBS_SCAN_LDS_MIN") ? (size_t)atol(getenv("TFBS_SCAN_LDS_MIN")) : 0;
    const size_t lds = std::max(staged ? staged_bytes : base, lds_min);
    const MfmaKernel kern = mfma_all_variant(staged);
    hipError_t e = hipSuccess;
    if (lds > 64 * 1024)
        e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("MFMA LDS attribute: ") + hipGetErrorString(e));
    int launches = 0;
    const uint64_t max_hg = (1ull << 31) - 1;
    for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
        const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
        const uint32_t h0 = (uint32_t)(g0 * hpb);
        ScanArgs a = a0;
        a.haps = a0.haps + h0;
        a.hd = a0.hd + h0;
        a.hd2 = a0.hd2 + h0;
        a.hap_base = a0.hap_base + h0;
        for (int c = 0; c < 2; c++) a.wlist_off[c] = a0.wlist_off[c] ? a0.wlist_off[c] + h0 : nullptr;
        a.gnarrow = a0.gnarrow ? a0.gnarrow + g0 : nullptr;
        a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
        a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
        a.region_base = (uint32_t)g0;
        if (*n_srcs >= (uint32_t)kMaxHitSrcs) return fail(TFBS_E_ARG, "matrix-core scan: too many launches");
        srcs[(*n_srcs)++] = HitSrc{(uint32_t)g0, 1, (uint32_t)g0, ng};
        a.mimg_max = (uint32_t)img_bytes;
        hipLaunchKernelGGL(kern, dim3(ng), dim3(kMBlock), lds, stream, a);
        launches++;
    }
    e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_mfma_all_kernel launch: ") + hipGetErrorString(e));
    return launches;
}

int launch_mfma(const ScanArgs &a0, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words,
                uint32_t n_haps, const hipStream_t *streams, uint32_t n_streams, HitSrc *srcs, uint32_t *n_srcs) {
    *n_srcs = 0;
    if (n_haps == 0 || n_supers == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    // candidate list entries: global strand < 2^24, haplotype in the group < 2^8
    const DevMSuper &last = supers[n_supers - 1];
    if ((uint64_t)(last.tile0 + last.tile_count) * kMStrands > (1u << 24) || hpb > kMMaxHapsPerBlock)
        return fail(TFBS_E_ARG, "matrix-core scan: more than 2^24 strands or 64 haplotypes per workgroup");
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const size_t static_lds =
        sizeof(s_qdata) + sizeof(s_qmeta) + sizeof(s_cand) + sizeof(s_went) + sizeof(s_hnext) + sizeof(s_hd) + sizeof(s_hd2);  // queues, descriptors
    uint32_t region = 0;
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
        static const bool shallow_first = getenv("TFBS_SCAN_SHALLOW_FIRST") && atoi(getenv("TFBS_SCAN_SHALLOW_FIRST"));
        const size_t gk = shallow_first ? gi : groups.size() - 1 - gi;  // (A/B: the launch order of the depths)
        const uint32_t s0 = groups[gk].first, s1 = groups[gk].second;
        const hipStream_t stream = streams[gi % n_streams];
        const uint32_t nk = supers[s0].nk;
        size_t img_bytes = 0;
        for (uint32_t k = s0; k < s1; k++) img_bytes = std::max<size_t>(img_bytes, supers[k].img_bytes);
        const uint32_t ns = s1 - s0;
        // stage the group's words in LDS when they fit beside the image at 4 workgroups per CU
        const size_t base = kMOnehotBytes + img_bytes + kMChunkBytes;  // (the padding: scan_segment's B prefetch)
        const size_t staged_bytes = base + ((size_t)group_words * 4 + 15) / 16 * 16;
        const bool staged = staged_bytes + static_lds <= kMStagedMax;
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
            a.hd = a0.hd + h0;
            a.hd2 = a0.hd2 + h0;
            a.hap_base = a0.hap_base + h0;
            for (int c = 0; c < 2; c++) a.wlist_off[c] = a0.wlist_off[c] ? a0.wlist_off[c] + h0 : nullptr;
            a.gnarrow = a0.gnarrow ? a0.gnarrow + g0 : nullptr;
            a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
            a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
            a.region_base = region;
            if (*n_srcs >= (uint32_t)kMaxHitSrcs) return fail(TFBS_E_ARG, "matrix-core scan: too many launches");
            srcs[(*n_srcs)++] = HitSrc{region, ns, (uint32_t)g0, ng};
            region += ns * ng;
            a.mimg_max = (uint32_t)img_bytes;
            hipLaunchKernelGGL(kern, dim3(ns * ng), dim3(kMBlock), lds, stream, a);
            launches++;
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_mfma_kernel launch: ") + hipGetErrorString(e));
    return launches;
}

}  // namespace tfbs
