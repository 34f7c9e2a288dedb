// MI355X (gfx950) scan kernels and the device context.
//
// The hot path of find-tfbs is `matches` (pattern.rs:141-171) called for every
// (distinct haplotype, pattern) of a merged region (main.rs:101-147), followed
// by the inner-peak overlap test of count_matches_by_sample (main.rs:503).
// Here one launch scores every window of every distinct haplotype of a batch
// of regions against every PWM strand and writes, per (haplotype, pattern_id,
// inner range), the number of windows with score > min_score whose match range
// [pos_i, pos_i + L - 1] overlaps the inner range (range.rs:18-21).
//
// Design (DESIGN.md has the numbers):
//  * Haplotypes are packed 2 bits/base (16 bases per u32).  A lane owns one
//    window start i and funnel-shifts a 64-bit image of bases i..i+31 out of
//    three words, once per (haplotype, tile), into eight 4-mer codes.
//  * Each PWM strand of length L <= 32 is ceil(L/4) 4-mer lookup tables (entry
//    = sum of the 4 column weights, i32 wrap).  Four strands of similar length
//    form a quad whose tables are interleaved, so ONE ds_read_b128 per 4-mer
//    returns the four strands' partial sums (16 columns of work per LDS read).
//  * A 512-thread workgroup stages one tile of quads (whole pattern_id groups,
//    both strands) in LDS; each of its 8 waves scores haplotypes against it.
//  * N (weight 0 in every column, types.rs:110) packs as A; haplotypes that
//    contain an N carry a bit mask and subtract w[j][A] for each N column.
//  * Hits are rare (p ~ 1e-4): a ballot of the threshold compare gates the
//    inner-range counting, which runs on SALU bit masks (s_and + s_bcnt1).
//  * Indel haplotypes carry explicit positions (inserted bases repeat a pos,
//    deletions skip some, haplotype.rs:130-139); SNV-only ones are affine.
//  * PWM strands longer than 32 columns go to a column-wise generic kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "batch.hpp"
#include "patterns.hpp"
#include "tfbs_internal.hpp"

using namespace tfbs;

#define HIP_TRY(expr)                                                                                       \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return tfbs::fail(TFBS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));               \
    } while (0)

namespace {

constexpr int kFastBlock = 512;  // 8 waves share one LDS tile
constexpr int kGenBlock = 256;
constexpr int kChunks = 4;       // 64-window chunks per lane group (256 windows per pass)

struct Inner {
    int32_t s;
    uint32_t span;  // e - s
};


// Count, for every inner range of this pass, the hit windows whose match range
// overlaps it (main.rs:503 with Range::overlaps, range.rs:18-21), and add the
// counts to the lane that owns the pattern_id slot.
template <int NCH>
__device__ __forceinline__ void count_hits(const uint64_t (&hit)[NCH], const int32_t (&pos)[NCH], uint32_t L,
                                           const Inner *in, uint32_t n_pass, uint32_t slot, uint32_t lane,
                                           uint32_t (&acc)[kMaxInnerPass]) {
#pragma unroll
    for (int kk = 0; kk < kMaxInnerPass; kk++) {
        if ((uint32_t)kk >= n_pass) break;
        const int32_t s = in[kk].s;
        const uint32_t span = in[kk].span;
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (!hit[c]) continue;
            int32_t p = pos[c];
            asm volatile("" : "+v"(p));  // keep the (rare) overlap test here, not hoisted into the hot loop
            const bool ov = (uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span;
            cnt += __popcll(hit[c] & __ballot(ov));
        }
        acc[kk] += (lane == slot) ? cnt : 0u;
    }
}

__device__ __forceinline__ uint32_t comp(const uint4 &v, int s) {
    return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

struct ScanArgs {
    const DevTile *tiles;
    uint32_t n_tiles;
    const DevQuad *quads;
    const int32_t *lut;
    const int32_t *colA;
    const DevHap *haps;
    uint32_t n_haps;
    const DevRegion *regions;
    const int32_t *inner;
    const uint32_t *words;
    const uint32_t *nmask;
    const int32_t *posrel;
    uint32_t *counts;
    uint32_t haps_per_block;
    unsigned long long *hits;  // debug (tfbs_matches): per (hap, pattern, 64-window chunk) hit masks
    uint32_t hits_wpp;
    uint32_t n_patterns_total;
};

// Partial sums of one quad over NCH chunks: nblk interleaved 4-mer lookups per
// window (ds_read_b128 each).  NB > 0 fixes the block count at compile time so
// every read can be issued ahead of its add; NB == 0 loops over Q.nblk.
template <int NCH>
struct Sums {
    uint4 v[NCH];
};

template <int NCH, int NB>
__device__ __forceinline__ Sums<NCH> quad_sums(const char *base, uint32_t nblk, const uint32_t (&code16)[NCH][8]) {
    Sums<NCH> r;
    uint4 (&sc)[NCH] = r.v;
#pragma unroll
    for (int c = 0; c < NCH; c++) sc[c] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        if (NB > 0 ? b >= NB : (uint32_t)b >= nblk) break;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(base + b * (kQuadBlockInts * 4) + code16[c][b]);
            sc[c].x += v.x;
            sc[c].y += v.y;
            sc[c].z += v.z;
            sc[c].w += v.w;
        }
    }
    return r;
}

// One quad of strands over NCH chunks: the lookups, then per strand the
// threshold ballot and, on a hit, the inner-range counting.
template <int NCH>
__device__ __forceinline__ void quad_body(const ScanArgs &A, const DevQuad &Q, const char *s_lut,
                                          const int32_t *s_col, const uint32_t (&code16)[NCH][8],
                                          const int32_t (&rem)[NCH], const int32_t (&pos)[NCH],
                                          const uint32_t (&nm)[NCH], bool has_n, uint32_t h, uint32_t cg,
                                          const Inner *in, uint32_t n_pass, bool write_hits, uint32_t lane,
                                          uint32_t (&acc)[kMaxInnerPass]) {
    const char *base = s_lut + (size_t)Q.lut_off * (kQuadBlockInts * 4);
    const uint32_t nblk = Q.nblk;
    Sums<NCH> S;
    if (NCH == 4) {
        switch (nblk) {
        case 1: S = quad_sums<NCH, 1>(base, nblk, code16); break;
        case 2: S = quad_sums<NCH, 2>(base, nblk, code16); break;
        case 3: S = quad_sums<NCH, 3>(base, nblk, code16); break;
        case 4: S = quad_sums<NCH, 4>(base, nblk, code16); break;
        case 5: S = quad_sums<NCH, 5>(base, nblk, code16); break;
        case 6: S = quad_sums<NCH, 6>(base, nblk, code16); break;
        case 7: S = quad_sums<NCH, 7>(base, nblk, code16); break;
        default: S = quad_sums<NCH, 8>(base, nblk, code16); break;
        }
    } else {
        S = quad_sums<NCH, 0>(base, nblk, code16);
    }
    const uint4 (&sc)[NCH] = S.v;
#pragma unroll
    for (int s = 0; s < kQuad; s++) {
        if (s >= Q.nstrand) break;
        const uint32_t L = Q.len[s];
        int32_t score[NCH];
#pragma unroll
        for (int c = 0; c < NCH; c++) score[c] = (int32_t)comp(sc[c], s);
        if (has_n) {
            const uint32_t lmask = L >= 32 ? 0xFFFFFFFFu : ((1u << L) - 1u);
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                uint32_t m = nm[c] & lmask;
                while (m) {
                    const uint32_t j = __builtin_ctz(m);
                    score[c] = (int32_t)((uint32_t)score[c] - (uint32_t)s_col[Q.col_off[s] + j]);
                    m &= m - 1;
                }
            }
        }
        uint64_t hit[NCH];
        uint64_t any = 0;
        const int32_t ms = Q.min_score[s];
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            hit[c] = __ballot(score[c] > ms && rem[c] >= (int32_t)L);
            any |= hit[c];
        }
        if (__builtin_expect(write_hits, 0) && lane == 0) {
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                const uint32_t wi = cg / 64 + c;
                if (wi < A.hits_wpp)
                    A.hits[((size_t)h * A.n_patterns_total + Q.orig_index[s]) * A.hits_wpp + wi] = hit[c];
            }
        }
        if (__builtin_expect(any != 0, 0)) count_hits<NCH>(hit, pos, L, in, n_pass, Q.slot_local[s], lane, acc);
    }
}

// Score NCH 64-window chunks starting at window cg against every quad of the tile.
template <int NCH>
__device__ __forceinline__ void scan_chunks(const ScanArgs &A, const DevTile &t, const char *s_lut,
                                            const DevQuad *s_quads, const int32_t *s_col, const DevHap &hm, uint32_t h, uint32_t cg,
                                            const Inner *in, uint32_t n_pass, bool write_hits, uint32_t lane,
                                            uint32_t (&acc)[kMaxInnerPass]) {
    const bool has_n = (hm.flags & HAP_HAS_N) != 0;
    const bool has_pos = (hm.flags & HAP_HAS_POS) != 0;
    uint32_t code16[NCH][8];  // byte offsets of the eight 4-mer codes in a quad-block (code * 16)
    int32_t rem[NCH], pos[NCH];
    uint32_t nm[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        const uint32_t i = cg + 64 * c + lane;
        const uint32_t ic = min(i, hm.len);  // keep reads inside the +3 word pad
        const uint32_t *w = A.words + hm.word_off + (ic >> 4);
        const uint32_t sh = 2 * (ic & 15);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh);
        const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, sh);
#pragma unroll
        for (int b = 0; b < 4; b++) {
            code16[c][b] = ((lo >> (8 * b)) & 0xFFu) << 4;
            code16[c][b + 4] = ((hi >> (8 * b)) & 0xFFu) << 4;
        }
        rem[c] = (int32_t)hm.len - (int32_t)i;
        pos[c] = has_pos ? (i < hm.len ? A.posrel[hm.pos_off + i] : 0) : (int32_t)i;
        if (has_n) {
            const uint32_t *m = A.nmask + hm.nmask_off + (ic >> 5);
            nm[c] = __builtin_amdgcn_alignbit(m[1], m[0], ic & 31);
        } else {
            nm[c] = 0;
        }
    }
    for (uint32_t qi = t.first; qi < t.last; qi++) {
        const DevQuad &Q = s_quads[qi - t.first];
        quad_body<NCH>(A, Q, s_lut, s_col, code16, rem, pos, nm, has_n, h, cg, in, n_pass, write_hits, lane, acc);
    }
}

// ---------------------------------------------------------------------------
// Fast kernel: PWM strands of length <= 32 via interleaved 4-mer LUTs in LDS.
// Grid: n_tiles x ceil(n_haps / haps_per_block); block 512 threads.
// ---------------------------------------------------------------------------
// MINW = minimum waves per SIMD (the register budget: 2 -> up to 256 VGPRs, one
// workgroup per CU; 4 -> 128 VGPRs, two workgroups per CU).
template <int MINW>
__global__ __launch_bounds__(kFastBlock, MINW) void scan_fast_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) int32_t smem[];
    const uint32_t tile_idx = blockIdx.x % A.n_tiles;
    const uint32_t hg = blockIdx.x / A.n_tiles;
    const DevTile t = A.tiles[tile_idx];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = kFastBlock / 64;

    // stage the tile's quad-blocks and A columns (16-byte loads)
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.lut + (size_t)t.lut_begin * kQuadBlockInts);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        const uint32_t n4 = t.nblocks * (kQuadBlockInts / 4);
        for (uint32_t i = threadIdx.x; i < n4; i += kFastBlock) dst[i] = src[i];
        // the tile's quad descriptors: read by every wave at uniform addresses (LDS broadcast)
        const uint32_t nq = t.last - t.first;
        const uint32_t *qsrc = reinterpret_cast<const uint32_t *>(A.quads + t.first);
        uint32_t *qdst = reinterpret_cast<uint32_t *>(smem + t.nblocks * kQuadBlockInts);
        for (uint32_t i = threadIdx.x; i < nq * (sizeof(DevQuad) / 4); i += kFastBlock) qdst[i] = qsrc[i];
        int32_t *scol = smem + t.nblocks * kQuadBlockInts + nq * (sizeof(DevQuad) / 4);
        for (uint32_t i = threadIdx.x; i < t.ncols; i += kFastBlock) scol[i] = A.colA[t.col_begin + i];
    }
    __syncthreads();
    const char *s_lut = reinterpret_cast<const char *>(smem);
    const DevQuad *s_quads = reinterpret_cast<const DevQuad *>(smem + t.nblocks * kQuadBlockInts);
    const int32_t *s_col = smem + t.nblocks * kQuadBlockInts + (t.last - t.first) * (sizeof(DevQuad) / 4);

    for (uint32_t hh = wave; hh < A.haps_per_block; hh += kWaves) {
        const uint32_t h = hg * A.haps_per_block + hh;
        if (h >= A.n_haps) break;
        const DevHap hm = A.haps[h];
        const DevRegion rg = A.regions[hm.region];
        const uint32_t n_inner = rg.n_inner;
        const uint32_t nwin = hm.len >= t.lmin ? hm.len - t.lmin + 1 : 0;
        const uint32_t n_passes =
            n_inner == 0 ? (A.hits ? 1u : 0u) : (n_inner + kMaxInnerPass - 1) / kMaxInnerPass;
        for (uint32_t pass = 0; pass < n_passes; pass++) {
            const uint32_t k0 = pass * kMaxInnerPass;
            const uint32_t n_pass = n_inner > k0 ? min((uint32_t)kMaxInnerPass, n_inner - k0) : 0u;
            Inner in[kMaxInnerPass];
#pragma unroll
            for (int kk = 0; kk < kMaxInnerPass; kk++) {
                if ((uint32_t)kk < n_pass) {
                    const int32_t s = A.inner[2 * (rg.inner_off + k0 + kk)];
                    const int32_t e = A.inner[2 * (rg.inner_off + k0 + kk) + 1];
                    in[kk].s = s;
                    in[kk].span = (uint32_t)(e - s);
                } else {
                    in[kk].s = 0;
                    in[kk].span = 0;
                }
            }
            uint32_t acc[kMaxInnerPass];
#pragma unroll
            for (int kk = 0; kk < kMaxInnerPass; kk++) acc[kk] = 0;
            const bool write_hits = A.hits != nullptr && pass == 0;
            for (uint32_t cg = 0; cg < nwin; cg += 64 * kChunks) {
                const uint32_t nch = min((uint32_t)kChunks, (nwin - cg + 63) / 64);
                if (nch >= 3)  // a 3-chunk tail scores one chunk of invalid windows (rem < L)
                    scan_chunks<4>(A, t, s_lut, s_quads, s_col, hm, h, cg, in, n_pass, write_hits, lane, acc);
                else if (nch == 2)
                    scan_chunks<2>(A, t, s_lut, s_quads, s_col, hm, h, cg, in, n_pass, write_hits, lane, acc);
                else
                    scan_chunks<1>(A, t, s_lut, s_quads, s_col, hm, h, cg, in, n_pass, write_hits, lane, acc);
            }
            if (n_pass && lane < t.nslots) {
                uint32_t *out = A.counts + hm.count_off + (size_t)(t.slot_begin + lane) * n_inner + k0;
#pragma unroll
                for (int kk = 0; kk < kMaxInnerPass; kk++)
                    if ((uint32_t)kk < n_pass) out[kk] = acc[kk];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Generic kernel: one pattern_id group whose strands include one longer than
// 32 columns; column-wise scoring with weights read through the cache.
// Grid: n_gen_tiles x ceil(n_haps / haps_per_block).
// ---------------------------------------------------------------------------
struct GenArgs {
    const DevTile *tiles;
    uint32_t n_tiles;
    const DevPattern *pats;
    const int32_t *gw;
    const DevHap *haps;
    uint32_t n_haps;
    const DevRegion *regions;
    const int32_t *inner;
    const uint32_t *words;
    const uint32_t *nmask;
    const int32_t *posrel;
    uint32_t *counts;
    uint32_t haps_per_block;
    unsigned long long *hits;
    uint32_t hits_wpp;
    uint32_t n_patterns_total;
};

__global__ __launch_bounds__(kGenBlock) void scan_generic_kernel(GenArgs A) {
    const uint32_t tile_idx = blockIdx.x % A.n_tiles;
    const uint32_t hg = blockIdx.x / A.n_tiles;
    const DevTile t = A.tiles[tile_idx];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = kGenBlock / 64;
    for (uint32_t hh = wave; hh < A.haps_per_block; hh += kWaves) {
        const uint32_t h = hg * A.haps_per_block + hh;
        if (h >= A.n_haps) break;
        const DevHap hm = A.haps[h];
        const DevRegion rg = A.regions[hm.region];
        const uint32_t n_inner = rg.n_inner;
        const bool has_n = (hm.flags & HAP_HAS_N) != 0;
        const bool has_pos = (hm.flags & HAP_HAS_POS) != 0;
        const uint32_t n_passes =
            n_inner == 0 ? (A.hits ? 1u : 0u) : (n_inner + kMaxInnerPass - 1) / kMaxInnerPass;
        for (uint32_t pass = 0; pass < n_passes; pass++) {
            const uint32_t k0 = pass * kMaxInnerPass;
            const uint32_t n_pass = n_inner > k0 ? min((uint32_t)kMaxInnerPass, n_inner - k0) : 0u;
            Inner in[kMaxInnerPass];
            for (int kk = 0; kk < kMaxInnerPass; kk++) {
                if ((uint32_t)kk < n_pass) {
                    in[kk].s = A.inner[2 * (rg.inner_off + k0 + kk)];
                    in[kk].span = (uint32_t)(A.inner[2 * (rg.inner_off + k0 + kk) + 1] - in[kk].s);
                } else {
                    in[kk].s = 0;
                    in[kk].span = 0;
                }
            }
            uint32_t acc[kMaxInnerPass];
            for (int kk = 0; kk < kMaxInnerPass; kk++) acc[kk] = 0;
            for (uint32_t cg = 0; cg < hm.len; cg += 64 * kChunks) {
                int32_t rem[kChunks], pos[kChunks];
#pragma unroll
                for (int c = 0; c < kChunks; c++) {
                    const uint32_t i = cg + 64 * c + lane;
                    rem[c] = (int32_t)hm.len - (int32_t)i;
                    pos[c] = has_pos ? (i < hm.len ? A.posrel[hm.pos_off + i] : 0) : (int32_t)i;
                }
                for (uint32_t pi = t.first; pi < t.last; pi++) {
                    const DevPattern p = A.pats[pi];
                    uint64_t hit[kChunks];
                    uint64_t any = 0;
#pragma unroll
                    for (int c = 0; c < kChunks; c++) {
                        const uint32_t i = cg + 64 * c + lane;
                        const bool valid = rem[c] >= (int32_t)p.len;
                        uint32_t sc = 0;
                        if (valid) {
                            for (uint32_t j = 0; j < p.len; j++) {
                                const uint32_t q = i + j;
                                uint32_t code = (A.words[hm.word_off + (q >> 4)] >> (2 * (q & 15))) & 3u;
                                if (has_n && ((A.nmask[hm.nmask_off + (q >> 5)] >> (q & 31)) & 1u)) code = 4;
                                sc += (uint32_t)A.gw[(size_t)(p.col_off + j) * 5 + code];
                            }
                        }
                        hit[c] = __ballot(valid && (int32_t)sc > p.min_score);
                        any |= hit[c];
                    }
                    if (A.hits && pass == 0 && lane == 0) {
                        for (int c = 0; c < kChunks; c++) {
                            const uint32_t wi = cg / 64 + c;
                            if (wi < A.hits_wpp)
                                A.hits[((size_t)h * A.n_patterns_total + p.orig_index) * A.hits_wpp + wi] = hit[c];
                        }
                    }
                    if (any) count_hits<kChunks>(hit, pos, p.len, in, n_pass, p.slot_local, lane, acc);
                }
            }
            if (n_pass && lane == 0) {
                uint32_t *out = A.counts + hm.count_off + (size_t)t.slot_begin * n_inner + k0;
                for (int kk = 0; kk < kMaxInnerPass; kk++)
                    if ((uint32_t)kk < n_pass) out[kk] = acc[kk];
            }
        }
    }
}

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;
    size_t n = 0;
    int ensure(size_t want) {
        n = want;
        if (want <= cap) return TFBS_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(want, 16);
        hipError_t e = hipMalloc(&p, c * sizeof(T));
        if (e != hipSuccess) return tfbs::fail(TFBS_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        cap = c;
        return TFBS_OK;
    }
    int put(const std::vector<T> &v, hipStream_t s) {
        int rc = ensure(v.size());
        if (rc) return rc;
        if (!v.empty()) HIP_TRY(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
        return TFBS_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = n = 0;
    }
};

}  // namespace

struct tfbs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    const Patterns *pats = nullptr;
    Plan plan;
    uint32_t tile_qblocks = 16;   // quad-blocks (4 KiB each) per LDS tile
    uint32_t haps_per_block = 64;
    int fast_minw = 2;            // scan_fast_kernel<MINW> instantiation
    size_t lds_bytes = 0;
    DevBuf<DevQuad> fast_quads;
    DevBuf<DevPattern> gen_pats;
    DevBuf<DevTile> fast_tiles, gen_tiles;
    DevBuf<int32_t> lut, colA, gen_w;
    // batch image
    DevBuf<uint32_t> words, nmask, counts;
    DevBuf<int32_t> posrel, inner;
    DevBuf<DevHap> haps;
    DevBuf<DevRegion> regions;
    DevBuf<unsigned long long> hits;
    const tfbs_batch *resident = nullptr;
    float last_ms = 0.f;
    int last_launches = 0;
    bool timing_pending = false;
};

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    if (!v || !*v) return dflt;
    return atoi(v);
}

static int launch_scan(tfbs_ctx *ctx, uint32_t n_haps, unsigned long long *hits, uint32_t hits_wpp) {
    const Plan &P = ctx->plan;
    const uint32_t hpb = ctx->haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const uint32_t n_pat_total = (uint32_t)ctx->pats->pats.size();
    int launches = 0;
    if (n_haps == 0) return 0;
    // keep every grid below 2^31 workgroups by splitting along haplotype groups
    if (!P.fast_tiles.empty()) {
        const uint32_t nt = (uint32_t)P.fast_tiles.size();
        const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / nt - 1);
        for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
            const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
            const uint32_t h0 = (uint32_t)(g0 * hpb);
            ScanArgs a{};
            a.tiles = ctx->fast_tiles.p;
            a.n_tiles = nt;
            a.quads = ctx->fast_quads.p;
            a.lut = ctx->lut.p;
            a.colA = ctx->colA.p;
            a.haps = ctx->haps.p + h0;
            a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
            a.regions = ctx->regions.p;
            a.inner = ctx->inner.p;
            a.words = ctx->words.p;
            a.nmask = ctx->nmask.p;
            a.posrel = ctx->posrel.p;
            a.counts = ctx->counts.p;
            a.haps_per_block = hpb;
            a.hits = hits ? hits + (size_t)h0 * n_pat_total * hits_wpp : nullptr;
            a.hits_wpp = hits_wpp;
            a.n_patterns_total = n_pat_total;
            if (ctx->fast_minw == 4)
                hipLaunchKernelGGL(scan_fast_kernel<4>, dim3(nt * ng), dim3(kFastBlock), ctx->lds_bytes, ctx->stream, a);
            else
                hipLaunchKernelGGL(scan_fast_kernel<2>, dim3(nt * ng), dim3(kFastBlock), ctx->lds_bytes, ctx->stream, a);
            launches++;
        }
    }
    if (!P.gen_tiles.empty()) {
        const uint32_t nt = (uint32_t)P.gen_tiles.size();
        const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / nt - 1);
        for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
            const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
            const uint32_t h0 = (uint32_t)(g0 * hpb);
            GenArgs a{};
            a.tiles = ctx->gen_tiles.p;
            a.n_tiles = nt;
            a.pats = ctx->gen_pats.p;
            a.gw = ctx->gen_w.p;
            a.haps = ctx->haps.p + h0;
            a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
            a.regions = ctx->regions.p;
            a.inner = ctx->inner.p;
            a.words = ctx->words.p;
            a.nmask = ctx->nmask.p;
            a.posrel = ctx->posrel.p;
            a.counts = ctx->counts.p;
            a.haps_per_block = hpb;
            a.hits = hits ? hits + (size_t)h0 * n_pat_total * hits_wpp : nullptr;
            a.hits_wpp = hits_wpp;
            a.n_patterns_total = n_pat_total;
            hipLaunchKernelGGL(scan_generic_kernel, dim3(nt * ng), dim3(kGenBlock), 0, ctx->stream, a);
            launches++;
        }
    }
    HIP_TRY(hipGetLastError());
    return launches;
}

extern "C" {

int tfbs_device_count(int *n) {
    if (!n) return tfbs::fail(TFBS_E_ARG, "null argument");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c == 0) {
        *n = 0;
        return tfbs::fail(TFBS_E_NODEVICE, "no HIP device visible");
    }
    *n = c;
    return TFBS_OK;
}

void tfbs_ctx_destroy(tfbs_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    ctx->fast_quads.release(); ctx->gen_pats.release(); ctx->fast_tiles.release(); ctx->gen_tiles.release();
    ctx->lut.release(); ctx->colA.release(); ctx->gen_w.release();
    ctx->words.release(); ctx->nmask.release(); ctx->counts.release(); ctx->posrel.release();
    ctx->inner.release(); ctx->haps.release(); ctx->regions.release(); ctx->hits.release();
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int tfbs_ctx_create(int device, const tfbs_patterns *p, tfbs_ctx **out) {
    if (!p || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    int n = 0;
    int rc = tfbs_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n) return tfbs::fail(TFBS_E_ARG, "device index out of range");
    auto *ctx = new tfbs_ctx();
    ctx->device = device;
    ctx->pats = &tfbs::patterns_of(p);
    ctx->tile_qblocks = (uint32_t)std::min(36, std::max(8, env_int("TFBS_TILE_QBLOCKS", 16)));
    ctx->haps_per_block = (uint32_t)std::max(8, env_int("TFBS_HAPS_PER_BLOCK", 64));
    ctx->fast_minw = env_int("TFBS_FAST_MINW", 2) == 4 ? 4 : 2;
    rc = ctx->pats->build_plan(ctx->tile_qblocks, &ctx->plan);
    if (rc) {
        delete ctx;
        return rc;
    }
    if (ctx->plan.zero_len_panics) {
        delete ctx;
        return tfbs::fail(TFBS_E_ZEROLEN, "length-0 PWM with negative min_score (pattern.rs:150-156)");
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
    if (e != hipSuccess) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_HIP, std::string("HIP init: ") + hipGetErrorString(e));
    }
    const Plan &P = ctx->plan;
    ctx->lds_bytes = (size_t)P.max_tile_blocks * kQuadBlockInts * 4 + (size_t)P.max_tile_quads * sizeof(DevQuad) +
                     (size_t)P.max_tile_cols * 4 + 16;
    if (ctx->lds_bytes > 160 * 1024) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_ARG, "pattern tile exceeds the 160 KiB LDS");
    }
    if (ctx->lds_bytes > 64 * 1024) {
        e = hipFuncSetAttribute((const void *)scan_fast_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)ctx->lds_bytes);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void *)scan_fast_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)ctx->lds_bytes);
        if (e != hipSuccess) {
            tfbs_ctx_destroy(ctx);
            return tfbs::fail(TFBS_E_HIP, std::string("LDS attribute: ") + hipGetErrorString(e));
        }
    }
    if ((rc = ctx->fast_quads.put(P.fast_quads, ctx->stream)) || (rc = ctx->fast_tiles.put(P.fast_tiles, ctx->stream)) ||
        (rc = ctx->lut.put(P.lut, ctx->stream)) || (rc = ctx->colA.put(P.colA, ctx->stream)) ||
        (rc = ctx->gen_pats.put(P.gen_pats, ctx->stream)) || (rc = ctx->gen_tiles.put(P.gen_tiles, ctx->stream)) ||
        (rc = ctx->gen_w.put(P.gen_w, ctx->stream))) {
        tfbs_ctx_destroy(ctx);
        return rc;
    }
    e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_HIP, std::string("upload: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return TFBS_OK;
}

int tfbs_ctx_sync(tfbs_ctx *ctx) {
    if (!ctx) return tfbs::fail(TFBS_E_ARG, "null ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return TFBS_OK;
}

float tfbs_ctx_last_scan_ms(const tfbs_ctx *ctx) {
    if (!ctx) return -1.f;
    auto *c = const_cast<tfbs_ctx *>(ctx);
    if (c->timing_pending) {
        if (hipEventSynchronize(c->ev1) == hipSuccess) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, c->ev0, c->ev1) == hipSuccess) c->last_ms = ms;
        }
        c->timing_pending = false;
    }
    return c->last_ms;
}

int tfbs_ctx_last_scan_launches(const tfbs_ctx *ctx) { return ctx ? ctx->last_launches : 0; }

int tfbs_batch_upload(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    Batch &B = b->b;
    if (B.pats != ctx->pats) return tfbs::fail(TFBS_E_ARG, "batch and ctx use different pattern sets");
    if (B.open) return tfbs::fail(TFBS_E_STATE, "region still open");
    if (B.slot_pid != ctx->plan.slot_pid) return tfbs::fail(TFBS_E_STATE, "batch slot order differs from the ctx plan");
    HIP_TRY(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ctx->words.put(B.words, ctx->stream)) || (rc = ctx->nmask.put(B.nmask, ctx->stream)) ||
        (rc = ctx->posrel.put(B.posrel, ctx->stream)) || (rc = ctx->haps.put(B.haps, ctx->stream)) ||
        (rc = ctx->regions.put(B.regions, ctx->stream)) || (rc = ctx->inner.put(B.inner, ctx->stream)) ||
        (rc = ctx->counts.ensure(B.n_counts)))
        return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->resident = b;
    return TFBS_OK;
}

int tfbs_scan(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not uploaded to this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    int n = launch_scan(ctx, (uint32_t)b->b.haps.size(), nullptr, 0);
    if (n < 0) return n;
    HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->last_launches = n;
    ctx->timing_pending = true;
    b->b.counts_valid = false;
    return TFBS_OK;
}

int tfbs_batch_download(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    B.counts.resize(B.n_counts);
    if (B.n_counts)
        HIP_TRY(hipMemcpyAsync(B.counts.data(), ctx->counts.p, B.n_counts * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    B.counts_valid = true;
    return TFBS_OK;
}

int tfbs_matches(tfbs_ctx *ctx, const uint8_t *nucs, const uint64_t *pos, size_t n, uint32_t *counts,
                 uint64_t *out_start, uint64_t *out_end, size_t cap, size_t *n_total) {
    if (!ctx || !n_total || !counts || (n && (!nucs || !pos))) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (n >= (1u << 30)) return tfbs::fail(TFBS_E_ARG, "haplotype too long");
    const Patterns &P = *ctx->pats;
    // pack one haplotype; no inner ranges, hit bitmaps only
    std::vector<uint32_t> words((n + 15) / 16 + 3, 0u), nmask;
    bool has_n = false;
    for (size_t i = 0; i < n; i++) {
        if (nucs[i] > 4) return tfbs::fail(TFBS_E_BADBASE, "nucleotide code > 4");
        uint32_t c = nucs[i];
        if (c == 4) {
            has_n = true;
            c = 0;
        }
        words[i / 16] |= c << (2 * (i % 16));
    }
    DevHap hm{};
    hm.len = (uint32_t)n;
    if (has_n) {
        hm.flags |= HAP_HAS_N;
        nmask.assign((n + 31) / 32 + 2, 0u);
        for (size_t i = 0; i < n; i++)
            if (nucs[i] == 4) nmask[i / 32] |= 1u << (i % 32);
    }
    std::vector<DevHap> haps{hm};
    std::vector<DevRegion> regions{DevRegion{0, 0}};
    std::vector<int32_t> inner{0, 0}, posrel{0};
    const uint32_t wpp = (uint32_t)((n + 255) / 256 * 4);
    HIP_TRY(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ctx->words.put(words, ctx->stream)) || (rc = ctx->nmask.put(nmask, ctx->stream)) ||
        (rc = ctx->posrel.put(posrel, ctx->stream)) || (rc = ctx->haps.put(haps, ctx->stream)) ||
        (rc = ctx->regions.put(regions, ctx->stream)) || (rc = ctx->inner.put(inner, ctx->stream)) ||
        (rc = ctx->counts.ensure(1)))
        return rc;
    ctx->resident = nullptr;
    const size_t nh = (size_t)P.pats.size() * wpp;
    if ((rc = ctx->hits.ensure(std::max<size_t>(nh, 1)))) return rc;
    if (nh) HIP_TRY(hipMemsetAsync(ctx->hits.p, 0, nh * 8, ctx->stream));
    int l = launch_scan(ctx, 1, ctx->hits.p, wpp);
    if (l < 0) return l;
    std::vector<unsigned long long> h(nh);
    if (nh) HIP_TRY(hipMemcpyAsync(h.data(), ctx->hits.p, nh * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    size_t total = 0;
    for (size_t pi = 0; pi < P.pats.size(); pi++) {
        const Pat &q = P.pats[pi];
        uint32_t c = 0;
        for (uint32_t w = 0; w < wpp; w++) {
            unsigned long long m = h[pi * wpp + w];
            while (m) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const size_t i = (size_t)w * 64 + bit;
                if (total < cap) {
                    out_start[total] = pos[i];
                    out_end[total] = pos[i] + q.len - 1;
                }
                total++;
                c++;
            }
        }
        counts[pi] = c;
    }
    *n_total = total;
    if (total > cap) return tfbs::fail(TFBS_E_ARG, "output capacity too small");
    return TFBS_OK;
}

}  // extern "C"
