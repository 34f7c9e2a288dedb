// MI355X (gfx950) scan kernels.
//
// The hot path of find-tfbs is `matches` (pattern.rs:141-171) called for every
// (distinct haplotype, pattern) of a merged region (main.rs:101-147), followed
// by the inner-peak overlap test of count_matches_by_sample (main.rs:503).
// One launch scores every window of every distinct haplotype of a batch of
// regions against every PWM strand and writes, per (haplotype, pattern_id,
// inner range), the number of windows with score > min_score whose match range
// [pos_i, pos_i + L - 1] overlaps the inner range (range.rs:18-21).
//
//  * Haplotypes are packed 2 bits/base (16 bases per u32).  A lane owns one
//    window start i and funnel-shifts a 64-bit image of bases i..i+31 out of
//    three words, once per (haplotype, tile), into eight 4-mer codes.
//  * PWM strands (L <= 32) are grouped in units whose 4-mer tables are
//    interleaved (plan.cpp): one ds_read_b128 per 4-mer returns the partial
//    sums of 8 strands (OCTET16: biased int16, accumulated with saturating
//    v_pk_add_i16) or 4 strands (QUAD32: wrapping int32).
//  * A 512-thread workgroup stages one tile of units in LDS; its 8 waves score
//    haplotypes against it.
//  * N (weight 0, types.rs:110) packs as A plus a per-haplotype bit mask; the
//    (rare) windows that contain an N are rescored exactly, column by column.
//  * Hits are rare (p ~ 1e-4): a ballot of the threshold compare gates the
//    inner-range counting, which runs on SALU bit masks (s_and + s_bcnt1).
//  * Indel haplotypes carry explicit positions (inserted bases repeat a pos,
//    deletions skip some, haplotype.rs:130-139); SNV-only ones are affine.
//  * PWM strands longer than 32 columns go to a column-wise generic kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "scan.hpp"

namespace tfbs {
namespace {

constexpr int kChunks = 4;

// Unit descriptors are read through the constant address space so that the
// wave-uniform field loads become scalar loads (s_load) even though the kernel
// also stores to global memory.
typedef const __attribute__((address_space(4))) DevUnit CUnit;  // 64-window chunks per lane group (256 windows per pass)
constexpr int kGenBlock = 256;

// Count, for every inner range of this pass, the hit windows whose match range
// overlaps it (main.rs:503 with Range::overlaps, range.rs:18-21), and add the
// counts to the lane that owns the pattern_id slot.  Rare: only runs when a
// ballot found a hit, so the inner ranges are loaded here, not kept in registers.
template <int NCH>
__device__ __forceinline__ void count_hits(const uint64_t (&hit)[NCH], const int32_t (&pos)[NCH], uint32_t L,
                                           const int32_t *inner, uint32_t n_pass, uint32_t slot, uint32_t lane,
                                           uint32_t (&acc)[kMaxInnerPass]) {
#pragma unroll
    for (int kk = 0; kk < kMaxInnerPass; kk++) {
        if ((uint32_t)kk >= n_pass) break;
        const int32_t s = inner[2 * kk];
        const uint32_t span = (uint32_t)(inner[2 * kk + 1] - s);
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if (!hit[c]) continue;
            int32_t p = pos[c];
            asm volatile("" : "+v"(p));  // keep the overlap test here, not hoisted into the hot loop
            const bool ov = (uint32_t)(p - s) <= span || (uint32_t)(p + (int32_t)L - 1 - s) <= span;
            cnt += __popcll(hit[c] & __ballot(ov));
        }
        acc[kk] += (lane == slot) ? cnt : 0u;
    }
}

// Exact score of the window starting at base i (pattern.rs:125-135), N = 0.
// Only lanes whose window contains an N run it.
__device__ __noinline__ int32_t exact_score(const uint32_t *words, uint32_t i, uint32_t nmbits, uint32_t L,
                                            const int32_t *w4) {
    uint32_t s = 0;
    for (uint32_t j = 0; j < L; j++) {
        if ((nmbits >> j) & 1u) continue;
        const uint32_t q = i + j;
        const uint32_t code = (words[q >> 4] >> (2 * (q & 15))) & 3u;
        s += (uint32_t)w4[4 * j + code];
    }
    return (int32_t)s;
}

template <int NCH>
struct Win {
    uint32_t code16[NCH][8];  // byte offsets of the eight 4-mer codes in a block (code * 16)
    int32_t rem[NCH];         // bases from the window start to the haplotype end
    int32_t pos[NCH];         // pos_i relative to ext_start
    uint32_t nm[NCH];         // N bits of bases i..i+31
};

__device__ __forceinline__ uint32_t pk_add_sat_i16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_add_i16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Table lookups of NB blocks for NCH chunks, added into sum.
// Threshold test of strand s of a unit for every chunk (hit ballots), with the
// windows that contain an N rescored exactly, then the counting on a hit.
template <int NCH, bool OCT>
__device__ __forceinline__ void strand_hits(const ScanArgs &A, CUnit &U, int s, const uint32_t (&sum)[NCH][4],
                                            const Win<NCH> &W, const DevHap &hm, bool has_n, uint32_t h, uint32_t cg,
                                            const int32_t *inner, uint32_t n_pass, bool write_hits, uint32_t lane,
                                            uint32_t (&acc)[kMaxInnerPass]) {
    const uint32_t L = U.len[s];
    uint64_t hit[NCH];
    uint64_t any = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        bool hb;
        if (OCT) {
            const uint32_t d = sum[c][s >> 1];
            hb = (s & 1) ? (int32_t)d >= 0 : (int32_t)(d << 16) >= 0;
        } else {
            hb = (int32_t)sum[c][s] > U.thr[s];
        }
        if (has_n) {
            const uint32_t lm = L >= 32 ? 0xFFFFFFFFu : ((1u << L) - 1u);
            const uint32_t m = W.nm[c] & lm;
            if (m && W.rem[c] >= (int32_t)L)
                hb = exact_score(A.words + hm.word_off, cg + 64 * c + lane, m, L, A.wfull + 4 * (size_t)U.wofs[s]) >
                     U.min_score[s];
        }
        hit[c] = __ballot(hb && W.rem[c] >= (int32_t)L);
        any |= hit[c];
    }
    if (__builtin_expect(write_hits, 0) && lane == 0) {
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const uint32_t wi = cg / 64 + c;
            if (wi < A.hits_wpp) A.hits[((size_t)h * A.n_patterns_total + U.orig_index[s]) * A.hits_wpp + wi] = hit[c];
        }
    }
    if (__builtin_expect(any != 0, 0)) count_hits<NCH>(hit, W.pos, L, inner, n_pass, U.slot_local[s], lane, acc);
}

// One unit over NCH chunks.  OCTET16: the halves start at -(thr + 1) and a
// strand hits iff its final half is >= 0, so the AND of every accumulator has
// a clear sign bit iff some strand of some window may hit -- one wave-uniform
// test gates the per-strand work.  QUAD32: per-strand compares.
template <int NCH, bool OCT>
__device__ __forceinline__ void unit_body(const ScanArgs &A, CUnit &U, const char *s_lut, const Win<NCH> &W,
                                          const DevHap &hm, bool has_n, uint32_t h, uint32_t cg, const int32_t *inner,
                                          uint32_t n_pass, bool write_hits, uint32_t lane,
                                          uint32_t (&acc)[kMaxInnerPass]) {
    const char *base = s_lut + (size_t)U.lut_off * kBlockBytes;
    const uint32_t nblk = U.nblk;
    uint32_t sum[NCH][4];
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
        for (int d = 0; d < 4; d++) sum[c][d] = OCT ? U.init[d] : 0u;
#pragma unroll
    for (int b = 0; b < 8; b++) {
        if ((uint32_t)b >= nblk) break;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(base + b * kBlockBytes + W.code16[c][b]);
            if (OCT) {
                sum[c][0] = pk_add_sat_i16(sum[c][0], v.x);
                sum[c][1] = pk_add_sat_i16(sum[c][1], v.y);
                sum[c][2] = pk_add_sat_i16(sum[c][2], v.z);
                sum[c][3] = pk_add_sat_i16(sum[c][3], v.w);
            } else {
                sum[c][0] += v.x;
                sum[c][1] += v.y;
                sum[c][2] += v.z;
                sum[c][3] += v.w;
            }
        }
    }
    if (OCT) {
        uint32_t all = 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < NCH; c++) all &= sum[c][0] & sum[c][1] & sum[c][2] & sum[c][3];
        const bool maybe = (all & 0x80008000u) != 0x80008000u;
        if (__builtin_expect(!has_n && !write_hits && __ballot(maybe) == 0, 1)) return;
    }
    constexpr int kStrands = OCT ? 8 : 4;
#pragma unroll
    for (int s = 0; s < kStrands; s++) {
        if ((uint32_t)s >= U.nstrand) break;
        strand_hits<NCH, OCT>(A, U, s, sum, W, hm, has_n, h, cg, inner, n_pass, write_hits, lane, acc);
    }
}

// Score NCH 64-window chunks starting at window cg against every unit of the tile.
template <int NCH>
__device__ __forceinline__ void scan_chunks(const ScanArgs &A, const DevTile &t, const char *s_lut,
                                            CUnit *s_units, const DevHap &hm, uint32_t h, uint32_t cg,
                                            const int32_t *inner, uint32_t n_pass, bool write_hits, uint32_t lane,
                                            uint32_t (&acc)[kMaxInnerPass]) {
    const bool has_n = (hm.flags & HAP_HAS_N) != 0;
    const bool has_pos = (hm.flags & HAP_HAS_POS) != 0;
    Win<NCH> W;
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
            W.code16[c][b] = ((lo >> (8 * b)) & 0xFFu) << 4;
            W.code16[c][b + 4] = ((hi >> (8 * b)) & 0xFFu) << 4;
        }
        W.rem[c] = (int32_t)hm.len - (int32_t)i;
        W.pos[c] = has_pos ? (i < hm.len ? A.posrel[hm.pos_off + i] : 0) : (int32_t)i;
        if (has_n) {
            const uint32_t *m = A.nmask + hm.nmask_off + (ic >> 5);
            W.nm[c] = __builtin_amdgcn_alignbit(m[1], m[0], ic & 31);
        } else {
            W.nm[c] = 0;
        }
    }
    for (uint32_t ui = 0; ui < t.last - t.first; ui++) {
        CUnit &U = s_units[ui];
        if (U.kind == UNIT_OCTET16)
            unit_body<NCH, true>(A, U, s_lut, W, hm, has_n, h, cg, inner, n_pass, write_hits, lane, acc);
        else
            unit_body<NCH, false>(A, U, s_lut, W, hm, has_n, h, cg, inner, n_pass, write_hits, lane, acc);
    }
}

// ---------------------------------------------------------------------------
// Fast kernel.  Grid: n_tiles x ceil(n_haps / haps_per_block); 512 threads.
// LDS: the tile's table blocks, then its unit descriptors.
// ---------------------------------------------------------------------------
template <int MINW>
__global__ __launch_bounds__(512, MINW) void scan_fast_kernel(ScanArgs A) {
    extern __shared__ __attribute__((aligned(16))) int32_t smem[];
    constexpr uint32_t kBlock = 512, kWaves = kBlock / 64;
    const uint32_t tile_idx = blockIdx.x % A.n_tiles;
    const uint32_t hg = blockIdx.x / A.n_tiles;
    const DevTile t = A.tiles[tile_idx];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.lut + (size_t)t.lut_begin * kBlockInts);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        const uint32_t n4 = t.nblocks * (kBlockInts / 4);
        for (uint32_t i = threadIdx.x; i < n4; i += kBlock) dst[i] = src[i];
    }
    __syncthreads();
    const char *s_lut = reinterpret_cast<const char *>(smem);
    // unit descriptors stay in global memory: wave-uniform, read with scalar loads
    CUnit *s_units = (CUnit *)(A.units + t.first);

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
            const int32_t *inner = A.inner + 2 * (size_t)(rg.inner_off + k0);
            uint32_t acc[kMaxInnerPass];
#pragma unroll
            for (int kk = 0; kk < kMaxInnerPass; kk++) acc[kk] = 0;
            const bool write_hits = A.hits != nullptr && pass == 0;
            for (uint32_t cg = 0; cg < nwin; cg += 64 * kChunks) {
                const uint32_t nch = min((uint32_t)kChunks, (nwin - cg + 63) / 64);
                if (nch >= 3)  // a 3-chunk tail scores one chunk of invalid windows (rem < L)
                    scan_chunks<4>(A, t, s_lut, s_units, hm, h, cg, inner, n_pass, write_hits, lane, acc);
                else if (nch == 2)
                    scan_chunks<2>(A, t, s_lut, s_units, hm, h, cg, inner, n_pass, write_hits, lane, acc);
                else
                    scan_chunks<1>(A, t, s_lut, s_units, hm, h, cg, inner, n_pass, write_hits, lane, acc);
            }
            if (n_pass && lane < t.nslots) {
                const size_t st = rg.count_stride;
                uint32_t *out = A.counts + hm.count_off + ((size_t)(t.slot_begin + lane) * n_inner + k0) * st;
#pragma unroll
                for (int kk = 0; kk < kMaxInnerPass; kk++)
                    if ((uint32_t)kk < n_pass) out[kk * st] = acc[kk];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Generic kernel: one pattern_id group whose strands include one longer than
// 32 columns; column-wise scoring with weights read through the cache.
// Grid: n_gen_tiles x ceil(n_haps / haps_per_block).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kGenBlock) void scan_generic_kernel(ScanArgs A) {
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
            const int32_t *inner = A.inner + 2 * (size_t)(rg.inner_off + k0);
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
                    const DevPattern p = A.gpats[pi];
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
                    if (any) count_hits<kChunks>(hit, pos, p.len, inner, n_pass, p.slot_local, lane, acc);
                }
            }
            if (n_pass && lane == 0) {
                const size_t st = rg.count_stride;
                uint32_t *out = A.counts + hm.count_off + ((size_t)t.slot_begin * n_inner + k0) * st;
                for (int kk = 0; kk < kMaxInnerPass; kk++)
                    if ((uint32_t)kk < n_pass) out[kk * st] = acc[kk];
            }
        }
    }
}

typedef void (*FastKernel)(ScanArgs);
FastKernel fast_variant(int minw) { return minw == 4 ? scan_fast_kernel<4> : scan_fast_kernel<2>; }

}  // namespace

int fast_kernel_set_lds(const LaunchConfig &cfg) {
    if (cfg.lds_bytes <= 64 * 1024) return TFBS_OK;
    hipError_t e = hipFuncSetAttribute((const void *)fast_variant(cfg.minw), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)cfg.lds_bytes);
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("LDS attribute: ") + hipGetErrorString(e));
    return TFBS_OK;
}

// Grids stay below 2^31 workgroups by splitting along haplotype groups.
int launch_fast(const ScanArgs &a0, const LaunchConfig &cfg, uint32_t n_haps, hipStream_t stream) {
    if (n_haps == 0 || a0.n_tiles == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / a0.n_tiles - 1);
    int launches = 0;
    for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
        const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
        const uint32_t h0 = (uint32_t)(g0 * hpb);
        ScanArgs a = a0;
        a.haps = a0.haps + h0;
        a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
        a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
        hipLaunchKernelGGL(fast_variant(cfg.minw), dim3(a0.n_tiles * ng), dim3(512), cfg.lds_bytes, stream, a);
        launches++;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_fast_kernel launch: ") + hipGetErrorString(e));
    return launches;
}

int launch_generic(const ScanArgs &a0, uint32_t n_haps, hipStream_t stream) {
    if (n_haps == 0 || a0.n_tiles == 0) return 0;
    const uint32_t hpb = a0.haps_per_block;
    const uint32_t n_hg = (n_haps + hpb - 1) / hpb;
    const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / a0.n_tiles - 1);
    int launches = 0;
    for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
        const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
        const uint32_t h0 = (uint32_t)(g0 * hpb);
        ScanArgs a = a0;
        a.haps = a0.haps + h0;
        a.n_haps = std::min<uint32_t>(n_haps - h0, ng * hpb);
        a.hits = a0.hits ? a0.hits + (size_t)h0 * a0.n_patterns_total * a0.hits_wpp : nullptr;
        hipLaunchKernelGGL(scan_generic_kernel, dim3(a0.n_tiles * ng), dim3(kGenBlock), 0, stream, a);
        launches++;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("scan_generic_kernel launch: ") + hipGetErrorString(e));
    return launches;
}

}  // namespace tfbs
