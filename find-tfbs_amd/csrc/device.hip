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
//    three words, once per haplotype, into eight 4-mer codes.
//  * Each PWM strand of length L <= 32 is a list of ceil(L/4) 4-mer lookup
//    tables (256 int32 each; entry = sum of the 4 column weights, i32 wrap).
//    A workgroup stages one tile of tables (several pattern_ids, both strands)
//    in LDS and every wave scores its haplotypes against the whole tile: one
//    LDS read + two VALU adds per 4 columns per window.
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

constexpr int kBlock = 256;     // 4 waves
constexpr int kWaves = kBlock / 64;
constexpr int kChunks = 4;      // 64-window chunks per lane group (256 windows per pass)

struct Inner {
    int32_t s;
    uint32_t span;  // e - s
};

// Count, for every inner range of this pass, the hit windows whose match range
// overlaps it (main.rs:503 with Range::overlaps, range.rs:18-21), and add the
// counts to the lane that owns the pattern_id slot.
__device__ __forceinline__ void count_hits(const uint64_t (&hit)[kChunks], const int32_t (&pos)[kChunks], uint32_t L,
                                           const Inner *in, uint32_t n_pass, uint32_t slot, uint32_t lane,
                                           uint32_t (&acc)[kMaxInnerPass]) {
#pragma unroll
    for (int kk = 0; kk < kMaxInnerPass; kk++) {
        if ((uint32_t)kk >= n_pass) break;
        const int32_t s = in[kk].s;
        const uint32_t span = in[kk].span;
        uint32_t cnt = 0;
#pragma unroll
        for (int c = 0; c < kChunks; c++) {
            if (!hit[c]) continue;
            const bool ov = (uint32_t)(pos[c] - s) <= span || (uint32_t)(pos[c] + (int32_t)L - 1 - s) <= span;
            cnt += __popcll(hit[c] & __ballot(ov));
        }
        acc[kk] += (lane == slot) ? cnt : 0u;
    }
}

// ---------------------------------------------------------------------------
// Fast kernel: PWM strands of length <= 32 via 4-mer LUTs staged in LDS.
// Grid: n_tiles x ceil(n_haps / haps_per_block); block 256 threads.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void scan_fast_kernel(
    const DevTile *__restrict__ tiles, uint32_t n_tiles, const DevPattern *__restrict__ pats,
    const int32_t *__restrict__ lut, const int32_t *__restrict__ colA, const DevHap *__restrict__ haps,
    uint32_t n_haps, const DevRegion *__restrict__ regions, const int32_t *__restrict__ inner,
    const uint32_t *__restrict__ words, const uint32_t *__restrict__ nmask, const int32_t *__restrict__ posrel,
    uint32_t *__restrict__ counts, uint32_t haps_per_block, unsigned long long *__restrict__ hits,
    uint32_t hits_wpp, uint32_t n_patterns_total) {
    extern __shared__ __attribute__((aligned(16))) int32_t smem[];
    const uint32_t tile_idx = blockIdx.x % n_tiles;
    const uint32_t hg = blockIdx.x / n_tiles;
    const DevTile t = tiles[tile_idx];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;

    // stage the tile's LUT blocks and A columns (16-byte loads)
    {
        const int4 *src = reinterpret_cast<const int4 *>(lut + (size_t)t.lut_begin * kLutEntries);
        int4 *dst = reinterpret_cast<int4 *>(smem);
        const uint32_t n4 = t.nblocks * (kLutEntries / 4);
        for (uint32_t i = threadIdx.x; i < n4; i += kBlock) dst[i] = src[i];
        int32_t *scol = smem + t.nblocks * kLutEntries;
        for (uint32_t i = threadIdx.x; i < t.ncols; i += kBlock) scol[i] = colA[t.col_begin + i];
    }
    __syncthreads();
    const char *s_lut = reinterpret_cast<const char *>(smem);
    const int32_t *s_col = smem + t.nblocks * kLutEntries;

    for (uint32_t hh = wave; hh < haps_per_block; hh += kWaves) {
        const uint32_t h = hg * haps_per_block + hh;
        if (h >= n_haps) break;
        const DevHap hm = haps[h];
        const DevRegion rg = regions[hm.region];
        const uint32_t n_inner = rg.n_inner;
        const bool has_n = (hm.flags & HAP_HAS_N) != 0;
        const bool has_pos = (hm.flags & HAP_HAS_POS) != 0;
        const uint32_t n_passes = n_inner == 0 ? (hits ? 1u : 0u) : (n_inner + kMaxInnerPass - 1) / kMaxInnerPass;
        for (uint32_t pass = 0; pass < n_passes; pass++) {
            const uint32_t k0 = pass * kMaxInnerPass;
            const uint32_t n_pass = n_inner > k0 ? min((uint32_t)kMaxInnerPass, n_inner - k0) : 0u;
            Inner in[kMaxInnerPass];
#pragma unroll
            for (int kk = 0; kk < kMaxInnerPass; kk++) {
                if ((uint32_t)kk < n_pass) {
                    const int32_t s = inner[2 * (rg.inner_off + k0 + kk)];
                    const int32_t e = inner[2 * (rg.inner_off + k0 + kk) + 1];
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

            for (uint32_t cg = 0; cg < hm.len; cg += 64 * kChunks) {
                uint32_t code4[kChunks][8];  // byte offsets of the 8 4-mer codes (code * 4)
                int32_t rem[kChunks], pos[kChunks];
                uint32_t nm[kChunks];
#pragma unroll
                for (int c = 0; c < kChunks; c++) {
                    const uint32_t i = cg + 64 * c + lane;
                    const uint32_t ic = min(i, hm.len);  // keep reads inside the +3 word pad
                    const uint32_t *w = words + hm.word_off + (ic >> 4);
                    const uint32_t sh = 2 * (ic & 15);
                    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                    const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, sh);
                    const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, sh);
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        code4[c][b] = ((lo >> (8 * b)) & 0xFFu) << 2;
                        code4[c][b + 4] = ((hi >> (8 * b)) & 0xFFu) << 2;
                    }
                    rem[c] = (int32_t)hm.len - (int32_t)i;
                    pos[c] = has_pos ? (i < hm.len ? posrel[hm.pos_off + i] : 0) : (int32_t)i;
                    if (has_n) {
                        const uint32_t *m = nmask + hm.nmask_off + (ic >> 5);
                        nm[c] = __builtin_amdgcn_alignbit(m[1], m[0], ic & 31);
                    } else {
                        nm[c] = 0;
                    }
                }
                for (uint32_t pi = t.pat_begin; pi < t.pat_end; pi++) {
                    const DevPattern p = pats[pi];
                    const char *base = s_lut + (size_t)p.lut_off * (kLutEntries * 4);
                    int32_t sc[kChunks];
#pragma unroll
                    for (int c = 0; c < kChunks; c++) sc[c] = 0;
#pragma unroll
                    for (int b = 0; b < 8; b++) {
                        if (b >= p.nblk) break;
#pragma unroll
                        for (int c = 0; c < kChunks; c++)
                            sc[c] = (int32_t)((uint32_t)sc[c] +
                                              (uint32_t)*reinterpret_cast<const int32_t *>(
                                                  base + b * (kLutEntries * 4) + code4[c][b]));
                    }
                    if (has_n) {
                        const uint32_t lmask = p.len >= 32 ? 0xFFFFFFFFu : ((1u << p.len) - 1u);
#pragma unroll
                        for (int c = 0; c < kChunks; c++) {
                            uint32_t m = nm[c] & lmask;
                            while (m) {
                                const uint32_t j = __builtin_ctz(m);
                                sc[c] = (int32_t)((uint32_t)sc[c] - (uint32_t)s_col[p.col_off + j]);
                                m &= m - 1;
                            }
                        }
                    }
                    uint64_t hit[kChunks];
                    uint64_t any = 0;
#pragma unroll
                    for (int c = 0; c < kChunks; c++) {
                        hit[c] = __ballot(sc[c] > p.min_score && rem[c] >= (int32_t)p.len);
                        any |= hit[c];
                    }
                    if (hits && pass == 0 && lane == 0) {
#pragma unroll
                        for (int c = 0; c < kChunks; c++) {
                            const uint32_t wi = cg / 64 + c;
                            if (wi < hits_wpp)
                                hits[((size_t)h * n_patterns_total + p.orig_index) * hits_wpp + wi] = hit[c];
                        }
                    }
                    if (any) count_hits(hit, pos, p.len, in, n_pass, p.slot_local, lane, acc);
                }
            }
            if (n_pass && lane < t.nslots) {
                uint32_t *out = counts + hm.count_off + (size_t)(t.slot_begin + lane) * n_inner + k0;
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
__global__ __launch_bounds__(kBlock) void scan_generic_kernel(
    const DevTile *__restrict__ tiles, uint32_t n_tiles, const DevPattern *__restrict__ pats,
    const int32_t *__restrict__ gw, const DevHap *__restrict__ haps, uint32_t n_haps,
    const DevRegion *__restrict__ regions, const int32_t *__restrict__ inner, const uint32_t *__restrict__ words,
    const uint32_t *__restrict__ nmask, const int32_t *__restrict__ posrel, uint32_t *__restrict__ counts,
    uint32_t haps_per_block, unsigned long long *__restrict__ hits, uint32_t hits_wpp, uint32_t n_patterns_total) {
    const uint32_t tile_idx = blockIdx.x % n_tiles;
    const uint32_t hg = blockIdx.x / n_tiles;
    const DevTile t = tiles[tile_idx];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    for (uint32_t hh = wave; hh < haps_per_block; hh += kWaves) {
        const uint32_t h = hg * haps_per_block + hh;
        if (h >= n_haps) break;
        const DevHap hm = haps[h];
        const DevRegion rg = regions[hm.region];
        const uint32_t n_inner = rg.n_inner;
        const bool has_n = (hm.flags & HAP_HAS_N) != 0;
        const bool has_pos = (hm.flags & HAP_HAS_POS) != 0;
        const uint32_t n_passes = n_inner == 0 ? (hits ? 1u : 0u) : (n_inner + kMaxInnerPass - 1) / kMaxInnerPass;
        for (uint32_t pass = 0; pass < n_passes; pass++) {
            const uint32_t k0 = pass * kMaxInnerPass;
            const uint32_t n_pass = n_inner > k0 ? min((uint32_t)kMaxInnerPass, n_inner - k0) : 0u;
            Inner in[kMaxInnerPass];
            for (int kk = 0; kk < kMaxInnerPass; kk++) {
                if ((uint32_t)kk < n_pass) {
                    in[kk].s = inner[2 * (rg.inner_off + k0 + kk)];
                    in[kk].span = (uint32_t)(inner[2 * (rg.inner_off + k0 + kk) + 1] - in[kk].s);
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
                    pos[c] = has_pos ? (i < hm.len ? posrel[hm.pos_off + i] : 0) : (int32_t)i;
                }
                for (uint32_t pi = t.pat_begin; pi < t.pat_end; pi++) {
                    const DevPattern p = pats[pi];
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
                                uint32_t code = (words[hm.word_off + (q >> 4)] >> (2 * (q & 15))) & 3u;
                                if (has_n && ((nmask[hm.nmask_off + (q >> 5)] >> (q & 31)) & 1u)) code = 4;
                                sc += (uint32_t)gw[(size_t)(p.col_off + j) * 5 + code];
                            }
                        }
                        hit[c] = __ballot(valid && (int32_t)sc > p.min_score);
                        any |= hit[c];
                    }
                    if (hits && pass == 0 && lane == 0) {
                        for (int c = 0; c < kChunks; c++) {
                            const uint32_t wi = cg / 64 + c;
                            if (wi < hits_wpp)
                                hits[((size_t)h * n_patterns_total + p.orig_index) * hits_wpp + wi] = hit[c];
                        }
                    }
                    if (any) count_hits(hit, pos, p.len, in, n_pass, p.slot_local, lane, acc);
                }
            }
            if (n_pass && lane == 0) {
                uint32_t *out = counts + hm.count_off + (size_t)t.slot_begin * n_inner + k0;
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
    uint32_t tile_blocks = 32;
    uint32_t haps_per_block = 64;
    size_t lds_bytes = 0;
    DevBuf<DevPattern> fast_pats, gen_pats;
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

static int env_u32(const char *name, uint32_t dflt) {
    const char *v = getenv(name);
    if (!v || !*v) return (int)dflt;
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
            const uint32_t nh = std::min<uint32_t>(n_haps - h0, ng * hpb);
            hipLaunchKernelGGL(scan_fast_kernel, dim3(nt * ng), dim3(kBlock), ctx->lds_bytes, ctx->stream,
                               ctx->fast_tiles.p, nt, ctx->fast_pats.p, ctx->lut.p, ctx->colA.p, ctx->haps.p + h0, nh,
                               ctx->regions.p, ctx->inner.p, ctx->words.p, ctx->nmask.p, ctx->posrel.p,
                               ctx->counts.p, hpb, hits ? hits + (size_t)h0 * n_pat_total * hits_wpp : nullptr,
                               hits_wpp, n_pat_total);
            launches++;
        }
    }
    if (!P.gen_tiles.empty()) {
        const uint32_t nt = (uint32_t)P.gen_tiles.size();
        const uint64_t max_hg = std::max<uint64_t>(1, (1ull << 31) / nt - 1);
        for (uint64_t g0 = 0; g0 < n_hg; g0 += max_hg) {
            const uint32_t ng = (uint32_t)std::min<uint64_t>(max_hg, n_hg - g0);
            const uint32_t h0 = (uint32_t)(g0 * hpb);
            const uint32_t nh = std::min<uint32_t>(n_haps - h0, ng * hpb);
            hipLaunchKernelGGL(scan_generic_kernel, dim3(nt * ng), dim3(kBlock), 0, ctx->stream, ctx->gen_tiles.p, nt,
                               ctx->gen_pats.p, ctx->gen_w.p, ctx->haps.p + h0, nh, ctx->regions.p, ctx->inner.p,
                               ctx->words.p, ctx->nmask.p, ctx->posrel.p, ctx->counts.p, hpb,
                               hits ? hits + (size_t)h0 * n_pat_total * hits_wpp : nullptr, hits_wpp, n_pat_total);
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
    ctx->fast_pats.release(); ctx->gen_pats.release(); ctx->fast_tiles.release(); ctx->gen_tiles.release();
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
    ctx->tile_blocks = (uint32_t)std::max(8, env_u32("TFBS_TILE_BLOCKS", 32));
    ctx->haps_per_block = (uint32_t)std::max(4, env_u32("TFBS_HAPS_PER_BLOCK", 64));
    rc = ctx->pats->build_plan(ctx->tile_blocks, &ctx->plan);
    if (rc) { delete ctx; return rc; }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->ev1);
    if (e != hipSuccess) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_HIP, std::string("HIP init: ") + hipGetErrorString(e));
    }
    const Plan &P = ctx->plan;
    ctx->lds_bytes = (size_t)P.max_tile_blocks * kLutEntries * 4 + (size_t)P.max_tile_cols * 4 + 16;
    if (ctx->lds_bytes > 64 * 1024) {
        e = hipFuncSetAttribute((const void *)scan_fast_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)ctx->lds_bytes);
        if (e != hipSuccess) {
            tfbs_ctx_destroy(ctx);
            return tfbs::fail(TFBS_E_HIP, std::string("LDS attribute: ") + hipGetErrorString(e));
        }
    }
    if ((rc = ctx->fast_pats.put(P.fast_pats, ctx->stream)) || (rc = ctx->fast_tiles.put(P.fast_tiles, ctx->stream)) ||
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
        if (c == 4) { has_n = true; c = 0; }
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
