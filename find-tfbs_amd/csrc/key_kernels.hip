// Per-region key assembly on the device.
//
// count_matches_by_sample (main.rs:500-534) builds, per key (bed, inner range,
// pattern_id), the per-sample L/R vectors; counts_as_genotypes (main.rs:439-498)
// emits a row only when the per-sample totals differ.  Every sample's total is
// a sum of two distinct haplotypes' counts, so a key can only produce a row if
// its counts over the region's distinct haplotypes are not constant.
//
// The matrix-core scan leaves no count matrix: per hit one (haplotype, key =
// slot * n_inner + range) pair in its workgroup's hit list (or the spill list),
// plus the region's reference hits (strand, window) that every HAP_DEDUP
// haplotype inherits in the window tiles it did not scan.  key_asm_kernel (one
// workgroup per region) counts them into a [key][distinct haplotype] block in
// LDS, a chunk of keys at a time -- the LUT/generic kernels' slots are copied
// from their dense counts -- and then either classifies every key (any count
// != 0 -> the key exists in the reference's HashMap; counts differ -> it may
// emit a row) and appends the varying keys' counts to a compact list (the run
// flow's reduction), or stores the block into the dense matrix (the debug
// download).
#include <hip/hip_runtime.h>

#include <mutex>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "keys.hpp"

namespace tfbs {
namespace {

constexpr int kAsmBlock = 256;
constexpr uint32_t kAsmWaves = kAsmBlock / 64;
constexpr uint32_t kAsmCounters = 6144;  // u32 counters of the LDS block (24 KiB)
constexpr uint32_t kAsmHaps = 1024;      // haplotypes whose diff runs sit in LDS (else read from L2)

constexpr uint32_t kAsmRuns = 2048;      // diff runs staged in LDS
constexpr uint32_t kAsmHits = 2048;      // own hits staged in LDS (else re-read from the lists per pass)
constexpr uint32_t kAsmRefs = 256;       // reference hits staged in LDS (else re-read)
constexpr uint32_t kAsmKeyWords = 2048;  // touched-key bitmap: keys handled per key window
constexpr uint32_t kAsmKeyWin = 32 * kAsmKeyWords;

// Region r's spill records (bucketed: [spill_off[r], spill_off[r + 1]) of spill_sorted).
__device__ __forceinline__ uint2 spill_range(const AsmArgs &A, uint32_t r) {
    return (A.spill_count && *A.spill_count) ? make_uint2(A.spill_off[r], A.spill_off[r + 1]) : make_uint2(0, 0);
}

// The inner ranges [k0, k0 + nk) a reference hit (window i of a strand of length L)
// overlaps (range.rs:18-21 as main.rs:503 uses it; the reference's positions are
// affine): bit k - k0.
__device__ __forceinline__ uint32_t ref_overlaps(const AsmArgs &A, const DevRegion &rg, uint32_t L, uint32_t i,
                                                 uint32_t k0, uint32_t nk) {
    const int32_t *inner = A.inner + 2 * (size_t)rg.inner_off;
    uint32_t mask = 0;
    for (uint32_t k = k0; k < k0 + nk; k++) {
        const int32_t s = inner[2 * k], en = inner[2 * k + 1];
        const uint32_t span = (uint32_t)(en - s);
        if ((uint32_t)((int32_t)i - s) <= span || (uint32_t)((int32_t)(i + L) - 1 - s) <= span) mask |= 1u << (k - k0);
    }
    return mask;
}

// A reference hit (strand g, window i) as the assembly uses it: {first key
// (slot * n_inner), window, L | (K depth - 1) << 16, inner ranges < 32 it overlaps}.
__device__ __forceinline__ uint4 make_ref(const AsmArgs &A, const DevRegion &rg, uint32_t g, uint32_t i) {
    const int32_t *meta = A.mmeta + (size_t)(g >> 6) * kGMetaInts;
    const uint32_t sn = g & 63u, L = (uint32_t)meta[kGStrandInts * sn + kGLen];
    const uint32_t dk = (uint32_t)meta[kGDepth] - 1;
    const uint32_t key0 = (uint32_t)meta[kGStrandInts * sn + kGSlot] * rg.n_inner;
    return make_uint4(key0, i, L | (dk << 16), ref_overlaps(A, rg, L, i, 0, min(rg.n_inner, 32u)));
}

// Every own hit (local haplotype l < U, key) of region r: the workgroup lists of the
// matrix-core launches (one wave per list), then the region's spill records.
template <class F>
__device__ __forceinline__ void visit_hits(const AsmArgs &A, uint32_t r, uint32_t hb, uint32_t U, F &&f) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t g_lo = hb / A.hpb, g_hi = (hb + U - 1) / A.hpb;
    for (uint32_t si = 0; si < A.n_srcs; si++) {
        const HitSrc src = A.srcs[si];
        const uint32_t ga = max(g_lo, src.g0), gb = min(g_hi + 1, src.g0 + src.ng);
        if (ga >= gb) continue;
        const uint32_t per_g = src.ns * kMBlockWaves, n_l = (gb - ga) * per_g;
        for (uint32_t li = wave; li < n_l; li += kAsmWaves) {
            const uint32_t g = ga + li / per_g, rem = li % per_g;
            const uint32_t wg = src.wg_base + (g - src.g0) * src.ns + rem / kMBlockWaves, w = rem % kMBlockWaves;
            const uint32_t n = A.hitn[(size_t)wg * kMBlockWaves + w];
            const uint2 *lst = reinterpret_cast<const uint2 *>(A.hitl) + (size_t)wg * A.cand_cap +
                               (size_t)w * (A.cand_cap / kMBlockWaves);
            for (uint32_t e = lane; e < n; e += 64) {
                const uint2 h = lst[e];
                if (h.x - hb < U) f(h.x - hb, h.y);
            }
        }
    }
    const uint2 sp = spill_range(A, r);
    for (uint32_t e = sp.x + threadIdx.x; e < sp.y; e += kAsmBlock) {
        const uint32_t *q = A.spill_sorted + 3 * (size_t)e;
        if (!(q[0] >> 31) && q[1] - hb < U) f(q[1] - hb, q[2]);
    }
}

// Every reference hit of region r (its list, then its spill records).
template <class F>
__device__ __forceinline__ void visit_refs(const AsmArgs &A, uint32_t r, const DevRegion &rg, F &&f) {
    const uint32_t nl = min(A.ref_count[r], kRefPerRegion);
    for (uint32_t t = threadIdx.x; t < nl; t += kAsmBlock)
        f(make_ref(A, rg, A.ref_hits[2 * ((size_t)r * kRefPerRegion + t)],
                   A.ref_hits[2 * ((size_t)r * kRefPerRegion + t) + 1]));
    const uint2 sp = spill_range(A, r);
    for (uint32_t e = sp.x + threadIdx.x; e < sp.y; e += kAsmBlock) {
        const uint32_t *q = A.spill_sorted + 3 * (size_t)e;
        if (q[0] >> 31) f(make_ref(A, rg, q[1], q[2]));
    }
}

// One region per iteration: every region (list == nullptr, grid = regions) or the
// *list_n regions at list over a fixed grid.
__global__ __launch_bounds__(kAsmBlock) void key_asm_kernel(AsmArgs A, const uint32_t *list, const uint32_t *list_n) {
    __shared__ uint32_t s_cnt[kAsmCounters];
    __shared__ uint32_t s_rh[kAsmHaps];    // per haplotype: first staged run | runs << 16 (0xFFFFFFFF: not HAP_DEDUP)
    __shared__ uint2 s_run[kAsmRuns];      // the region's diff runs
    __shared__ uint2 s_hit[kAsmHits];      // (local haplotype, key)
    __shared__ uint4 s_ref[kAsmRefs];      // make_ref
    __shared__ uint32_t s_bits[kAsmKeyWords], s_rbase[kAsmKeyWords];  // touched keys of the window, rows before each word
    __shared__ uint32_t s_scan[kAsmBlock];
    __shared__ uint32_t s_nhit, s_nref, s_nvar, s_nput;
    __shared__ unsigned long long s_vbase, s_obase;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (list && A.report && blockIdx.x == 0 && tid < 2) A.report[tid] = A.report_src ? A.report_src[tid] : 0u;
    const uint32_t n_it = list ? *list_n : gridDim.x;
    for (uint32_t it = blockIdx.x; it < n_it; it += gridDim.x) {
    const uint32_t r = list ? list[it] : it;
    __syncthreads();  // the previous region's LDS readers are done
    [&]() {
    const DevRegion rg = A.regions[r];
    const uint32_t U = rg.hap_count, n_inner = rg.n_inner;
    const uint32_t K = A.n_slots * n_inner;
    const uint64_t ko = (uint64_t)rg.inner_off * A.n_slots;
    if (U == 0 || K == 0) {  // no samples: no haplotype, no match, no key
        if (A.mode == 0)
            for (uint32_t j = tid; j < K; j += kAsmBlock) {
                A.key_first[ko + j] = 0;
                A.key_flags[ko + j] = 0;
            }
        return;
    }
    const uint32_t hb = rg.hap_begin;
    // the diff runs of the region's HAP_DEDUP haplotypes (consecutive in the batch's
    // run array) in LDS when they fit
    uint32_t run0 = 0, run1 = 0;
    for (uint32_t l = 0; l < U; l++)  // uniform: the first and last HAP_DEDUP haplotype's runs
        if (A.haps[hb + l].flags & HAP_DEDUP) {
            run0 = A.haps[hb + l].rrun_off;
            break;
        }
    for (uint32_t l = U; l-- > 0;)
        if (A.haps[hb + l].flags & HAP_DEDUP) {
            run1 = A.haps[hb + l].rrun_off + A.haps[hb + l].n_rruns;
            break;
        }
    const bool lds_haps = U <= kAsmHaps && run1 - run0 <= kAsmRuns;
    if (lds_haps) {
        for (uint32_t l = tid; l < U; l += kAsmBlock) {
            const DevHap h = A.haps[hb + l];
            s_rh[l] = (h.flags & HAP_DEDUP) ? (h.rrun_off - run0) | (h.n_rruns << 16) : 0xFFFFFFFFu;
        }
        for (uint32_t k = tid; k < run1 - run0; k += kAsmBlock)
            s_run[k] = make_uint2(A.druns[2 * (run0 + k)], A.druns[2 * (run0 + k) + 1]);
    }
    const bool refs_on = A.mfma && rg.ref_hap != UINT32_MAX;
    // stage the region's own hits and reference hits in LDS (the lists are read once)
    if (tid == 0) s_nhit = s_nref = 0;
    __syncthreads();
    if (A.mfma) {
        visit_hits(A, r, hb, U, [&](uint32_t l, uint32_t key) {
            const uint32_t at = atomicAdd(&s_nhit, 1u);
            if (at < kAsmHits) s_hit[at] = make_uint2(l, key);
        });
        if (refs_on)
            visit_refs(A, r, rg, [&](const uint4 &q) {
                const uint32_t at = atomicAdd(&s_nref, 1u);
                if (at < kAsmRefs) s_ref[at] = q;
            });
    }
    __syncthreads();
    const uint32_t nhit = s_nhit, nref = s_nref;
    const bool hits_lds = nhit <= kAsmHits, refs_lds = nref <= kAsmRefs;
    auto each_hit = [&](auto &&f) {
        if (!A.mfma) return;
        if (hits_lds) {
            for (uint32_t e = tid; e < nhit; e += kAsmBlock) f(s_hit[e].x, s_hit[e].y);
        } else {
            visit_hits(A, r, hb, U, f);
        }
    };
    auto each_ref = [&](auto &&f) {  // thread-parallel over the reference hits
        if (!refs_on) return;
        if (refs_lds) {
            for (uint32_t t = tid; t < nref; t += kAsmBlock) f(s_ref[t]);
        } else {
            visit_refs(A, r, rg, f);
        }
    };
    // the keys a reference hit adds to: its ranges past 32 recomputed, the others in q.w
    auto ref_keys = [&](const uint4 &q, auto &&f) {
        const uint32_t L = q.z & 0xFFFFu;
        for (uint32_t kb = 0; kb < n_inner; kb += 32)
            for (uint32_t m = kb ? ref_overlaps(A, rg, L, q.y, kb, min(32u, n_inner - kb)) : q.w; m; m &= m - 1)
                f(q.x + kb + __builtin_ctz(m));
    };
    const uint64_t dense_base = A.dense_base ? A.haps[hb].count_off : 0;
    const bool lds_cnt = U <= kAsmCounters;
    const uint32_t rows_per = lds_cnt ? kAsmCounters / U : 1;
    uint32_t *cnt = lds_cnt ? s_cnt : A.scratch + rg.big_off;
    for (uint32_t kw0 = 0; kw0 < K; kw0 += kAsmKeyWin) {  // key windows (one unless 65536 keys)
        const uint32_t kwn = min(kAsmKeyWin, K - kw0), nw = (kwn + 31) / 32;
        __syncthreads();
        for (uint32_t w = tid; w < nw; w += kAsmBlock) s_bits[w] = 0;
        __syncthreads();
        // touched keys: own hits, reference hits, every key of a LUT/generic slot
        each_hit([&](uint32_t, uint32_t key) {
            const uint32_t j = key - kw0;
            if (j < kwn) atomicOr(&s_bits[j >> 5], 1u << (j & 31));
        });
        each_ref([&](const uint4 &q) {
            ref_keys(q, [&](uint32_t key) {
                const uint32_t j = key - kw0;
                if (j < kwn) atomicOr(&s_bits[j >> 5], 1u << (j & 31));
            });
        });
        if (A.any_dense)
            for (uint32_t j = tid; j < kwn; j += kAsmBlock)
                if (!A.slot_mfma[(kw0 + j) / n_inner]) atomicOr(&s_bits[j >> 5], 1u << (j & 31));
        __syncthreads();
        // rows: touched keys in key order (block scan of the words' popcounts)
        constexpr uint32_t per = kAsmKeyWords / kAsmBlock;
        uint32_t mine = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nw) mine += __popc(s_bits[w]);
        }
        s_scan[tid] = mine;
        __syncthreads();
        for (uint32_t o = 1; o < kAsmBlock; o <<= 1) {
            const uint32_t t = tid >= o ? s_scan[tid - o] : 0;
            __syncthreads();
            s_scan[tid] += t;
            __syncthreads();
        }
        {
            uint32_t run = s_scan[tid] - mine;
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t w = tid * per + q;
                if (w < nw) {
                    s_rbase[w] = run;
                    run += __popc(s_bits[w]);
                }
            }
        }
        const uint32_t T = s_scan[kAsmBlock - 1];
        __syncthreads();
        auto row_of = [&](uint32_t j) { return s_rbase[j >> 5] + __popc(s_bits[j >> 5] & ((1u << (j & 31)) - 1u)); };
        auto key_of_row = [&](uint32_t t) {  // the word whose rows start at or before t, then its bit
            uint32_t lo = 0, hi = nw - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (s_rbase[mid] <= t) lo = mid;
                else hi = mid - 1;
            }
            uint32_t b = s_bits[lo];
            for (uint32_t k = t - s_rbase[lo]; k; k--) b &= b - 1;
            return 32 * lo + __builtin_ctz(b);
        };
        // untouched keys: no match -- no key in the reference's HashMap (zeros in the dense matrix)
        for (uint32_t j = tid; j < kwn; j += kAsmBlock) {
            if ((s_bits[j >> 5] >> (j & 31)) & 1u) continue;
            if (A.mode == 0) {
                A.key_first[ko + kw0 + j] = 0;
                A.key_flags[ko + kw0 + j] = 0;
            } else {
                for (uint32_t l = 0; l < U; l++) A.counts[dense_base + (uint64_t)(kw0 + j) * rg.count_stride + l] = 0;
            }
        }
        for (uint32_t t0 = 0; t0 < T; t0 += rows_per) {
            const uint32_t nrow = min(rows_per, T - t0);
            __syncthreads();  // the previous chunk's readers are done
            for (uint32_t rr = wave; rr < nrow; rr += kAsmWaves) {  // a LUT/generic key: its dense counts
                const uint32_t j = kw0 + key_of_row(t0 + rr);
                const bool dense = A.any_dense && !A.slot_mfma[j / n_inner];
                for (uint32_t l = lane; l < U; l += 64)
                    cnt[rr * U + l] = dense ? A.counts[dense_base + (uint64_t)j * rg.count_stride + l] : 0u;
            }
            __syncthreads();
            each_hit([&](uint32_t l, uint32_t key) {
                const uint32_t j = key - kw0;
                if (j >= kwn) return;
                const uint32_t t = row_of(j) - t0;
                if (t < nrow) atomicAdd(&cnt[t * U + l], 1u);
            });
            // reference hits: +1 to every HAP_DEDUP haplotype for which the hit's
            // window is not dirty (in the reference's columns: the haplotype has the
            // window's bases from its start position on, the scan lists no hit there;
            // tfbs_internal.hpp run_meets, span L)
            auto dirty = [&](uint32_t l, uint32_t L, uint32_t w) {
                const uint32_t S = L;
                if (lds_haps) {
                    const uint32_t x = s_rh[l];
                    if (x == 0xFFFFFFFFu) return true;
                    for (uint32_t k = x & 0xFFFFu, e = k + (x >> 16); k < e; k++)
                        if (run_meets(s_run[k].x, s_run[k].y, w, S)) return true;
                    return false;
                }
                const DevHap &h = A.haps[hb + l];
                if (!(h.flags & HAP_DEDUP)) return true;
                for (uint32_t k = h.rrun_off; k < h.rrun_off + h.n_rruns; k++)
                    if (run_meets(A.druns[2 * k], A.druns[2 * k + 1], w, S)) return true;
                return false;
            };
            if (refs_on && refs_lds && U <= 32 * kAsmBlock) {
                for (uint32_t q0 = 0; q0 < nref; q0++) {  // workgroup-uniform; threads over the haplotypes
                    const uint4 q = s_ref[q0];
                    const uint32_t L = q.z & 0xFFFFu;
                    bool here = false;  // uniform: a key of the hit is in this chunk
                    ref_keys(q, [&](uint32_t key) {
                        here = here || (key - kw0 < kwn && row_of(key - kw0) - t0 < nrow);
                    });
                    if (!here) continue;
                    uint32_t keep = 0;  // bit j: haplotype tid + j kAsmBlock inherits the hit
                    for (uint32_t l = tid, j = 0; l < U; l += kAsmBlock, j++)
                        if (!dirty(l, L, q.y)) keep |= 1u << j;
                    ref_keys(q, [&](uint32_t key) {
                        const uint32_t t = key - kw0 < kwn ? row_of(key - kw0) - t0 : UINT32_MAX;
                        if (t >= nrow) return;
                        for (uint32_t m = keep; m; m &= m - 1)
                            atomicAdd(&cnt[t * U + tid + kAsmBlock * __builtin_ctz(m)], 1u);
                    });
                }
            } else if (refs_on) {  // too many for LDS (rare): each thread walks its hits' haplotypes
                visit_refs(A, r, rg, [&](const uint4 &q) {
                    const uint32_t L = q.z & 0xFFFFu;
                    ref_keys(q, [&](uint32_t key) {
                        const uint32_t t = key - kw0 < kwn ? row_of(key - kw0) - t0 : UINT32_MAX;
                        if (t >= nrow) return;
                        for (uint32_t l = 0; l < U; l++)
                            if (!dirty(l, L, q.y)) atomicAdd(&cnt[t * U + l], 1u);
                    });
                });
            }
            __syncthreads();
            if (A.mode == 1) {  // dense: the matrix-core slots' counts into the count matrix
                for (uint32_t rr = wave; rr < nrow; rr += kAsmWaves) {
                    const uint32_t j = kw0 + key_of_row(t0 + rr);
                    if (!A.slot_mfma[j / n_inner]) continue;
                    for (uint32_t l = lane; l < U; l += 64)
                        A.counts[dense_base + (uint64_t)j * rg.count_stride + l] = cnt[rr * U + l];
                }
                continue;
            }
            // classify: one wave per row
            if (tid == 0) s_nvar = 0;
            __syncthreads();
            for (uint32_t rr = wave; rr < nrow; rr += kAsmWaves) {
                const uint32_t j = kw0 + key_of_row(t0 + rr);
                const uint32_t *col = cnt + rr * U;
                const uint32_t c0 = col[0];
                uint32_t any = 0, diff = 0;
                for (uint32_t l = lane; l < U; l += 64) {
                    const uint32_t c = col[l];
                    any |= c;
                    diff |= c ^ c0;
                }
                const bool a = __ballot(any != 0) != 0, v = __ballot(diff != 0) != 0;
                if (lane == 0) {
                    A.key_first[ko + j] = c0;
                    A.key_flags[ko + j] = (uint8_t)((a ? KEY_ANY : 0) | (v ? KEY_VARIES : 0));
                    if (v) atomicAdd(&s_nvar, 1u);
                }
            }
            __syncthreads();
            const uint32_t nvar = s_nvar;  // (reset only after the next chunk's first barrier)
            if (nvar == 0) continue;
            if (tid == 0) {  // the chunk's share of the compact lists
                s_vbase = atomicAdd(A.var_tot, (unsigned long long)nvar);
                s_obase = atomicAdd(A.var_tot + 1, (unsigned long long)nvar * U);
                s_nput = 0;
            }
            __syncthreads();
            for (uint32_t rr = wave; rr < nrow; rr += kAsmWaves) {
                const uint32_t *col = cnt + rr * U;
                const uint32_t c0 = col[0];
                uint32_t diff = 0;
                for (uint32_t l = lane; l < U; l += 64) diff |= col[l] ^ c0;
                if (__ballot(diff != 0) == 0) continue;
                const uint32_t j = kw0 + key_of_row(t0 + rr);
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(&s_nput, 1u);
                at = __shfl(at, 0);
                const uint64_t vi = s_vbase + at;
                const uint64_t off = s_obase + (uint64_t)at * U;
                if (vi < A.var_keys_cap && off + U <= A.var_cap) {
                    if (lane == 0) A.var_keys[vi] = DevVarKey{r, j, off};
                    for (uint32_t l = lane; l < U; l += 64) A.var_counts[off + l] = col[l];
                }
            }
        }
    }
    }();
    }
}

// ---------------------------------------------------------------------------
// key_fast_kernel: the reduction (mode 0) of one region per workgroup with
// every list in LDS.  A distinct haplotype l's count on key j is
//     own(l, j) + [HAP_DEDUP l] * (R(j) - D(l, j))
// (own: its hits, all in windows the scan read; R: the reference hits on j;
// D: those whose window is dirty for l -- the scan read that window of l, so
// its own hits already cover it).  So the region's work is its own hits plus,
// per HAP_DEDUP haplotype, the reference hits inside its few dirty windows
// (found by walking its diff runs over the reference hits sorted by window):
// one "correction" list of (key, l, +1 | -1) entries (in LDS, or for a region
// with many haplotypes a share of a launch-wide arena in global memory), then
// per chunk of touched keys a [key][haplotype] block in LDS that starts at the
// base (R(j) or 0, or the dense count of a LUT/generic slot) and takes the
// corrections with LDS atomics.  A region past the kernel's limits (haplotypes,
// keys, hit lists, reference hits, diff runs, arena) is appended to A.redo and
// left to key_asm_kernel.
#ifndef TFBS_KF_BLOCK
#define TFBS_KF_BLOCK 256
#endif
constexpr uint32_t kFMaxU = 2048;     // distinct haplotypes (11 bits of a correction)
constexpr uint32_t kFKeyWords = 512;  // touched-key bitmap: keys <= 16384
constexpr uint32_t kFBatch = 8;       // hit-list entries each thread has in flight
constexpr uint32_t kFNone = 0xFFFFFFFFu;
// Two shapes of the kernel: the common one (TFBS_KF_BLOCK threads, ~40 KB of LDS,
// four regions per CU) and one for regions of many distinct haplotypes (1 024
// threads and ~154 KB of LDS: a whole CU, counter chunks of 24 Ki u32 -- 17 rows of
// 1 400 haplotypes instead of 2, which sent such a region's counters to the
// global arena).  HAP_LDS: haplotypes whose reuse descriptor sits in LDS (the
// others: read again); COR: corrections in LDS; REFS: reference hits; CNT: u32
// counters of a chunk (rows x U); ROWS: rows (touched keys) per chunk; LISTS: scan
// hit lists staged at a time.
template <int BLOCK, uint32_t HAP_LDS, uint32_t COR, uint32_t REFS, uint32_t CNT, uint32_t ROWS, uint32_t LISTS>
struct KfShape {
    static constexpr int kBlock = BLOCK;
    static constexpr uint32_t kWaves = BLOCK / 64, kHapLds = HAP_LDS, kCor = COR, kRefs = REFS, kCnt = CNT,
                              kRuns = CNT / 2, kRows = ROWS, kLists = LISTS;
    static_assert(kFMaxU % BLOCK == 0 && HAP_LDS % BLOCK == 0 && LISTS <= BLOCK && REFS <= BLOCK,
                  "key_fast_kernel's per-thread shares");
};
constexpr int kFB = TFBS_KF_BLOCK;
#ifdef TFBS_KF_LDS3  // (A/B: the round-4 start's ~51 KB shape, three regions per CU)
using KfSmall = KfShape<kFB, 4 * kFB, 16 * kFB, kFB, 16 * kFB, 2 * kFB, kFB>;
#elif defined(TFBS_KF_LDS6)  // (A/B: ~26 KB, six regions per CU)
using KfSmall = KfShape<kFB, 2 * kFB, 7 * kFB, kFB, 6 * kFB, kFB, kFB / 2>;
#elif defined(TFBS_KF_LDS8)  // (A/B: ~19 KB, eight regions per CU)
using KfSmall = KfShape<kFB, kFB, 4 * kFB, kFB / 2, 4 * kFB, kFB / 2, kFB / 2>;
#else  // ~40 KB: four regions per CU
using KfSmall = KfShape<kFB, 2 * kFB, 14 * kFB, kFB, 12 * kFB, kFB, kFB / 2>;
#endif
using KfBig = KfShape<1024, 2048, 8192, 256, 24576, 1024, 256>;
constexpr uint32_t kFBigU = 384;  // regions of more distinct haplotypes take KfBig

// correction: key << 12 | (-1) << 11 | local haplotype (key < 2^20)
__device__ __forceinline__ uint32_t cor_entry(uint32_t key, uint32_t l, uint32_t neg) {
    return (key << 12) | (neg << 11) | l;
}
__device__ __forceinline__ uint32_t cor_key(uint32_t c) { return c >> 12; }
__device__ __forceinline__ bool cor_neg(uint32_t c) { return (c >> 11) & 1u; }
__device__ __forceinline__ uint32_t cor_hap(uint32_t c) { return c & 2047u; }

// Appends v from the wave's lanes with want set, in lane order (one LDS atomic
// per wave); *n counts every attempt (> cap: overflow).
__device__ __forceinline__ void wave_push(uint32_t *list, uint32_t *n, uint32_t cap, bool want, uint32_t v) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(n, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)leader);
    if (want) {
        const uint32_t at = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (at < cap) list[at] = v;
    }
}

// Exclusive prefix of v over the workgroup (wave scans + the waves' totals in s_w).
template <uint32_t kFWaves>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_w, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kFWaves; w++) {
        const uint32_t t = s_w[w];
        pre += w < wave ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

#ifndef TFBS_KF_WAVES
#define TFBS_KF_WAVES 1
#endif
template <class C>
__global__ __launch_bounds__(C::kBlock) __attribute__((amdgpu_waves_per_eu(C::kBlock == 1024 ? 1 : TFBS_KF_WAVES)))
void key_fast_kernel(AsmArgs A, uint32_t first, uint32_t count, uint32_t which) {
    constexpr int kFBlock = C::kBlock;
    constexpr uint32_t kFWaves = C::kWaves, kFHapLds = C::kHapLds, kFCor = C::kCor, kFRefs = C::kRefs,
                       kFCnt = C::kCnt, kFRuns = C::kRuns, kFRows = C::kRows, kFLists = C::kLists;
    constexpr uint32_t kPerW = kFKeyWords >= (uint32_t)kFBlock ? kFKeyWords / kFBlock : 1u;  // key words per thread
    __shared__ uint32_t s_cor[kFCor];
    __shared__ uint4 s_ref[kFRefs];          // make_ref, sorted by window
    __shared__ uint32_t s_hap[kFHapLds];     // HAP_DEDUP: its first run (from the region's first) | runs << 16; else kFNone
    __shared__ uint32_t s_cnt[kFCnt];        // the counters; before them the diff runs (s_run)
    uint2 *const s_run = reinterpret_cast<uint2 *>(s_cnt);
    __shared__ uint32_t s_bits[kFKeyWords], s_rbase[kFKeyWords];
    __shared__ uint32_t s_rkey[kFRows], s_rr[kFRows];  // per row of a chunk: its key; R(key), then its varying slot
    __shared__ uint32_t s_loff[kFLists + 1], s_lidx[kFLists];
    __shared__ uint32_t s_w[kFWaves];
    __shared__ uint32_t s_ncor, s_nref, s_run0, s_run1, s_nvar, s_arena, s_ndirty, s_lmax;
    __shared__ unsigned long long s_vbase, s_obase;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    auto process = [&](const uint32_t r) {  // one region (every exit is workgroup-uniform)
    // TFBS_KF_PROF: phase times 0-7 (wall_clock64: 100 MHz), then sizes (U, entries, dirty reference hits, rows, chunks)
    auto stamp = [&](uint32_t k, uint64_t v) {
        if (A.prof && tid == 0) A.prof[16 * (size_t)r + k] = v;
    };
    stamp(0, wall_clock64());
    const DevRegion rg = A.regions[r];
    const uint32_t U = rg.hap_count, n_inner = rg.n_inner, K = A.n_slots * n_inner;
    const uint64_t ko = (uint64_t)rg.inner_off * A.n_slots;
    if (U == 0 || K == 0) {  // no samples: no haplotype, no match, no key
        for (uint32_t j = tid; j < K; j += kFBlock) {
            A.key_first[ko + j] = 0;
            A.key_flags[ko + j] = 0;
        }
        return;
    }
    auto give_up = [&](uint32_t why) {  // workgroup-uniform, before any output
        if (tid == 0) {
            A.redo[atomicAdd(A.redo_n, 1u)] = r;
            if (A.why) atomicAdd(A.why + why, 1u);  // (TFBS_DEBUG_OVER: the reasons)
        }
    };
    if (U > (kFMaxU < A.fast_max_u ? kFMaxU : A.fast_max_u) || K > 32 * kFKeyWords || n_inner > 32) return give_up(0);
    const uint32_t hb = rg.hap_begin;
    const bool refs_on = A.mfma && rg.ref_hap != UINT32_MAX;
    if (tid == 0) {
        s_ncor = s_nref = s_run1 = s_ndirty = s_lmax = 0;
        s_run0 = kFNone;
    }
    __syncthreads();
    // descriptors: which haplotypes reuse the reference's windows, and their runs
    constexpr uint32_t kPer = kFMaxU / kFBlock;
    uint32_t roff[kPer], rn[kPer], lmax = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPer; q++) {
        const uint32_t l = tid + q * kFBlock;
        roff[q] = kFNone;
        rn[q] = 0;
        if (l < U) {
            const DevHap &h = A.haps[hb + l];
            lmax = max(lmax, h.len);
            if (h.flags & HAP_DEDUP) {  // its runs in the reference's columns
                roff[q] = h.rrun_off;
                rn[q] = h.n_rruns;
                atomicMin(&s_run0, h.rrun_off);
                atomicMax(&s_run1, h.rrun_off + h.n_rruns);
            }
        }
    }
    // own hits: the scan workgroups' lists over the region's haplotype groups (one
    // hitn load per thread), their entries read flat over the workgroup below
    uint32_t nl = 0;
    const uint32_t g_lo = hb / A.hpb, g_hi = (hb + U - 1) / A.hpb;
    if (A.mfma)
        for (uint32_t si = 0; si < A.n_srcs; si++) {
            const HitSrc src = A.srcs[si];
            const uint32_t ga = max(g_lo, src.g0), gb = min(g_hi + 1, src.g0 + src.ng);
            if (ga < gb) nl += (gb - ga) * src.ns * kMBlockWaves;
        }
    auto list_idx = [&](uint32_t t) -> uint32_t {  // list t of the region's: its wave list (wg x 8 + wave)
        for (uint32_t si = 0; si < A.n_srcs; si++) {
            const HitSrc src = A.srcs[si];
            const uint32_t ga = max(g_lo, src.g0), gb = min(g_hi + 1, src.g0 + src.ng);
            if (ga >= gb) continue;
            const uint32_t per_g = src.ns * kMBlockWaves;
            if (t < (gb - ga) * per_g) {
                const uint32_t g = ga + t / per_g, rem = t % per_g;
                const uint32_t wg = src.wg_base + (g - src.g0) * src.ns + rem / kMBlockWaves;
                return wg * kMBlockWaves + rem % kMBlockWaves;
            }
            t -= (gb - ga) * per_g;
        }
        return 0;
    };
    uint32_t lcnt = 0, lidx = 0;  // the region's entries (an upper bound of its hits: groups are shared)
    for (uint32_t t = tid; t < nl; t += kFBlock) {
        const uint32_t i = list_idx(t);
        if (t == tid) lidx = i;
        lcnt += A.hitn[i];
    }
    uint32_t n_ent = 0;
    const uint32_t loff = block_excl_scan<kFWaves>(lcnt, s_w, n_ent);  // (barriers: s_run0 / s_run1 are final)
    if (tid == 0 && rg.ref_hap != UINT32_MAX) lmax = max(lmax, A.haps[rg.ref_hap].len);  // (R's haplotype)
    if (lmax) atomicMax(&s_lmax, lmax);
    const bool lists_staged = nl <= kFLists;  // one list per thread: its offset and index kept for the list pass
    if (lists_staged && tid < nl) {
        s_lidx[tid] = lidx;
        s_loff[tid] = loff;
    }
    if (lists_staged && tid == 0) s_loff[nl] = n_ent;
    stamp(1, wall_clock64());
    const uint32_t run0 = s_run0, nruns = s_run0 == kFNone ? 0u : s_run1 - s_run0;
    if (nruns >= 65536) return give_up(2);
#pragma unroll
    for (uint32_t q = 0; q < kFHapLds / kFBlock; q++) {
        const uint32_t l = tid + q * kFBlock;
        if (l < U) s_hap[l] = roff[q] == kFNone ? kFNone : (roff[q] - run0) | (rn[q] << 16);
    }
    auto hap_info = [&](uint32_t l) -> uint32_t {  // s_hap's entry of any haplotype
        if (l < kFHapLds) return s_hap[l];
        const DevHap &h = A.haps[hb + l];
        return (h.flags & HAP_DEDUP) ? (h.rrun_off - run0) | (h.n_rruns << 16) : kFNone;
    };
    // the runs in LDS when they fit, else read from global memory (L2)
    const uint2 *const runs = nruns <= kFRuns ? s_run : reinterpret_cast<const uint2 *>(A.druns) + run0;
    if (nruns <= kFRuns)
        for (uint32_t k = tid; k < nruns; k += kFBlock)
            s_run[k] = make_uint2(A.druns[2 * (run0 + k)], A.druns[2 * (run0 + k) + 1]);
    // reference hits: the region's list, then its spill records of kind 1
    const uint2 sp = spill_range(A, r);
    if (refs_on) {
        const uint32_t n = min(A.ref_count[r], kRefPerRegion);
        if (tid < n) {
            const size_t o = 2 * ((size_t)r * kRefPerRegion + tid);
            const uint32_t at = atomicAdd(&s_nref, 1u);
            if (at < kFRefs) s_ref[at] = make_ref(A, rg, A.ref_hits[o], A.ref_hits[o + 1]);
        }
        for (uint32_t e = sp.x + tid; e < sp.y; e += kFBlock) {
            const uint32_t *q = A.spill_sorted + 3 * (size_t)e;
            if (q[0] >> 31) {
                const uint32_t at = atomicAdd(&s_nref, 1u);
                if (at < kFRefs) s_ref[at] = make_ref(A, rg, q[1], q[2]);
            }
        }
    }
    __syncthreads();
    const uint32_t nref = s_nref;
    if (nref > kFRefs) return give_up(3);
    // D: per HAP_DEDUP haplotype the reference hits in its dirty windows (a run
    // [a, b] meets the columns [w, w + L - 1] of window w).  Up to 64 Ki (haplotype,
    // reference hit) pairs are tested pairwise -- a wave's lanes are hpw haplotypes x
    // rpl hits, every run of the lane's haplotype tried (<= 16) -- so the waves share
    // the work and no lane walks a chain of LDS reads; past that the hits are sorted
    // by window and each haplotype walks its runs over them (a hit in [a - 31, b] of
    // run [a, b] tested once: runs ascend, the cursor only moves forward).
    // f(l, ref hit, dirty): in pairwise mode called by every lane of the wave together
    // (uniform = true), else only for dirty pairs.
    const bool pairwise = (uint64_t)U * nref <= 65536;
    if (!pairwise) {  // the reference hits by window (rank sort; ties by list position)
        uint4 mine = make_uint4(0, 0, 0, 0);
        uint32_t rank = 0;
        if (tid < nref) {
            mine = s_ref[tid];
            for (uint32_t j = 0; j < nref; j++) {
                const uint32_t w = s_ref[j].y;
                rank += (w < mine.y || (w == mine.y && j < tid)) ? 1u : 0u;
            }
        }
        __syncthreads();
        if (tid < nref) s_ref[rank] = mine;
        __syncthreads();
    }
    stamp(2, wall_clock64());
    const uint32_t rpl = nref <= 1 ? 1u : nref >= 64 ? 64u : 1u << (32 - __clz(nref - 1));  // hits per lane group
    const uint32_t hpw = 64 / rpl;                                                         // haplotypes per wave
    auto each_dirty = [&](auto &&f) {
        if (!nref) return;
        if (pairwise) {
            for (uint32_t l0 = wave * hpw; l0 < U; l0 += kFWaves * hpw) {
                const uint32_t l = l0 + lane / rpl;
                for (uint32_t p0 = 0; p0 < nref; p0 += rpl) {
                    const uint32_t p = p0 + lane % rpl;
                    uint4 q = make_uint4(0, 0, 0, 0);
                    bool dirty = false;
                    if (l < U && p < nref) {
                        const uint32_t x = hap_info(l);
                        if (x != kFNone) {
                            q = s_ref[p];
                            const uint32_t k0 = x & 0xFFFFu, k1 = k0 + (x >> 16);
                            for (uint32_t k = k0; k < k1 && !dirty; k++)
                                dirty = run_meets(runs[k].x, runs[k].y, q.y, q.z & 0xFFFFu);
                        }
                    }
                    f(l, q, dirty, true);
                }
            }
            return;
        }
        for (uint32_t l = tid; l < U; l += kFBlock) {
            const uint32_t x = hap_info(l);
            if (x == kFNone) continue;
            const uint32_t k0 = x & 0xFFFFu, k1 = k0 + (x >> 16);
            uint32_t p = 0;
            for (uint32_t k = k0; k < k1 && p < nref; k++) {
                const uint32_t a = runs[k].x, b = runs[k].y;
                const uint32_t lo = a >= kMChunkCols * kMMaxChunks - 1 ? a - (kMChunkCols * kMMaxChunks - 1) : 0u;
                while (p < nref && s_ref[p].y < lo) p++;
                for (; p < nref && s_ref[p].y <= b; p++) {
                    const uint4 q = s_ref[p];
                    bool dirty = false;
                    for (uint32_t k2 = k0; k2 < k1 && !dirty; k2++)
                        dirty = run_meets(runs[k2].x, runs[k2].y, q.y, q.z & 0xFFFFu);
                    if (dirty) f(l, q, true, false);
                }
            }
        }
    };
    // the slot of a lane's first of c entries: one counter atomic per wave (an
    // inclusive scan of the lanes' counts) when the wave calls together, else per lane
    auto slots = [&](uint32_t c, bool uniform, uint32_t *ctr) -> uint32_t {
        if (!uniform) return atomicAdd(ctr, c);
        if (!__ballot(c > 1)) {  // (one entry per lane at most: a ballot prefix)
            const uint64_t m = __ballot(c != 0);
            if (!m) return 0;
            const uint32_t leader = (uint32_t)__builtin_ctzll(m);
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
            return (uint32_t)__shfl((int)base, (int)leader) +
                   __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        }
        uint32_t x = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (lane >= (uint32_t)o) x += y;
        }
        const uint32_t tot = (uint32_t)__shfl((int)x, 63);
        uint32_t base = 0;
        if (lane == 0 && tot) base = atomicAdd(ctr, tot);
        return (uint32_t)__shfl((int)base, 0) + x - c;
    };
    // pairwise mode lists the dirty corrections while counting them, at the top of
    // s_cor downwards (the first kFCor); the walk lists them in a second pass
    // (a wave of at most 64 pairwise steps keeps a bit per step and lists its
    // corrections after the pass: one slot reservation for the wave, no atomic per step)
    const uint32_t n_p = (nref + rpl - 1) / rpl;
    const uint32_t n_l0 = U > wave * hpw ? (U - wave * hpw + kFWaves * hpw - 1) / (kFWaves * hpw) : 0u;
    const bool stepbits = pairwise && n_l0 * n_p <= 64;
    uint32_t nd = 0, it = 0;
    uint64_t dm = 0;  // steps whose pair is dirty
    each_dirty([&](uint32_t l, const uint4 &q, bool dirty, bool uniform) {
        const uint32_t c = dirty ? __popc(q.w) : 0u;
        nd += c;
        if (!uniform) return;
        if (stepbits) {
            if (c) dm |= 1ull << it;
            it++;
            return;
        }
        uint32_t at = slots(c, true, &s_ndirty);
        for (uint32_t m = q.w; c && m; m &= m - 1, at++)
            if (at < kFCor) s_cor[kFCor - 1 - at] = cor_entry(q.x + __builtin_ctz(m), l, 1);
    });
    if (stepbits && nref) {
        uint32_t at = slots(nd, true, &s_ndirty);
        for (uint64_t m = dm; m; m &= m - 1) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            const uint32_t l = wave * hpw + (k / n_p) * kFWaves * hpw + lane / rpl;
            const uint4 q = s_ref[(k % n_p) * rpl + lane % rpl];
            for (uint32_t b = q.w; b; b &= b - 1, at++)
                if (at < kFCor) s_cor[kFCor - 1 - at] = cor_entry(q.x + __builtin_ctz(b), l, 1);
        }
    }
    uint32_t nD = 0;
    (void)block_excl_scan<kFWaves>(nd, s_w, nD);
    const bool dirty_listed = pairwise && nD <= kFCor;
    // the corrections' list: LDS when they fit (own hits from the bottom, the dirty
    // ones at the top), else a share of the launch's arena (the dirty ones first)
    const uint32_t need = n_ent + (sp.y - sp.x) + nD;  // (an upper bound: entries of other regions' haplotypes)
    const bool in_lds = need <= (kFCor < A.cor_lds ? kFCor : A.cor_lds);
    if (tid == 0) {
        s_arena = kFNone;
        if (!in_lds) {
            const uint32_t at = atomicAdd(A.cor_used, need);
            if (at <= A.cor_cap && need <= A.cor_cap - at) s_arena = at;
            if (dirty_listed) s_ncor = nD;
        }
    }
    __syncthreads();
    if (!in_lds && s_arena == kFNone) return give_up(4);  // the host grows the arena for the next call
    stamp(3, wall_clock64());
    uint32_t *const cor = in_lds ? s_cor : A.cor_arena + s_arena;
    if (!in_lds && dirty_listed)
        for (uint32_t e = tid; e < nD; e += kFBlock) cor[e] = s_cor[kFCor - 1 - e];
    const uint2 *hitl = reinterpret_cast<const uint2 *>(A.hitl);
    for (uint32_t l0 = 0; l0 < nl; l0 += kFLists) {  // kFLists lists at a time: their offsets in LDS
        const uint32_t nlc = min(kFLists, nl - l0);
        uint32_t tot = n_ent;
        if (!lists_staged) {
            uint32_t lc = 0;
            if (tid < nlc) {
                const uint32_t idx = list_idx(l0 + tid);
                lc = A.hitn[idx];
                s_lidx[tid] = idx;
            }
            const uint32_t off = block_excl_scan<kFWaves>(lc, s_w, tot);
            if (tid < nlc) s_loff[tid] = off;
            if (tid == 0) s_loff[nlc] = tot;
            __syncthreads();
        }
        for (uint32_t e0 = 0; e0 < tot; e0 += kFBlock * kFBatch) {  // kFBatch loads in flight per thread
            uint2 h[kFBatch];
#pragma unroll
            for (uint32_t q = 0; q < kFBatch; q++) {
                const uint32_t e = e0 + q * kFBlock + tid;
                h[q] = make_uint2(hb + U, 0);  // (no entry: not the region's)
                if (e < tot) {
                    uint32_t lo = 0, hi = nlc - 1;  // the list holding entry e: the last with s_loff <= e
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi + 1) / 2;
                        if (s_loff[mid] <= e) lo = mid;
                        else hi = mid - 1;
                    }
                    const uint32_t idx = s_lidx[lo];
                    h[q] = hitl[(size_t)(idx / kMBlockWaves) * A.cand_cap +
                                (size_t)(idx % kMBlockWaves) * (A.cand_cap / kMBlockWaves) + (e - s_loff[lo])];
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < kFBatch; q++)
                wave_push(cor, &s_ncor, need, h[q].x - hb < U, cor_entry(h[q].y, h[q].x - hb, 0));
        }
        __syncthreads();  // s_loff / s_lidx reused by the next lists
    }
    for (uint32_t e0 = sp.x; e0 < sp.y; e0 += kFBlock) {  // own hits of the spill list (kind 0)
        const uint32_t e = e0 + tid;
        bool want = false;
        uint32_t v = 0;
        if (e < sp.y) {
            const uint32_t *q = A.spill_sorted + 3 * (size_t)e;
            want = !(q[0] >> 31) && q[1] - hb < U;
            v = cor_entry(q[2], q[1] - hb, 0);
        }
        wave_push(cor, &s_ncor, need, want, v);
    }
    if (!dirty_listed)
        each_dirty([&](uint32_t l, const uint4 &q, bool dirty, bool uniform) {
            const uint32_t c = dirty ? __popc(q.w) : 0u;
            uint32_t at = slots(c, uniform, &s_ncor);
            for (uint32_t m = q.w; c && m; m &= m - 1, at++)
                if (at < need) cor[at] = cor_entry(q.x + __builtin_ctz(m), l, 1);
        });
    const uint32_t nw = (K + 31) / 32;
    for (uint32_t w = tid; w < nw; w += kFBlock) s_bits[w] = 0;
    __syncthreads();
    stamp(4, wall_clock64());
    // the corrections: [0, nA) and, listed at the top of s_cor, [kFCor - nB, kFCor)
    const uint32_t nA = s_ncor, nB = in_lds && dirty_listed ? nD : 0u, ncor = nA + nB;  // (nA <= need)
    auto cor_at = [&](uint32_t e) -> uint32_t & { return e < nA ? cor[e] : s_cor[kFCor - nB + (e - nA)]; };
    // touched keys: own hits (the dirty reference hits' keys are reference keys),
    // reference hits, every key of a LUT/generic slot; rows in key order
    for (uint32_t e = tid; e < nA; e += kFBlock) {
        const uint32_t c = cor[e];
        if (!cor_neg(c)) atomicOr(&s_bits[cor_key(c) >> 5], 1u << (cor_key(c) & 31u));
    }
    if (tid < nref)
        for (uint32_t m = s_ref[tid].w; m; m &= m - 1) {
            const uint32_t key = s_ref[tid].x + __builtin_ctz(m);
            atomicOr(&s_bits[key >> 5], 1u << (key & 31u));
        }
    if (A.any_dense)
        for (uint32_t j = tid; j < K; j += kFBlock)
            if (!A.slot_mfma[j / n_inner]) atomicOr(&s_bits[j >> 5], 1u << (j & 31u));
    __syncthreads();
    uint32_t T = 0;
    {
        constexpr uint32_t per = kPerW;
        uint32_t mine = 0;
#pragma unroll
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nw) mine += __popc(s_bits[w]);
        }
        uint32_t run = block_excl_scan<kFWaves>(mine, s_w, T);
#pragma unroll
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t w = tid * per + q;
            if (w < nw) {
                s_rbase[w] = run;
                run += __popc(s_bits[w]);
            }
        }
    }
    stamp(5, wall_clock64());
    auto row_of = [&](uint32_t j) { return s_rbase[j >> 5] + __popc(s_bits[j >> 5] & ((1u << (j & 31)) - 1u)); };
    // the counter block: LDS chunks of rows x U, or -- when that would take more than
    // 32 chunks (hundreds of haplotypes and keys: each chunk re-reads every
    // correction and costs a few barriers) -- chunks of kFRows rows in a share of
    // the arena (global atomics)
    // u16 counters in LDS (two per word) when no count can reach 2^16, also while the
    // corrections land: a key's count on a haplotype is at most its 2 strands'
    // windows (< 2 x length), but the unordered atomics can add every +1 (own hits,
    // < 2 x length) to the base R (< 2 x length) before any -1, so the bound is
    // 4 x length; the -1 corrections never take a count below 0 (a haplotype's
    // dirty reference hits on a key are some of its base R), so a packed pair
    // never borrows or carries
    const bool half = 4 * (s_lmax + 64) < 65536 && A.cor_lds != 0;
    uint32_t rows_per = min((half ? 2 : 1) * kFCnt / U, kFRows);
    uint32_t *cnt = s_cnt;
    uint16_t *const cnt16 = reinterpret_cast<uint16_t *>(s_cnt);
    bool h16 = half;
    if ((T + rows_per - 1) / rows_per > 32 || A.cor_lds == 0) {  // (cor_lds 0: the tests' all-global path)
        h16 = false;
        rows_per = min(T, kFRows);
        if (tid == 0) {
            s_arena = kFNone;
            const uint32_t want = rows_per * U, at = atomicAdd(A.cor_used, want);
            if (at <= A.cor_cap && want <= A.cor_cap - at) s_arena = at;
        }
        __syncthreads();
        if (s_arena == kFNone) return give_up(5);  // the host grows the arena for the next call
        cnt = A.cor_arena + s_arena;
    }
    // untouched keys: no match -- no key in the reference's HashMap
    for (uint32_t j = tid; j < K; j += kFBlock)
        if (!((s_bits[j >> 5] >> (j & 31)) & 1u)) {
            A.key_first[ko + j] = 0;
            A.key_flags[ko + j] = 0;
        }
    const uint64_t dense_base = A.dense_base ? A.haps[hb].count_off : 0;
    // the corrections by row (key << 12 becomes row << 12: no row_of per chunk)
    for (uint32_t e = tid; e < ncor; e += kFBlock) {
        uint32_t &c = cor_at(e);
        c = (row_of(cor_key(c)) << 12) | (c & 4095u);
    }
    uint32_t dedup_bits = 0;  // bit i: haplotype lane + 64 i takes the reference's counts as its base
    for (uint32_t i = 0, l = lane; l < U; i++, l += 64)
        if (hap_info(l) != kFNone) dedup_bits |= 1u << i;
    uint64_t t_atomics = 0;  // (TFBS_KF_PROF)
    for (uint32_t t0 = 0; t0 < T; t0 += rows_per) {
        const uint32_t nrow = min(rows_per, T - t0);
        __syncthreads();  // s_rbase / cor rows written, the previous chunk's readers done
        if (tid == 0) s_nvar = 0;
        {  // each row's key, from the key words this thread scanned (rows [s_rbase[w], ..))
            constexpr uint32_t per = kPerW;
#pragma unroll
            for (uint32_t q = 0; q < per; q++) {
                const uint32_t w = tid * per + q;
                if (w >= nw) continue;
                uint32_t t = s_rbase[w], b = s_bits[w];
                if (t >= t0 + nrow || t + __popc(b) <= t0) continue;
                for (; b; b &= b - 1, t++)
                    if (t - t0 < nrow) s_rkey[t - t0] = 32 * w + __builtin_ctz(b);
            }
        }
        for (uint32_t rr = tid; rr < nrow; rr += kFBlock) s_rr[rr] = 0;
        __syncthreads();
        if (tid < nref)  // R: reference hits per key
            for (uint32_t m = s_ref[tid].w; m; m &= m - 1) {
                const uint32_t t = row_of(s_ref[tid].x + __builtin_ctz(m)) - t0;
                if (t < nrow) atomicAdd(&s_rr[t], 1u);
            }
        __syncthreads();
        for (uint32_t rr = wave; rr < nrow; rr += kFWaves) {  // the base of every haplotype
            const uint32_t j = s_rkey[rr], R = s_rr[rr];
            const bool dense = A.any_dense && !A.slot_mfma[j / n_inner];
            for (uint32_t i = 0, l = lane; l < U; i++, l += 64) {
                const uint32_t v = dense ? A.counts[dense_base + (uint64_t)j * rg.count_stride + l]
                                         : ((dedup_bits >> i) & 1u ? R : 0u);
                if (h16) cnt16[rr * U + l] = (uint16_t)v;
                else cnt[rr * U + l] = v;
            }
        }
        __syncthreads();
        for (uint32_t e = tid; e < ncor; e += kFBlock) {
            const uint32_t c = cor_at(e);
            const uint32_t t = cor_key(c) - t0;  // (its row)
            if (t < nrow) {
                const uint32_t x = t * U + cor_hap(c);
                if (h16) atomicAdd(&cnt[x >> 1], (cor_neg(c) ? 0xFFFFFFFFu : 1u) << (16 * (x & 1u)));
                else atomicAdd(&cnt[x], cor_neg(c) ? 0xFFFFFFFFu : 1u);
            }
        }
        __syncthreads();
        auto count_at = [&](uint32_t x) -> uint32_t { return h16 ? (uint32_t)cnt16[x] : cnt[x]; };
        // classify: one wave per row
        for (uint32_t rr = wave; rr < nrow; rr += kFWaves) {
            const uint32_t c0 = count_at(rr * U);
            uint32_t any = 0, diff = 0;
            for (uint32_t l = lane; l < U; l += 64) {
                const uint32_t c = count_at(rr * U + l);
                any |= c;
                diff |= c ^ c0;
            }
            const bool a = __ballot(any != 0) != 0, v = __ballot(diff != 0) != 0;
            if (lane == 0) {
                const uint32_t j = s_rkey[rr];
                A.key_first[ko + j] = c0;
                A.key_flags[ko + j] = (uint8_t)((a ? KEY_ANY : 0) | (v ? KEY_VARIES : 0));
                s_rr[rr] = v ? atomicAdd(&s_nvar, 1u) : kFNone;
            }
        }
        __syncthreads();
        const uint64_t ta = A.prof ? wall_clock64() : 0;
        if (tid == 0 && s_nvar) {  // the chunk's share of the compact lists
            s_vbase = atomicAdd(A.var_tot, (unsigned long long)s_nvar);
            s_obase = atomicAdd(A.var_tot + 1, (unsigned long long)s_nvar * U);
        }
        __syncthreads();
        if (A.prof) t_atomics += wall_clock64() - ta;
        for (uint32_t rr = wave; rr < nrow; rr += kFWaves) {
            const uint32_t slot = s_rr[rr];
            if (slot == kFNone) continue;
            const uint64_t vi = s_vbase + slot, off = s_obase + (uint64_t)slot * U;
            if (vi >= A.var_keys_cap || off + U > A.var_cap) continue;  // the host grows the lists and reruns
            if (lane == 0) A.var_keys[vi] = DevVarKey{r, s_rkey[rr], off};
            for (uint32_t l = lane; l < U; l += 64) A.var_counts[off + l] = count_at(rr * U + l);
        }
    }
    stamp(6, wall_clock64());
    stamp(7, t_atomics);
    stamp(8, U);
    stamp(9, n_ent);
    stamp(10, nD);
    stamp(11, ncor);
    stamp(12, T);
    stamp(13, (T + rows_per - 1) / rows_per);
    stamp(14, blockIdx.x | (which << 24));  // (the workgroup: its timeline in the report)
    stamp(15, nref);
    };
    // regions [first, first + count) in A.order's order (most haplotypes first): with
    // A.persist a grid of a few workgroups per CU takes them -- its first region by
    // workgroup index, the next ones from the counter A.next[which] (gridDim.x + ticket),
    // the ticket for the next region taken as this one starts, so that its latency hides
    // behind the region's first loads --, else one per workgroup.  A grid with one
    // workgroup per region takes no ticket (1 000 tickets at once cost microseconds).
    __shared__ uint32_t s_tk;
    const bool tickets = A.persist && gridDim.x < count;
    uint32_t i = blockIdx.x;
    while (i < count) {
        uint32_t tk = 0;
        if (tickets && tid == 0) tk = gridDim.x + atomicAdd(A.next + which, 1u);
        process(A.order ? A.order[first + i] : first + i);
        if (!tickets) break;
        if (tid == 0) s_tk = tk;
        __syncthreads();
        i = s_tk;
        __syncthreads();
    }
}

// Spill bucketing: per-region record counts, their exclusive scan (one
// workgroup), and the scatter into region order.
__global__ __launch_bounds__(256) void spill_hist_kernel(const uint32_t *__restrict__ over, uint32_t cap,
                                                          const uint32_t *__restrict__ spill, uint32_t *__restrict__ bcnt) {
    const uint32_t n = min(over[0], cap);
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256)
        atomicAdd(&bcnt[spill[3 * (size_t)e] & 0x7FFFFFFFu], 1u);
}

__global__ __launch_bounds__(1024) void spill_scan_kernel(const uint32_t *__restrict__ over, uint32_t *__restrict__ bcnt,
                                                          uint32_t n, uint32_t *__restrict__ boff) {
    __shared__ uint32_t s[1024];
    if (over[0] == 0) return;  // no records: the readers skip the buckets (AsmArgs::spill_count)
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < n ? bcnt[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
            const uint32_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n) {
            boff[i] = carry + s[threadIdx.x] - v;
            bcnt[i] = 0;  // the scatter's fill counters
        }
        carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) boff[n] = carry;
}

__global__ __launch_bounds__(256) void spill_scatter_kernel(const uint32_t *__restrict__ over, uint32_t cap,
                                                            const uint32_t *__restrict__ spill,
                                                            const uint32_t *__restrict__ boff,
                                                            uint32_t *__restrict__ bfill, uint32_t *__restrict__ out) {
    const uint32_t n = min(over[0], cap);
    for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const uint32_t r = spill[3 * (size_t)e] & 0x7FFFFFFFu;
        const uint32_t at = boff[r] + atomicAdd(&bfill[r], 1u);
        out[3 * (size_t)at] = spill[3 * (size_t)e];
        out[3 * (size_t)at + 1] = spill[3 * (size_t)e + 1];
        out[3 * (size_t)at + 2] = spill[3 * (size_t)e + 2];
    }
}

// A region's distinct (left, right) haplotype pairs: sample s carries distinct
// haplotypes (a, b) = (memb[2 s], memb[2 s + 1]) of its u16 membership row.  The
// pairs (key a | b << 16) go into an LDS hash table with their sample counts
// (one insert per wave for the lanes sharing lane 0's pair, which is most of
// them: the reference group on both sides), are listed at r * kEncMaxPairs of
// pab / pcnt in table order, and each sample gets its pair's index in pidx.
// More than kEncMaxPairs pairs: pair_n[r] = UINT32_MAX (the host path).
constexpr int kPairBlock = 512;
constexpr uint32_t kPairSlots = 2 * kEncMaxPairs;
constexpr uint32_t kPairEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t pair_slot(uint32_t key) { return (key * 0x9E3779B1u) >> (32 - 14); }
static_assert(kPairSlots == 1u << 14, "pair_slot hashes into 2^14 slots");

__global__ __launch_bounds__(kPairBlock) void pair_table_kernel(const uint64_t *__restrict__ rows, uint32_t n_samples,
                                                                uint32_t *__restrict__ pab, uint32_t *__restrict__ pcnt,
                                                                uint32_t *__restrict__ pair_n,
                                                                uint16_t *__restrict__ pidx) {
    __shared__ uint32_t s_key[kPairSlots];
    __shared__ uint32_t s_val[kPairSlots];  // sample counts, then the pairs' indices
    __shared__ uint32_t s_n, s_over, s_pos;
    const uint32_t r = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const uint16_t *m = reinterpret_cast<const uint16_t *>(rows[r]);
    if (!m) {
        if (tid == 0) pair_n[r] = kPairEmpty;
        return;
    }
    for (uint32_t t = tid; t < kPairSlots; t += kPairBlock) {
        s_key[t] = kPairEmpty;
        s_val[t] = 0;
    }
    if (tid == 0) {
        s_n = 0;
        s_over = 0;
        s_pos = 0;
    }
    __syncthreads();
    auto insert = [&](uint32_t key, uint32_t add) {
        uint32_t sl = pair_slot(key);
        while (!*(volatile uint32_t *)&s_over) {
            const uint32_t old = atomicCAS(&s_key[sl], kPairEmpty, key);
            if (old == kPairEmpty && atomicAdd(&s_n, 1u) >= kEncMaxPairs) atomicOr(&s_over, 1u);
            if (old == kPairEmpty || old == key) {
                atomicAdd(&s_val[sl], add);
                return;
            }
            sl = (sl + 1) & (kPairSlots - 1);
        }
    };
    for (uint32_t s0 = 0; s0 < n_samples; s0 += kPairBlock) {
        const uint32_t s = s0 + tid;
        const bool valid = s < n_samples;
        const uint32_t key = valid ? (uint32_t)m[2 * s] | ((uint32_t)m[2 * s + 1] << 16) : kPairEmpty;
        const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
        const unsigned long long same = __ballot(valid && key == k0);
        if (valid && key == k0) {
            if (lane == (uint32_t)__builtin_ctzll(same)) insert(k0, (uint32_t)__popcll(same));
        } else if (valid) {
            insert(key, 1u);
        }
    }
    __syncthreads();
    if (s_over) {
        if (tid == 0) pair_n[r] = kPairEmpty;
        return;
    }
    const size_t p0 = (size_t)r * kEncMaxPairs;
    for (uint32_t t = tid; t < kPairSlots; t += kPairBlock)
        if (s_key[t] != kPairEmpty) {
            const uint32_t i = atomicAdd(&s_pos, 1u);
            pab[p0 + i] = s_key[t];
            pcnt[p0 + i] = s_val[t];
            s_val[t] = i;
        }
    __syncthreads();
    uint16_t *out = pidx + (size_t)r * n_samples;
    for (uint32_t s = tid; s < n_samples; s += kPairBlock) {
        const uint32_t key = (uint32_t)m[2 * s] | ((uint32_t)m[2 * s + 1] << 16);
        uint32_t sl = pair_slot(key);
        while (s_key[sl] != key) sl = (sl + 1) & (kPairSlots - 1);
        out[s] = (uint16_t)s_val[sl];
    }
    if (tid == 0) pair_n[r] = s_n;
}

// counts_as_genotypes' per-sample half (main.rs:439-498) for one varying key.
// A sample's total is C[a] + C[b] for its two haplotypes' distinct indices (a,
// b); pair_table_kernel lists each region's distinct (a, b) pairs with their
// sample counts and gives every sample its pair index, so the key's totals, min
// / max, distinct values (a bitmap of hi - lo + 1 bits), their ranks and sample
// counts are computed over the P pairs, not the N samples (no per-sample
// atomics); the one per-sample pass packs code[pair[s]].  The range
// multiplicity and the text stay on the host, which formats a row from the
// value table and the codes (aggregate.cpp).
constexpr int kEncBlock = 256;
constexpr uint32_t kEncWords = kEncMaxRange / 32;
constexpr uint32_t kEncWordsPerThread = kEncWords / kEncBlock;  // the rank scan's share of the bitmap

__global__ __launch_bounds__(kEncBlock) void key_encode_kernel(const uint32_t *__restrict__ var_counts,
                                                                 const DevVarKey *__restrict__ keys,
                                                                 const uint32_t *__restrict__ pab,
                                                                 const uint32_t *__restrict__ pcnt,
                                                                 const uint32_t *__restrict__ pair_n,
                                                                 const uint16_t *__restrict__ pidx, uint32_t region0,
                                                                 uint32_t n_samples, EncHdr *__restrict__ hdr,
                                                                 uint32_t *__restrict__ vals,
                                                                 uint32_t *__restrict__ hist,
                                                                 uint8_t *__restrict__ codes) {
    __shared__ uint32_t s_v[kEncMaxPairs];   // the pairs' totals, then their codes
    __shared__ uint32_t s_bits[kEncWords];
    __shared__ uint16_t s_rank[kEncWords];   // distinct values in the words before
    __shared__ uint32_t s_hist[kEncMaxVals + 1];
    __shared__ uint32_t s_red[2 * kEncBlock / 64];
    __shared__ uint32_t s_tsum[kEncBlock];
    const uint32_t k = blockIdx.x, tid = threadIdx.x;
    const DevVarKey vk = keys[k];
    const uint32_t r = vk.region - region0;
    const size_t p0 = (size_t)r * kEncMaxPairs;
    const uint32_t P = pair_n[r];
    // each pair's total (u32 wrapping, as the reference's additions) from the key's
    // distinct-haplotype counts (a region's U counts, cache-resident); the host
    // sends only keys of regions with <= kEncMaxPairs pairs
    const uint32_t *cnt = var_counts + vk.out_off;
    uint32_t lo = UINT32_MAX, hi = 0;
    {
        for (uint32_t p = tid; p < P; p += kEncBlock) {
            const uint32_t ab = pab[p0 + p];
            const uint32_t v = cnt[ab & 0xFFFFu] + cnt[ab >> 16];
            s_v[p] = v;
            if (pcnt[p0 + p] == 0) continue;  // the reference group's pair when every sample carries a variant
            lo = min(lo, v);
            hi = max(hi, v);
        }
    }
    for (int o = 32; o; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    const uint32_t wave = tid >> 6;
    if ((tid & 63) == 0) {
        s_red[wave] = lo;
        s_red[kEncBlock / 64 + wave] = hi;
    }
    for (uint32_t w = tid; w < kEncWords; w += kEncBlock) s_bits[w] = 0;
    for (uint32_t i = tid; i <= kEncMaxVals; i += kEncBlock) s_hist[i] = 0;
    __syncthreads();
    lo = s_red[0];
    hi = s_red[kEncBlock / 64];
    for (int w = 1; w < kEncBlock / 64; w++) {
        lo = min(lo, s_red[w]);
        hi = max(hi, s_red[kEncBlock / 64 + w]);
    }
    if (hi - lo >= kEncMaxRange) {
        if (tid == 0) hdr[k] = EncHdr{lo, hi, 0, 1, 0};
        return;
    }
    // which totals occur: one bit per pair (P LDS ORs, not N)
    for (uint32_t p = tid; p < P; p += kEncBlock) {
        if (pcnt[p0 + p] == 0) continue;
        const uint32_t d = s_v[p] - lo;
        atomicOr(&s_bits[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    // ranks: each thread's words summed, a block scan of the sums, the words' prefixes
    const uint32_t nw = (hi - lo) / 32 + 1;
    uint32_t mine = 0;
    for (uint32_t q = 0; q < kEncWordsPerThread; q++) {
        const uint32_t w = tid * kEncWordsPerThread + q;
        if (w < nw) mine += __popc(s_bits[w]);
    }
    s_tsum[tid] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < kEncBlock; o <<= 1) {
        const uint32_t t = tid >= o ? s_tsum[tid - o] : 0;
        __syncthreads();
        s_tsum[tid] += t;
        __syncthreads();
    }
    {
        uint32_t run = s_tsum[tid] - mine;
        for (uint32_t q = 0; q < kEncWordsPerThread; q++) {
            const uint32_t w = tid * kEncWordsPerThread + q;
            if (w < nw) {
                s_rank[w] = (uint16_t)min(run, 0xFFFFu);
                run += __popc(s_bits[w]);
            }
        }
    }
    const uint32_t nv = s_tsum[kEncBlock - 1];
    __syncthreads();
    if (nv > kEncMaxVals) {
        if (tid == 0) hdr[k] = EncHdr{lo, hi, nv, 1, 0};
        return;
    }
    for (uint32_t w = tid; w < nw; w += kEncBlock) {  // the sorted value table
        uint32_t b = s_bits[w], rk = s_rank[w];
        while (b) {
            const uint32_t t = __ffs(b) - 1;
            b &= b - 1;
            vals[(size_t)k * (kEncMaxVals + 1) + rk++] = lo + 32 * w + t;
        }
    }
    // each pair's code and its samples into the histogram (P LDS adds)
    for (uint32_t p = tid; p < P; p += kEncBlock) {
        const uint32_t n = pcnt[p0 + p];
        if (n == 0) {  // no sample has this pair: no code (its total may lie outside [lo, hi])
            s_v[p] = 0;
            continue;
        }
        const uint32_t d = s_v[p] - lo, w = d >> 5;
        const uint32_t c = s_rank[w] + __popc(s_bits[w] & ((1u << (d & 31)) - 1u));
        s_v[p] = c;
        atomicAdd(&s_hist[c], n);
    }
    __syncthreads();
    // the per-sample pass: code[pair[s]] packed (each thread writes whole bytes)
    const uint32_t width = nv <= 4 ? 2 : (nv <= 16 ? 4 : 8), per = 8 / width;
    uint8_t *out = codes + (size_t)k * n_samples;
    const uint16_t *pi = pidx + (size_t)r * n_samples;
    const uint32_t nbytes = (n_samples + per - 1) / per;
    for (uint32_t byte = tid; byte < nbytes; byte += kEncBlock) {
        uint32_t packed = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t smp = byte * per + q;
            if (smp >= n_samples) break;
            packed |= s_v[pi[smp]] << (q * width);
        }
        out[byte] = (uint8_t)packed;
    }
    for (uint32_t i = tid; i < nv; i += kEncBlock) hist[(size_t)k * (kEncMaxVals + 1) + i] = s_hist[i];
    if (tid == 0) hdr[k] = EncHdr{lo, hi, nv, 0, width};
}

// Membership rows of host-built regions from their non-reference lists: row k
// (Hp u16 at k * Hp) is the region's reference group everywhere (meta[2k + 1]),
// then its entries [meta[2k], meta[2k + 2]) of ids / loc scattered over it.
__global__ __launch_bounds__(256) void memb_fill_kernel(const uint32_t *__restrict__ meta, const uint32_t *__restrict__ ids,
                                                        const uint16_t *__restrict__ loc, uint32_t Hp,
                                                        uint16_t *__restrict__ memb) {
    const uint32_t k = blockIdx.x;
    const uint32_t o0 = meta[2 * k], o1 = meta[2 * k + 2], ref = meta[2 * k + 1] & 0xFFFFu;
    uint16_t *row = memb + (size_t)k * Hp;
    const uint32_t v = ref | (ref << 16);
    for (uint32_t i = threadIdx.x; i < Hp / 8; i += 256) reinterpret_cast<uint4 *>(row)[i] = uint4{v, v, v, v};
    __syncthreads();
    for (uint32_t i = o0 + threadIdx.x; i < o1; i += 256) row[ids[i]] = loc[i];
}

// Copies each key's packed codes (at k * n_samples) to off[k] of a contiguous buffer.
__global__ __launch_bounds__(256) void code_compact_kernel(const uint8_t *__restrict__ codes, uint32_t n_samples,
                                                           const uint64_t *__restrict__ off, uint8_t *__restrict__ dst) {
    const uint32_t k = blockIdx.x;
    const uint64_t o = off[k], n = off[k + 1] - o;
    const uint8_t *src = codes + (size_t)k * n_samples;
    for (uint64_t i = threadIdx.x; i < n; i += 256) dst[o + i] = src[i];
}

// Each key's n_vals value-table entries and histogram counts (of kEncMaxVals + 1
// slots) back to back at off[k].
__global__ __launch_bounds__(64) void val_compact_kernel(const uint32_t *__restrict__ vals,
                                                         const uint32_t *__restrict__ hist,
                                                         const uint32_t *__restrict__ off, uint32_t *__restrict__ ov,
                                                         uint32_t *__restrict__ oh) {
    const uint32_t k = blockIdx.x, o = off[k], n = off[k + 1] - o;
    for (uint32_t i = threadIdx.x; i < n; i += 64) {
        ov[o + i] = vals[(size_t)k * (kEncMaxVals + 1) + i];
        oh[o + i] = hist[(size_t)k * (kEncMaxVals + 1) + i];
    }
}

}  // namespace

int launch_val_compact(const uint32_t *vals, const uint32_t *hist, uint32_t n_keys, const uint32_t *off, uint32_t *ov,
                       uint32_t *oh, hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(val_compact_kernel, dim3(n_keys), dim3(64), 0, stream, vals, hist, off, ov, oh);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("val_compact_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_memb_fill(const uint32_t *meta, const uint32_t *ids, const uint16_t *loc, uint32_t n_rows, uint32_t Hp,
                     uint16_t *memb, hipStream_t stream) {
    if (n_rows == 0) return TFBS_OK;
    hipLaunchKernelGGL(memb_fill_kernel, dim3(n_rows), dim3(256), 0, stream, meta, ids, loc, Hp, memb);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("memb_fill_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_pair_table(const uint64_t *rows, uint32_t n_regions, uint32_t n_samples, uint32_t *pab, uint32_t *pcnt,
                      uint32_t *pair_n, uint16_t *pidx, hipStream_t stream) {
    if (n_regions == 0) return TFBS_OK;
    hipLaunchKernelGGL(pair_table_kernel, dim3(n_regions), dim3(kPairBlock), 0, stream, rows, n_samples, pab, pcnt,
                       pair_n, pidx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("pair_table_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_key_encode(const uint32_t *var_counts, const DevVarKey *keys, uint32_t n_keys, const uint32_t *pab,
                      const uint32_t *pcnt, const uint32_t *pair_n, const uint16_t *pidx, uint32_t region0,
                      uint32_t n_samples, EncHdr *hdr, uint32_t *vals, uint32_t *hist, uint8_t *codes,
                      hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(key_encode_kernel, dim3(n_keys), dim3(kEncBlock), 0, stream, var_counts, keys, pab, pcnt,
                       pair_n, pidx, region0, n_samples, hdr, vals, hist, codes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_encode_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_code_compact(const uint8_t *codes, uint32_t n_keys, uint32_t n_samples, const uint64_t *off, uint8_t *dst,
                        hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(code_compact_kernel, dim3(n_keys), dim3(256), 0, stream, codes, n_samples, off, dst);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("code_compact_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_spill_buckets(const uint32_t *over, uint32_t cap, const uint32_t *spill, uint32_t n_regions, uint32_t *bcnt,
                         uint32_t *boff, uint32_t *sorted, hipStream_t stream, bool bcnt_zeroed) {
    hipError_t e = bcnt_zeroed ? hipSuccess : hipMemsetAsync(bcnt, 0, (size_t)(n_regions + 1) * 4, stream);
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("spill bucket memset: ") + hipGetErrorString(e));
    hipLaunchKernelGGL(spill_hist_kernel, dim3(64), dim3(256), 0, stream, over, cap, spill, bcnt);
    hipLaunchKernelGGL(spill_scan_kernel, dim3(1), dim3(1024), 0, stream, over, bcnt, n_regions, boff);
    hipLaunchKernelGGL(spill_scatter_kernel, dim3(64), dim3(256), 0, stream, over, cap, spill, boff, bcnt, sorted);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("spill bucket kernels: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_key_asm(const AsmArgs &a, uint32_t n_regions, hipStream_t stream) {
    if (n_regions == 0) return TFBS_OK;
    hipLaunchKernelGGL(key_asm_kernel, dim3(n_regions), dim3(kAsmBlock), 0, stream, a, (const uint32_t *)nullptr,
                       (const uint32_t *)nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_asm_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

static size_t key_fast_lds_bytes(bool big) {
    hipFuncAttributes fa{};
    const hipError_t e = big ? hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(key_fast_kernel<KfBig>))
                             : hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(key_fast_kernel<KfSmall>));
    return e == hipSuccess ? fa.sharedSizeBytes : 0;
}

int launch_key_fast(const AsmArgs &a, uint32_t n_regions, uint32_t n_big, hipStream_t stream, hipStream_t side,
                    hipEvent_t fork, hipEvent_t join, bool leftover) {
    if (n_regions == 0) return TFBS_OK;
    if (!a.order || !side) n_big = 0;
    n_big = std::min(n_big, n_regions);
    // persistent grids (a.persist): the workgroups of each shape that fit the device at
    // once, queried once per device (the calling thread's current device: the ctx's),
    // thread-safe for contexts on several threads
    struct Fit {
        int n_cu = 256, per_small = 2, per_big = 1;
    };
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static Fit fits[kMaxDev];
    int dev = 0;
    (void)hipGetDevice(&dev);
    dev = std::min(std::max(dev, 0), kMaxDev - 1);
    std::call_once(once[dev], [dev] {
        Fit &f = fits[dev];
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) f.n_cu = v;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, key_fast_kernel<KfSmall>, KfSmall::kBlock, 0) ==
                hipSuccess && v > 0)
            f.per_small = v;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, key_fast_kernel<KfBig>, KfBig::kBlock, 0) == hipSuccess &&
            v > 0)
            f.per_big = v;
        (void)hipGetLastError();
        if (getenv("TFBS_KF_PROF"))
            fprintf(stderr, "[kf prof] device %d: CUs %d, workgroups per CU: %d (%d threads, %zu B LDS), %d (%d threads, %zu B LDS)\n",
                    dev, f.n_cu, f.per_small, KfSmall::kBlock, key_fast_lds_bytes(false), f.per_big, KfBig::kBlock,
                    key_fast_lds_bytes(true));
    });
    const Fit &fit = fits[dev];
    const int n_cu = fit.n_cu, per_small = fit.per_small, per_big = fit.per_big;
    auto grid = [&](uint32_t n, int per) { return a.persist ? std::min<uint32_t>(n, (uint32_t)(n_cu * per)) : n; };
    hipError_t e = hipSuccess;
    // two shapes at once: the regions of many haplotypes (order[0, n_big), whole-CU
    // workgroups) go first on `stream` -- queued ahead, they take their CUs before the
    // others fill every CU -- and the rest on `side`, forked before and joined after
    const bool two = n_big && n_regions > n_big;
    if (two) {
        if ((e = hipEventRecord(fork, stream)) == hipSuccess) e = hipStreamWaitEvent(side, fork, 0);
        if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_fast_kernel fork: ") + hipGetErrorString(e));
    }
    if (n_big)
        hipLaunchKernelGGL(key_fast_kernel<KfBig>, dim3(grid(n_big, per_big)), dim3(KfBig::kBlock), 0, stream, a, 0u,
                           n_big, 1u);
    if (n_regions > n_big)
        hipLaunchKernelGGL(key_fast_kernel<KfSmall>, dim3(grid(n_regions - n_big, per_small)), dim3(KfSmall::kBlock), 0,
                           two ? side : stream, a, n_big, n_regions - n_big, 0u);
    if (two) {
        if ((e = hipEventRecord(join, side)) == hipSuccess) e = hipStreamWaitEvent(stream, join, 0);
        if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_fast_kernel join: ") + hipGetErrorString(e));
    }
    // the regions it left: a fixed grid over the list (no host round trip)
    if (leftover)
        hipLaunchKernelGGL(key_asm_kernel, dim3(std::min<uint32_t>(n_regions, 256)), dim3(kAsmBlock), 0, stream, a,
                           (const uint32_t *)a.redo, (const uint32_t *)a.redo_n);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_fast_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

__global__ void asm_report_kernel(const uint32_t *__restrict__ over, uint32_t *__restrict__ ctr) {
    if (threadIdx.x < 2) ctr[threadIdx.x] = over ? over[threadIdx.x] : 0u;
}

int launch_asm_report(const uint32_t *over, uint32_t *ctr, hipStream_t stream) {
    hipLaunchKernelGGL(asm_report_kernel, dim3(1), dim3(64), 0, stream, over, ctr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("asm_report_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

uint32_t key_asm_lds_counters() { return kAsmCounters; }
uint32_t key_fast_big_u() { return kFBigU; }

}  // namespace tfbs
