// Launch interface of the scan kernels (scan_kernels.hip), used by device.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "tfbs_internal.hpp"

namespace tfbs {

// Everything a scan launch reads or writes (device pointers).
struct ScanArgs {
    const DevTile *tiles;
    uint32_t n_tiles;
    const DevUnit *units;       // fast path: units; generic path: unused
    const DevPattern *gpats;    // generic path
    const int32_t *lut;         // fast path: 4 KiB table blocks
    const int32_t *wfull;       // fast path: [A,C,G,T] per column (windows containing N)
    const int32_t *gw;          // generic path: 5 weights per column
    const DevHap *haps;
    uint32_t n_haps;
    uint32_t hap_base;          // batch index of haps[0] (a launch over a later part of the batch)
    const DevRegion *regions;
    const int32_t *inner;
    const uint32_t *words;
    const uint32_t *nmask;
    const int32_t *posrel;
    // dense counts [count_off + key * count_stride] of the slots the LUT and generic
    // kernels score (stores); nullptr when every slot is on the matrix cores
    uint32_t *counts;
    uint32_t haps_per_block;
    const DevMSuper *msupers;   // matrix-core path
    uint32_t n_msupers;
    const int32_t *mimage;
    const int32_t *mweights;    // exact weights of the matrix-core strands
    const int32_t *mmeta;       // their per-tile rescoring fields
    uint32_t mimg_max;          // LDS bytes reserved for the largest super tile image
    unsigned long long *hits;   // debug (tfbs_matches): per (hap, pattern, 64-window chunk) hit masks
    uint32_t hits_wpp;
    uint32_t n_patterns_total;
    // matrix-core candidates (scan_mfma.hip): one region of cand_cap (strand |
    // haplotype in the group << 24, window) pairs per scan workgroup (region
    // region_base + blockIdx.x), an equal share per wave, each wave's filled and
    // rescored by the wave
    uint32_t *cands;  // kCandWords per entry
    uint32_t cand_cap;
    uint32_t region_base;
    // matrix-core hits, sparse (no count matrix, no atomics): the wave that
    // rescores its candidates appends one (haplotype, key = slot * n_inner +
    // range) pair per hit and overlapped inner range to its part of the
    // workgroup's hit list (hitl + 2 (wg cand_cap + wave cand_cap / 8), the same
    // geometry as the candidate list) and stores their number at hitn[8 wg +
    // wave]; the excess goes to the spill list
    uint32_t *hitl;
    uint32_t *hitn;
    uint32_t *candn;  // per wave (as hitn): the candidates it found (tfbs_ctx_scan_counters; no atomics)
    // matrix-core window lists (build_window_lists), per depth class (2, 4): the
    // windows the scan reads, haplotype-major, entry = window << 6 | the haplotype's
    // index in its group of haps_per_block (<= 64); haplotype h's entries start at
    // wlist_off[c][h] (n_haps + 1 offsets, relative to this launch's haps); a
    // narrow group (gnarrow[g], relative to this launch's groups: every haplotype of
    // at most kWlNarrowLen bases, so window << 6 | haplotype fits 16 bits) has its
    // entries at the same offsets of wlist16[c] instead (half the bytes to read)
    const uint32_t *wlist[2];
    const uint16_t *wlist16[2];
    const uint4 *hd;   // matrix-core scan: per haplotype (word_off, len, flags, nmask_off) of haps (build_window_lists)
    const uint4 *hd2;  // and (region, pos_off, drun_off, n_druns): the rescoring's
    const uint8_t *gnarrow;
    // scan_mfma_all_kernel: workgroup b scans haplotype group gorder[b] (the groups in
    // descending order of work, so the launch ends on the small ones); null: group b
    const uint32_t *gorder;
    const uint64_t *wlist_off[2];
    // reference-window reuse (HAP_DEDUP haplotypes, tfbs_internal.hpp): dedup
    // != 0 scans only their dirty windows (the lists); the HAP_REF haplotypes' hits
    // (strand, window) are listed per region (ref_count[r] of kRefPerRegion at
    // ref_hits + 2 kRefPerRegion r), the excess in the spill list
    uint32_t dedup;
    // HAP_DEDUP haplotypes' diff runs: a hit of one in a window whose strand columns
    // [i, i + L - 1] meet no run is the reference's (the key assembly adds it), so
    // the rescoring does not list it
    const uint32_t *druns;
    uint32_t n_regions;
    uint32_t *ref_hits;
    uint32_t *ref_count;
    // spill list: (region | kind << 31, x, y) records -- kind 0 a hit (haplotype,
    // key), kind 1 a reference hit (strand, window) -- counted at over[0] (of
    // spill_cap), bucketed by region after the scan (launch_spill_buckets)
    uint32_t *spill;
    uint32_t *over;  // [0] spill records, [1] candidates past a wave's list
    uint32_t spill_cap;
    // candidates past a wave's list region: (haplotype, strand, window) triples,
    // rescored by a kernel after the scan (launch_post_scan)
    uint32_t *cand_over;
    uint32_t cand_over_cap;
    // fused post-scan (tfbs_step's lean steps): scan_mfma_all_kernel's last workgroup to
    // finish (ticket post_done) does post_scan_kernel's work -- the overflow candidates'
    // rescoring, the overflow counters to post_report, the spill records bucketed by
    // region (post_need_wide set when they are too many) -- instead of a launch after
    // the scan; post_done null: no fusion
    uint32_t *post_done;
    uint32_t post_regions;
    uint32_t *post_bcnt, *post_boff, *post_sorted, *post_report, *post_need_wide;
    // TFBS_SCAN_PROF builds of scan_mfma.hip (tools/variant_build.sh): per wave of
    // workgroup region_base + blockIdx.x, kScanProfWords clock stamps and counts
    // (tools/scan_prof.py); null otherwise
    unsigned long long *prof;
};
constexpr uint32_t kScanProfWords = 16;
constexpr uint32_t kRefPerRegion = 64;
constexpr uint32_t kMBlockWaves = 8;  // waves per matrix-core workgroup (hit list parts per workgroup)
constexpr uint32_t kCandWords = 2;  // candidate list entry: strand | haplotype in the group << 24, window

struct LaunchConfig {
    int minw = 2;               // __launch_bounds__ min waves per SIMD of the fast kernel
    size_t lds_bytes = 0;       // dynamic LDS of the fast kernel
};

// Enqueues the fast and/or generic scan over n_haps haplotypes on `stream`
// (grids split below 2^31 workgroups).  Returns launches issued or <0.
int launch_fast(const ScanArgs &a, const LaunchConfig &cfg, uint32_t n_haps, hipStream_t stream);
int launch_generic(const ScanArgs &a, uint32_t n_haps, hipStream_t stream);
// Opts the fast kernel into more than 64 KiB of dynamic LDS.
int fast_kernel_set_lds(const LaunchConfig &cfg);
// The workgroups of one matrix-core launch: hap groups [g0, g0 + ng) x ns super
// tiles, workgroup wg_base + (g - g0) ns + super; their hit lists are read back
// per region by the key assembly (key_kernels.hip).
struct HitSrc {
    uint32_t wg_base, ns, g0, ng;
};
constexpr int kMaxHitSrcs = 64;
constexpr uint32_t kMWaveCands = 48;  // a scan wave's candidates kept in LDS before its global list
// Matrix-core scan (scan_mfma.hip): sparse hits (hitl / hitn / spill), no counts.
// group_words: the most packed words any haplotype group of haps_per_block spans.
// One launch per K depth, spread round-robin over `streams` (deepest first);
// supers: the host copy of a.msupers (sorted by depth); srcs receives one
// HitSrc per launch (*n_srcs of kMaxHitSrcs).
int launch_mfma(const ScanArgs &a, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words, uint32_t n_haps,
                const hipStream_t *streams, uint32_t n_streams, HitSrc *srcs, uint32_t *n_srcs);
// The same in one launch on `stream`: one workgroup per haplotype group scans it
// against every super tile in turn (scan_mfma_all_kernel); one HitSrc with ns = 1.
int launch_mfma_all(const ScanArgs &a, const DevMSuper *supers, uint32_t n_supers, uint32_t group_words, uint32_t n_haps,
                    hipStream_t stream, HitSrc *srcs, uint32_t *n_srcs);
// Rescores the candidates past the waves' lists (after launch_mfma on the same stream).
int launch_post_scan(const ScanArgs &a, hipStream_t stream);
// The same (when cand) and the spill records' buckets by region (boff[0 .. n_regions],
// sorted) in one launch; *done and bcnt[0 .. n_regions] must be zero.
// wide: also the grid-wide spill bucketing (more than kPostSerial records); report /
// need_wide: post_scan_kernel's optional outputs (see there); cand_grid: the rescoring's
// workgroups (1 when the batch's last scan had no candidate past the lists: the same
// result, without 256 workgroups' dispatch and tickets)
constexpr uint32_t kPostSerial = 8192;  // spill records post_scan_kernel's last workgroup buckets itself
int launch_post_fused(const ScanArgs &a, bool cand, uint32_t *done, uint32_t n_regions, uint32_t *bcnt, uint32_t *boff,
                      uint32_t *sorted, hipStream_t stream, bool wide = true, uint32_t *report = nullptr,
                      uint32_t *need_wide = nullptr, uint32_t cand_grid = 256);
uint32_t mfma_group_words(const DevHap *haps, uint32_t n_haps, uint32_t hpb);
constexpr uint32_t kMMaxHapsPerBlock = 64;  // 6 bits of a window list entry
// Builds the window lists of every haplotype of the batch for the depth classes
// c (0: class 2, 1: class 4) with lmin[c] != 0 (the class's shortest strand):
// all windows [0, len - lmin + 1) of a haplotype, only the dirty ones of a
// HAP_DEDUP haplotype when dedup -- a run meeting the window's first span[c]
// columns, span[c] the class's longest strand (tfbs_internal.hpp) --; off[c] gets n_haps + 1
// offsets, list[c] (grown with ensure_list) the entries.  Synchronises `stream`.
constexpr uint32_t kWlNarrowLen = 1024;  // haplotypes of a narrow group: windows < 2^10
struct WindowListBufs {
    uint64_t *off[2];      // n_haps + 1 each
    uint64_t *scan_tmp;    // >= scan_tmp_words(n_haps + 1)
    uint32_t *list[2];
    uint16_t *list16[2];   // the narrow groups' entries (gnarrow: one flag per group of hpb)
    const uint8_t *gnarrow;
    uint4 *hd;             // n_haps compact descriptors (ScanArgs::hd), written here
    uint4 *hd2;            // and ScanArgs::hd2
    uint64_t list_cap[2];  // entries
};
size_t scan_tmp_words(size_t n);
// Per haplotype group of hpb (n_groups): the window tiles of its lists, cost[g] =
// pairs of class 2 x w[0] + pairs of class 4 x w[1] (w: the per-pair work of each
// depth class's super tiles), for the scan's workgroup order.
int group_costs(const uint64_t *off0, const uint64_t *off1, uint32_t n_haps, uint32_t hpb, uint32_t w0, uint32_t w1,
                uint32_t *cost, hipStream_t stream);
int build_window_lists(const DevHap *haps, uint32_t n_haps, const uint32_t *druns, const uint32_t lmin[2],
                       const uint32_t span[2], uint32_t hpb, uint32_t dedup, WindowListBufs &bufs, uint64_t total[2], hipStream_t stream,
                       int (*ensure_list)(void *ctx, int c, uint64_t n, uint32_t **p, uint16_t **p16),
                       void *ensure_ctx);
// Super tile image budgets per K depth (1-8) that let each depth's kernel reach
// the waves per SIMD its registers allow.
void mfma_depth_budgets(uint32_t out[9]);
size_t mfma_lds_fixed();  // LDS bytes the MFMA kernel needs besides the image and words

}  // namespace tfbs
