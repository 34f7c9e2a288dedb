// Launch interface of the key kernels (key_kernels.hip), used by device.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "batch.hpp"
#include "scan.hpp"

namespace tfbs {

// Everything key_asm_kernel reads and writes (device pointers; see key_kernels.hip).
struct AsmArgs {
    const DevHap *haps;
    const uint32_t *druns;  // HAP_DEDUP haplotypes' diff runs (tfbs_internal.hpp)
    const DevRegion *regions;
    const int32_t *inner;
    const int32_t *mmeta;       // matrix-core tiles' rescoring fields (strand length, slot, depth)
    const uint8_t *slot_mfma;   // per slot: 1 = matrix-core hits, 0 = the LUT/generic kernels' dense counts
    uint32_t any_dense;         // some slot is not on the matrix cores
    uint32_t n_slots;
    uint32_t hpb;               // haplotypes per matrix-core workgroup
    // the matrix-core launches' hit lists (ScanArgs::hitl / hitn)
    const uint32_t *hitl, *hitn;
    uint32_t cand_cap;
    const HitSrc *srcs;
    uint32_t n_srcs;
    uint32_t mfma;              // 0: the matrix-core kernel did not run (no hit lists, no reference hits)
    // reference hits per region, and the spill records bucketed by region
    const uint32_t *ref_hits, *ref_count;
    const uint32_t *spill_sorted, *spill_off;
    // the scan's spill record count (device, ScanArgs::over[0]; 0: spill_off is not
    // read), bucketed up to spill_cap records
    const uint32_t *spill_count;
    uint32_t spill_cap;
    uint32_t *counts;           // dense counts: read (LUT/generic slots) / written (mode 1)
    uint32_t dense_base;        // != 0: counts exist (haps' count_off are valid)
    uint32_t *scratch;          // counters of regions with more haplotypes than the LDS block holds
    int mode;                   // 0: classify + compact varying keys, 1: dense counts
    // mode 0 outputs: per key (region inner_off * n_slots + j) the first
    // haplotype's count and KeyFlags; the varying keys (var_tot[0] of
    // var_keys_cap) with their counts (var_tot[1] of var_cap u32)
    uint32_t *key_first;
    uint8_t *key_flags;
    DevVarKey *var_keys;
    uint32_t var_keys_cap;
    uint32_t *var_counts;
    uint64_t var_cap;
    unsigned long long *var_tot;
    // regions key_fast_kernel leaves to key_asm_kernel (*redo_n of them at redo):
    // written by key_fast_kernel, worked through by key_asm_kernel's list pass
    uint32_t *redo, *redo_n;
    uint32_t fast_max_u;  // key_fast_kernel takes regions of at most this many haplotypes (TFBS_KEY_FAST_MAXU)
    // key_fast_kernel's corrections of regions past its LDS list: shares of cor_arena
    // (cor_cap u32) taken from *cor_used (zeroed by launch_key_fast; read back by the host)
    uint32_t *cor_arena;
    uint32_t cor_cap;
    uint32_t *cor_used;
    uint32_t cor_lds;  // corrections kept in LDS at most (TFBS_KEY_COR_LDS, tests: the arena path)
    uint32_t *why;     // debug (TFBS_DEBUG_OVER): key_fast_kernel's give-ups per reason (8 counters), or null
    // launch_key_fast's list pass also copies report_src[0..1] (the scan's overflow
    // counters; null: zeros) to report[0..1] (null: not)
    const uint32_t *report_src;
    uint32_t *report;
    // key_fast_kernel: workgroup b takes region order[b] (regions by distinct haplotypes,
    // most first: the longest regions start first and do not trail the launch), or b
    const uint32_t *order;
    // key_fast_kernel: a persistent grid (a few workgroups per CU taking regions from
    // the counters next[0] / next[1] of the two shapes, zeroed before the launch),
    // else one region per workgroup
    uint32_t persist;
    uint32_t *next;
    uint64_t *prof;  // debug (TFBS_KF_PROF): key_fast_kernel's phase clocks and sizes, 16 per region, or null
};

// key_asm_kernel over every region (mode 0 or 1).
int launch_key_asm(const AsmArgs &a, uint32_t n_regions, hipStream_t stream);
// The reduction (mode 0) in two launches, no host round trip: key_fast_kernel
// takes every region within its limits (all of them at BASELINE shapes) and
// appends the others to a.redo, which key_asm_kernel then works through (a fixed
// grid looping over the list).  *a.redo_n, *a.cor_used and a.var_tot must be zero.
// a.order lists the regions with the n_big of more than key_fast_big_u() distinct
// haplotypes first: those take the 1 024-thread kernel on `stream`, queued ahead of
// the others' on `side` (forked from and joined back into `stream` with the events).
// leftover: also key_asm_kernel over the regions key_fast_kernel gave up (left out when the
// batch's last assembly had none: the host reruns the assembly if this one did)
int launch_key_fast(const AsmArgs &a, uint32_t n_regions, uint32_t n_big, hipStream_t stream, hipStream_t side,
                    hipEvent_t fork, hipEvent_t join, bool leftover = true);
uint32_t key_fast_big_u();
// ctr[0], ctr[1] = over[0], over[1] (the scan's overflow counters next to the
// assembly's, for one copy back).
int launch_asm_report(const uint32_t *over, uint32_t *ctr, hipStream_t stream);
uint32_t key_asm_lds_counters();  // regions with more distinct haplotypes use AsmArgs::scratch
// Buckets the spill records (ScanArgs::spill, *over of cap) by region: boff[r]
// .. boff[r + 1] of sorted (bcnt: n_regions + 1 scratch counters, zeroed here
// unless bcnt_zeroed).
int launch_spill_buckets(const uint32_t *over, uint32_t cap, const uint32_t *spill, uint32_t n_regions, uint32_t *bcnt,
                         uint32_t *boff, uint32_t *sorted, hipStream_t stream, bool bcnt_zeroed = false);
// A region's distinct haplotype pairs and each sample's pair (rows[r]: the device
// address of region r's u16 membership row, 0 to skip it): pab / pcnt at
// r * kEncMaxPairs, pair_n[r] (UINT32_MAX: skipped or too many pairs), pidx at r * n_samples.
int launch_pair_table(const uint64_t *rows, uint32_t n_regions, uint32_t n_samples, uint32_t *pab, uint32_t *pcnt,
                      uint32_t *pair_n, uint16_t *pidx, hipStream_t stream);
// Host-built regions' u16 membership rows made on the device (Hp, a multiple of 8,
// u16 per row): row k = the reference group (meta[2k + 1]) with the entries
// [meta[2k], meta[2k + 2]) of (ids, loc) -- haplotype id, distinct index -- over it.
int launch_memb_fill(const uint32_t *meta, const uint32_t *ids, const uint16_t *loc, uint32_t n_rows, uint32_t Hp,
                     uint16_t *memb, hipStream_t stream);
// One workgroup per key: counts_as_genotypes' per-sample half over the
// region's distinct haplotype pairs (launch_pair_table's, region - region0):
// pab = a | b << 16 (the distinct indices of a sample's two haplotypes), pcnt
// the samples with that pair, pidx each sample's pair.  Writes hdr[k], vals[k *
// 256 ..] (sorted distinct totals), hist[k * 256 ..] (samples per value) and
// codes[k * n_samples ..].
int launch_key_encode(const uint32_t *var_counts, const DevVarKey *keys, uint32_t n_keys, const uint32_t *pab,
                      const uint32_t *pcnt, const uint32_t *pair_n, const uint16_t *pidx, uint32_t region0,
                      uint32_t n_samples, EncHdr *hdr, uint32_t *vals, uint32_t *hist, uint8_t *codes,
                      hipStream_t stream);
// Key k's first (off[k + 1] - off[k]) value-table and histogram entries to off[k] of ov / oh.
int launch_val_compact(const uint32_t *vals, const uint32_t *hist, uint32_t n_keys, const uint32_t *off, uint32_t *ov,
                       uint32_t *oh, hipStream_t stream);
int launch_code_compact(const uint8_t *codes, uint32_t n_keys, uint32_t n_samples, const uint64_t *off, uint8_t *dst,
                        hipStream_t stream);

}  // namespace tfbs
