/*
 * tfbs_amd.h -- C ABI of the MI355X-native PWM scanner that drops in for
 * find-tfbs's per-haplotype TFBS scoring path (Helkafen/find-tfbs v1.0.1).
 *
 * The reference has no FFI on this path: it is the Rust `Pattern` enum
 * (types.rs:86-90) dispatched by `matches` (pattern.rs:141-171), fed by
 * `load_haplotypes` (haplotype.rs:77-88) and consumed by
 * `count_matches_by_sample` / `counts_as_genotypes` (main.rs:439-534).  Each
 * entry point below names the reference function it replaces; INTEGRATION.md
 * shows the Rust `extern "C"` block a maintainer would add to bind them.
 *
 * Conventions
 *  - Every entry returns int: TFBS_OK (0) or a negative TFBS_E_* code;
 *    tfbs_last_error() returns this thread's message for the last failure.
 *    The reference panics where these codes are returned (cited per code).
 *  - Caller owns every buffer it passes for the duration of the call; the
 *    library copies what it keeps.  Opaque objects are freed by their
 *    *_destroy.  No callbacks.
 *  - tfbs_patterns is immutable after creation and may be shared across
 *    threads.  tfbs_ctx and tfbs_batch are single-threaded objects; use one
 *    ctx per host thread / per GPU (the reference runs one reader per worker,
 *    main.rs:333-371).
 *  - Nucleotide codes are the reference enum order A=0 C=1 G=2 T=3 N=4
 *    (types.rs:5-8); weights are milli-log-odds int32 per column [A,C,G,T,N]
 *    with N = 0 (types.rs:103-114).
 *  - Haplotype ids are 2*sample + side, side 0 = Left, 1 = Right
 *    (types.rs:29-30, 66-70).
 */
#ifndef TFBS_AMD_H
#define TFBS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFBS_OK 0
#define TFBS_E_ARG (-1)         /* bad argument / call order */
#define TFBS_E_BADBASE (-2)     /* util.rs:15 "Unknown nucleotide" panic */
#define TFBS_E_REFMISMATCH (-3) /* haplotype.rs:126-128 panic */
#define TFBS_E_MNP (-4)         /* haplotype.rs:141-142 "Missing case" panic */
#define TFBS_E_PLOIDY (-5)      /* haplotype.rs:32 assert */
#define TFBS_E_RANGE (-6)       /* main.rs:407 u64 underflow / FASTA seek failure */
#define TFBS_E_PARSE (-7)       /* pattern.rs parse().unwrap()/expect panics */
#define TFBS_E_IO (-8)          /* file open/read failures (pattern.rs:116, bed.rs:34, ...) */
#define TFBS_E_HIP (-9)         /* HIP runtime error */
#define TFBS_E_NODEVICE (-10)   /* no HIP device: the product never falls back to the CPU */
#define TFBS_E_ALLELES (-11)    /* haplotype.rs:22 alleles[1] on a record with one allele */
#define TFBS_E_ZEROLEN (-12)    /* pattern.rs:150-156 index past the end for a length-0 PWM */
#define TFBS_E_NOPATTERN (-13)  /* main.rs:238 assert!(pwm_list.len() > 0) */
#define TFBS_E_STATE (-14)      /* object used out of order */
#define TFBS_E_NOMEM (-15)

const char *tfbs_strerror(int code);
const char *tfbs_last_error(void);
const char *tfbs_version(void);

/* ------------------------------------------------------------------ */
/* Patterns: the plugin surface (types.rs:86-114; README.md:68-72)      */
/* ------------------------------------------------------------------ */
#define TFBS_KIND_PWM 0   /* Pattern::PWM */
#define TFBS_KIND_OTHER 1 /* Pattern::OtherPattern: length 0, never matches */
#define TFBS_DIR_P 0      /* PWMDirection::P ("+") */
#define TFBS_DIR_N 1      /* PWMDirection::N ("-") */

typedef struct tfbs_pattern_desc {
    uint16_t pattern_id;    /* shared by both strands of one PWM (pattern.rs:73-77) */
    uint8_t direction;      /* TFBS_DIR_* */
    uint8_t kind;           /* TFBS_KIND_* */
    uint32_t length;        /* columns (pattern_length, types.rs:92-101) */
    const int32_t *weights; /* length x 5 ints [A,C,G,T,N]; the N column is ignored (always 0) */
    int32_t min_score;      /* a window matches iff score > min_score (pattern.rs:151) */
    const char *name;       /* pattern_id -> name (main.rs:239-250) */
} tfbs_pattern_desc;

typedef struct tfbs_patterns tfbs_patterns;

/* Replaces building Vec<Pattern> by hand: copies n descriptors. */
int tfbs_patterns_create(const tfbs_pattern_desc *descs, size_t n, tfbs_patterns **out);
/* Replaces parse_pwm_files (pattern.rs:37-87): names_csv is --pwm_names,
 * add_reverse = !--forward_only.  Fails with TFBS_E_NOPATTERN when nothing loads. */
int tfbs_patterns_from_files(const char *pwm_file, const char *threshold_dir, float pwm_threshold,
                             const char *names_csv, int add_reverse, tfbs_patterns **out);
size_t tfbs_patterns_count(const tfbs_patterns *p);
/* Pointers in *out stay valid while p lives. */
int tfbs_patterns_get(const tfbs_patterns *p, size_t i, tfbs_pattern_desc *out);
/* Name for a pattern_id (main.rs:239-250, last writer wins); NULL if unknown. */
const char *tfbs_patterns_name_of(const tfbs_patterns *p, uint16_t pattern_id);
/* max pattern_length over all patterns (main.rs:404). */
uint32_t tfbs_patterns_max_length(const tfbs_patterns *p);
void tfbs_patterns_destroy(tfbs_patterns *p);
/* Host-only diagnostics of the device plan the scan would use with tiles of
 * tile_blocks 4 KiB table blocks (and, if mfma, the matrix-core path): strands
 * on the 16-bit octet path, the 32-bit quad path, the generic (L > 32) kernel
 * and the FP4 x FP6 MFMA path, and their tiles. */
typedef struct tfbs_plan_stats {
    uint32_t n_octet_strands, n_quad_strands, n_generic_strands;
    uint32_t n_fast_tiles, n_fast_units, n_generic_tiles, max_tile_blocks;
    uint64_t lut_bytes;
    uint32_t n_mfma_strands, n_mfma_tiles, n_mfma_supers;
} tfbs_plan_stats;
int tfbs_patterns_plan_stats(const tfbs_patterns *p, uint32_t tile_blocks, int mfma, tfbs_plan_stats *out);
/* Host-only diagnostic of the matrix-core bound (mfma.cpp) for pattern i and
 * one window of pattern_length bases (0-3 = A,C,G,T, 4 = N): the window's
 * bound digit sum q8 = 8 Q, the strand's threshold t8, its scale and column
 * offset c.  The bound is c + scale * q8 / 8 >= apply_pwm (pattern.rs:125-135);
 * the window is a candidate iff q8 > t8, which every window with
 * score > min_score (pattern.rs:151) is.  eligible = 0: the pattern is scored
 * by the LUT kernels instead (the other fields are 0). */
typedef struct tfbs_mfma_bound {
    int32_t eligible;
    int64_t q8, t8, scale, c;
} tfbs_mfma_bound;
int tfbs_patterns_mfma_bound(const tfbs_patterns *p, size_t i, const uint8_t *bases, tfbs_mfma_bound *out);

/* pattern.rs:13-16 parse_weight: (f32(s) * 1000f32).round() as i32. */
int tfbs_parse_weight(const char *s, int32_t *out);
/* pattern.rs:18-35 parse_threshold_file: returns 1 (found, *out set), 0 (None) or an error. */
int tfbs_parse_threshold_file(const char *path, float pwm_threshold, int32_t *out);

/* ------------------------------------------------------------------ */
/* Device context: one GPU, one HIP stream, the pattern tables in HBM   */
/* ------------------------------------------------------------------ */
typedef struct tfbs_ctx tfbs_ctx;

int tfbs_device_count(int *n);
/* Uploads the 4-mer lookup tables of p to `device`.  p must outlive ctx. */
int tfbs_ctx_create(int device, const tfbs_patterns *p, tfbs_ctx **out);
void tfbs_ctx_destroy(tfbs_ctx *ctx);
int tfbs_ctx_sync(tfbs_ctx *ctx);
/* Host threads the ctx's host-side work may use (tfbs_batch_encode's staging;
 * default min(16, hardware threads)): a run with one ctx per device passes its share. */
int tfbs_ctx_set_host_threads(tfbs_ctx *ctx, uint32_t threads);
/* Device time (HIP events on the ctx stream) of the last tfbs_scan, ms. */
float tfbs_ctx_last_scan_ms(const tfbs_ctx *ctx);
/* Number of scan-kernel launches issued by the last tfbs_scan. */
int tfbs_ctx_last_scan_launches(const tfbs_ctx *ctx);
/* Device time (ms) of the last tfbs_scan's matrix-core kernel launches alone
 * (HIP events on the ctx stream), or -1 if the scan ran no MFMA tile. */
float tfbs_ctx_last_mfma_ms(const tfbs_ctx *ctx);
/* The matrix-core window lists of the uploaded batch (built by tfbs_batch_upload):
 * entries[c] = windows depth class c (0: strands of 1-2 K chunks, 1: 3-4) reads,
 * *seconds = the build's wall time.  Zeros before an upload or without MFMA strands. */
int tfbs_ctx_window_lists(const tfbs_ctx *ctx, uint64_t entries[2], double *seconds);
/* The last matrix-core scan's list counters (waits for it): out[0] spill records,
 * out[1] candidates past the waves' lists (rescored by post_scan_kernel), out[2]
 * candidates found, out[3] of them written to the waves' global lists (past the
 * LDS ones), out[4] (haplotype, key) pairs in the hit lists.  Zeros without one. */
int tfbs_ctx_scan_counters(tfbs_ctx *ctx, uint64_t out[5]);

/* Replaces matches() (pattern.rs:141-171) for ONE haplotype against every
 * pattern, on the GPU.  nucs are codes 0..4, pos the NucleotidePos.pos values.
 * Writes match ranges grouped by pattern index (in creation order): for each
 * pattern i, counts[i] matches; the ranges are concatenated into out_start /
 * out_end (start = pos[w], end = pos[w] + L - 1) in window order.  *n_total
 * receives the total; TFBS_E_ARG if cap is too small (then *n_total is the need). */
int tfbs_matches(tfbs_ctx *ctx, const uint8_t *nucs, const uint64_t *pos, size_t n, uint32_t *counts,
                 uint64_t *out_start, uint64_t *out_end, size_t cap, size_t *n_total);

/* ------------------------------------------------------------------ */
/* Haplotype reconstruction (haplotype.rs:94-156)                       */
/* ------------------------------------------------------------------ */
/* patch_haplotype over a reference window.  Diffs are flattened: diff d has
 * ref codes dref[roff..roff+dnref[d]) and alt codes dalt[aoff..aoff+dnalt[d]).
 * Writes at most cap bases; *n_out gets the length (TFBS_E_ARG if > cap). */
int tfbs_patch_haplotype(uint64_t range_start, uint64_t range_end, size_t n_diffs, const uint64_t *dpos,
                         const uint8_t *dref, const uint32_t *dnref, const uint8_t *dalt, const uint32_t *dnalt,
                         const uint8_t *ref_nucs, const uint64_t *ref_pos, size_t n_ref, uint8_t *out_nucs,
                         uint64_t *out_pos, size_t cap, size_t *n_out);

/* ------------------------------------------------------------------ */
/* Region batches: load_haplotypes + find_all_matches + counting          */
/* (haplotype.rs:13-88, main.rs:94-154, 395-436, 439-534)                */
/* ------------------------------------------------------------------ */
typedef struct tfbs_batch tfbs_batch;

/* n_samples = selected samples (main.rs:293-314).  keep_membership = 0 drops
 * per-haplotype group membership (scan-only use; rows then unavailable). */
int tfbs_batch_create(const tfbs_patterns *p, uint32_t n_samples, int keep_membership, tfbs_batch **out);
void tfbs_batch_destroy(tfbs_batch *b);
/* Registers a BED source by basename (bed.rs:49-60); returns its index >= 0. */
int tfbs_batch_add_bed(tfbs_batch *b, const char *basename);
/* main.rs:404: L_max of the halo-extended windows, if wider than the pattern set's
 * longest strand (>= it; before the first region).  A batch scanning a shard of the
 * pattern_ids passes the whole set's L_max so that its windows, distinct haplotypes
 * and counts are those of the unsharded run (SURVEY.md 8(e) region x PWM shard). */
int tfbs_batch_set_window_lmax(tfbs_batch *b, uint32_t lmax);
/* load_diffs / group_by_diffs / load_haplotypes (haplotype.rs:16-88) on a device
 * (before the first region; device < 0: host only): a region whose applied
 * records are all SNVs inside its window (REF = the window's base, ALT another of
 * A/C/G/T, at most 64, one per position, carrier ids ascending) and whose window
 * has no N gets its haplotypes' diff masks, distinct groups, patched and packed
 * haplotypes and membership computed there (the membership stays on the device, a
 * u16 distinct index per haplotype id, fetched only when a host path needs it).  A
 * region with indels or N whose applied records are at most 64 distinct diffs with
 * ascending carriers is grouped there (distinct masks, carrier counts, membership:
 * the O(haplotypes x records) part) and the host patches only its distinct groups
 * (TFBS_DEV_PATCH=0: built on the host).  Every other region, and one of more than
 * 2 047 distinct diff masks, is built on the host.  The batch is the same either
 * way (tfbs_batch_region_input_digest). */
int tfbs_batch_set_build_device(tfbs_batch *b, int device);
/* Regions grouped on the device / built on the host so far. */
int tfbs_batch_build_stats(const tfbs_batch *b, uint64_t *dev_regions, uint64_t *host_regions);
/* Of the regions grouped on the device, those whose distinct groups the host
 * patched (indels / N). */
int tfbs_batch_patch_stats(const tfbs_batch *b, uint64_t *patched_regions);
/* main.rs:404-407: the halo-extended window of a merged region. */
int tfbs_batch_region_ext(const tfbs_batch *b, uint64_t merged_start, uint64_t merged_end, uint64_t *ext_start,
                          uint64_t *ext_end);
/* Starts a merged region; ref_ascii = FASTA bases from ext_start (main.rs:156-161,
 * may be shorter than the window at a contig end). */
int tfbs_batch_region_begin(tfbs_batch *b, uint64_t merged_start, uint64_t merged_end, const char *ref_ascii,
                            size_t n_ref);
/* One inner peak selected by select_inner_peaks (main.rs:62-72); duplicates count twice. */
int tfbs_batch_region_add_inner(tfbs_batch *b, uint32_t bed, uint64_t start, uint64_t end);
/* One BCF record (haplotype.rs:16-60): gt = 2 raw BCF GT ints per selected
 * sample, INT32_MIN+1 = vector_end.  Left carries ALT iff gt0 == 4 (Unphased(1)),
 * Right iff gt1 == 5 (Phased(1)). */
int tfbs_batch_region_add_record_gt(tfbs_batch *b, uint64_t pos, uint32_t n_alleles, const char *ref,
                                    const char *alt, const int32_t *gt);
/* Same with the carrying haplotype ids given directly (phased synthetic data). */
int tfbs_batch_region_add_record_carriers(tfbs_batch *b, uint64_t pos, const char *ref, const char *alt,
                                          const uint32_t *hap_ids, size_t n);
/* Groups, patches, deduplicates and packs the region's distinct haplotypes. */
int tfbs_batch_region_end(tfbs_batch *b);

size_t tfbs_batch_num_regions(const tfbs_batch *b);
size_t tfbs_batch_num_haplotypes(const tfbs_batch *b); /* distinct haplotypes (number_of_haplotypes, main.rs:97-130) */
/* Windows the scan scores: sum over distinct haplotypes and PWM patterns of max(0, len - L + 1). */
uint64_t tfbs_batch_num_windows(const tfbs_batch *b);
/* Column lookups the scan performs: sum over windows of the pattern length L. */
uint64_t tfbs_batch_num_cell_ops(const tfbs_batch *b);
/* Per-sample-weighted windows (each distinct haplotype times its carrier count). */
uint64_t tfbs_batch_num_effective_windows(const tfbs_batch *b);
/* Windows and column lookups the scan executes: a window of an SNV-only haplotype
   whose bases and positions equal the region's reference window takes the
   reference window's result (reference-window reuse, TFBS_DEDUP=0 disables it);
   helper reference haplotypes of regions without a reference group count here. */
uint64_t tfbs_batch_num_scan_windows(const tfbs_batch *b);
uint64_t tfbs_batch_num_scan_cell_ops(const tfbs_batch *b);
/* Packed bytes the scan reads from HBM per launch (sequence + masks + positions + metadata). */
uint64_t tfbs_batch_input_bytes(const tfbs_batch *b);
/* Bytes of the dense u32 counts (the LUT / generic kernels' slots, and the debug
   download tfbs_batch_download fills); the matrix-core path writes sparse hit lists. */
uint64_t tfbs_batch_output_bytes(const tfbs_batch *b);

/* Copies the packed batch into ctx device memory (H2D). */
int tfbs_batch_upload(tfbs_ctx *ctx, tfbs_batch *b);
/* Scans the uploaded batch on the GPU (the work of matches() over every distinct
 * haplotype, main.rs:101-147, plus the overlap test of main.rs:503): sparse hit
 * lists -- one (distinct haplotype, pattern_id slot x inner range) entry per hit
 * and overlapped range from the matrix-core kernel, the region's reference
 * haplotype's hits listed for reference-window reuse -- and, for strands the
 * LUT / generic kernels score, dense counts.  Asynchronous on the ctx stream;
 * tfbs_batch_assemble / tfbs_batch_reduce / tfbs_batch_download turn the lists
 * into per-key counts. */
int tfbs_scan(tfbs_ctx *ctx, tfbs_batch *b);
/* D2H copy of the counts into the batch. */
int tfbs_batch_download(tfbs_ctx *ctx, tfbs_batch *b);
/* Alternative to tfbs_batch_download for row emission (the gather half of
 * count_matches_by_sample, main.rs:500-534, moved to the device): classifies
 * every (region, pattern_id, inner range) key on the GPU (some distinct
 * haplotype matched / distinct haplotypes disagree) and downloads only the
 * flags and one count per key; the per-haplotype counts of the disagreeing keys
 * stay on the device (tfbs_batch_encode / tfbs_batch_rows_bgzf read them there)
 * and are downloaded when a host key / row function first needs them -- the ctx
 * makes that copy itself before it reduces another batch or is destroyed.  The
 * key / row functions below then work as after a download. */
int tfbs_batch_reduce(tfbs_ctx *ctx, tfbs_batch *b);
/* The device half of tfbs_batch_reduce, enqueued behind tfbs_scan with no host
 * wait (main.rs:94-154's per-region result + count_matches_by_sample's key
 * vectors, main.rs:500-534): candidates past the scan's lists rescored, spill
 * records bucketed, every region's keys assembled from its hit lists -- each
 * HAP_DEDUP haplotype's count is the reference haplotype's plus its own hits
 * minus the reference hits inside its dirty windows -- classified, and the
 * varying keys' counts compacted on the device.  tfbs_batch_assemble_wait
 * waits for it and checks every list (a scan list that overflowed is rescanned
 * larger, a full varying-key list reassembled); tfbs_batch_reduce then only
 * downloads.  One step of scan + assembly = tfbs_scan, tfbs_batch_assemble,
 * tfbs_batch_assemble_wait. */
int tfbs_batch_assemble(tfbs_ctx *ctx, tfbs_batch *b);
int tfbs_batch_assemble_wait(tfbs_ctx *ctx, tfbs_batch *b);
/* One step of the resident batch: tfbs_scan + tfbs_batch_assemble +
 * tfbs_batch_assemble_wait, same results.  From the third step alike on (same
 * batch, no buffer regrown), the scan's and the assembly's launches run as one
 * hipGraph captured on the third (TFBS_STEP_GRAPH=0: never); graph steps leave
 * the timing queries (tfbs_ctx_last_scan_ms, ...) at the last plain step's. */
int tfbs_step(tfbs_ctx *ctx, tfbs_batch *b);
/* Device time (ms, HIP events on the ctx stream) of the last assembly, -1 if none ran. */
float tfbs_ctx_last_assemble_ms(const tfbs_ctx *ctx);
/* counts_as_genotypes' per-sample half on the device (main.rs:439-534, SURVEY.md
 * 8(f) f1) for the varying keys of regions [r0, r1) after tfbs_batch_reduce:
 * per key v[s] = C[hap(2s)] + C[hap(2s+1)] over the samples, min / max, the
 * sorted distinct values with their sample counts, and one u8 code per sample;
 * rows of these regions are then formatted from the codes (no per-sample
 * count gather on the host).  Keys whose region has > 65 535 distinct haplotypes
 * (u16 membership) or > 8 192 distinct (left, right) haplotype pairs (the LDS pair
 * table, pair_table_kernel), or with > 255 distinct totals or a total range >= 65 536,
 * keep the host path (tfbs_internal.hpp kEncMax*). */
int tfbs_batch_encode(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1);
/* tfbs_batch_encode with flags: TFBS_ENC_DEVICE_CODES keeps the per-sample codes on
 * the device only (for tfbs_batch_rows_bgzf; host row functions then take their
 * slower path for these keys). */
#define TFBS_ENC_DEVICE_CODES 1
int tfbs_batch_encode_flags(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, int flags);

/* The rows of regions [r0, r1) (main.rs:415-429, same text as tfbs_batch_rows) as
 * BGZF blocks (main.rs:258-290's BGzWriter) built on the GPU
 * after tfbs_batch_encode over them: row heads formatted on the host, the
 * per-sample genotype text generated from the device codes and deflated there
 * (deflate, CRC32), so the text never crosses PCIe.  Whole blocks -- the last one
 * shorter -- are written to file descriptor fd (after the header's blocks);
 * *fake_position is the POS counter, advanced per row; *bytes / *n_rows /
 * *text_bytes (optional) receive the bytes written, the rows and their
 * uncompressed bytes. */
int tfbs_batch_rows_bgzf(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, const char *chromosome,
                         uint32_t min_maf, uint32_t *fake_position, int fd, uint64_t *bytes, uint64_t *n_rows,
                         uint64_t *text_bytes);
/* Seconds spent in tfbs_batch_rows_bgzf on this ctx so far: out[0] the row plan on
 * the host (heads, token tables), out[1] the rest (uploads, kernels, copy-back, write). */
int tfbs_ctx_rows_bgzf_seconds(const tfbs_ctx *ctx, double *out);

/* After download: count_matches_by_sample (main.rs:500-534), keys ordered by
 * (inner.start, inner.end, bed basename, pattern_id).  keys are per region. */
int tfbs_batch_region_num_keys(const tfbs_batch *b, size_t region, size_t *n);
int tfbs_batch_region_key(const tfbs_batch *b, size_t region, size_t k, uint32_t *bed, uint64_t *start,
                          uint64_t *end, uint16_t *pattern_id, uint32_t *left, uint32_t *right);
/* counts_as_genotypes + row emission (main.rs:415-429, 439-498) for every
 * region, in region order.  Appends rows to *text (malloc'd; free with
 * tfbs_free); *fake_position is the POS counter, advanced per row. */
int tfbs_batch_rows(const tfbs_batch *b, const char *chromosome, uint32_t min_maf, uint32_t *fake_position,
                    char **text, size_t *len);
/* The rows of one region (main.rs:415-429 for one process_peak call), same
 * format and POS handling as tfbs_batch_rows. */
int tfbs_batch_region_rows(const tfbs_batch *b, size_t region, const char *chromosome, uint32_t min_maf,
                           uint32_t *fake_position, char **text, size_t *len);
/* 64-bit digest of one region's keys at the distinct-haplotype level (key
 * identity in row order + every distinct haplotype's count): equal digests
 * from the dense download and the device reduction, or from a sharded and an
 * unsharded batch, mean equal count_matches_by_sample maps (main.rs:500-534). */
int tfbs_batch_region_digest(const tfbs_batch *b, size_t region, uint64_t *digest);
/* Order-free digest: the sum over the region's keys of a hash of the key (bed,
 * range, multiplicity, pattern_id) and its distinct haplotypes' counts.  Batches
 * over disjoint pattern_id shards of one pattern set (same windows: see
 * tfbs_batch_set_window_lmax) sum to the unsharded batch's digest. */
int tfbs_batch_region_key_digest_sum(const tfbs_batch *b, size_t region, uint64_t *digest);
/* Digest of what the host prep packed for a region (window, inner keys, distinct
 * haplotypes' bases / N masks / positions, carriers, membership): equal for the
 * same region built in any batch or shard. */
int tfbs_batch_region_input_digest(const tfbs_batch *b, size_t region, uint64_t *digest);
/* Canonical per-region digests of regions [r0, r1) (the full-size golden files of
 * tests/golden/, made by the oracle's orc_job_digests; no reference counterpart):
 * keys[i] = the sum over the region's keys of a hash of (bed index, start, end,
 * pattern_id, S) with S = sum over samples s of L[s] w(2s) + R[s] w(2s + 1) mod 2^64
 * (w = splitmix64; count_matches_by_sample's vectors, main.rs:500-534, as a linear
 * sketch computed from the distinct haplotypes' counts and the membership);
 * rows[i] = XXH64 (seed 0) of the region's rows with their "<chr>\t<POS>\t"
 * prefix removed (main.rs:415-429), n_rows[i] their number.  Regions run on
 * `threads` host threads; keys or rows (with n_rows) may be null to skip that digest.
 * Needs the counts (download or reduce) and the membership. */
int tfbs_batch_region_digests(const tfbs_batch *b, size_t r0, size_t r1, uint32_t min_maf, uint32_t threads,
                              uint64_t *keys, uint64_t *rows, uint64_t *n_rows);
/* Distinct haplotypes (number_of_haplotypes, main.rs:97-130) and records (variant_count) of a region. */
int tfbs_batch_region_stats(const tfbs_batch *b, size_t region, uint32_t *n_haplotypes, uint32_t *n_variants);
/* Formats the rows of regions [r0, r1) (main.rs:415-429) on `threads` host threads and
 * discards them: the row count and bytes (without POS digits).  The bench's
 * end-to-end leg times it; tfbs_run writes the same rows. */
int tfbs_batch_format_rows(const tfbs_batch *b, const char *chromosome, uint32_t min_maf, uint32_t threads,
                           size_t r0, size_t r1, uint64_t *n_rows, uint64_t *n_bytes);
/* Host prep seconds of the batch's synthetic fills (out[4]): generation and
 * build_region (thread CPU-seconds, summed), build_region + the serial commit
 * (wall: the prep a BCF reader's records go through) and the whole fill (wall,
 * generation included). */
int tfbs_batch_prep_seconds(const tfbs_batch *b, double *out);
void tfbs_free(void *p);

/* counts_as_genotypes alone (main.rs:439-498): 1 = row (strings written), 0 = no variation. */
int tfbs_counts_as_genotypes(const uint32_t *left, const uint32_t *right, size_t n, uint32_t *maf, char *info,
                             size_t info_cap, char *genotypes, size_t gt_cap);

/* ------------------------------------------------------------------ */
/* The find-tfbs command flow (main.rs:163-393) and its file formats     */
/* (f2 BCF, f3 CLI + BGZF writer, f4 FASTA/BED)  */
/* ------------------------------------------------------------------ */
typedef struct tfbs_run_args {
    const char *chromosome;        /* --chromosome */
    const char *bcf;               /* --input */
    const char *bed_files;         /* --bed (comma list) */
    const char *reference;         /* --reference (FASTA with .fai) */
    const char *samples_file;      /* --samples, NULL = all BCF samples */
    const char *pwm_file;          /* --pwm_file */
    const char *pwm_threshold_dir; /* --pwm_threshold_directory */
    const char *pwm_names;         /* --pwm_names (comma list) */
    const char *output;            /* --output (BGZF VCF) */
    float pwm_threshold;           /* --pwm_threshold */
    int forward_only;              /* --forward_only */
    uint32_t min_maf;              /* --min_maf */
    uint32_t threads;              /* --threads: host threads building regions */
    uint64_t after_position;       /* --after_position */
    int tabix;                     /* --tabix */
    int verbose;                   /* --verbose */
    int device;                    /* HIP device (when devices is NULL/empty) */
    uint32_t regions_per_batch;    /* merged regions per GPU batch (0 = 512) */
    const char *devices;           /* comma list of HIP devices, one region shard each ("0,1,2,3";
                                      a device may repeat); NULL/"" = just `device` */
} tfbs_run_args;
/* Replaces run() (main.rs:234-393): writes <output>.part, renames it to output.
 * The merged regions go in batches of regions_per_batch (the reference's 50-peak
 * chunks over worker threads, main.rs:332-381); each batch is built (BCF records,
 * load_diffs; SNV-only regions grouped on the GPU), scanned, reduced, encoded and
 * its rows made as BGZF blocks on the device.  Several devices:
 * batch g runs on device g % n, each device with its own pipeline (BCF reader --
 * CSI-indexed seek when <bcf>.csi exists --, FASTA reader, host prep thread,
 * ctx); batch g's first POS is batch g - 1's plus its row count (published before
 * either deflates) and the batches' blocks are written in order, so the output
 * text is identical for any device list. */
int tfbs_run(const tfbs_run_args *args);

typedef struct tfbs_bcf tfbs_bcf;
/* Replaces rust-htslib IndexedReader::from_path / header().samples() (main.rs:46-52, 255). */
int tfbs_bcf_open(const char *path, tfbs_bcf **out);
void tfbs_bcf_close(tfbs_bcf *b);
size_t tfbs_bcf_num_samples(const tfbs_bcf *b);
/* 1 if <path>.csi was loaded: fetches that would rewind or skip ahead seek to the
 * index's chunk start (IndexedReader::fetch, haplotype.rs:78-79); 0 = streaming sweep. */
int tfbs_bcf_indexed(const tfbs_bcf *b);
const char *tfbs_bcf_sample_name(const tfbs_bcf *b, size_t i);
/* Samples whose GT is decoded, in this order (default: all); main.rs:293-314's sample selection,
 * applied while decoding.  Rewinds the stream. */
int tfbs_bcf_select(tfbs_bcf *b, const size_t *idx, size_t n);
/* Replaces reader.fetch(rid, beg, end) (haplotype.rs:79): records with pos < end && pos + rlen > beg,
 * in file order.  Streams the file: queries with nondecreasing beg on one contig read it once,
 * an earlier beg or another contig rewinds to the start. */
int tfbs_bcf_fetch(tfbs_bcf *b, const char *chrom, uint64_t beg, uint64_t end, size_t *n_records);
/* Record i of the last fetch: raw GT ints, 2 per selected sample, INT32_MIN+1 = vector_end; alt NULL
 * for a single-allele record. */
int tfbs_bcf_record(const tfbs_bcf *b, size_t i, uint64_t *pos, uint32_t *rlen, uint32_t *n_alleles, const char **ref,
                    const char **alt, const int32_t **gt);
/* Carriers mode (on != 0; rewinds the stream): records keep load_diffs' carrier ids of a bi-allelic
 * record (haplotype.rs:16-41: 2 k iff GT[0] = Unphased(1), 2 k + 1 iff GT[1] = Phased(1), k the
 * selected sample), found on the reader's threads while decoding, instead of raw GT (tfbs_bcf_record
 * then returns gt NULL).  tfbs_run reads its BCF this way. */
int tfbs_bcf_set_carriers_mode(tfbs_bcf *b, int on);
/* The BCF reader's raw DEFLATE decoder (RFC 1951; BGZF blocks, htslib's bgzf.c
 * reads them with zlib): in_len bytes into exactly out_len bytes.  TFBS_OK, or
 * TFBS_E_PARSE for a stream it does not decode exactly (the reader then inflates
 * that block with zlib).  Exported for its tests. */
int tfbs_inflate_raw(const void *in, size_t in_len, void *out, size_t out_len);
/* Record i of the last fetch in carriers mode: ascending carrier ids and the ploidy check
 * (TFBS_OK, or TFBS_E_PLOIDY when a selected sample's GT does not hold 2 alleles,
 * haplotype.rs:24-26); 0 ids for a record that is not bi-allelic. */
int tfbs_bcf_record_carriers(const tfbs_bcf *b, size_t i, const uint32_t **ids, size_t *n, int *gt_status);
/* Replaces bio fasta IndexedReader fetch(chrom, start, stop) + read (main.rs:156-161). */
int tfbs_fasta_fetch(const char *fasta, const char *chrom, uint64_t start, uint64_t stop, char **out, size_t *n);
/* BGZF writer as BGzWriter (main.rs:267-276): data blocks, `flushes` empty blocks, EOF block. */
int tfbs_bgzf_write_file(const char *path, const char *text, size_t n, int flushes);
int tfbs_bgzf_read_file(const char *path, char **out, size_t *n);
/* RangeStack (range.rs:43-87): out arrays need n entries. */
int tfbs_merge_ranges(const uint64_t *starts, const uint64_t *ends, size_t n, uint64_t *out_s, uint64_t *out_e,
                      size_t *n_out);

/* ------------------------------------------------------------------ */
/* Synthetic workloads                            */
/* ------------------------------------------------------------------ */
/* Writes <dir>/pwms.txt and <dir>/thr/<name>.thr for n PWMs; lengths follow
 * config 2 (L = 8..15) or 3 (L = 8 + i%15, the last 30 L = 23 + i%8) or
 * 5 (L = 25..30).  names_csv (malloc'd) lists the names. */
int tfbs_synth_write_pwms(const char *dir, uint32_t n_pwms, int length_config, uint64_t seed, char **names_csv);
typedef struct tfbs_synth_region tfbs_synth_region;
/* Region `index` of a synthetic chromosome: BED row [1000+400*index, 1200+400*index],
 * Poisson(20) distinct variant sites over the ext window of max length lmax,
 * carriers with P(k) ~ 1/k on 1..H/10; indel_pct % of sites are 1-10 bp indels. */
int tfbs_synth_region_make(uint64_t seed, uint64_t index, uint32_t n_samples, uint32_t lmax, uint32_t indel_pct,
                           tfbs_synth_region **out);
void tfbs_synth_region_destroy(tfbs_synth_region *r);
void tfbs_synth_region_info(const tfbs_synth_region *r, uint64_t *merged_start, uint64_t *merged_end,
                            uint64_t *ext_start, const char **ref_ascii, size_t *n_ref, size_t *n_records);
void tfbs_synth_region_record(const tfbs_synth_region *r, size_t i, uint64_t *pos, const char **ref,
                              const char **alt, const uint32_t **carriers, size_t *n_carriers);
/* Adds regions [first, first+count) to b (one bed source "synthetic.bed" is
 * registered on first use; each region's inner peak is its BED row). */
int tfbs_synth_fill_batch(tfbs_batch *b, uint64_t seed, uint64_t first, uint64_t count, uint32_t indel_pct);

#ifdef __cplusplus
}
#endif
#endif /* TFBS_AMD_H */
