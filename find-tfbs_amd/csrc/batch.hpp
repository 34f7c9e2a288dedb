// Host-side region batch: the distinct haplotypes of many merged regions,
// packed for the scan kernels, plus what the count aggregation needs.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {
// std::allocator whose value-less construct leaves a trivial element uninitialised: a
// vector grown with resize(n) is not zero-filled first.  The batch's largest host arrays
// use it -- commit_regions fills every element on its threads (a serial zero-fill of the
// positions and words took 0.2-0.4 s per 4 000 C5 regions, most of the commit).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    template <class U>
    void construct(U *p) noexcept {
        ::new ((void *)p) U;
    }
    template <class U, class... Args>
    void construct(U *p, Args &&...args) {
        ::new ((void *)p) U(std::forward<Args>(args)...);
    }
};
template <class T>
using RawVec = std::vector<T, NoInitAlloc<T>>;
}  // namespace tfbs

namespace tfbs {

struct Record {  // one BCF record as load_diffs sees it (haplotype.rs:16-60)
    uint64_t pos = 0;
    uint32_t n_alleles = 2;
    std::vector<uint8_t> ref, alt;   // nucleotide codes
    std::vector<uint32_t> carriers;  // haplotype ids carrying alt (2*sample + side)
};

struct InnerKey {   // one (bed, inner range) of select_inner_peaks (main.rs:62-72)
    uint32_t bed;
    uint64_t s, e;
    uint32_t mult;  // duplicates of the same range in one bed list count twice (main.rs:503-505)
    int32_t slot;   // distinct-range slot in the kernel output, -1 if the range is empty (e < s)
};

struct RegionH {
    uint64_t ms = 0, me = 0, es = 0, ee = 0;
    uint32_t hap_begin = 0, hap_count = 0;  // distinct haplotypes (batch-global indices)
    int32_t ref_local = -1;                 // local index of the reference-group haplotype, -1 if none
    uint32_t n_variants = 0;
    uint64_t key_off = 0;                   // first key (slot * n_inner + range) in the reduced arrays
    std::vector<InnerKey> keys;             // sorted by (s, e, bed)
    std::vector<std::pair<uint64_t, uint64_t>> ranges;  // distinct non-empty inner ranges
    // membership: haplotype id -> local distinct index; ids not listed use ref_local.
    // A region grouped on the device (memb_dev != 0) keeps its membership there, one
    // u16 per haplotype id; the lists are filled from it when a host path asks
    // (region_membership).
    mutable std::vector<uint32_t> nonref_id, nonref_local;
    uint64_t memb_dev = 0;          // device address of the membership row, 0 if host-built
    mutable bool memb_host = true;  // nonref_id / nonref_local are valid
};

// Page-locked host bytes (hipHostMalloc): device downloads land at full PCIe rate.
struct PinnedBytes {
    uint8_t *p = nullptr;
    size_t cap = 0;
    bool pinned = false;    // hipHostMalloc'd (else malloc'd: page-locked memory ran out)
    int reserve(size_t n);  // keeps nothing; TFBS_E_NOMEM on failure
    void release();
    const uint8_t *data() const { return p; }
    ~PinnedBytes();
    PinnedBytes() = default;
    PinnedBytes(const PinnedBytes &) = delete;
    PinnedBytes &operator=(const PinnedBytes &) = delete;
};

// Device grouping (haplotype.rs:16-88 on the GPU): regions whose
// applied diffs are all SNVs get their haplotypes' diff masks, distinct groups and
// membership computed on a device (build_gpu.hip).  One chunk of regions:
// carrier ids back to back (each record's list), the records and the regions.
struct GrpRecord {
    uint32_t off, n;     // carriers [off, off + n) of the chunk's carrier array
    uint32_t rank;       // the diff's rank in Vec<Diff> order (its bit in the masks)
    uint32_t region;     // chunk region index
};
struct GrpRegion {
    uint32_t rec_off, n_rec;  // records [rec_off, rec_off + n_rec) of the chunk
};
constexpr uint32_t kGrpMax = 2047;  // distinct diff masks of a device-grouped region (the LDS table)
struct GroupOut {                 // per chunk region
    std::vector<uint32_t> n_groups;  // distinct non-empty masks, UINT32_MAX: more than kGrpMax (host build)
    std::vector<uint32_t> first;     // the region's first mask in masks / counts
    std::vector<uint64_t> masks;     // per region n_groups masks, ascending Vec<Diff> order
    std::vector<uint32_t> counts;    // carriers per mask
    std::vector<uint64_t> memb;      // device address of each region's membership row
    void *memb_alloc = nullptr;      // the chunk's rows' allocation (the batch hands it back: recycle)
};
struct DevGrouper {
    virtual ~DevGrouper() {}
    virtual int device() const = 0;
    // staging for n carrier ids (page-locked, valid until the next group call)
    virtual uint32_t *carriers(size_t n) = 0;
    virtual int group(size_t n_car, const std::vector<GrpRecord> &recs, const std::vector<GrpRegion> &regs,
                      uint32_t H, GroupOut &out) = 0;
    // one membership row (H u16) to the host
    virtual int fetch(uint64_t memb, uint32_t H, uint16_t *out) = 0;
    // membership allocations of a batch going away, kept for later chunks (a grouper
    // shared by a run's batches allocates once; thread-safe)
    virtual void recycle(std::vector<void *> &allocs) = 0;
};
DevGrouper *make_gpu_grouper(int device);  // build_gpu.hip
// The HIP runtime and these devices' contexts initialised (0.1-0.4 s in a fresh process):
// tfbs_run starts it on a thread before it parses its inputs.  build_gpu.hip
void warm_devices(const std::vector<int> &devices);

struct Batch {
    const Patterns *pats = nullptr;
    uint32_t n_samples = 0;
    bool keep_membership = true;
    uint32_t n_slots = 0;                 // pattern_id slots (Plan::slot_pid)
    std::vector<uint16_t> slot_pid;       // slot -> pattern_id (slots ordered for the kernels)
    std::vector<uint32_t> slots_by_pid;   // slots in ascending pattern_id (row order)
    std::vector<std::string> beds;        // registered bed basenames
    std::vector<std::pair<uint32_t, uint32_t>> pwm_len_hist;  // (length, strands) of scannable strands

    // packed device image
    RawVec<uint32_t> words;               // 2-bit bases, 16 per word, LSB first, +3 pad words per hap
    RawVec<uint32_t> nmask;               // N masks (+2 pad words per hap)
    RawVec<int32_t> posrel;               // positions relative to ext_start (non-affine haps only)
    RawVec<uint32_t> druns;               // HAP_DEDUP haplotypes' diff runs, (a, b) pairs (tfbs_internal.hpp)
    std::vector<DevHap> haps;
    std::vector<DevRegion> regions;
    std::vector<int32_t> inner;           // (s_rel, e_rel) pairs
    std::vector<uint32_t> hap_carriers;   // carriers per distinct hap
    uint64_t n_counts = 0;                // u32 counts the scan writes
    std::vector<uint32_t> counts;         // downloaded counts
    bool counts_valid = false;
    // on-device key reduction (tfbs_batch_reduce): per key
    // (region, slot, range) the first distinct haplotype's count and flags
    // (KEY_ANY: some count != 0, KEY_VARIES: counts differ); varying keys keep
    // every distinct haplotype's count at var_off[key] in var_counts.
    std::vector<uint32_t> key_first;
    std::vector<uint8_t> key_flags;
    std::vector<uint32_t> var_off;        // UINT32_MAX unless the key varies
    PinnedBytes var_counts;  // u32 counts, host copy (made on first use: ensure_host_var_counts)
    // tfbs_batch_reduce leaves the varying counts on the device (the device encode
    // and BGZF rows need no host copy); var_dev / var_n / var_device locate them
    // while var_ctx holds them (its next reduction of another batch, or its
    // destruction, makes the host copy first)
    mutable std::mutex var_mu;
    const void *var_dev = nullptr;
    size_t var_n = 0;
    int var_device = -1;
    struct ::tfbs_ctx *var_ctx = nullptr;
    bool var_host = true;   // var_counts holds the counts
    int var_err = 0;        // the host copy's failure, if any
    std::vector<DevVarKey> var_keys;      // the varying keys in reduction order
    std::vector<uint32_t> var_idx;        // key -> index in var_keys, UINT32_MAX unless it varies
    bool reduced = false;
    // device-side per-sample encoding of the varying keys of regions
    // [enc_r0, enc_r1) (tfbs_batch_encode): per encoded key (index in enc_key
    // order) its header, value table, per-value sample counts and codes;
    // enc_idx[var key index] = encoded key or UINT32_MAX
    uint32_t enc_r0 = 0, enc_r1 = 0;
    std::vector<uint32_t> enc_idx;
    std::vector<EncHdr> enc_hdr;
    std::vector<uint32_t> enc_vals, enc_hist;  // per encoded key its n_vals entries at enc_val_off[key]
    std::vector<uint32_t> enc_val_off;         // per encoded key, + the end
    PinnedBytes enc_codes;                     // packed codes of every encoded key, back to back
    bool enc_codes_host = true;                // enc_codes downloaded (not with TFBS_ENC_DEVICE_CODES)
    std::vector<uint64_t> enc_code_off;        // per encoded key, + the end

    std::vector<RegionH> rh;
    uint64_t windows = 0, eff_windows = 0, cell_ops = 0;
    // reference-window reuse (HAP_DEDUP, TFBS_DEDUP=0 turns it off): windows and
    // column lookups the scan executes (helper reference haplotypes included)
    bool dedup = true;
    bool dev_patch = true;   // device grouping + host patching of indel regions (TFBS_DEV_PATCH=0: off)
    uint64_t scan_windows = 0, scan_cell_ops = 0;
    // host prep seconds (tfbs_batch_prep_seconds): synthetic generation (thread
    // CPU-seconds), build_region (thread CPU-seconds), serial commit (wall), whole fill (wall)
    double prep_s[4] = {0, 0, 0, 0};

    // region under construction
    bool open = false;
    RegionH cur;
    std::vector<uint8_t> cur_ref;         // nucleotide codes of the fetched window
    std::vector<Record> cur_rec;
    std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> cur_inner;
    int status = TFBS_OK;

    // L_max of the halo-extended window (main.rs:404-407): the pattern set's
    // longest strand unless set wider (tfbs_batch_set_window_lmax: a shard of
    // the patterns keeps the whole set's windows, so its counts are the whole
    // run's for its pattern_ids)
    uint32_t window_lmax = 0;
    uint32_t lmax() const { return window_lmax ? window_lmax : pats->max_length(); }

    // device grouping of SNV-only regions (tfbs_batch_set_build_device, or one
    // grouper shared by a run's batches on a device); the batch's membership rows
    // (memb_allocs) go back to it when the batch goes
    std::shared_ptr<DevGrouper> grouper;
    std::vector<void *> memb_allocs;
    ~Batch() {
        if (grouper) grouper->recycle(memb_allocs);
    }
    uint64_t dev_regions = 0, host_regions = 0;  // regions grouped on the device / built on the host
    uint64_t patched_regions = 0;                // of dev_regions: distinct groups patched on the host

    uint64_t device_bytes() const;
};

enum KeyFlags : uint8_t { KEY_ANY = 1, KEY_VARIES = 2 };

struct RegionInput {  // one merged region as the reader hands it over
    RegionH R;                        // ms, me, es, ee set
    std::vector<uint8_t> ref;         // nucleotide codes from es
    std::vector<Record> recs;         // records in BCF order
    std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> inner;  // (bed, (s, e))
};

// A haplotype's positions (haplotype.rs's pos vector) as maximal runs of consecutive
// positions: run k covers bases [r[k].at, r[k + 1].at) (the last to n) at positions
// r[k].p, r[k].p + 1, ...  One run unless an indel breaks it, so a distinct haplotype
// holds ~1 byte per base instead of 9 (the batch build's first-touch page faults were
// most of a cold C5 build).  The runs are canonical (each starts where the previous
// one's positions stop being consecutive), so equal runs <=> equal position vectors.
struct PosRun {
    uint32_t at;
    uint64_t p;
    bool operator==(const PosRun &o) const { return at == o.at && p == o.p; }
};
struct PosRuns {
    std::vector<PosRun> r;
    uint32_t n = 0;  // positions
    bool extends(uint64_t p) const { return n && r.back().p + (n - r.back().at) == p; }
    void push(uint64_t p) {  // one position
        if (!extends(p)) r.push_back({n, p});
        n++;
    }
    void push_range(uint64_t lo, uint64_t hi) {  // positions lo ..= hi
        if (!extends(lo)) r.push_back({n, lo});
        n += (uint32_t)(hi - lo + 1);
    }
    static PosRuns affine(uint64_t start, size_t count) {  // start, start + 1, ...
        PosRuns x;
        if (count) x.push_range(start, start + count - 1);
        return x;
    }
    bool is_affine(uint64_t start) const { return n == 0 || (r.size() == 1 && r[0].p == start); }
    uint32_t end(size_t k) const { return k + 1 < r.size() ? r[k + 1].at : n; }
    template <class T, class F>
    void expand(T *out, F &&f) const {  // out[i] = f(position of base i)
        for (size_t k = 0; k < r.size(); k++)
            for (uint32_t i = r[k].at, e = end(k); i < e; i++) out[i] = f(r[k].p + (i - r[k].at));
    }
    bool operator==(const PosRuns &o) const { return n == o.n && r == o.r; }
};

struct Distinct {  // one distinct haplotype (a key of load_haplotypes' HashMap)
    std::vector<uint8_t> nuc;
    PosRuns pos;
    int32_t group;
};

struct RegionBuilt {
    RegionH R;
    std::vector<Distinct> dist;
    std::vector<uint32_t> carriers;
    bool helper = false;  // dist.back() is a helper reference haplotype (no carriers, no keys)
    // grouped on the device: distinct haplotype i is the reference window with the
    // SNVs of masks[i] (bit k = snv_rel[k] / snv_alt[k]; 0 = the reference group or
    // the helper); dist stays empty
    bool dev = false;
    // grouped on the device, patched on the host (regions with indels, N or diffs
    // outside the window): dist holds the patched groups, the membership row stays
    // on the device unless two groups patched to one sequence
    bool dev_grouped = false;
    std::vector<uint64_t> masks;
    std::vector<uint32_t> snv_rel;
    std::vector<uint8_t> snv_alt;
    std::vector<uint8_t> ref;
    size_t n_haps() const { return dev ? masks.size() : dist.size(); }
};

int build_region(const Batch &B, RegionInput &&in, RegionBuilt &out);
// Builds regions (on the device grouper where they qualify, see batch.cpp),
// `threads` host threads; *build_s (optional) += the host threads' seconds.
//
// Field ownership (tfbs_synth_fill_batch runs build_regions of chunk k + 1 while
// commit_regions of chunk k runs on another thread, TFBS_PREP_OVERLAP): build_regions
// writes only grouper, memb_allocs and the dev_ / host_ / patched_regions counters;
// commit_regions writes rh, regions, inner, haps, words, nmask, posrel, druns,
// hap_carriers, windows and the other scan / count totals.  Both only read the
// batch's configuration (n_samples, dedup, dev_patch, the patterns).  A field written
// by both would be a data race: keep the two sets disjoint
// (tests/test_capi_cpu.py::test_prep_overlap_same_batch checks the digests).
int build_regions(Batch &B, std::vector<RegionInput> &ins, uint32_t threads, std::vector<RegionBuilt> &built,
                  double *build_s);
// The region's nonref_id / nonref_local (fetched from the device if grouped there).
int region_membership(const Batch &B, const RegionH &R);
void commit_region(Batch &B, RegionBuilt &&built);
void commit_regions(Batch &B, std::vector<RegionBuilt> &built, uint32_t threads);
// Capacity for `factor` times the batch's current contents (a caller that knows how
// many more regions follow: no regrowth copies of the packed arrays).
void reserve_batch(Batch &B, double factor);
// The varying keys' counts of the last tfbs_batch_reduce on the host (downloaded on
// first use; thread-safe, idempotent); every host reader of var_counts calls it.
int ensure_host_var_counts(const Batch &B);
// A batch going away: its ctx forgets it as the holder of its device counts.
void forget_var_counts(Batch &B);
int add_regions(Batch &B, std::vector<RegionInput> &ins, uint32_t threads);
int make_record_gt(uint32_t n_samples, uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                   const int32_t *gt, Record &r);
// The same from a record whose carriers the BCF reader found while decoding it
// (Bcf::set_carriers_mode): gt_status is its ploidy check, raised here as
// make_record_gt would (after the allele count and the REF / ALT bases).
int make_record_ids(uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                    const std::vector<uint32_t> &carriers, int gt_status, Record &r);
int make_record_ids(uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                    std::vector<uint32_t> &&carriers, int gt_status, Record &r);  // (carriers moved in)

// haplotype.rs:94-156 over a reference window given as codes for positions
// [ref_start, ref_start + n_ref).  Diffs are pointers to records.
int patch(uint64_t rs, uint64_t re, std::vector<const Record *> diffs, const uint8_t *ref, uint64_t ref_start,
          size_t n_ref, std::vector<uint8_t> &nucs, std::vector<uint64_t> &pos);

}  // namespace tfbs

struct tfbs_batch {
    tfbs::Batch b;
};
