// Internal declarations shared by the host C++ and the HIP translation units.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/tfbs_amd.h"

namespace tfbs {

// Sets this thread's last-error message and returns code.
int fail(int code, const std::string &msg);

// util.rs:4-16 to_nucleotide: ASCII -> 0..4, or -1.
inline int to_nuc(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    case 'N': case 'n': return 4;
    default: return -1;
    }
}

// ---------------------------------------------------------------------------
// Device-side descriptors (POD, shared with the kernels).  All fields are
// 32-bit: the kernels read descriptors at wave-uniform addresses and gfx950
// scalar loads (s_load) exist only at dword granularity.
// ---------------------------------------------------------------------------
constexpr int kLutEntries = 256;   // one 4-mer block: 4^4 codes
constexpr int kBlockBytes = 4096;  // one table block: 256 codes x 16 bytes (one ds_read_b128 per lookup)
constexpr int kBlockInts = kBlockBytes / 4;
constexpr int kUnitMax = 8;        // strands per unit (octet)
constexpr int kFastMaxLen = 32;    // the LUT path reads a 64-bit (32-base) window per lane
constexpr int kMaxInnerPass = 8;   // inner ranges handled per pass (accumulators per lane)
constexpr int kMaxTileSlots = 64;  // pattern_id slots per tile: one lane each
constexpr uint32_t kMaxHapLen = 1u << 26;  // haplotype bases: window starts fit the window lists' 26-bit fields

enum UnitKind : uint32_t {
    // 8 strands, int16 partial sums biased to <= 0 per block, saturating packed adds:
    // hit iff sum > thr where thr = min_score - sum(block maxima) (exact, see plan)
    UNIT_OCTET16 = 0,
    // 4 strands, int32 partial sums (wrapping like the reference's i32)
    UNIT_QUAD32 = 1,
};

// A unit of strands scored together: their 4-mer tables are interleaved so one
// 16-byte LDS read returns every strand's partial sum for a code.
struct DevUnit {
    uint32_t lut_off;              // block offset inside the tile's LDS image
    uint32_t nblk;                 // max ceil(len / 4) over the strands
    uint32_t nstrand;              // real strands (the rest never match)
    uint32_t kind;                 // UnitKind
    uint32_t init[4];              // OCTET16: packed accumulator start -(thr + 1) per strand
    int32_t thr[kUnitMax];         // OCTET16: biased threshold; QUAD32: min_score
    int32_t min_score[kUnitMax];   // pattern.rs:151 threshold (windows containing N)
    uint32_t len[kUnitMax];
    uint32_t slot_local[kUnitMax]; // pattern_id slot relative to the tile's first slot
    uint32_t orig_index[kUnitMax]; // index in creation order (tfbs_matches)
    uint32_t wofs[kUnitMax];       // first column of the strand in the full weight table
};

struct DevPattern {        // one long strand (generic kernel)
    uint32_t col_off;      // offset of this pattern's columns in the generic weights (x5)
    int32_t min_score;
    uint32_t len;
    uint32_t slot_local;
    uint32_t orig_index;
    uint32_t pad;
};

struct DevTile {
    uint32_t first, last;         // unit range (fast) or pattern range (generic)
    uint32_t lut_begin;           // first block (global)
    uint32_t nblocks;             // blocks in the tile
    uint32_t slot_begin;          // global pattern_id slot of local slot 0
    uint32_t nslots;
    uint32_t lmin;                // shortest strand (bounds the windows to scan)
    uint32_t pad;
};

// Matrix-core path (scan_mfma.hip).  Each strand's weights are bounded above
// by C + s q per window (mfma.cpp): q <= 0 FP6 (e2m3) digits, s a per-strand
// scale, U = 8 Q an integer.  Two strands share one column of the
// v_mfma_scale_f32_32x32x64_f8f6f4 GEMM: the first's digits in K block 0, the
// second's in K block 1, whose A scale is 2^11, and the accumulator starts at
// 2^23 + (1023 - T0) (1 + 2^11).  Every output is then an integer in
// [2^23, 2^24) whose mantissa holds two 11-bit fields V = U + 1023 - T0, one
// per strand; a window is a candidate (U > T0, T0 the super tile's common
// threshold) iff its field's bit 10 is set, so one OR tree tests two strands
// per element.  Candidates are rescored exactly from the strand's weights.
// K chunk (64) = 2 strands x 8 columns x 4 bases: k = 32 h + 4 t + c <->
// strand 2 n + h, column 8 kc + t, base c.
constexpr int kMStrands = 64;      // strands per MFMA tile (32 columns of strand pairs)
constexpr int kMWindows = 32;      // windows per MFMA tile (the M dimension)
constexpr int kMChunkCols = 8;     // columns per strand per K chunk
constexpr int kMMaxChunks = 4;     // L <= 32
constexpr int kMSuperMaxTiles = 64;  // tiles per super tile (6 bits in a candidate entry)
// one strand tile of nk chunks in LDS: per chunk 64 lanes x 16 bytes (B dwords
// 0-3) and 64 lanes x 8 bytes (dwords 4-5)
constexpr inline uint32_t mfma_tile_bytes(uint32_t nk) { return nk * 1536; }
constexpr int kMFieldBits = 11;    // bits per strand field of an output
constexpr int kMFieldBias = 1023;  // V = U + kMFieldBias - T0: candidate iff V >= 1024
// The fields only the candidate rescoring reads live in global memory
// (Plan::m_meta, kGMetaInts per tile, strand sn = 2 n + h): min_score, offset of
// the exact weights (4 per column), len and slot at kGStrandInts * sn + field
// (one 16-byte load), the pattern index at kGOrig + sn.
enum MGMeta { kGMin = 0, kGWoff = 1, kGLen = 2, kGSlot = 3, kGStrandInts = 4, kGOrig = 256, kGDepth = 320 };
constexpr int kGMetaInts = 384;  // [kGDepth]: the tile's K depth (one int)

// The strand tiles one workgroup stages in LDS: tile_count tiles of K depth
// 1..nk (nk = 2 for tiles of depth 1-2, 4 for 3-4: one kernel, one A fragment
// build per window tile for each class), sorted by depth: byte seg d - 1 of
// `seg` = the first tile deeper than d; the tiles lie back to back, each
// mfma_tile_bytes(its depth); tile t's rescoring fields at
// Plan::m_meta[(tile0 + t) * kGMetaInts].  t0: the common candidate threshold
// of its strands' bounds (U > t0), acc0 the accumulator's start value
// 2^23 + (1023 - t0) (1 + 2^11) as f32 bits.
struct DevMSuper {
    uint32_t tile_count;
    uint32_t nk;        // the depth class: K chunks of the A fragments (2 or 4)
    uint32_t img_off;   // byte offset of the LDS image in Plan::m_image
    uint32_t img_bytes;
    int32_t t0;
    uint32_t lmin;      // shortest strand
    uint32_t tile0;     // global index of tile 0 (Plan::m_meta)
    uint32_t acc0;
    uint32_t seg;       // depth segment ends, one byte per depth
    uint32_t lmax;      // longest strand
    uint32_t pad[2];
};
constexpr inline uint32_t mfma_depth_class(uint32_t nk) { return nk <= 2 ? 2u : 4u; }

// HAP_REF: the region's reference haplotype (the reference group's, or a
// helper with no carriers after the region's distinct haplotypes); its
// matrix-core hits are listed for the reference-window reuse.  HAP_DEDUP: a
// haplotype of at most kDedupMaxWindows bases whose columns outside its
// *segments* (runs of columns equal to the reference column at their position,
// positions consecutive: the reference shifted by the indels before them;
// batch.cpp commit_regions) form at most kMaxDiffRuns runs (diff runs [a, b],
// inclusive, ascending, at DevHap::drun_off of the batch's run array; a run
// [a, a - 1] marks two touching segments).  Window i of a strand of length L is
// *dirty* iff some run meets its columns [i, i + L - 1]; every other window lies
// in one segment and has the bases and the start position of the reference
// window at i + its shift, so its hit (or none) is that window's, which the key
// assembly adds (key_kernels.hip, with the runs in the reference's columns:
// DevHap::rrun_off).  The matrix-core scan reads the windows dirty for the span
// S = the longest strand of their depth class (DevMSuper::lmax, or 8 nk when the
// class's span is not given; S >= L: a superset; the window list, scan_mfma.hip)
// and lists only the hits of windows dirty for the strand's L.
enum HapFlags : uint32_t { HAP_HAS_N = 1u, HAP_HAS_POS = 2u, HAP_REF = 4u, HAP_DEDUP = 8u };
constexpr uint32_t kDedupMaxWindows = 1024;  // longest HAP_DEDUP haplotype (and reference)
constexpr uint32_t kMaxDiffRuns = 16;        // diff runs of a HAP_DEDUP haplotype
constexpr uint32_t kRunToEnd = 0xFFFFFFFFu;  // a run's end past either sequence's end

struct DevHap {
    uint32_t word_off;   // packed 2-bit bases, 16 per u32, LSB first
    uint32_t len;        // bases
    uint32_t region;     // batch region index
    uint32_t flags;      // HapFlags
    uint32_t nmask_off;  // u32 words of the N mask (bit i = base i is N), if HAP_HAS_N
    uint32_t pos_off;    // int32 positions relative to ext_start, if HAP_HAS_POS
    uint64_t count_off;  // counts[count_off + (slot * n_inner + k) * DevRegion::count_stride]
    uint32_t drun_off;   // HAP_DEDUP: its diff runs, (a, b) u32 pairs at druns + 2 drun_off
    uint32_t n_druns;
    // HAP_DEDUP: the same runs in the reference's columns (the reference hits it
    // takes: key_kernels.hip); = drun_off / n_druns unless it has an indel
    uint32_t rrun_off;
    uint32_t n_rruns;
};

// Window w of span S (a strand's L, or a depth class's longest strand) is dirty for a
// haplotype with diff runs r (HAP_DEDUP): some run meets its columns [w, w + S - 1].
inline constexpr bool run_meets(uint32_t a, uint32_t b, uint32_t w, uint32_t S) { return a <= w + S - 1 && b >= w; }

struct DevRegion {
    uint32_t inner_off;  // into the inner (s_rel, e_rel) pair array
    uint32_t n_inner;    // distinct inner ranges
    uint32_t hap_begin;  // first distinct haplotype (their count blocks are consecutive)
    uint32_t hap_count;  // distinct haplotypes (a helper reference haplotype follows them)
    uint32_t ref_hap;    // the HAP_REF haplotype, UINT32_MAX if none
    // the region's counts are [key = slot * n_inner + range][haplotype]: a key's
    // counts for every haplotype of the region (the helper's included) are
    // consecutive, count_stride apart from the next key's
    uint32_t count_stride;
    // key assembly scratch (u32 counters) of a region with more distinct
    // haplotypes than the assembly's LDS block holds (key_kernels.hip)
    uint64_t big_off;
};

// Per-sample encoding of one varying key (tfbs_batch_encode, key_encode_kernel):
// v[s] = C[hap(2s)] + C[hap(2s+1)] over the samples (counts before the inner
// range's multiplicity), its min / max, the sorted distinct values (COUNTS=,
// main.rs:466-470) with their sample counts, and one u8 code per sample = the
// rank of v[s] among them, packed at 2, 4 or 8 bits.  status != 0: too many
// distinct values or too wide a
// range for the encoding -- the rows take the host path for that key.
struct EncHdr {
    uint32_t lo, hi, n_vals, status;
    uint32_t width;  // bits per code (2, 4 or 8): codes packed LSB first, n_samples * width / 8 bytes
};
constexpr uint32_t kEncMaxVals = 255;       // u8 codes
constexpr uint32_t kEncMaxRange = 1u << 16;  // value bitmap of hi - lo + 1 bits in LDS
constexpr uint32_t kEncMaxHaps = 65535;     // u16 membership: distinct haplotypes per region
constexpr uint32_t kEncMaxPairs = 8192;     // distinct (left, right) haplotype pairs per region (LDS)

// One key (region, slot * n_inner + range) whose distinct-haplotype counts differ;
// the gather copies its hap_count counts to out_off (tfbs_batch_reduce).
struct DevVarKey {
    uint32_t region;
    uint32_t j;
    uint64_t out_off;
};

}  // namespace tfbs
