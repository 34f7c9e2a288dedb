// Device context and the device-side C-ABI (tfbs_ctx_*, tfbs_batch_upload,
// tfbs_scan, tfbs_batch_download, tfbs_matches).  The kernels live in
// scan_kernels.hip; this file owns device memory, the stream and timing.
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "batch.hpp"
#include "bgzf_gpu.hpp"
#include "patterns.hpp"
#include "keys.hpp"
#include "rows.hpp"
#include "scan.hpp"
#include "tfbs_internal.hpp"

using namespace tfbs;

#define HIP_TRY(expr)                                                                                       \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return tfbs::fail(TFBS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));               \
    } while (0)

namespace {
template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;
    size_t n = 0;
    int ensure(size_t want) {
        n = want;
        if (want <= cap) return TFBS_OK;
        // geometric growth (hipFree waits for the device: a buffer regrown per call
        // would serialise the pipelined callers), the exact size if that fails
        size_t c = std::max<size_t>({want, cap + cap / 2, 16});
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, c * sizeof(T));
        if (e != hipSuccess && c > want) {
            (void)hipGetLastError();
            c = want;
            e = hipMalloc(&p, c * sizeof(T));
        }
        if (e != hipSuccess) return tfbs::fail(TFBS_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        cap = c;
        return TFBS_OK;
    }
    template <class Alloc>
    int put(const std::vector<T, Alloc> &v, hipStream_t s) {
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
    hipEvent_t evk0 = nullptr, evk1 = nullptr;  // around the dominant kernel (the MFMA launches)
    // the per-depth MFMA launches run on kSide + 1 streams so that they overlap
    static constexpr int kSide = 3;
    hipStream_t side[kSide] = {};
    hipEvent_t fork = nullptr, join[kSide] = {};
    hipEvent_t kf_fork = nullptr, kf_join = nullptr;  // the big-region key assembly on side[0]
    bool kernel_timed = false;
    float last_kernel_ms = 0.f;
    const Patterns *pats = nullptr;
    Plan plan;
    uint32_t tile_blocks = 20;    // table blocks (4 KiB each) per LDS tile: 80 KiB, two workgroups per CU
    uint32_t haps_per_block = 128;
    LaunchConfig cfg;
    DevBuf<DevUnit> fast_units;
    DevBuf<DevPattern> gen_pats;
    DevBuf<DevTile> fast_tiles, gen_tiles;
    DevBuf<int32_t> lut, wfull, gen_w, m_image, m_weights, m_meta;
    DevBuf<uint8_t> slot_mfma;           // Plan::slot_mfma
    DevBuf<uint32_t> cands;              // matrix-core candidate lists (scan.hpp)
    DevBuf<uint32_t> hitl, hitn;         // matrix-core hit lists (scan.hpp)
    DevBuf<uint32_t> candn;              // per wave: candidates found (tfbs_ctx_scan_counters)
    DevBuf<uint32_t> ref_hits, ref_count;  // reference-window reuse (scan.hpp)
    DevBuf<uint32_t> spill, over;        // spill records, [0] their count, [1] candidates past the wave lists
    uint32_t spill_cap = 1u << 16;
    DevBuf<uint32_t> spill_sorted, spill_bcnt, spill_boff;  // the spill records in region order
    DevBuf<uint32_t> cand_over;  // candidates past the waves' list regions (scan.hpp)
    uint32_t cand_over_cap = 1u << 20;
    // the last scan's overflow counters, copied back asynchronously (checked,
    // and the scan redone with larger lists, before its results are read)
    uint32_t *over_host = nullptr;       // pinned [spill records, candidates past the lists]
    hipEvent_t over_ev = nullptr;
    bool over_pending = false;
    bool over_copied = false;  // the last scan's overflow counters copied to over_host
    bool post_done = false;              // the last scan's overflow candidates were rescored (launch_post_scan)
    HitSrc srcs_host[kMaxHitSrcs] = {};
    HitSrc srcs_dev[kMaxHitSrcs] = {};   // what srcs holds (copied from here: stable while the copy runs)
    bool srcs_on_dev = false;
    ScanArgs last_margs{};               // the last matrix-core scan's arguments (launch_post_scan)
    uint32_t n_srcs = 0;
    DevBuf<HitSrc> srcs;
    bool debug_over = false;  // TFBS_DEBUG_OVER: print the overflow lists' fill after each check
    uint32_t n_regions = 0;                // of the resident batch
    uint32_t cand_cap = 1024;            // per scan workgroup (TFBS_CAND_CAP), per super tile it scans
    bool mfma_merged = true;             // TFBS_SCAN_MERGED=0: one launch per depth class (a workgroup per super tile)
    uint32_t scan_cand_cap = 1024;       // the last scan's list entries per workgroup (ScanArgs::cand_cap)
    DevBuf<DevMSuper> m_supers;
    bool mfma = true;             // int8 matrix-core path for eligible strands (TFBS_MFMA=0: LUT only)
    uint32_t mfma_lds = 44 * 1024;  // LDS image budget of one MFMA super tile
    uint32_t mfma_hpb = 64;         // haplotypes per MFMA workgroup
    uint32_t mfma_group_words = 0;  // packed words of the largest haplotype group (LDS staging)
    // batch image
    DevBuf<uint32_t> words, nmask, counts;  // counts: dense, for the LUT/generic slots (and tfbs_batch_download)
    bool counts_live = false;             // counts allocated for the resident batch
    DevBuf<int32_t> posrel, inner;
    DevBuf<DevHap> haps;
    DevBuf<uint32_t> druns;               // HAP_DEDUP haplotypes' diff runs
    // matrix-core window lists per depth class (ScanArgs::wlist), built at upload
    DevBuf<uint64_t> wl_off[2], wl_tmp;
    DevBuf<uint32_t> wl[2];
    DevBuf<uint16_t> wl16[2];  // the narrow groups' window lists
    DevBuf<uint8_t> gnarrow;   // per haplotype group of mfma_hpb: every haplotype <= kWlNarrowLen bases
    DevBuf<uint32_t> gorder;   // the merged scan's group order (most work first; TFBS_SCAN_LPT=0: none)
    DevBuf<uint32_t> gcost;    // (its per-group work estimates)
    bool wl_any_narrow = false, wl_any_wide = false;  // the resident batch has narrow / other groups
    DevBuf<uint4> hd, hd2;     // the matrix-core scan's compact haplotype descriptors
    uint64_t wl_entries[2] = {0, 0};
    double wl_seconds = 0;                // the last build's wall time
    DevBuf<DevRegion> regions;
    DevBuf<unsigned long long> hits;
    DevBuf<uint32_t> asm_scratch;         // key assembly counters of regions with many distinct haplotypes
    // key reduction (tfbs_batch_reduce)
    DevBuf<uint32_t> key_first, var_counts, asm_redo;   // asm_redo: the regions left to key_asm_kernel
    // the assembly's counters (one memset, one copy back): [0..1] the scan's spill /
    // candidate overflow counts (asm_report_kernel), [2] regions left, [3] the arena's
    // fill, [4..7] the varying keys and counts (u64), [8..15] give-up reasons (debug)
    DevBuf<uint32_t> asm_ctr;
    DevBuf<uint32_t> cor_arena;                          // key_fast_kernel's corrections past its LDS list
    uint32_t cor_cap = 1u << 22;
    DevBuf<uint8_t> key_flags;
    DevBuf<DevVarKey> var_keys, enc_keys;
    uint32_t var_keys_cap = 1u << 16;
    uint32_t key_fast_max_u = 1u << 30;  // TFBS_KEY_FAST_MAXU (0: every region through key_asm_kernel)
    uint32_t key_cor_lds = 1u << 30;     // TFBS_KEY_COR_LDS (0: every region's corrections in the arena)
    uint64_t var_cap = 1u << 24;
    bool var_cap_forced = false;     // TFBS_VAR_CAP applied (tfbs_batch_reduce)
    Batch *var_owner = nullptr;      // the batch whose varying counts are only in var_counts (device)
    uint32_t *asm_host = nullptr;  // asm_ctr copied back (pinned)
    bool asm_ctr_zeroed = false;   // launch_scan zeroed asm_ctr (for the scan's first assembly)
    hipEvent_t asm_ev = nullptr, asm_t0 = nullptr, asm_t1 = nullptr;
    const Batch *asm_batch = nullptr;    // the batch the enqueued assembly is for
    int asm_state = 0;                   // 0 none, 1 enqueued, 2 complete (checked)
    bool asm_timed = false;
    float last_asm_ms = 0.f;
    // per-sample encoding (tfbs_batch_encode)
    DevBuf<uint8_t> enc_codes, enc_packed;
    DevBuf<uint16_t> enc_pidx;            // per sample its haplotype pair
    DevBuf<uint32_t> enc_pab, enc_pcnt, enc_pair_n;  // per pair its distinct indices a | b << 16, its samples
    DevBuf<uint16_t> enc_memb;            // membership rows of host-built regions (u16 per haplotype id)
    DevBuf<uint32_t> enc_nr_ids, enc_nr_meta;  // host-built regions' non-reference ids, per row (offset, reference)
    DevBuf<uint16_t> enc_nr_loc;               // and their distinct indices (launch_memb_fill)
    DevBuf<uint64_t> enc_rows;            // per region the device address of its membership row
    tfbs::PinnedBytes enc_memb_host;  // host-built regions' membership rows staged for upload (reused)
    uint32_t host_threads = 16;      // host threads of tfbs_batch_encode (tfbs_ctx_set_host_threads)
    DevBuf<uint64_t> enc_off;
    DevBuf<EncHdr> enc_hdr;
    DevBuf<uint32_t> enc_vals, enc_hist;  // kEncMaxVals + 1 per key
    DevBuf<uint32_t> enc_vals_c, enc_hist_c, enc_val_off;  // compacted for the download
    // device BGZF rows (tfbs_batch_rows_bgzf)
    DevBuf<DevRow> bg_rows;
    DevBuf<char> bg_heads, bg_tok_text;
    DevBuf<uint8_t> bg_tok_len, bg_plans, bg_tok_litn;
    DevBuf<uint4> bg_tok_lit;
    DevBuf<uint32_t> bg_cum, bg_crc;  // bg_crc: byte table | shift operators
    DevBuf<uint64_t> bg_prof;         // TFBS_BGZF_PROF: bgzf_wave_kernel phase clocks
    uint32_t bg_crc_full = 0;         // bgzf_crc_tables' full-block CRC init term
    DevBuf<uint64_t> kf_prof;         // TFBS_KF_PROF: key_fast_kernel phase clocks and sizes per region
    DevBuf<uint32_t> bg_check;  // TFBS_BGZF_CHECK=1: the checked BGZF wave kernel's violation count
    DevBuf<unsigned long long> scan_prof;  // TFBS_SCAN_PROF=<file>: scan_mfma_kernel's per-wave stamps (prof builds)
    DevBuf<uint32_t> asm_order;       // the resident batch's regions by distinct haplotypes, most first
    uint32_t asm_order_n = 0;         // regions asm_order holds (0: none)
    uint32_t asm_order_big = 0;       // the first of them with more than key_fast_big_u() haplotypes
    bool kf_prof_on = false;
    bool kf_persistent = true;        // TFBS_KF_PERSIST=0: one workgroup per region
    // two slots of block batches (one being made, one copied back and written)
    static constexpr int kBgSlots = 3;  // batches of blocks in flight: two queued while one is written out
    DevBuf<uint8_t> bg_out[kBgSlots], bg_packed[kBgSlots];
    DevBuf<uint32_t> bg_out_len[kBgSlots];
    DevBuf<uint64_t> bg_off[kBgSlots];
    tfbs::PinnedBytes bg_host[kBgSlots];  // compressed blocks staged for the host
    uint64_t *bg_total_host = nullptr;  // pinned: each slot's packed bytes
    hipEvent_t bg_done[kBgSlots] = {}, bg_copied[kBgSlots] = {};
    hipStream_t copy_stream = nullptr;
    double rows_s[2] = {0, 0};            // tfbs_batch_rows_bgzf seconds: row plan (host), the rest
    double drain_s[3] = {0, 0, 0};        // of rows_s[1]: bgzf_drain's waits for the blocks, the copy back, the write
    // rows_set_async (the run flow's one-device path): a drained slot's blocks are
    // copied back and written by this ctx's writer thread, in order, while the caller
    // goes on; the slot's device buffers are reused once its copy is enqueued (the
    // stream waits for bg_copied), its host buffer once its write is done (rows_flush:
    // every write done)
    struct RowsWriter {
        std::thread th;
        std::mutex mu;
        std::condition_variable cv;
        struct Job {
            int fd, k;
            uint64_t n;
        };
        std::deque<Job> q, wq;                     // to copy back; copied, to write (in order)
        std::thread th2;                           // the writes (th: the copies back)
        bool copier_done = false;
        bool busy[3] = {false, false, false};      // a job of the slot is queued or running
        bool recorded[3] = {false, false, false};  // its copy back is enqueued (bg_copied[k] recorded)
        bool stop = false;
        int rc = 0;
        std::string err;
        double copy_s = 0, write_s = 0;
    } rw;
    bool rows_async = false;
    uint64_t rows_text_last = 0;          // the last call's uncompressed row bytes
    const tfbs_batch *resident = nullptr;
    bool scanned = false;                 // the resident batch has been scanned (its lists exist)
    float last_ms = 0.f;
    int last_launches = 0;
    bool timing_pending = false;
    // tfbs_step: one step's scan and assembly launches captured as a hipGraph and
    // replayed while the resident batch and every buffer they use stay as captured
    hipGraph_t step_graph = nullptr;
    hipGraphExec_t step_exec = nullptr;
    uint64_t step_sig = 0;       // step_signature() of the graph (or of the last plain step)
    bool step_sig_seen = false;  // the last plain step had step_sig: the next one is captured
    bool capturing = false;      // the timing events and asm_ev are left out of a capture
    uint64_t upload_gen = 0;     // tfbs_batch_upload calls (a new batch image: a new graph)
    bool step_graphs = true;     // TFBS_STEP_GRAPH=0: plain launches
    // lean assemblies: the wide spill bucketing and the leftover key pass are left out
    // when the batch's last assembly needed neither (C2 is launch-bound); the kernels
    // flag what they could not do and the wait reruns the assembly in full.
    // TFBS_ASM_LEAN: 0 never, 1 predicted (default), 2 always (the tests' rerun path)
    int asm_lean_mode = 1;
    uint32_t prev_spill = UINT32_MAX, prev_redo = UINT32_MAX;  // the last checked assembly's (unknown: max)
    uint32_t prev_cand = UINT32_MAX;                           // and its scan's candidates past the lists
    bool asm_wide = true, asm_leftover = true;                 // what the enqueued assembly launched
    bool asm_full = false;                                     // (a rerun: everything)
    // fused post-scan (ScanArgs::post_done): tfbs_step allows it for its lean steps
    // (TFBS_POST_FUSE=0: never); post_fused: the last scan did it (its assembly skips the launch)
    bool post_fuse_env = true, post_fuse_ok = false, post_fused = false;
};

namespace tfbs {
int PinnedBytes::reserve(size_t n) {
    if (n <= cap) return TFBS_OK;
    // geometric with headroom (page-locking is slow: ~5 ms per 20 MB; the BGZF slots' batches
    // vary 2x in size, and each regrowth stalled the GPU between a batch and its copy back).
    // (The old capacity is read before release() clears it: until round 6 it was read after,
    // so every growth was to the exact size.)
    size_t want = std::max<size_t>({n + n / 2, 2 * cap, (size_t)1 << 20});
    release();
    if (hipHostMalloc((void **)&p, want, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        want = n;  // the exact size, then pageable memory
        if (hipHostMalloc((void **)&p, want, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
        }
    }
    pinned = p != nullptr;
    if (!pinned) {  // page-locked memory exhausted: pageable memory (slower copies, same results)
        p = static_cast<uint8_t *>(malloc(want));
        if (!p) return tfbs::fail(TFBS_E_NOMEM, "host staging buffer");
    }
    cap = want;
    return TFBS_OK;
}
void PinnedBytes::release() {
    if (p) {
        if (pinned) (void)hipHostFree(p);
        else free(p);
    }
    p = nullptr;
    cap = 0;
}
PinnedBytes::~PinnedBytes() { release(); }

}  // namespace tfbs

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    if (!v || !*v) return dflt;
    return atoi(v);
}

// The matrix-core window lists of the haplotypes just put on the device (one
// per depth class the plan has; scan.hpp build_window_lists).
static int build_lists(tfbs_ctx *ctx, uint32_t n_haps, const std::vector<uint8_t> &narrow) {
    const Plan &P = ctx->plan;
    if (P.m_supers.empty()) return TFBS_OK;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t lmin[2] = {0, 0}, span[2] = {0, 0};  // per depth class: shortest and longest strand
    for (const DevMSuper &S : P.m_supers) {
        uint32_t &l = lmin[S.nk > 2 ? 1 : 0];
        l = l ? std::min(l, S.lmin) : S.lmin;
        span[S.nk > 2 ? 1 : 0] = std::max(span[S.nk > 2 ? 1 : 0], S.lmax);
    }
    int rc;
    for (int c = 0; c < 2; c++)
        if (lmin[c] && (rc = ctx->wl_off[c].ensure((size_t)n_haps + 1))) return rc;
    if ((rc = ctx->wl_tmp.ensure(scan_tmp_words((size_t)n_haps + 1))) ||
        (rc = ctx->druns.ensure(std::max<size_t>(ctx->druns.n, 1))))
        return rc;
    if ((rc = ctx->gnarrow.put(narrow, ctx->stream))) return rc;
    WindowListBufs bufs{};
    for (int c = 0; c < 2; c++) {
        bufs.off[c] = lmin[c] ? ctx->wl_off[c].p : nullptr;
        bufs.list[c] = nullptr;
        bufs.list16[c] = nullptr;
    }
    bufs.gnarrow = narrow.empty() ? nullptr : ctx->gnarrow.p;
    if ((rc = ctx->hd.ensure(std::max<uint32_t>(n_haps, 1))) || (rc = ctx->hd2.ensure(std::max<uint32_t>(n_haps, 1))))
        return rc;
    bufs.hd = ctx->hd.p;
    bufs.hd2 = ctx->hd2.p;
    bufs.scan_tmp = ctx->wl_tmp.p;
    // a group's entries are all in one of the two lists (16-bit: a narrow group), both
    // indexed by the same offsets: a list no group uses gets no room
    ctx->wl_any_narrow = ctx->wl_any_wide = false;
    for (uint8_t g : narrow) (g ? ctx->wl_any_narrow : ctx->wl_any_wide) = true;
    if (narrow.empty()) ctx->wl_any_wide = true;
    auto ensure = [](void *x, int c, uint64_t n, uint32_t **p, uint16_t **p16) {
        tfbs_ctx *cx = static_cast<tfbs_ctx *>(x);
        if (int e = cx->wl[c].ensure(cx->wl_any_wide ? n : 1)) return e;
        if (int e = cx->wl16[c].ensure(cx->wl_any_narrow ? n : 1)) return e;
        *p = cx->wl[c].p;
        *p16 = cx->wl16[c].p;
        return TFBS_OK;
    };
    if ((rc = build_window_lists(ctx->haps.p, n_haps, ctx->druns.p, lmin, span, ctx->mfma_hpb, 1, bufs, ctx->wl_entries,
                                 ctx->stream, ensure, ctx)))
        return rc;
    for (int c = 0; c < 2; c++)
        if (!lmin[c]) ctx->wl_off[c].release(), ctx->wl[c].release(), ctx->wl16[c].release();
    // The merged scan's workgroup order: groups by descending work (window pairs x the
    // per-pair MFMAs + rounds of each depth class's super tiles), so that the launch
    // ends on its smallest groups instead of a late large one (LPT).
    ctx->gorder.release();
    if (env_int("TFBS_SCAN_LPT", 1) && n_haps) {
        uint32_t w[2] = {0, 0};
        for (const DevMSuper &S : P.m_supers) {
            uint32_t prev = 0;
            for (uint32_t d = 1; d <= 4; d++) {
                const uint32_t e = (S.seg >> (8 * (d - 1))) & 255u;
                if (e > prev) w[S.nk > 2 ? 1 : 0] += (e - prev) * (2 * d + 1);
                prev = std::max(prev, e);
            }
        }
        const uint32_t hpb = ctx->mfma_hpb, ng = (n_haps + hpb - 1) / hpb;
        if ((rc = ctx->gcost.ensure(ng)) ||
            (rc = group_costs(lmin[0] ? ctx->wl_off[0].p : nullptr, lmin[1] ? ctx->wl_off[1].p : nullptr, n_haps, hpb,
                              w[0], w[1], ctx->gcost.p, ctx->stream)))
            return rc;
        std::vector<uint32_t> cost(ng), order(ng);
        HIP_TRY(hipMemcpyAsync(cost.data(), ctx->gcost.p, (size_t)ng * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        for (uint32_t g = 0; g < ng; g++) order[g] = g;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
        if ((rc = ctx->gorder.put(order, ctx->stream))) return rc;
        HIP_TRY(hipStreamSynchronize(ctx->stream));  // (order is copied from the host's stack)
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->wl_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return TFBS_OK;
}

// asm_ctr's counter words (layout at enqueue_assembly), the spill buckets after them
constexpr size_t kAsmCtrWords = 24;

// The scan's counters (reference hits per region, the overflow pair) and the
// assembly's (asm_ctr) zeroed in one launch at the scan's start, instead of three
// memsets on either side of it (C2 is launch-bound).
__global__ void zero3_kernel(uint32_t *__restrict__ a, uint32_t na, uint32_t *__restrict__ b, uint32_t nb,
                             uint32_t *__restrict__ c, uint32_t nc) {
    const uint32_t s = gridDim.x * blockDim.x;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < na || k < nb || k < nc; k += s) {
        if (k < na) a[k] = 0;
        if (k < nb) b[k] = 0;
        if (k < nc) c[k] = 0;
    }
}

static int launch_scan(tfbs_ctx *ctx, uint32_t n_haps, unsigned long long *hits, uint32_t hits_wpp) {
    const Plan &P = ctx->plan;
    if (n_haps == 0) return 0;
    ScanArgs a{};
    a.haps = ctx->haps.p;
    a.n_haps = n_haps;
    a.hap_base = 0;
    a.regions = ctx->regions.p;
    a.inner = ctx->inner.p;
    a.words = ctx->words.p;
    a.nmask = ctx->nmask.p;
    a.posrel = ctx->posrel.p;
    a.counts = ctx->counts_live ? ctx->counts.p : nullptr;
    a.haps_per_block = ctx->haps_per_block;
    a.hits = hits;
    a.hits_wpp = hits_wpp;
    a.n_patterns_total = (uint32_t)ctx->pats->pats.size();
    int launches = 0;
    ctx->n_srcs = 0;
    if (!P.m_supers.empty()) {  // sparse hits: no count matrix to zero
        ScanArgs m = a;
        m.msupers = ctx->m_supers.p;
        m.n_msupers = (uint32_t)P.m_supers.size();
        m.mimage = ctx->m_image.p;
        m.mweights = ctx->m_weights.p;
        m.mmeta = ctx->m_meta.p;
        m.haps_per_block = ctx->mfma_hpb;
        // one candidate list and one hit list per scan workgroup (super tile x haplotype
        // group; merged: one workgroup per group scans every super tile, its lists hold
        // their candidates)
        const uint64_t n_groups = (n_haps + ctx->mfma_hpb - 1) / ctx->mfma_hpb;
        const uint64_t n_wg = ctx->mfma_merged ? n_groups : (uint64_t)P.m_supers.size() * n_groups;
        const uint32_t cand_cap = ctx->mfma_merged
                                      ? (uint32_t)std::min<uint64_t>(1u << 16, (uint64_t)ctx->cand_cap * P.m_supers.size())
                                      : ctx->cand_cap;
        int rc;
        if ((rc = ctx->cands.ensure(n_wg * cand_cap * kCandWords)) || (rc = ctx->hitl.ensure(n_wg * cand_cap * 2)) ||
            (rc = ctx->hitn.ensure(n_wg * (kMBlockWaves))) || (rc = ctx->candn.ensure(n_wg * (kMBlockWaves))))
            return rc;
        m.cands = ctx->cands.p;
        m.cand_cap = cand_cap;
        ctx->scan_cand_cap = cand_cap;
        m.hitl = ctx->hitl.p;
        m.hitn = ctx->hitn.p;
        m.candn = ctx->candn.p;
        const uint32_t nr = std::max<uint32_t>(1, ctx->n_regions);
        if ((rc = ctx->ref_count.ensure(nr)) || (rc = ctx->ref_hits.ensure((size_t)nr * kRefPerRegion * 2)) ||
            (rc = ctx->over.ensure(2)) || (rc = ctx->spill.ensure((size_t)ctx->spill_cap * 3)) ||
            (rc = ctx->cand_over.ensure((size_t)ctx->cand_over_cap * 3)) ||
            (rc = ctx->spill_sorted.ensure((size_t)ctx->spill_cap * 3)) || (rc = ctx->spill_bcnt.ensure(nr + 1)) ||
            (rc = ctx->spill_boff.ensure(nr + 1)))
            return rc;
        m.dedup = 1;
        m.gnarrow = ctx->gnarrow.n ? ctx->gnarrow.p : nullptr;
        m.gorder = ctx->mfma_merged && ctx->gorder.n ? ctx->gorder.p : nullptr;
        m.hd = ctx->hd.p;
        m.hd2 = ctx->hd2.p;
        m.druns = ctx->druns.p;
        m.n_regions = ctx->n_regions;
        m.ref_hits = ctx->ref_hits.p;
        m.ref_count = ctx->ref_count.p;
        m.spill = ctx->spill.p;
        m.over = ctx->over.p;
        m.spill_cap = ctx->spill_cap;
        m.cand_over = ctx->cand_over.p;
        m.cand_over_cap = ctx->cand_over_cap;
        static const char *prof_path = getenv("TFBS_SCAN_PROF");
        if (prof_path && *prof_path) {
            if ((rc = ctx->scan_prof.ensure(n_wg * kMBlockWaves * kScanProfWords))) return rc;
            HIP_TRY(hipMemsetAsync(ctx->scan_prof.p, 0, ctx->scan_prof.n * 8, ctx->stream));
            m.prof = ctx->scan_prof.p;
        }
        for (int c = 0; c < 2; c++) {
            m.wlist[c] = ctx->wl[c].p;
            m.wlist16[c] = ctx->wl16[c].p;
            m.wlist_off[c] = ctx->wl_off[c].p;
        }
        {
            const uint32_t na = (uint32_t)(kAsmCtrWords + nr + 1);
            if ((rc = ctx->asm_ctr.ensure(na))) return rc;
            hipLaunchKernelGGL(zero3_kernel, dim3(std::min<uint32_t>(256, (std::max(na, nr) + 255) / 256)), dim3(256), 0,
                               ctx->stream, ctx->ref_count.p, nr, ctx->over.p, 2u, ctx->asm_ctr.p, na);
            HIP_TRY(hipGetLastError());
            ctx->asm_ctr_zeroed = true;  // (for this scan's first assembly)
        }
        // the post-scan work in the scan's last workgroup when the assembly that follows
        // (tfbs_step) would launch it lean: neither the grid-wide bucketing nor overflow
        // candidates last time (it handles both anyway: too many spill records set
        // need_wide, and the assembly reruns with the wide kernels)
        ctx->post_fused = ctx->post_fuse_ok && ctx->post_fuse_env && ctx->mfma_merged && ctx->asm_lean_mode != 0 &&
                          !ctx->asm_full && (ctx->asm_lean_mode == 2 || ctx->prev_spill <= kPostSerial) &&
                          ctx->prev_cand == 0;
        if (ctx->post_fused) {
            m.post_done = ctx->asm_ctr.p + 21;
            m.post_regions = nr;
            m.post_bcnt = ctx->asm_ctr.p + kAsmCtrWords;
            m.post_boff = ctx->spill_boff.p;
            m.post_sorted = ctx->spill_sorted.p;
            m.post_report = ctx->asm_ctr.p;
            m.post_need_wide = ctx->asm_ctr.p + 20;
        }
        if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->evk0, ctx->stream));
        // one stream per depth launch (launch_mfma: one per K depth), side streams
        // forked and joined only when there is more than one (small batches: no
        // cross-stream waits)
        int n_depths = 0;
        for (size_t k = 0; k < P.m_supers.size(); k++)
            n_depths += (k == 0 || P.m_supers[k].nk != P.m_supers[k - 1].nk) ? 1 : 0;
        if (ctx->mfma_merged) n_depths = 1;  // one launch
        const int n_side = std::min(n_depths - 1, (int)tfbs_ctx::kSide);
        hipStream_t streams[tfbs_ctx::kSide + 1] = {ctx->stream};
        if (n_side > 0) HIP_TRY(hipEventRecord(ctx->fork, ctx->stream));
        for (int i = 0; i < n_side; i++) {
            HIP_TRY(hipStreamWaitEvent(ctx->side[i], ctx->fork, 0));
            streams[i + 1] = ctx->side[i];
        }
        const int n = ctx->mfma_merged
                          ? launch_mfma_all(m, P.m_supers.data(), (uint32_t)P.m_supers.size(), ctx->mfma_group_words,
                                            n_haps, ctx->stream, ctx->srcs_host, &ctx->n_srcs)
                          : launch_mfma(m, P.m_supers.data(), (uint32_t)P.m_supers.size(), ctx->mfma_group_words,
                                        n_haps, streams, (uint32_t)n_side + 1, ctx->srcs_host, &ctx->n_srcs);
        if (n < 0) return n;
        for (int i = 0; i < n_side; i++) {
            HIP_TRY(hipEventRecord(ctx->join[i], ctx->side[i]));
            HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->join[i], 0));
        }
        if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->evk1, ctx->stream));
        ctx->kernel_timed = true;
        launches += n;
        if (m.prof) {  // (profiling runs only) the stamps, appended to the file: launches, then the waves
            std::vector<unsigned long long> h(ctx->scan_prof.n);
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            HIP_TRY(hipMemcpy(h.data(), ctx->scan_prof.p, h.size() * 8, hipMemcpyDeviceToHost));
            if (FILE *f = fopen(prof_path, "ab")) {
                unsigned long long hdr[2] = {ctx->n_srcs, h.size()};
                fwrite(hdr, 8, 2, f);
                for (uint32_t i = 0; i < ctx->n_srcs; i++) {
                    const HitSrc &q = ctx->srcs_host[i];
                    unsigned long long v[5] = {q.wg_base, q.ns, q.g0, q.ng, i};  // launches: deepest class first
                    fwrite(v, 8, 5, f);
                }
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
        ctx->last_margs = m;  // the overflow candidates are rescored when the results are read (check_overflow)
        ctx->post_done = false;
        if ((rc = ctx->srcs.ensure(kMaxHitSrcs))) return rc;
        if (!ctx->srcs_on_dev || memcmp(ctx->srcs_dev, ctx->srcs_host, sizeof(ctx->srcs_host)) != 0) {
            // (a rescan of the same batch launches the same workgroups: no copy)
            memcpy(ctx->srcs_dev, ctx->srcs_host, sizeof(ctx->srcs_host));
            HIP_TRY(hipMemcpyAsync(ctx->srcs.p, ctx->srcs_dev, sizeof(ctx->srcs_dev), hipMemcpyHostToDevice,
                                   ctx->stream));
            ctx->srcs_on_dev = true;
        }
        // the overflow counters are checked before the results are read: by the
        // assembly's list pass, or by check_overflow (which copies them back first)
        ctx->over_pending = true;
        ctx->over_copied = false;
    }
    if (!P.fast_tiles.empty()) {
        ScanArgs f = a;
        f.tiles = ctx->fast_tiles.p;
        f.n_tiles = (uint32_t)P.fast_tiles.size();
        f.units = ctx->fast_units.p;
        f.lut = ctx->lut.p;
        f.wfull = ctx->wfull.p;
        const int n = launch_fast(f, ctx->cfg, n_haps, ctx->stream);
        if (n < 0) return n;
        launches += n;
    }
    if (!P.gen_tiles.empty()) {
        ScanArgs g = a;
        g.tiles = ctx->gen_tiles.p;
        g.n_tiles = (uint32_t)P.gen_tiles.size();
        g.gpats = ctx->gen_pats.p;
        g.gw = ctx->gen_w.p;
        const int n = launch_generic(g, n_haps, ctx->stream);
        if (n < 0) return n;
        launches += n;
    }
    return launches;
}

// The last scan's overflow lists must have held every entry (a dropped
// candidate may hide a hit, a dropped spill record is a lost count): read the
// counters copied back after it and, if one overflowed, grow the lists and scan
// again.  Then the candidates past the waves' lists are rescored (their hits
// join the spill list) and the spill records bucketed by region -- work only
// when there is any.  Runs before anything reads the scan's results.
static int check_overflow(tfbs_ctx *ctx, uint32_t n_haps, unsigned long long *hits = nullptr, uint32_t wpp = 0) {
    auto grow = [](uint32_t &cap, uint32_t need, uint64_t lim) {
        if (need > cap) cap = (uint32_t)std::min<uint64_t>(lim, (uint64_t)need * 5 / 4 + 1024);
    };
    for (int round = 0; ctx->over_pending; round++) {
        if (round == 8) return tfbs::fail(TFBS_E_NOMEM, "scan overflow lists still full after 8 rescans");
        if (!ctx->over_copied) {  // (the scan's counters: nothing after it on the stream changes them)
            if (!ctx->over_host) HIP_TRY(hipHostMalloc((void **)&ctx->over_host, 8, hipHostMallocDefault));
            HIP_TRY(hipMemcpyAsync(ctx->over_host, ctx->over.p, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipEventRecord(ctx->over_ev, ctx->stream));
            ctx->over_copied = true;
        }
        HIP_TRY(hipEventSynchronize(ctx->over_ev));
        uint32_t nspill = ctx->over_host[0];
        const uint32_t ncand = ctx->over_host[1];
        if (ncand > 0 && ncand <= ctx->cand_over_cap && !ctx->post_done) {  // rescore them: their hits add spill records
            const int f = launch_post_scan(ctx->last_margs, ctx->stream);
            if (f < 0) return f;
            HIP_TRY(hipMemcpyAsync(ctx->over_host, ctx->over.p, 8, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            nspill = ctx->over_host[0];
        }
        if (ctx->debug_over) {
            fprintf(stderr, "tfbs_scan overflow lists: spill %u/%u candidates %u/%u\n", nspill, ctx->spill_cap, ncand,
                    ctx->cand_over_cap);
            // the hits of the scan workgroups' lists
            const size_t nw = ctx->hitn.n;
            std::vector<uint32_t> hn(nw);
            HIP_TRY(hipMemcpy(hn.data(), ctx->hitn.p, nw * 4, hipMemcpyDeviceToHost));
            uint64_t sh = 0, mh = 0;
            for (size_t i = 0; i < nw; i++) sh += hn[i], mh = std::max<uint64_t>(mh, hn[i]);
            fprintf(stderr, "tfbs_scan hit pairs %llu (max per wave %llu) over %zu waves\n", (unsigned long long)sh,
                    (unsigned long long)mh, nw);
        }
        if (nspill <= ctx->spill_cap && ncand <= ctx->cand_over_cap) {
            ctx->over_pending = false;
            ctx->post_done = true;
            if (nspill) {
                const uint32_t nr = std::max<uint32_t>(1, ctx->n_regions);
                const int rc = launch_spill_buckets(ctx->over.p, ctx->spill_cap, ctx->spill.p, nr, ctx->spill_bcnt.p,
                                                    ctx->spill_boff.p, ctx->spill_sorted.p, ctx->stream);
                if (rc) return rc;
            }
            return TFBS_OK;
        }
        grow(ctx->spill_cap, ncand > ctx->cand_over_cap ? 2 * std::max(nspill, 1024u) : nspill, UINT32_MAX / 4);
        grow(ctx->cand_over_cap, ncand, UINT32_MAX / 4);
        const int n = launch_scan(ctx, n_haps, hits, wpp);
        if (n < 0) return n;
    }
    return TFBS_OK;
}

static int assembly_wait(tfbs_ctx *ctx, Batch &B);

static AsmArgs asm_args(tfbs_ctx *ctx, const Batch &B, int mode) {
    AsmArgs a{};
    a.haps = ctx->haps.p;
    a.druns = ctx->druns.p;
    a.regions = ctx->regions.p;
    a.inner = ctx->inner.p;
    a.mmeta = ctx->m_meta.p;
    a.slot_mfma = ctx->slot_mfma.p;
    a.any_dense = (!ctx->plan.fast_tiles.empty() || !ctx->plan.gen_tiles.empty()) ? 1 : 0;
    a.n_slots = B.n_slots;
    a.hpb = ctx->mfma_hpb;
    a.hitl = ctx->hitl.p;
    a.hitn = ctx->hitn.p;
    a.cand_cap = ctx->scan_cand_cap;
    a.srcs = ctx->srcs.p;
    a.mfma = ctx->plan.m_supers.empty() ? 0 : 1;
    a.n_srcs = a.mfma ? ctx->n_srcs : 0;
    a.ref_hits = ctx->ref_hits.p;
    a.ref_count = ctx->ref_count.p;
    a.spill_sorted = ctx->spill_sorted.p;
    a.spill_off = ctx->spill_boff.p;
    a.spill_count = ctx->plan.m_supers.empty() ? nullptr : ctx->over.p;
    a.spill_cap = ctx->spill_cap;
    a.counts = ctx->counts_live ? ctx->counts.p : nullptr;
    a.dense_base = ctx->counts_live ? 1 : 0;
    a.scratch = ctx->asm_scratch.p;
    a.mode = mode;
    return a;
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
    if (ctx->rw.th.joinable()) {  // the jobs still queued go out first
        {
            std::lock_guard<std::mutex> l(ctx->rw.mu);
            ctx->rw.stop = true;
        }
        ctx->rw.cv.notify_all();
        ctx->rw.th.join();
        if (ctx->rw.th2.joinable()) ctx->rw.th2.join();
    }
    if (ctx->var_owner) {  // its varying counts to the host before var_counts goes
        (void)tfbs::ensure_host_var_counts(*ctx->var_owner);
        std::lock_guard<std::mutex> g(ctx->var_owner->var_mu);
        if (ctx->var_owner->var_ctx == ctx) ctx->var_owner->var_ctx = nullptr;
        ctx->var_owner = nullptr;
    }
    ctx->fast_units.release(); ctx->gen_pats.release(); ctx->fast_tiles.release(); ctx->gen_tiles.release();
    ctx->lut.release(); ctx->wfull.release(); ctx->gen_w.release(); ctx->slot_mfma.release();
    ctx->m_image.release(); ctx->m_weights.release(); ctx->m_meta.release(); ctx->m_supers.release();
    ctx->cands.release(); ctx->hitl.release(); ctx->hitn.release(); ctx->candn.release(); ctx->cand_over.release(); ctx->ref_hits.release();
    ctx->ref_count.release(); ctx->spill.release(); ctx->over.release(); ctx->spill_sorted.release();
    ctx->spill_bcnt.release(); ctx->spill_boff.release(); ctx->srcs.release();
    if (ctx->over_host) (void)hipHostFree(ctx->over_host);
    if (ctx->asm_host) (void)hipHostFree(ctx->asm_host);
    if (ctx->asm_ev) (void)hipEventDestroy(ctx->asm_ev);
    if (ctx->asm_t0) (void)hipEventDestroy(ctx->asm_t0);
    if (ctx->asm_t1) (void)hipEventDestroy(ctx->asm_t1);
    ctx->words.release(); ctx->nmask.release(); ctx->counts.release(); ctx->posrel.release();
    ctx->druns.release(); ctx->wl_tmp.release();
    for (int c = 0; c < 2; c++) ctx->wl_off[c].release(), ctx->wl[c].release(), ctx->wl16[c].release();
    ctx->gnarrow.release();
    ctx->gorder.release();
    ctx->gcost.release();
    ctx->hd.release();
    ctx->hd2.release();
    ctx->inner.release(); ctx->haps.release(); ctx->regions.release(); ctx->hits.release(); ctx->asm_scratch.release();
    ctx->key_first.release(); ctx->var_counts.release(); ctx->asm_ctr.release(); ctx->key_flags.release();
    ctx->asm_redo.release(); ctx->cor_arena.release();
    ctx->var_keys.release();
    ctx->enc_keys.release(); ctx->enc_pidx.release(); ctx->enc_pab.release(); ctx->enc_pcnt.release();
    ctx->enc_pair_n.release(); ctx->enc_memb.release(); ctx->enc_nr_ids.release(); ctx->enc_nr_meta.release();
    ctx->enc_nr_loc.release(); ctx->enc_rows.release(); ctx->enc_codes.release();
    ctx->enc_hdr.release();
    ctx->enc_vals.release(); ctx->enc_hist.release(); ctx->enc_packed.release(); ctx->enc_off.release();
    ctx->enc_vals_c.release(); ctx->enc_hist_c.release(); ctx->enc_val_off.release();
    ctx->bg_rows.release(); ctx->bg_heads.release(); ctx->bg_tok_text.release(); ctx->bg_tok_len.release();
    ctx->bg_tok_lit.release(); ctx->bg_tok_litn.release();
    ctx->bg_cum.release(); ctx->bg_crc.release(); ctx->bg_plans.release(); ctx->bg_prof.release(); ctx->kf_prof.release(); ctx->asm_order.release();
    for (int k = 0; k < tfbs_ctx::kBgSlots; k++) {
        ctx->bg_out[k].release(); ctx->bg_packed[k].release(); ctx->bg_out_len[k].release(); ctx->bg_off[k].release();
        ctx->bg_host[k].release();
        if (ctx->bg_done[k]) (void)hipEventDestroy(ctx->bg_done[k]);
        if (ctx->bg_copied[k]) (void)hipEventDestroy(ctx->bg_copied[k]);
    }
    if (ctx->bg_total_host) (void)hipHostFree(ctx->bg_total_host);
    if (ctx->copy_stream) {
        (void)hipStreamSynchronize(ctx->copy_stream);
        (void)hipStreamDestroy(ctx->copy_stream);
    }
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->evk0) (void)hipEventDestroy(ctx->evk0);
    if (ctx->evk1) (void)hipEventDestroy(ctx->evk1);
    if (ctx->over_ev) (void)hipEventDestroy(ctx->over_ev);
    for (int i = 0; i < tfbs_ctx::kSide; i++) {
        if (ctx->side[i]) (void)hipStreamSynchronize(ctx->side[i]);
        if (ctx->side[i]) (void)hipStreamDestroy(ctx->side[i]);
        if (ctx->join[i]) (void)hipEventDestroy(ctx->join[i]);
    }
    if (ctx->step_exec) (void)hipGraphExecDestroy(ctx->step_exec);
    if (ctx->step_graph) (void)hipGraphDestroy(ctx->step_graph);
    if (ctx->fork) (void)hipEventDestroy(ctx->fork);
    if (ctx->kf_fork) (void)hipEventDestroy(ctx->kf_fork);
    if (ctx->kf_join) (void)hipEventDestroy(ctx->kf_join);
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
    ctx->tile_blocks = (uint32_t)std::min(36, std::max(8, env_int("TFBS_TILE_BLOCKS", 20)));
    ctx->haps_per_block = (uint32_t)std::max(8, env_int("TFBS_HAPS_PER_BLOCK", 128));
    ctx->cfg.minw = env_int("TFBS_FAST_MINW", 2) == 4 ? 4 : 2;
    ctx->mfma = env_int("TFBS_MFMA", 1) != 0;
    ctx->mfma_lds = (uint32_t)std::min(144, std::max(8, env_int("TFBS_MFMA_LDS_KB", 44))) * 1024u;
    ctx->mfma_hpb = (uint32_t)std::min((int)kMMaxHapsPerBlock, std::max(4, env_int("TFBS_MFMA_HAPS_PER_BLOCK", 64)));  // 6 bits in a window list entry
    ctx->cand_cap = (uint32_t)std::min(1 << 16, std::max(64, env_int("TFBS_CAND_CAP", 1024)));
    ctx->mfma_merged = env_int("TFBS_SCAN_MERGED", 1) != 0;
    ctx->debug_over = env_int("TFBS_DEBUG_OVER", 0) != 0;
    ctx->kf_prof_on = env_int("TFBS_KF_PROF", 0) != 0;
    ctx->kf_persistent = env_int("TFBS_KF_PERSIST", 1) != 0;
    ctx->asm_lean_mode = env_int("TFBS_ASM_LEAN", 1);
    ctx->post_fuse_env = env_int("TFBS_POST_FUSE", 0) != 0;  // (measured: C2 0.083 vs 0.068 ms -- a ticket atomic per scan workgroup)
    ctx->step_graphs = env_int("TFBS_STEP_GRAPH", 1) != 0 && !getenv("TFBS_SCAN_PROF") && !ctx->kf_prof_on &&
                       !ctx->debug_over;
    ctx->key_fast_max_u = (uint32_t)std::max(0, env_int("TFBS_KEY_FAST_MAXU", 1 << 30));
    ctx->key_cor_lds = (uint32_t)std::max(0, env_int("TFBS_KEY_COR_LDS", 1 << 30));
    ctx->cor_cap = (uint32_t)std::max(1, env_int("TFBS_KEY_COR_CAP", 1 << 22));
    ctx->host_threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    ctx->cand_over_cap = (uint32_t)std::max(1, env_int("TFBS_CAND_OVER_CAP", 1 << 20));  // grows on demand (tfbs_scan)
    PlanOptions opt;
    opt.tile_blocks = ctx->tile_blocks;
    opt.mfma = ctx->mfma;
    opt.mfma_lds_bytes = ctx->mfma_lds;
    if (env_int("TFBS_MFMA_LDS_BY_DEPTH", 0)) mfma_depth_budgets(opt.mfma_lds_by_nk);
    rc = ctx->pats->build_plan(opt, &ctx->plan);
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
    if (e == hipSuccess) e = hipEventCreate(&ctx->evk0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->evk1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->kf_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->kf_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->over_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->asm_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreate(&ctx->asm_t0);
    if (e == hipSuccess) e = hipEventCreate(&ctx->asm_t1);
    for (int i = 0; i < tfbs_ctx::kSide; i++) {
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->side[i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->join[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_HIP, std::string("HIP init: ") + hipGetErrorString(e));
    }
    const Plan &P = ctx->plan;
    ctx->cfg.lds_bytes = (size_t)P.max_tile_blocks * kBlockBytes;
    if (ctx->cfg.lds_bytes > 160 * 1024) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_ARG, "pattern tile exceeds the 160 KiB LDS");
    }
    if (P.max_super_bytes + mfma_lds_fixed() > 160 * 1024) {
        tfbs_ctx_destroy(ctx);
        return tfbs::fail(TFBS_E_ARG, "MFMA super tile exceeds the 160 KiB LDS");
    }
    if ((rc = fast_kernel_set_lds(ctx->cfg))) {
        tfbs_ctx_destroy(ctx);
        return rc;
    }
    if ((rc = ctx->fast_units.put(P.fast_units, ctx->stream)) || (rc = ctx->fast_tiles.put(P.fast_tiles, ctx->stream)) ||
        (rc = ctx->lut.put(P.lut, ctx->stream)) || (rc = ctx->wfull.put(P.wfull, ctx->stream)) ||
        (rc = ctx->gen_pats.put(P.gen_pats, ctx->stream)) || (rc = ctx->gen_tiles.put(P.gen_tiles, ctx->stream)) ||
        (rc = ctx->gen_w.put(P.gen_w, ctx->stream)) || (rc = ctx->m_image.put(P.m_image, ctx->stream)) ||
        (rc = ctx->m_weights.put(P.m_weights, ctx->stream)) || (rc = ctx->m_meta.put(P.m_meta, ctx->stream)) ||
        (rc = ctx->m_supers.put(P.m_supers, ctx->stream)) || (rc = ctx->slot_mfma.put(P.slot_mfma, ctx->stream))) {
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

int tfbs_ctx_set_host_threads(tfbs_ctx *ctx, uint32_t threads) {
    if (!ctx || threads == 0) return tfbs::fail(TFBS_E_ARG, "null ctx or zero threads");
    ctx->host_threads = threads;
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
            ms = 0.f;
            if (c->kernel_timed && hipEventElapsedTime(&ms, c->evk0, c->evk1) == hipSuccess) c->last_kernel_ms = ms;
        }
        c->timing_pending = false;
    }
    return c->last_ms;
}

int tfbs_ctx_last_scan_launches(const tfbs_ctx *ctx) { return ctx ? ctx->last_launches : 0; }

int tfbs_ctx_rows_bgzf_seconds(const tfbs_ctx *ctx, double *out) {
    if (!ctx || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    out[0] = ctx->rows_s[0];
    out[1] = ctx->rows_s[1];
    return TFBS_OK;
}

int tfbs_ctx_scan_counters(tfbs_ctx *ctx, uint64_t out[5]) {
    if (!ctx || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    for (int i = 0; i < 5; i++) out[i] = 0;
    if (!ctx->over.p || !ctx->candn.p || !ctx->hitn.p || !ctx->scan_cand_cap) return TFBS_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    const size_t nw = std::min(ctx->hitn.n, ctx->candn.n);
    std::vector<uint32_t> hn(nw), cn(nw);
    uint32_t ov[2];
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(hn.data(), ctx->hitn.p, nw * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(cn.data(), ctx->candn.p, nw * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(ov, ctx->over.p, sizeof ov, hipMemcpyDeviceToHost));
    const uint64_t cap = ctx->scan_cand_cap / kMBlockWaves, lcap = std::min<uint64_t>(cap, kMWaveCands);
    out[0] = ov[0];
    out[1] = ov[1];
    for (size_t i = 0; i < nw; i++) {  // (the waves of every workgroup the last scan launched)
        out[2] += cn[i];
        out[3] += cn[i] > lcap ? std::min<uint64_t>(cn[i], lcap + cap) - lcap : 0;
        out[4] += hn[i];
    }
    return TFBS_OK;
}

int tfbs_ctx_window_lists(const tfbs_ctx *ctx, uint64_t entries[2], double *seconds) {
    if (!ctx || !entries || !seconds) return tfbs::fail(TFBS_E_ARG, "null argument");
    entries[0] = ctx->wl_entries[0];
    entries[1] = ctx->wl_entries[1];
    *seconds = ctx->wl_seconds;
    return TFBS_OK;
}

float tfbs_ctx_last_mfma_ms(const tfbs_ctx *ctx) {
    if (!ctx) return -1.f;
    tfbs_ctx_last_scan_ms(ctx);  // resolves the pending events
    return ctx->kernel_timed ? ctx->last_kernel_ms : -1.f;
}

int tfbs_batch_upload(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    Batch &B = b->b;
    if (B.pats != ctx->pats) return tfbs::fail(TFBS_E_ARG, "batch and ctx use different pattern sets");
    if (B.open) return tfbs::fail(TFBS_E_STATE, "region still open");
    if (B.slot_pid != ctx->plan.slot_pid) return tfbs::fail(TFBS_E_STATE, "batch slot order differs from the ctx plan");
    HIP_TRY(hipSetDevice(ctx->device));
    // key assembly scratch for regions of more distinct haplotypes than its LDS block holds
    uint64_t big = 0;
    for (DevRegion &rg : B.regions) {
        rg.big_off = big;
        if (rg.hap_count > key_asm_lds_counters()) big += rg.hap_count;
    }
    // dense counts only for the LUT / generic kernels' slots (they store theirs)
    const bool dense = !ctx->plan.fast_tiles.empty() || !ctx->plan.gen_tiles.empty();
    int rc;
    if ((rc = ctx->words.put(B.words, ctx->stream)) || (rc = ctx->nmask.put(B.nmask, ctx->stream)) ||
        (rc = ctx->posrel.put(B.posrel, ctx->stream)) || (rc = ctx->haps.put(B.haps, ctx->stream)) ||
        (rc = ctx->druns.put(B.druns, ctx->stream)) ||
        (rc = ctx->regions.put(B.regions, ctx->stream)) || (rc = ctx->inner.put(B.inner, ctx->stream)) ||
        (rc = ctx->asm_scratch.ensure(std::max<uint64_t>(big, 1))) ||
        (dense && (rc = ctx->counts.ensure(std::max<uint64_t>(B.n_counts, 1)))))
        return rc;
    std::vector<uint32_t> order(B.regions.size());  // (alive until the stream sync below)
    {  // key_fast_kernel's region order: most distinct haplotypes first (their workgroups run longest)
        for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
            return B.regions[x].hap_count > B.regions[y].hap_count;
        });
        if ((rc = ctx->asm_order.put(order, ctx->stream))) return rc;
        ctx->asm_order_n = (uint32_t)order.size();
        ctx->asm_order_big = 0;
        static const int big_u = env_int("TFBS_KF_BIGU", (int)key_fast_big_u());  // (0: every region on one shape)
        while (big_u > 0 && ctx->asm_order_big < order.size() &&
               B.regions[order[ctx->asm_order_big]].hap_count > (uint32_t)big_u)
            ctx->asm_order_big++;
    }
    std::vector<uint8_t> narrow((B.haps.size() + ctx->mfma_hpb - 1) / ctx->mfma_hpb, 1);  // (alive until the sync)
    for (size_t h = 0; h < B.haps.size(); h++)
        if (B.haps[h].len > kWlNarrowLen) narrow[h / ctx->mfma_hpb] = 0;
    if ((rc = build_lists(ctx, (uint32_t)B.haps.size(), narrow))) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->counts_live = dense;
    ctx->resident = b;
    ctx->upload_gen++;
    ctx->prev_spill = ctx->prev_redo = ctx->prev_cand = UINT32_MAX;
    ctx->mfma_group_words = mfma_group_words(B.haps.data(), (uint32_t)B.haps.size(), ctx->mfma_hpb);
    ctx->n_regions = (uint32_t)B.regions.size();
    ctx->over_pending = false;
    ctx->scanned = false;
    ctx->asm_state = 0;
    return TFBS_OK;
}

int tfbs_scan(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not uploaded to this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    ctx->kernel_timed = false;
    // asynchronous: the overflow lists are checked (and the scan redone if one
    // overflowed) when its results are read (tfbs_batch_reduce / download)
    const int n = launch_scan(ctx, (uint32_t)b->b.haps.size(), nullptr, 0);
    if (n < 0) return n;
    ctx->scanned = true;
    ctx->asm_state = 0;
    if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->last_launches = n;
    ctx->timing_pending = true;
    b->b.counts_valid = b->b.reduced = false;
    b->b.enc_r0 = b->b.enc_r1 = 0;
    return TFBS_OK;
}

int tfbs_batch_download(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    if (!ctx->scanned) return tfbs::fail(TFBS_E_STATE, "batch not scanned (tfbs_scan)");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    int rc;
    if (ctx->asm_state == 1 && ctx->asm_batch == &B && (rc = assembly_wait(ctx, B))) return rc;
    if ((rc = check_overflow(ctx, (uint32_t)B.haps.size()))) return rc;
    if (!ctx->counts_live) {  // no LUT/generic slots: the matrix is the assembly's alone
        if ((rc = ctx->counts.ensure(std::max<uint64_t>(B.n_counts, 1)))) return rc;
    }
    AsmArgs a = asm_args(ctx, B, 1);
    a.counts = ctx->counts.p;
    a.dense_base = 1;
    if ((rc = launch_key_asm(a, (uint32_t)B.regions.size(), ctx->stream))) return rc;
    B.counts.resize(B.n_counts);
    if (B.n_counts)
        HIP_TRY(hipMemcpyAsync(B.counts.data(), ctx->counts.p, B.n_counts * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    B.counts_valid = true;
    return TFBS_OK;
}

}  // extern "C"

// The device half of the key reduction, enqueued on the ctx stream behind the scan
// with no host wait: the candidates past the waves' lists rescored and the spill
// records bucketed by region (post: once per scan -- the rescoring appends spill
// records), then the key assembly (launch_key_fast); the overflow and list
// counters are copied back for assembly_wait.  Buffers are sized from the batch
// (1/16 of its keys and dense counts for the varying lists: no regrowth at C3
// shapes; TFBS_VAR_CAP=n starts at n keys and 4 n counts -- the regrow path's test).
// asm_ctr: [0, 2) the scan's overflow counters (copied), 2 regions left to key_asm,
// 3 arena words used, [4, 8) the varying keys' and counts' u64 totals, [8, 16) debug
// give-up reasons, 16 / 17 key_fast_kernel's region counters, 18 / 19 post_scan_kernel's and
// spill_hist_wide_kernel's finished workgroups, [20, 24) spare; the spill buckets after.

static int enqueue_assembly(tfbs_ctx *ctx, Batch &B, bool post) {
    int rc;
    const uint64_t n_keys = (uint64_t)(B.inner.size() / 2) * B.n_slots;
    const uint32_t nr = (uint32_t)B.regions.size();
    if ((rc = ctx->key_first.ensure(std::max<uint64_t>(n_keys, 1))) ||
        (rc = ctx->key_flags.ensure(std::max<uint64_t>(n_keys, 1))) || (rc = ctx->asm_ctr.ensure(kAsmCtrWords + (size_t)std::max<uint32_t>(1, nr) + 1)) ||
        (rc = ctx->asm_redo.ensure((size_t)nr + 1)) || (rc = ctx->cor_arena.ensure(ctx->cor_cap)))
        return rc;
    if (!ctx->asm_host) HIP_TRY(hipHostMalloc((void **)&ctx->asm_host, 4 * kAsmCtrWords, hipHostMallocDefault));
    if (const int vc = env_int("TFBS_VAR_CAP", 0); vc > 0) {
        if (!ctx->var_cap_forced) {
            ctx->var_keys_cap = (uint32_t)vc;
            ctx->var_cap = 4ull * (uint32_t)vc;
            ctx->var_cap_forced = true;
        }
    } else {
        ctx->var_keys_cap = std::max<uint32_t>(ctx->var_keys_cap, (uint32_t)std::min<uint64_t>(n_keys / 16, 1u << 26));
        ctx->var_cap = std::max<uint64_t>(ctx->var_cap, std::min<uint64_t>(B.n_counts / 16, 1ull << 28));
    }
    if ((rc = ctx->var_keys.ensure(ctx->var_keys_cap)) || (rc = ctx->var_counts.ensure(ctx->var_cap))) return rc;
    if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->asm_t0, ctx->stream));
    const bool mfma = !ctx->plan.m_supers.empty();
    // the assembly's counters and the spill buckets' (at asm_ctr + kAsmCtrWords): zeroed
    // by the scan for its first assembly, else one memset
    if (!(mfma && post && ctx->asm_ctr_zeroed && ctx->n_regions == nr))
        HIP_TRY(hipMemsetAsync(ctx->asm_ctr.p, 0,
                               (kAsmCtrWords + (mfma && post ? (size_t)std::max<uint32_t>(1, nr) + 1 : 0)) * 4,
                               ctx->stream));
    ctx->asm_ctr_zeroed = false;
    // lean (see tfbs_ctx): left out what the batch's last checked assembly did not need
    const bool lean = mfma && post && !ctx->asm_full && ctx->asm_lean_mode != 0;
    ctx->asm_wide = !(lean && (ctx->asm_lean_mode == 2 || ctx->prev_spill <= kPostSerial));
    ctx->asm_leftover = !(lean && (ctx->asm_lean_mode == 2 || ctx->prev_redo == 0));
    if (mfma && post) {  // overflow candidates rescored (once per scan: they append spill records) + spill buckets
        // (without the leftover pass post_scan_kernel copies the overflow counters to
        // asm_ctr[0, 2); asm_ctr[20]: set when the records needed the wide kernels)
        if (ctx->post_fused) {  // the scan's last workgroup did it (lean: no wide kernels)
            ctx->asm_wide = false;
        } else if ((rc = launch_post_fused(ctx->last_margs, !ctx->post_done, ctx->asm_ctr.p + 18,
                                           std::max<uint32_t>(1, nr), ctx->asm_ctr.p + kAsmCtrWords, ctx->spill_boff.p,
                                           ctx->spill_sorted.p, ctx->stream, ctx->asm_wide, ctx->asm_ctr.p,
                                           ctx->asm_ctr.p + 20, lean && ctx->prev_cand == 0 ? 1u : 256u))) {
            return rc;
        }
        ctx->post_done = true;
    }
    ctx->post_fused = false;
    AsmArgs a = asm_args(ctx, B, 0);
    a.key_first = ctx->key_first.p;
    a.key_flags = ctx->key_flags.p;
    a.var_keys = ctx->var_keys.p;
    a.var_keys_cap = ctx->var_keys_cap;
    a.var_counts = ctx->var_counts.p;
    a.var_cap = ctx->var_cap;
    a.var_tot = reinterpret_cast<unsigned long long *>(ctx->asm_ctr.p + 4);
    a.redo = ctx->asm_redo.p;
    a.redo_n = ctx->asm_ctr.p + 2;
    a.fast_max_u = ctx->key_fast_max_u;
    a.cor_arena = ctx->cor_arena.p;
    a.cor_cap = ctx->cor_cap;
    a.cor_used = ctx->asm_ctr.p + 3;
    a.cor_lds = ctx->key_cor_lds;
    a.why = ctx->debug_over ? ctx->asm_ctr.p + 8 : nullptr;
    a.report_src = mfma ? ctx->over.p : nullptr;  // (copied by the list pass: no report launch)
    a.report = ctx->asm_ctr.p;
    a.order = ctx->asm_order_n == nr ? ctx->asm_order.p : nullptr;
    a.persist = ctx->kf_persistent ? 1u : 0u;
    a.next = ctx->asm_ctr.p + 16;
    if (ctx->kf_prof_on && nr) {
        if ((rc = ctx->kf_prof.ensure((size_t)nr * 16))) return rc;
        HIP_TRY(hipMemsetAsync(ctx->kf_prof.p, 0, (size_t)nr * 128, ctx->stream));
        a.prof = ctx->kf_prof.p;
    }
    if ((rc = launch_key_fast(a, nr, a.order ? ctx->asm_order_big : 0, ctx->stream, ctx->side[0], ctx->kf_fork,
                              ctx->kf_join, ctx->asm_leftover)) ||
        (nr == 0 && (rc = launch_asm_report(a.report_src, ctx->asm_ctr.p, ctx->stream))))
        return rc;
    if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->asm_t1, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->asm_host, ctx->asm_ctr.p, 4 * kAsmCtrWords, hipMemcpyDeviceToHost, ctx->stream));
    if (!ctx->capturing) HIP_TRY(hipEventRecord(ctx->asm_ev, ctx->stream));
    ctx->over_pending = false;  // the assembly's check covers this scan's overflow lists
    ctx->asm_batch = &B;
    ctx->asm_state = 1;
    ctx->asm_timed = true;
    return TFBS_OK;
}

// Waits for the enqueued assembly and checks its lists: a scan overflow list that
// dropped entries means a rescan with larger lists (and a new assembly), a full
// varying-key list a new assembly with larger ones.
static uint64_t t_lo_all(const std::vector<uint64_t> &h, uint32_t nr) {
    uint64_t t = UINT64_MAX;
    for (uint32_t r = 0; r < nr; r++)
        if (h[(size_t)r * 16 + 6]) t = std::min(t, h[(size_t)r * 16]);
    return t;
}
static uint64_t t_hi_all(const std::vector<uint64_t> &h, uint32_t nr) {
    uint64_t t = 0;
    for (uint32_t r = 0; r < nr; r++) t = std::max(t, h[(size_t)r * 16 + 6]);
    return t;
}

// TFBS_KF_PROF: key_fast_kernel's mean phase cycles and sizes over the regions it
// finished (debug; synchronises).
static int kf_prof_report(tfbs_ctx *ctx, uint32_t nr) {
    std::vector<uint64_t> h((size_t)nr * 16);
    HIP_TRY(hipMemcpy(h.data(), ctx->kf_prof.p, h.size() * 8, hipMemcpyDeviceToHost));
    double ph[6] = {0, 0, 0, 0, 0, 0}, sz[8] = {0, 0, 0, 0, 0, 0, 0, 0}, mx = 0, at = 0;
    uint32_t n = 0;
    for (uint32_t r = 0; r < nr; r++) {
        const uint64_t *p = &h[(size_t)r * 16];
        if (!p[6]) continue;  // empty, or left to key_asm_kernel
        n++;
        for (int k = 0; k < 6; k++) ph[k] += (double)(p[k + 1] - p[k]);
        mx = std::max(mx, (double)(p[6] - p[0]));
        at += (double)p[7];
        for (int k = 0; k < 8; k++) sz[k] += (double)p[8 + k];
    }
    std::vector<std::pair<double, uint32_t>> tot;  // (cycles, region)
    for (uint32_t r = 0; r < nr; r++)
        if (h[(size_t)r * 16 + 6]) tot.push_back({(double)(h[(size_t)r * 16 + 6] - h[(size_t)r * 16]), r});
    std::sort(tot.begin(), tot.end());
    if (!tot.empty()) {
        auto pct = [&](double f) { return tot[std::min(tot.size() - 1, (size_t)(f * tot.size()))].first; };
        fprintf(stderr, "[kf prof] total ticks p50 %.0f p90 %.0f p99 %.0f max %.0f; slowest regions (ticks U rows chunks "
                        "corrections refs):", pct(0.5), pct(0.9), pct(0.99), tot.back().first);
        for (size_t i = tot.size(); i-- > 0 && i + 6 > tot.size();) {
            const uint64_t *p = &h[(size_t)tot[i].second * 16];
            fprintf(stderr, " [%.0f %llu %llu %llu %llu %llu]", tot[i].first, (unsigned long long)p[8],
                    (unsigned long long)p[12], (unsigned long long)p[13], (unsigned long long)p[11],
                    (unsigned long long)p[15]);
        }
        fprintf(stderr, "\n");
    }
    uint64_t t_lo = UINT64_MAX, t_hi = 0;
    double busy = 0;
    for (uint32_t r = 0; r < nr; r++) {
        const uint64_t *p = &h[(size_t)r * 16];
        if (!p[6]) continue;
        t_lo = std::min(t_lo, p[0]);
        t_hi = std::max(t_hi, p[6]);
        busy += (double)(p[6] - p[0]);
    }
    {  // per workgroup: its regions in start order -> gaps between them, late start, early end
        std::vector<std::pair<std::pair<uint64_t, uint64_t>, uint32_t>> ev;  // ((workgroup, start), region)
        for (uint32_t r = 0; r < nr; r++)
            if (h[(size_t)r * 16 + 6]) ev.push_back({{h[(size_t)r * 16 + 14], h[(size_t)r * 16]}, r});
        std::sort(ev.begin(), ev.end());
        double gap = 0, late = 0, early_end = 0;
        uint32_t n_gap = 0, n_wg = 0;
        for (size_t i = 0; i < ev.size(); i++) {
            const uint64_t *p = &h[(size_t)ev[i].second * 16];
            const bool first = i == 0 || ev[i - 1].first.first != ev[i].first.first;
            const bool last = i + 1 == ev.size() || ev[i + 1].first.first != ev[i].first.first;
            if (first) {
                n_wg++;
                late += (double)(p[0] - t_lo_all(h, nr));
            } else {
                gap += (double)(p[0] - h[(size_t)ev[i - 1].second * 16 + 6]);
                n_gap++;
            }
            if (last) early_end += (double)(t_hi_all(h, nr) - p[6]);
        }
        if (n_wg)
            fprintf(stderr, "[kf prof] %u workgroups: mean gap between a workgroup's regions %.1f us (%u gaps), first "
                            "region start after the kernel's first %.1f us, last end before the kernel's last %.1f us\n",
                    n_wg, n_gap ? gap / n_gap / 100.0 : 0.0, n_gap, late / n_wg / 100.0, early_end / n_wg / 100.0);
    }
    uint32_t early = 0;  // regions started in the first 10 us: the workgroups resident at the start
    for (uint32_t r = 0; r < nr; r++)
        if (h[(size_t)r * 16 + 6] && h[(size_t)r * 16] < t_lo + 1000) early++;
    if (t_hi > t_lo)
        fprintf(stderr, "[kf prof] span %.1f us (first region start to last end, 100 MHz ticks), region-time %.1f us: "
                        "%.0f regions in flight on average; %u regions started in the first 10 us\n",
                (t_hi - t_lo) / 100.0, busy / 100.0, busy / (double)(t_hi - t_lo), early);
    const double d = n ? n : 1;
    fprintf(stderr,
            "[kf prof] regions %u of %u ticks/region: descr+hitn %.0f refs %.0f dirty %.0f lists %.0f keys %.0f "
            "chunks %.0f (of which var-list atomics %.0f) (max total %.0f); per region: U %.1f entries %.1f dirty-refs %.1f corrections %.1f rows "
            "%.1f chunks %.2f in-LDS %.2f refs %.1f\n",
            n, nr, ph[0] / d, ph[1] / d, ph[2] / d, ph[3] / d, ph[4] / d, ph[5] / d, at / d, mx, sz[0] / d, sz[1] / d,
            sz[2] / d, sz[3] / d, sz[4] / d, sz[5] / d, sz[6] / d, sz[7] / d);
    return TFBS_OK;
}

static int assembly_wait(tfbs_ctx *ctx, Batch &B) {
    auto grow = [](uint32_t &cap, uint32_t need, uint64_t lim) {
        if (need > cap) cap = (uint32_t)std::min<uint64_t>(lim, (uint64_t)need * 5 / 4 + 1024);
    };
    for (int round = 0; ctx->asm_state == 1; round++) {
        if (round == 8) return tfbs::fail(TFBS_E_NOMEM, "scan / key lists still full after 8 reruns");
        HIP_TRY(hipEventSynchronize(ctx->asm_ev));
        const uint32_t nspill = ctx->asm_host[0], ncand = ctx->asm_host[1];
        const uint64_t *vt = reinterpret_cast<const uint64_t *>(ctx->asm_host + 4);
        const uint64_t nk = vt[0], nc = vt[1];
        if (ctx->debug_over && ctx->asm_host[2]) {  // the regions left to key_asm_kernel: their shapes
            std::vector<uint32_t> redo(ctx->asm_host[2]);
            HIP_TRY(hipMemcpy(redo.data(), ctx->asm_redo.p, redo.size() * 4, hipMemcpyDeviceToHost));
            uint64_t su = 0, sr = 0;
            uint32_t mu = 0, mi = 0;
            for (uint32_t r : redo) {
                const DevRegion &rg = B.regions[r];
                su += rg.hap_count;
                mu = std::max(mu, rg.hap_count);
                mi = std::max(mi, rg.n_inner);
                for (uint32_t l = 0; l < rg.hap_count; l++) sr += B.haps[rg.hap_begin + l].n_druns;
            }
            const uint32_t *why = ctx->asm_host + 8;
            fprintf(stderr, "tfbs assembly: %zu regions left to key_asm: mean haplotypes %.1f (max %u), max inner %u, "
                            "mean diff runs %.1f; reasons: shape %u lists %u runs %u refs %u arena(cor) %u arena(cnt) %u\n",
                    redo.size(), (double)su / redo.size(), mu, mi, (double)sr / redo.size(), why[0], why[1], why[2],
                    why[3], why[4], why[5]);
        }
        if (ctx->debug_over)
            fprintf(stderr, "tfbs assembly: spill %u/%u candidates %u/%u left to key_asm %u arena %u/%u varying keys "
                            "%llu/%u counts %llu/%llu\n", nspill, ctx->spill_cap, ncand, ctx->cand_over_cap,
                    ctx->asm_host[2], ctx->asm_host[3], ctx->cor_cap,
                    (unsigned long long)nk, ctx->var_keys_cap, (unsigned long long)nc,
                    (unsigned long long)ctx->var_cap);
        int rc;
        // a lean assembly that needed what it left out (more spill records than post_scan_kernel
        // buckets, or regions key_fast_kernel gave up): again with everything
        if ((!ctx->asm_wide && ctx->asm_host[20]) || (!ctx->asm_leftover && ctx->asm_host[2])) {
            ctx->asm_full = true;
            rc = enqueue_assembly(ctx, B, true);
            ctx->asm_full = false;
            if (rc) return rc;
            continue;
        }
        if (ctx->asm_host[3] > ctx->cor_cap)  // regions that found the arena full went to key_asm_kernel: larger next time
            ctx->cor_cap = (uint32_t)std::min<uint64_t>((uint64_t)ctx->asm_host[3] * 5 / 4, 1u << 30);
        if (nspill > ctx->spill_cap || ncand > ctx->cand_over_cap) {
            grow(ctx->spill_cap, ncand > ctx->cand_over_cap ? 2 * std::max(nspill, 1024u) : nspill, UINT32_MAX / 4);
            grow(ctx->cand_over_cap, ncand, UINT32_MAX / 4);
            const int n = launch_scan(ctx, (uint32_t)B.haps.size(), nullptr, 0);
            if (n < 0) return n;
            if ((rc = enqueue_assembly(ctx, B, true))) return rc;
            continue;
        }
        if (nk > ctx->var_keys_cap || nc > ctx->var_cap) {
            if (nk >= (1ull << 32) || nc >= (1ull << 40)) return tfbs::fail(TFBS_E_NOMEM, "too many varying counts");
            ctx->var_keys_cap = (uint32_t)std::max<uint64_t>(ctx->var_keys_cap, std::min<uint64_t>(nk + nk / 4 + 1024, UINT32_MAX));
            ctx->var_cap = std::max<uint64_t>(ctx->var_cap, nc + nc / 4 + 4096);
            if ((rc = enqueue_assembly(ctx, B, false))) return rc;
            continue;
        }
        ctx->asm_state = 2;
        ctx->prev_spill = nspill;
        ctx->prev_redo = ctx->asm_host[2];
        ctx->prev_cand = ncand;
        if (ctx->kf_prof_on && (rc = kf_prof_report(ctx, (uint32_t)B.regions.size()))) return rc;
    }
    return TFBS_OK;
}

extern "C" {

int tfbs_batch_assemble(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    if (!ctx->scanned) return tfbs::fail(TFBS_E_STATE, "batch not scanned (tfbs_scan)");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    if (ctx->asm_state != 0 && ctx->asm_batch == &B) return TFBS_OK;  // this scan's assembly is on its way
    // another batch's varying counts live in var_counts: to its host copy first
    if (ctx->var_owner && ctx->var_owner != &B) {
        int rc;
        if ((rc = tfbs::ensure_host_var_counts(*ctx->var_owner))) return rc;
        std::lock_guard<std::mutex> g(ctx->var_owner->var_mu);
        if (ctx->var_owner->var_ctx == ctx) ctx->var_owner->var_ctx = nullptr;
        ctx->var_owner = nullptr;
    }
    return enqueue_assembly(ctx, B, true);
}

}  // extern "C"

// What a step's launches depend on besides the batch image: the resident batch and
// its upload, every buffer's address and every list capacity the scan and the
// assembly pass to their kernels.  A step whose signature equals the captured
// graph's replays it.
static uint64_t step_signature(const tfbs_ctx *ctx, const tfbs_batch *b) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    auto mix = [&](uint64_t v) {
        h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
        h *= 0xBF58476D1CE4E5B9ull;
    };
    auto buf = [&](const auto &d) {
        mix((uint64_t)(uintptr_t)d.p);
        mix(d.n);
    };
    mix((uint64_t)(uintptr_t)b);
    mix((uint64_t)(uintptr_t)ctx->resident);
    mix(ctx->upload_gen);
    buf(ctx->cands); buf(ctx->hitl); buf(ctx->hitn); buf(ctx->candn); buf(ctx->ref_hits); buf(ctx->ref_count); buf(ctx->spill);
    buf(ctx->over); buf(ctx->spill_sorted); buf(ctx->spill_bcnt); buf(ctx->spill_boff); buf(ctx->cand_over);
    buf(ctx->srcs); buf(ctx->words); buf(ctx->nmask); buf(ctx->counts); buf(ctx->posrel); buf(ctx->inner);
    buf(ctx->haps); buf(ctx->druns); buf(ctx->gnarrow); buf(ctx->gorder); buf(ctx->hd); buf(ctx->hd2); buf(ctx->regions);
    buf(ctx->hits); buf(ctx->asm_scratch); buf(ctx->key_first); buf(ctx->var_counts); buf(ctx->asm_redo);
    buf(ctx->asm_ctr); buf(ctx->cor_arena); buf(ctx->key_flags); buf(ctx->var_keys); buf(ctx->asm_order);
    for (int c = 0; c < 2; c++) {
        buf(ctx->wl_off[c]);
        buf(ctx->wl[c]);
        buf(ctx->wl16[c]);
    }
    for (uint64_t v : {(uint64_t)ctx->spill_cap, (uint64_t)ctx->cand_over_cap, (uint64_t)ctx->cand_cap,
                       (uint64_t)ctx->scan_cand_cap, (uint64_t)ctx->var_keys_cap, ctx->var_cap,
                       (uint64_t)ctx->cor_cap, (uint64_t)ctx->n_regions, (uint64_t)ctx->asm_order_n,
                       (uint64_t)ctx->asm_order_big, (uint64_t)ctx->n_srcs, (uint64_t)ctx->srcs_on_dev,
                       (uint64_t)ctx->counts_live, (uint64_t)ctx->mfma_group_words,
                       (uint64_t)(uintptr_t)ctx->var_owner, (uint64_t)ctx->asm_lean_mode,
                       (uint64_t)(ctx->prev_spill <= kPostSerial), (uint64_t)(ctx->prev_redo == 0),
                       (uint64_t)(ctx->prev_cand == 0)})
        mix(v);
    return h;
}

// The host state a step leaves (tfbs_scan + tfbs_batch_assemble), set after a replay.
static void step_state(tfbs_ctx *ctx, Batch &B) {
    ctx->scanned = true;
    ctx->kernel_timed = false;  // (no timing events in a graph: the timing queries keep the last plain step's)
    ctx->timing_pending = false;
    ctx->asm_timed = false;
    ctx->asm_ctr_zeroed = false;
    ctx->post_done = true;
    ctx->over_pending = false;
    ctx->over_copied = false;
    ctx->asm_batch = &B;
    ctx->asm_state = 1;
    B.counts_valid = B.reduced = false;
    B.enc_r0 = B.enc_r1 = 0;
}

extern "C" {

int tfbs_step(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not uploaded to this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    auto plain = [&]() -> int {
        int rc;
        ctx->post_fuse_ok = true;  // (the assembly follows the scan at once)
        rc = tfbs_scan(ctx, b);
        ctx->post_fuse_ok = false;
        if (rc || (rc = tfbs_batch_assemble(ctx, b))) return rc;
        return TFBS_OK;
    };
    auto drop = [&]() {
        if (ctx->step_exec) (void)hipGraphExecDestroy(ctx->step_exec);
        if (ctx->step_graph) (void)hipGraphDestroy(ctx->step_graph);
        ctx->step_exec = nullptr;
        ctx->step_graph = nullptr;
    };
    // (another batch's varying counts in var_counts: tfbs_batch_assemble hands them over first)
    const bool eligible = ctx->step_graphs && (!ctx->var_owner || ctx->var_owner == &B);
    const uint64_t sig = step_signature(ctx, b);
    int rc;
    if (eligible && ctx->step_exec && sig == ctx->step_sig) {  // replay
        HIP_TRY(hipGraphLaunch(ctx->step_exec, ctx->stream));
        HIP_TRY(hipEventRecord(ctx->asm_ev, ctx->stream));
        step_state(ctx, B);
        ctx->last_launches = 1;
        return assembly_wait(ctx, B);
    }
    drop();
    if (eligible && ctx->step_sig_seen && sig == ctx->step_sig) {  // the second step alike: capture it
        hipGraph_t g = nullptr;
        HIP_TRY(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
        ctx->capturing = true;
        rc = plain();
        ctx->capturing = false;
        const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
        hipGraphExec_t x = nullptr;
        const bool ok = !rc && e == hipSuccess && g && hipGraphInstantiate(&x, g, nullptr, nullptr, 0) == hipSuccess;
        const uint64_t after = step_signature(ctx, b);  // (a buffer that moved while capturing: no graph)
        if (ok && after == sig) {
            ctx->step_graph = g;
            ctx->step_exec = x;
            ctx->step_sig = sig;
            HIP_TRY(hipGraphLaunch(ctx->step_exec, ctx->stream));
            HIP_TRY(hipEventRecord(ctx->asm_ev, ctx->stream));
            step_state(ctx, B);
            ctx->last_launches = 1;
            return assembly_wait(ctx, B);
        }
        (void)hipGetLastError();
        if (x) (void)hipGraphExecDestroy(x);
        if (g) (void)hipGraphDestroy(g);
        ctx->step_sig_seen = false;  // nothing ran: the step again, plainly
        if ((rc = plain())) return rc;
        return assembly_wait(ctx, B);
    }
    if ((rc = plain())) return rc;
    rc = assembly_wait(ctx, B);
    ctx->step_sig = step_signature(ctx, b);  // (after the wait: a rescan's regrown lists count)
    ctx->step_sig_seen = ctx->step_sig == sig;
    return rc;
}

int tfbs_batch_assemble_wait(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b || ctx->asm_state == 0 || ctx->asm_batch != &b->b)
        return tfbs::fail(TFBS_E_STATE, "no assembly of this batch on this ctx (tfbs_batch_assemble)");
    HIP_TRY(hipSetDevice(ctx->device));
    return assembly_wait(ctx, b->b);
}

float tfbs_ctx_last_assemble_ms(const tfbs_ctx *ctx) {
    if (!ctx || !ctx->asm_timed) return -1.f;
    auto *c = const_cast<tfbs_ctx *>(ctx);
    float ms = -1.f;
    if (hipEventSynchronize(c->asm_t1) == hipSuccess && hipEventElapsedTime(&ms, c->asm_t0, c->asm_t1) == hipSuccess)
        c->last_asm_ms = ms;
    return c->last_asm_ms;
}

int tfbs_batch_reduce(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    if (!ctx->scanned) return tfbs::fail(TFBS_E_STATE, "batch not scanned (tfbs_scan)");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    int rc;
    if ((rc = tfbs_batch_assemble(ctx, b)) || (rc = assembly_wait(ctx, B))) return rc;
    const uint64_t n_keys = (uint64_t)(B.inner.size() / 2) * B.n_slots;
    const uint64_t *vt = reinterpret_cast<const uint64_t *>(ctx->asm_host + 4);
    const uint32_t nk = (uint32_t)vt[0];
    const uint64_t nc = vt[1];
    if (nc >= UINT32_MAX) return tfbs::fail(TFBS_E_NOMEM, "too many varying counts (u32 offsets)");
    B.key_first.resize(n_keys);
    B.key_flags.resize(n_keys);
    std::vector<DevVarKey> vk(nk);
    if (n_keys) {
        HIP_TRY(hipMemcpyAsync(B.key_first.data(), ctx->key_first.p, n_keys * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipMemcpyAsync(B.key_flags.data(), ctx->key_flags.p, n_keys, hipMemcpyDeviceToHost, ctx->stream));
    }
    if (nk) HIP_TRY(hipMemcpyAsync(vk.data(), ctx->var_keys.p, nk * sizeof(DevVarKey), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    // the varying keys in (region, key) order -- a counting sort by region, then each
    // region's few keys by key; their counts stay where the device put them
    {
        std::vector<uint32_t> at(B.regions.size() + 1, 0);
        for (const DevVarKey &k : vk) at[k.region + 1]++;
        for (size_t r = 0; r < B.regions.size(); r++) at[r + 1] += at[r];
        std::vector<DevVarKey> by(nk);
        {
            std::vector<uint32_t> put(at.begin(), at.end() - 1);
            for (const DevVarKey &k : vk) by[put[k.region]++] = k;
        }
        for (size_t r = 0; r < B.regions.size(); r++)
            std::sort(by.begin() + at[r], by.begin() + at[r + 1],
                      [](const DevVarKey &x, const DevVarKey &y) { return x.j < y.j; });
        vk.swap(by);
    }
    B.var_off.assign(n_keys, UINT32_MAX);
    B.var_idx.assign(n_keys, UINT32_MAX);
    for (uint32_t i = 0; i < nk; i++) {
        const uint64_t k = (uint64_t)B.regions[vk[i].region].inner_off * B.n_slots + vk[i].j;
        B.var_off[k] = (uint32_t)vk[i].out_off;
        B.var_idx[k] = i;
    }
    B.var_keys = std::move(vk);
    // (a batch reduced before on another ctx: B.var_ctx moves here; that ctx drops B
    // as its owner when it next looks -- it checks B.var_ctx under B.var_mu)
    {  // the varying counts stay on the device until a host reader needs them
        std::lock_guard<std::mutex> g(B.var_mu);
        B.var_dev = ctx->var_counts.p;
        B.var_n = nc;
        B.var_device = ctx->device;
        B.var_ctx = ctx;
        B.var_host = false;
        B.var_err = 0;
    }
    ctx->var_owner = &B;
    B.enc_r0 = B.enc_r1 = 0;
    B.enc_idx.clear();
    B.reduced = true;
    return TFBS_OK;
}

int tfbs_batch_encode(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1) {
    return tfbs_batch_encode_flags(ctx, b, r0, r1, 0);
}

int tfbs_batch_encode_flags(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, int flags) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    Batch &B = b->b;
    if (!B.reduced) return tfbs::fail(TFBS_E_STATE, "keys not reduced (tfbs_batch_reduce)");
    if (!B.keep_membership) return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    {  // the varying counts the encode reads are this ctx's (var_counts, at the offsets of its reduction)
        std::lock_guard<std::mutex> g(B.var_mu);
        if (B.var_ctx != ctx) return tfbs::fail(TFBS_E_STATE, "batch last reduced on another ctx (tfbs_batch_reduce here)");
    }
    r1 = std::min(r1, B.rh.size());
    r0 = std::min(r0, r1);
    HIP_TRY(hipSetDevice(ctx->device));
    B.enc_r0 = B.enc_r1 = 0;
    B.enc_idx.assign(B.var_keys.size(), UINT32_MAX);
    B.enc_hdr.clear();
    B.enc_vals.clear();
    B.enc_hist.clear();
    B.enc_val_off.assign(1, 0);
    B.enc_code_off.assign(1, 0);
    const uint32_t N = B.n_samples, H = 2 * N;
    if (N == 0 || r0 == r1) {
        B.enc_r0 = (uint32_t)r0;
        B.enc_r1 = (uint32_t)r1;
        return TFBS_OK;
    }
    // every region's u16 membership row on this device -- a device-grouped region's
    // own, the others' made by the host threads in the ctx's pinned staging and
    // uploaded -- then its distinct (left, right) haplotype pairs and each sample's
    // pair on the device (launch_pair_table)
    const size_t nr = r1 - r0;
    int rc;
    std::vector<uint64_t> rows(nr, 0);
    std::vector<size_t> hostr;
    for (size_t r = r0; r < r1; r++) {
        const RegionH &R = B.rh[r];
        if (R.hap_count > kEncMaxHaps) continue;
        if (!R.memb_host && B.grouper && B.grouper->device() == ctx->device) rows[r - r0] = R.memb_dev;
        else hostr.push_back(r);
    }
    for (size_t r : hostr)
        if ((rc = region_membership(B, B.rh[r]))) return rc;
    const size_t Hp = ((size_t)H + 7) / 8 * 8;
    if (!hostr.empty()) {
        // their non-reference lists (haplotype id, distinct index) go up, the rows are
        // filled on the device (launch_memb_fill): a few MB instead of Hp u16 per region
        std::vector<uint32_t> meta(2 * (hostr.size() + 1), 0);
        uint64_t tot = 0;
        for (size_t k = 0; k < hostr.size(); k++) {
            const RegionH &R = B.rh[hostr[k]];
            meta[2 * k] = (uint32_t)tot;
            meta[2 * k + 1] = (uint32_t)(R.ref_local < 0 ? 0 : R.ref_local);
            tot += R.nonref_id.size();
        }
        if (tot >= UINT32_MAX) return tfbs::fail(TFBS_E_NOMEM, "too many non-reference haplotypes in one call");
        meta[2 * hostr.size()] = (uint32_t)tot;
        if ((rc = ctx->enc_memb_host.reserve(std::max<uint64_t>(tot, 1) * 6)) ||
            (rc = ctx->enc_memb.ensure(hostr.size() * Hp)) || (rc = ctx->enc_nr_ids.ensure(std::max<uint64_t>(tot, 1))) ||
            (rc = ctx->enc_nr_loc.ensure(std::max<uint64_t>(tot, 1))) || (rc = ctx->enc_nr_meta.put(meta, ctx->stream)))
            return rc;
        uint32_t *const ids = reinterpret_cast<uint32_t *>(ctx->enc_memb_host.p);
        uint16_t *const loc = reinterpret_cast<uint16_t *>(ctx->enc_memb_host.p + 4 * std::max<uint64_t>(tot, 1));
        const uint32_t T = std::max(1u, std::min(ctx->host_threads, (uint32_t)hostr.size()));
        std::atomic<size_t> next(0);
        auto work = [&]() {
            for (size_t k; (k = next.fetch_add(1)) < hostr.size();) {
                const RegionH &R = B.rh[hostr[k]];
                const size_t o = meta[2 * k];
                for (size_t i = 0; i < R.nonref_id.size(); i++) {
                    ids[o + i] = R.nonref_id[i];
                    loc[o + i] = (uint16_t)R.nonref_local[i];
                }
            }
        };
        std::vector<std::thread> ts;
        for (uint32_t t = 1; t < T; t++) ts.emplace_back(work);
        work();
        for (auto &t : ts) t.join();
        if (tot) {
            HIP_TRY(hipMemcpyAsync(ctx->enc_nr_ids.p, ids, tot * 4, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(ctx->enc_nr_loc.p, loc, tot * 2, hipMemcpyHostToDevice, ctx->stream));
        }
        if ((rc = launch_memb_fill(ctx->enc_nr_meta.p, ctx->enc_nr_ids.p, ctx->enc_nr_loc.p, (uint32_t)hostr.size(),
                                   (uint32_t)Hp, ctx->enc_memb.p, ctx->stream)))
            return rc;
    }
    for (size_t k = 0; k < hostr.size(); k++) rows[hostr[k] - r0] = (uint64_t)(uintptr_t)(ctx->enc_memb.p + k * Hp);
    std::vector<uint32_t> pair_n(nr);
    if ((rc = ctx->enc_rows.put(rows, ctx->stream)) || (rc = ctx->enc_pab.ensure(nr * kEncMaxPairs)) ||
        (rc = ctx->enc_pcnt.ensure(nr * kEncMaxPairs)) || (rc = ctx->enc_pair_n.ensure(nr)) ||
        (rc = ctx->enc_pidx.ensure(std::max<size_t>(nr * (size_t)N, 1))))
        return rc;
    if ((rc = launch_pair_table(ctx->enc_rows.p, (uint32_t)nr, N, ctx->enc_pab.p, ctx->enc_pcnt.p,
                                ctx->enc_pair_n.p, ctx->enc_pidx.p, ctx->stream)))
        return rc;
    HIP_TRY(hipMemcpyAsync(pair_n.data(), ctx->enc_pair_n.p, nr * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    // the keys to encode: varying keys of [r0, r1) whose region's pairs were listed
    // (<= kEncMaxHaps distinct haplotypes, <= kEncMaxPairs pairs; the others keep the host path)
    std::vector<DevVarKey> ek;
    // (B.var_keys is in region order: tfbs_batch_reduce)
    auto region_lb = [&](size_t r) {
        return (uint32_t)(std::lower_bound(B.var_keys.begin(), B.var_keys.end(), r,
                                           [](const DevVarKey &k, size_t x) { return k.region < x; }) -
                          B.var_keys.begin());
    };
    for (uint32_t i = region_lb(r0), i1 = region_lb(r1); i < i1; i++) {
        const DevVarKey &k = B.var_keys[i];
        if (pair_n[k.region - r0] == UINT32_MAX) continue;
        B.enc_idx[i] = (uint32_t)ek.size();
        ek.push_back(k);
    }
    const size_t nk = ek.size();
    if ((rc = ctx->enc_keys.put(ek, ctx->stream)) || (rc = ctx->enc_hdr.ensure(std::max<size_t>(nk, 1))) ||
        (rc = ctx->enc_vals.ensure(std::max<size_t>(nk, 1) * (kEncMaxVals + 1))) ||
        (rc = ctx->enc_hist.ensure(std::max<size_t>(nk, 1) * (kEncMaxVals + 1))) ||
        (rc = ctx->enc_codes.ensure(std::max<size_t>(nk, 1) * N)))
        return rc;
    if ((rc = launch_key_encode(ctx->var_counts.p, ctx->enc_keys.p, (uint32_t)nk, ctx->enc_pab.p, ctx->enc_pcnt.p,
                                ctx->enc_pair_n.p, ctx->enc_pidx.p, (uint32_t)r0, N, ctx->enc_hdr.p, ctx->enc_vals.p,
                                ctx->enc_hist.p, ctx->enc_codes.p, ctx->stream)))
        return rc;
    B.enc_hdr.resize(nk);
    B.enc_val_off.assign(nk + 1, 0);
    if (nk) {
        HIP_TRY(hipMemcpyAsync(B.enc_hdr.data(), ctx->enc_hdr.p, nk * sizeof(EncHdr), hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        // the value tables and histograms, and the packed codes, back to back (a key's
        // number of values and code width are known only now)
        B.enc_code_off.resize(nk + 1);
        for (size_t k = 0; k < nk; k++) {
            const EncHdr &h = B.enc_hdr[k];
            const uint64_t bytes = h.status ? 0 : ((uint64_t)N * h.width + 7) / 8;
            B.enc_code_off[k + 1] = B.enc_code_off[k] + bytes;
            B.enc_val_off[k + 1] = B.enc_val_off[k] + (h.status ? 0u : h.n_vals);
        }
        const uint32_t nv_tot = B.enc_val_off[nk];
        if ((rc = ctx->enc_val_off.put(B.enc_val_off, ctx->stream)) ||
            (rc = ctx->enc_vals_c.ensure(std::max<uint32_t>(nv_tot, 1))) ||
            (rc = ctx->enc_hist_c.ensure(std::max<uint32_t>(nv_tot, 1))))
            return rc;
        if ((rc = launch_val_compact(ctx->enc_vals.p, ctx->enc_hist.p, (uint32_t)nk, ctx->enc_val_off.p,
                                     ctx->enc_vals_c.p, ctx->enc_hist_c.p, ctx->stream)))
            return rc;
        B.enc_vals.resize(nv_tot);
        B.enc_hist.resize(nv_tot);
        if (nv_tot) {
            HIP_TRY(hipMemcpyAsync(B.enc_vals.data(), ctx->enc_vals_c.p, (size_t)nv_tot * 4, hipMemcpyDeviceToHost,
                                   ctx->stream));
            HIP_TRY(hipMemcpyAsync(B.enc_hist.data(), ctx->enc_hist_c.p, (size_t)nv_tot * 4, hipMemcpyDeviceToHost,
                                   ctx->stream));
        }
        const uint64_t total = B.enc_code_off[nk];
        if ((rc = ctx->enc_off.put(B.enc_code_off, ctx->stream)) ||
            (rc = ctx->enc_packed.ensure(total + 16)) ||  // (the BGZF staging reads whole dwords)
            (!(flags & TFBS_ENC_DEVICE_CODES) && (rc = B.enc_codes.reserve(total))))
            return rc;
        if ((rc = launch_code_compact(ctx->enc_codes.p, (uint32_t)nk, N, ctx->enc_off.p, ctx->enc_packed.p,
                                      ctx->stream)))
            return rc;
        if (total && !(flags & TFBS_ENC_DEVICE_CODES))
            HIP_TRY(hipMemcpyAsync(B.enc_codes.p, ctx->enc_packed.p, total, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    B.enc_r0 = (uint32_t)r0;
    B.enc_r1 = (uint32_t)r1;
    B.enc_codes_host = !(flags & TFBS_ENC_DEVICE_CODES);
    return TFBS_OK;
}

namespace {

// The BGZF batches of one tfbs_batch_rows_bgzf call, across its pieces: batch i uses
// slot i % kBgSlots; a launched batch is written out once two more are queued behind
// it (also across pieces), so the GPU never waits for a copy back or a file write.
int bgzf_drain(tfbs_ctx *ctx, int k, int fd, uint64_t &written);
struct BgPipe {
    uint64_t next = 0;                      // the call's next batch
    int pending[tfbs_ctx::kBgSlots] = {};   // launched batches not yet written (their slots, oldest first)
    int n_pending = 0;
    uint64_t written = 0;
    int drain_oldest(tfbs_ctx *ctx, int fd) {
        const int rc = bgzf_drain(ctx, pending[0], fd, written);
        for (int i = 1; i < n_pending; i++) pending[i - 1] = pending[i];
        n_pending--;
        return rc;
    }
};

// n bytes to fd at its offset, which moves past them.  A large write goes out as
// positioned pieces on a few threads (a page-cache copy runs ~2-3 GB/s per thread:
// one thread made the rows' write the run flow's longest host step); a descriptor
// without an offset (a pipe) takes plain writes.
static int write_out(int fd, const char *p, uint64_t n) {
    auto seq = [](int fd, const char *p, uint64_t n, int64_t at) -> int {  // at < 0: write()
        for (uint64_t o = 0; o < n;) {
            const size_t m = (size_t)std::min<uint64_t>(n - o, 1u << 30);
            const ssize_t w = at < 0 ? ::write(fd, p + o, m) : ::pwrite(fd, p + o, m, (off_t)(at + (int64_t)o));
            if (w < 0) {
                if (errno == EINTR) continue;
                return errno ? errno : EIO;
            }
            o += (uint64_t)w;
        }
        return 0;
    };
    constexpr uint64_t kPiece = 32u << 20;
    const off_t at = n >= 2 * kPiece ? lseek(fd, 0, SEEK_CUR) : (off_t)-1;
    int err = 0;
    if (at < 0) {
        err = seq(fd, p, n, -1);
    } else {
        const uint32_t T = (uint32_t)std::min<uint64_t>(4, n / kPiece);
        std::vector<int> errs(T, 0);
        std::vector<std::thread> ts;
        for (uint32_t t = 1; t < T; t++)
            ts.emplace_back([&, t] { errs[t] = seq(fd, p + n * t / T, n * (t + 1) / T - n * t / T, at + (int64_t)(n * t / T)); });
        errs[0] = seq(fd, p, n / T, at);
        for (auto &x : ts) x.join();
        for (int e : errs) err = err ? err : e;
        if (!err && lseek(fd, at + (off_t)n, SEEK_SET) < 0) err = errno;
    }
    return err ? tfbs::fail(TFBS_E_IO, std::string("write: ") + strerror(err)) : TFBS_OK;
}

// The launched batch in slot k: its packed blocks back (copy stream) and to fd.
static_assert(tfbs_ctx::kBgSlots == 3, "RowsWriter::busy has a flag per slot");

// The threads of rows_set_async: the copier takes the drained slots in order, copies
// each back (the main thread waits for its event to be recorded before it launches
// into the slot again) and hands it to the writer, which writes them in order -- a
// slot's copy overlaps the previous slot's write.  TFBS_ROWS_WRITER_DELAY_US: a pause
// before each copy (tests: the caller runs ahead of the copies).
static void rows_copier_loop(tfbs_ctx *ctx) {
    auto &w = ctx->rw;
    for (;;) {
        tfbs_ctx::RowsWriter::Job j;
        {
            std::unique_lock<std::mutex> l(w.mu);
            w.cv.wait(l, [&] { return w.stop || !w.q.empty(); });
            if (w.q.empty()) {  // (stop with nothing queued)
                w.copier_done = true;
                w.cv.notify_all();
                return;
            }
            j = w.q.front();
            w.q.pop_front();
        }
        const double t0 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        int rc = TFBS_OK;
        std::string err;
        {
            std::lock_guard<std::mutex> l(w.mu);
            rc = w.rc;  // (after a failure the rest are dropped)
        }
        const int delay_us = env_int("TFBS_ROWS_WRITER_DELAY_US", 0);
        if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
        hipError_t he = hipSetDevice(ctx->device);
        if (!rc && (rc = ctx->bg_host[j.k].reserve(std::max<uint64_t>(j.n, 1)))) err = tfbs_last_error();
        if (!rc && he == hipSuccess && j.n)
            he = hipMemcpyAsync(ctx->bg_host[j.k].p, ctx->bg_packed[j.k].p, j.n, hipMemcpyDeviceToHost, ctx->copy_stream);
        if (he == hipSuccess) he = hipEventRecord(ctx->bg_copied[j.k], ctx->copy_stream);
        {
            std::lock_guard<std::mutex> l(w.mu);
            w.recorded[j.k] = true;  // (also on failure: the stream's wait must not block)
        }
        w.cv.notify_all();
        if (he == hipSuccess) he = hipEventSynchronize(ctx->bg_copied[j.k]);
        if (!rc && he != hipSuccess) {
            rc = TFBS_E_HIP;
            err = std::string("rows copy back: ") + hipGetErrorString(he);
        }
        const double t1 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        {
            std::lock_guard<std::mutex> l(w.mu);
            w.copy_s += t1 - t0;
            if (rc && !w.rc) {
                w.rc = rc;
                w.err = err;
            }
            w.wq.push_back(j);
        }
        w.cv.notify_all();
    }
}

static void rows_writer_loop(tfbs_ctx *ctx) {
    auto &w = ctx->rw;
    for (;;) {
        tfbs_ctx::RowsWriter::Job j;
        int rc;
        {
            std::unique_lock<std::mutex> l(w.mu);
            w.cv.wait(l, [&] { return !w.wq.empty() || (w.stop && w.copier_done); });
            if (w.wq.empty()) return;
            j = w.wq.front();
            w.wq.pop_front();
            rc = w.rc;
        }
        const double t0 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        std::string err;
        if (!rc && (rc = write_out(j.fd, reinterpret_cast<const char *>(ctx->bg_host[j.k].p), j.n))) err = tfbs_last_error();
        const double t1 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        {
            std::lock_guard<std::mutex> l(w.mu);
            w.busy[j.k] = false;
            w.write_s += t1 - t0;
            if (rc && !w.rc) {
                w.rc = rc;
                w.err = err;
            }
        }
        w.cv.notify_all();
    }
}

// Waits until slot k's last job is done (k >= 0), until its copy back is enqueued
// (recorded), or until every queued job is done (k < 0); the writer's first failure.
static int rows_wait(tfbs_ctx *ctx, int k, bool recorded = false) {
    auto &w = ctx->rw;
    std::unique_lock<std::mutex> l(w.mu);
    w.cv.wait(l, [&] {
        if (k >= 0) return !w.busy[k] || (recorded && w.recorded[k]);
        for (bool b : w.busy)
            if (b) return false;
        return w.q.empty() && w.wq.empty();
    });
    return w.rc ? tfbs::fail(w.rc, w.err) : TFBS_OK;
}

int bgzf_drain(tfbs_ctx *ctx, int k, int fd, uint64_t &written) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = now();
    HIP_TRY(hipEventSynchronize(ctx->bg_done[k]));
    const double t1 = now();
    const uint64_t total = ctx->bg_total_host[k];
    int r;
    if (ctx->rows_async) {  // the writer thread copies it back and writes it (in order)
        if (!ctx->rw.th.joinable()) {
            ctx->rw.th = std::thread(rows_copier_loop, ctx);
            ctx->rw.th2 = std::thread(rows_writer_loop, ctx);
        }
        if ((r = rows_wait(ctx, k))) return r;  // slot k's last job is done (its host buffer free)
        {
            std::lock_guard<std::mutex> l(ctx->rw.mu);
            ctx->rw.busy[k] = true;
            ctx->rw.recorded[k] = false;
            ctx->rw.q.push_back({fd, k, total});
        }
        ctx->rw.cv.notify_all();
        ctx->drain_s[0] += t1 - t0;
        written += total;
        return TFBS_OK;
    }
    if ((r = ctx->bg_host[k].reserve(std::max<uint64_t>(total, 1)))) return r;
    if (total)
        HIP_TRY(hipMemcpyAsync(ctx->bg_host[k].p, ctx->bg_packed[k].p, total, hipMemcpyDeviceToHost, ctx->copy_stream));
    HIP_TRY(hipEventRecord(ctx->bg_copied[k], ctx->copy_stream));
    HIP_TRY(hipEventSynchronize(ctx->bg_copied[k]));
    const double t2 = now();
    ctx->drain_s[0] += t1 - t0;
    ctx->drain_s[1] += t2 - t1;
    written += total;
    if ((r = write_out(fd, reinterpret_cast<const char *>(ctx->bg_host[k].p), total))) return r;  // the blocks as they are
    ctx->drain_s[2] += now() - t2;
    return TFBS_OK;
}

// The device half of tfbs_batch_rows_bgzf: one row plan's BGZF blocks launched on the
// GPU (older batches written out as newer ones queue: BgPipe).  plan and heads (its
// heads as uploaded) must stay untouched until one of this piece's batches has been
// written out.

// TFBS_BGZF_PROF: the launch's bgzf_wave_kernel phase clocks (debug; synchronises).
static int bgzf_prof_report(tfbs_ctx *ctx, uint32_t nb) {
    std::vector<uint64_t> h((size_t)nb * 32);
    HIP_TRY(hipMemcpyAsync(h.data(), ctx->bg_prof.p, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    double ph[5] = {0, 0, 0, 0, 0}, items = 0, st[16] = {}, list_a = 0;
    uint32_t nw = 0;
    for (uint32_t b = 0; b < nb; b++) {
        const uint64_t *p = &h[(size_t)b * 32];
        if (!p[5]) continue;  // a bgzf_block_kernel block
        nw++;
        for (int k = 0; k < 5; k++) ph[k] += (double)(p[k + 1] - p[k]);
        if (p[7]) list_a += (double)(p[7] - p[1]);
        items += (double)p[6];
        for (int k = 0; k < 16; k++) st[k] += (double)p[8 + k];
    }
    const double d = nw ? nw : 1;
    fprintf(stderr,
            "[bgzf prof] blocks %u wave %u cycles/block: stage %.0f list %.0f items %.0f crc %.0f out %.0f; per block: "
            "items %.1f spins %.1f all-run %.1f look-back %.1f token-lit %.1f byte-lit %.1f heads %.1f newlines %.1f\n",
            nb, nw, ph[0] / d, ph[1] / d, ph[2] / d, ph[3] / d, ph[4] / d, items / d, st[0] / d, st[1] / d, st[2] / d,
            st[3] / d, st[4] / d, st[5] / d, st[6] / d);
    // wave-cycles per block: counting run groups / other groups, the deferred emits, the
    // groups with byte literals; other groups, those on the sample-by-sample look-back
    fprintf(stderr,
            "[bgzf prof] item cycles/block: count run groups %.0f, other groups %.0f; emit %.0f; byte-literal groups "
            "%.0f; other groups %.1f, on the serial look-back %.1f; listing: literal codes and run tests %.0f\n",
            st[8] / d, st[11] / d, st[9] / d, st[12] / d, st[7] / d, st[14] / d, list_a / d);
    return TFBS_OK;
}

int rows_bgzf_device(tfbs_ctx *ctx, const Batch &B, tfbs::RowPlan &plan, std::vector<char> &heads, int fd,
                     BgPipe &pp) {
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    int rc;
    struct Done {  // the device part's seconds, on every exit
        tfbs_ctx *c;
        double t;
        double (*f)();
        ~Done() { c->rows_s[1] += f() - t; }
    } done{ctx, now(), +[] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }};
    const uint32_t N = B.n_samples, ng = (N + kCumGroup - 1) / kCumGroup;
    const uint64_t n_blocks = (plan.text_bytes + kBgzfRaw - 1) / kBgzfRaw;
    if ((uint64_t)plan.rows.size() * (ng + 1) >= UINT32_MAX) return tfbs::fail(TFBS_E_NOMEM, "too many rows in one call");
    for (size_t i = 0; i < plan.rows.size(); i++) plan.rows[i].cum_off = (uint32_t)(i * (ng + 1));
    if (!n_blocks) {  // nothing launched: the pending batches go out now (their pieces' host data is released)
        while (pp.n_pending)
            if ((rc = pp.drain_oldest(ctx, fd))) return rc;
        return TFBS_OK;
    }
    if (!ctx->bg_crc.n) {  // CRC32 byte table, shift operators and slice tables, once per ctx
        std::vector<uint32_t> t(tfbs::kBgzfCrcWords);
        ctx->bg_crc_full = tfbs::bgzf_crc_tables(t.data(), t.data() + 256, t.data() + 256 + 32 * kBgzfOps,
                                                 t.data() + 256 + 32 * kBgzfOps + 768);
        if ((rc = ctx->bg_crc.put(t, ctx->stream))) return rc;
        HIP_TRY(hipStreamSynchronize(ctx->stream));  // (t goes out of scope)
    }
    heads.assign(plan.heads.begin(), plan.heads.end());
    if ((rc = ctx->bg_rows.put(plan.rows, ctx->stream)) || (rc = ctx->bg_heads.put(heads, ctx->stream)) ||
        (rc = ctx->bg_tok_text.put(plan.tok_text, ctx->stream)) ||
        (rc = ctx->bg_tok_len.put(plan.tok_len, ctx->stream)) ||
        (rc = ctx->bg_tok_lit.ensure(std::max<size_t>(plan.tok_len.size(), 1))) ||
        (rc = ctx->bg_tok_litn.ensure(std::max<size_t>(plan.tok_len.size(), 1))) ||
        (rc = ctx->bg_cum.ensure(std::max<size_t>(plan.rows.size() * (ng + 1), 1))))
        return rc;
    tfbs::BgArgs a{};
    a.rows = ctx->bg_rows.p;
    a.n_rows = (uint32_t)plan.rows.size();
    a.heads = ctx->bg_heads.p;
    a.tok_text = ctx->bg_tok_text.p;
    a.tok_len = ctx->bg_tok_len.p;
    a.tok_lit = ctx->bg_tok_lit.p;
    a.tok_litn = ctx->bg_tok_litn.p;
    a.codes = ctx->enc_packed.p;
    a.cum = ctx->bg_cum.p;
    a.n_samples = N;
    a.text_bytes = plan.text_bytes;
    a.crc_tab = ctx->bg_crc.p;
    a.crc_ops = ctx->bg_crc.p + 256;
    a.crc_slice = ctx->bg_crc.p + 256 + 32 * kBgzfOps;
    a.crc_lane = ctx->bg_crc.p + 256 + 32 * kBgzfOps + 768;
    a.crc_full = ctx->bg_crc_full;
    a.stored = env_int("TFBS_BGZF_STORED", 0) != 0 ? 1u : 0u;
    const bool bg_check = env_int("TFBS_BGZF_CHECK", 0) != 0;  // (debug: checked every launch, synchronously)
    if (bg_check) {
        if ((rc = ctx->bg_check.ensure(1))) return rc;
        HIP_TRY(hipMemsetAsync(ctx->bg_check.p, 0, 4, ctx->stream));
        a.check = ctx->bg_check.p;
    }
    if ((rc = tfbs::launch_tok_lit(a, (uint32_t)plan.tok_len.size(), ctx->stream)) ||
        (rc = tfbs::launch_row_cum(a, ctx->stream)))
        return rc;
    // blocks per launch (512 MiB of block slots); TFBS_BGZF_BATCH_BLOCKS=n: smaller
    // launches, so one call cycles the kBgSlots slots (the tests' path)
    const uint64_t kBatchBlocks = (uint64_t)std::max(1, env_int("TFBS_BGZF_BATCH_BLOCKS", 8192));
    const uint64_t n_batches = (n_blocks + kBatchBlocks - 1) / kBatchBlocks;
    if (!ctx->bg_total_host)
        HIP_TRY(hipHostMalloc((void **)&ctx->bg_total_host, 8 * tfbs_ctx::kBgSlots, hipHostMallocDefault));
    for (int k = 0; k < tfbs_ctx::kBgSlots; k++) {
        if (!ctx->bg_done[k]) HIP_TRY(hipEventCreateWithFlags(&ctx->bg_done[k], hipEventDisableTiming));
        if (!ctx->bg_copied[k]) HIP_TRY(hipEventCreateWithFlags(&ctx->bg_copied[k], hipEventDisableTiming));
    }
    if (!ctx->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    for (uint64_t i = 0; i < n_batches; i++, pp.next++) {
        const int k = (int)(pp.next % tfbs_ctx::kBgSlots);
        const uint64_t b0 = i * kBatchBlocks;
        const uint32_t nb = (uint32_t)std::min(kBatchBlocks, n_blocks - b0);
        if (ctx->rw.th.joinable()) {
            // async rows: slot k's last copy back -- of this call or of an earlier one, which
            // returned before its copies ran -- must be enqueued by the writer thread before
            // the stream may wait for it (below), and done before the slot's buffers grow
            // (a reallocation under a pending copy sent zeros to the file)
            const bool grows = ctx->bg_out[k].cap < (size_t)nb * kBgzfMax || ctx->bg_packed[k].cap < (size_t)nb * kBgzfMax ||
                               ctx->bg_out_len[k].cap < nb || ctx->bg_off[k].cap < (size_t)nb + 1;
            if ((rc = rows_wait(ctx, k, !grows))) return rc;
        }
        if ((rc = ctx->bg_out[k].ensure((size_t)nb * kBgzfMax)) || (rc = ctx->bg_out_len[k].ensure(nb)) ||
            (rc = ctx->bg_off[k].ensure(nb + 1)) || (rc = ctx->bg_packed[k].ensure((size_t)nb * kBgzfMax)) ||
            (rc = ctx->bg_plans.ensure((size_t)nb * tfbs::bgzf_plan_bytes())))
            return rc;
        // slot k's packed blocks were copied back (kBgSlots batches ago) before they are overwritten
        if (ctx->rw.th.joinable()) {  // (waited for above)
            HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->bg_copied[k], 0));
        } else if (pp.next >= (uint64_t)tfbs_ctx::kBgSlots) {  // (an earlier call's copies are done)
            HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->bg_copied[k], 0));
        }
        a.plans = ctx->bg_plans.p;
        a.block0 = b0;
        a.out = ctx->bg_out[k].p;
        a.out_len = ctx->bg_out_len[k].p;
        static const bool prof = env_int("TFBS_BGZF_PROF", 0) != 0;
        if (prof) {
            if ((rc = ctx->bg_prof.ensure((size_t)nb * 32))) return rc;
            HIP_TRY(hipMemsetAsync(ctx->bg_prof.p, 0, (size_t)nb * 256, ctx->stream));
            a.prof = ctx->bg_prof.p;
        }
        if ((rc = tfbs::launch_bgzf_blocks(a, nb, ctx->stream)) || (prof && (rc = bgzf_prof_report(ctx, nb))) ||
            (rc = tfbs::launch_bgzf_compact(ctx->bg_out[k].p, ctx->bg_out_len[k].p, ctx->bg_off[k].p, nb,
                                            ctx->bg_packed[k].p, ctx->stream)))
            return rc;
        if (bg_check) {
            uint32_t bad = 0;
            HIP_TRY(hipMemcpyAsync(&bad, ctx->bg_check.p, 4, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            if (bad)
                return fail(TFBS_E_STATE, "bgzf_wave_kernel: " + std::to_string(bad) +
                                                 " block-text writes met bits already set (TFBS_BGZF_CHECK)");
        }
        HIP_TRY(hipMemcpyAsync(ctx->bg_total_host + k, ctx->bg_off[k].p + nb, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipEventRecord(ctx->bg_done[k], ctx->stream));
        pp.pending[pp.n_pending++] = k;
        if (pp.n_pending == tfbs_ctx::kBgSlots && (rc = pp.drain_oldest(ctx, fd))) return rc;
    }
    return TFBS_OK;
}

}  // namespace

}  // extern "C"

namespace tfbs {

void rows_bgzf_drain_seconds(const ::tfbs_ctx *ctx, double out[3]) {
    for (int i = 0; i < 3; i++) out[i] = ctx ? ctx->drain_s[i] : 0.0;
    if (ctx) {  // (the writer thread's, read after rows_flush)
        out[1] += ctx->rw.copy_s;
        out[2] += ctx->rw.write_s;
    }
}

void rows_set_async(::tfbs_ctx *ctx, bool on) {
    if (ctx) ctx->rows_async = on;
}

int rows_flush(::tfbs_ctx *ctx) {
    if (!ctx || !ctx->rw.th.joinable()) return TFBS_OK;
    return rows_wait(ctx, -1);
}

// tfbs_batch_rows_bgzf; pos_base (optional): the POS base is asked for once the
// call's rows are counted (every piece's row parts built first).
int rows_bgzf_chained(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, const char *chromosome, uint32_t min_maf,
                      uint32_t *fake_position, int fd, uint64_t *bytes, uint64_t *n_rows,
                      const std::function<int(uint64_t, uint32_t *)> &pos_base) {
    if (!ctx || !b || !chromosome || !fake_position || fd < 0) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    Batch &B = b->b;
    r1 = std::min(r1, B.rh.size());
    r0 = std::min(r0, r1);
    if (!B.reduced || B.enc_r0 > r0 || B.enc_r1 < r1)
        return tfbs::fail(TFBS_E_STATE, "regions not encoded on this ctx (tfbs_batch_encode)");
    HIP_TRY(hipSetDevice(ctx->device));
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    // the regions in pieces of >= 64 (at most 8): a helper thread formats piece j + 1's
    // rows (the host row plan: heads, POS, token tables) while the GPU makes piece j's
    // blocks; every piece starts a new BGZF block (the decompressed stream is the same).
    // kBgSlots + 1 plan slots: piece j's host data (uploaded by its device half) stays
    // put until one of its batches has been written out -- by then the host has waited
    // for an event after its uploads -- which BgPipe's lag guarantees before the helper
    // builds piece j + kBgSlots + 1 into the same slot.
    const size_t n = r1 - r0;
    const size_t pieces = std::max<size_t>(1, std::min<size_t>(8, n / 64));
    auto cut = [&](size_t j) { return r0 + n * j / pieces; };
    const std::string chrom(chromosome);
    constexpr size_t kPlanSlots = tfbs_ctx::kBgSlots + 1;
    tfbs::RowPlan plans[kPlanSlots];
    std::vector<char> heads[kPlanSlots];
    std::shared_ptr<RowParts> parts;  // pos_base: every piece's rows before the first POS
    if (pos_base) {
        const double t0 = now();
        uint64_t nr = 0;
        int rc = build_row_parts(B, r0, r1, min_maf, ctx->host_threads, parts, &nr);
        ctx->rows_s[0] += now() - t0;
        if (rc || (rc = pos_base(nr, fake_position))) return rc;
    }
    auto build = [&](size_t j) {
        const double t0 = now();
        const int r = parts ? plan_from_parts(B, *parts, cut(j), cut(j + 1), chrom, fake_position, plans[j % kPlanSlots])
                            : tfbs::build_row_plan(B, cut(j), cut(j + 1), chrom, min_maf, fake_position,
                                                   ctx->host_threads, plans[j % kPlanSlots]);
        ctx->rows_s[0] += now() - t0;
        return r;
    };
    int rc = build(0);
    if (rc) return rc;
    BgPipe pp;
    uint64_t rows = 0, text = 0;
    for (size_t j = 0; j < pieces; j++) {
        int next_rc = TFBS_OK;
        std::thread helper;
        if (j + 1 < pieces) helper = std::thread([&, j] { next_rc = build(j + 1); });
        tfbs::RowPlan &plan = plans[j % kPlanSlots];
        rows += plan.n_rows;
        text += plan.text_bytes;
        rc = rows_bgzf_device(ctx, B, plan, heads[j % kPlanSlots], fd, pp);
        if (helper.joinable()) helper.join();
        if (rc) return rc;
        if (next_rc) return next_rc;
    }
    {
        const double t0 = now();
        while (pp.n_pending && !rc) rc = pp.drain_oldest(ctx, fd);
        ctx->rows_s[1] += now() - t0;
        if (rc) return rc;
    }
    if (n_rows) *n_rows = rows;
    if (bytes) *bytes = pp.written;
    ctx->rows_text_last = text;
    return TFBS_OK;
}

}  // namespace tfbs

extern "C" {

int tfbs_batch_rows_bgzf(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, const char *chromosome,
                         uint32_t min_maf, uint32_t *fake_position, int fd, uint64_t *bytes, uint64_t *n_rows,
                         uint64_t *text_bytes) {
    const int rc = tfbs::rows_bgzf_chained(ctx, b, r0, r1, chromosome, min_maf, fake_position, fd, bytes, n_rows, {});
    if (!rc && text_bytes) *text_bytes = ctx->rows_text_last;
    return rc;
}

int tfbs_matches(tfbs_ctx *ctx, const uint8_t *nucs, const uint64_t *pos, size_t n, uint32_t *counts,
                 uint64_t *out_start, uint64_t *out_end, size_t cap, size_t *n_total) {
    if (!ctx || !n_total || !counts || (n && (!nucs || !pos))) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (n >= kMaxHapLen) return tfbs::fail(TFBS_E_ARG, "haplotype longer than 2^26 - 1 bases");
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
    std::vector<DevRegion> regions{DevRegion{0, 0, 0, 1, UINT32_MAX, 1, 0}};
    std::vector<int32_t> inner{0, 0}, posrel{0};
    ctx->asm_order_n = 0;  // (this one-haplotype upload replaces the resident batch)
    const uint32_t wpp = (uint32_t)((n + 255) / 256 * 4);
    HIP_TRY(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ctx->words.put(words, ctx->stream)) || (rc = ctx->nmask.put(nmask, ctx->stream)) ||
        (rc = ctx->posrel.put(posrel, ctx->stream)) || (rc = ctx->haps.put(haps, ctx->stream)) ||
        (rc = ctx->regions.put(regions, ctx->stream)) || (rc = ctx->inner.put(inner, ctx->stream)) ||
        (rc = ctx->counts.ensure(std::max<uint64_t>(P.pats.size(), 1))) || (rc = ctx->druns.ensure(1)) ||
        (rc = build_lists(ctx, 1, std::vector<uint8_t>{(uint8_t)(n <= kWlNarrowLen)})))
        return rc;
    ctx->counts_live = true;
    ctx->resident = nullptr;
    ctx->scanned = false;
    ctx->mfma_group_words = mfma_group_words(haps.data(), 1, ctx->mfma_hpb);
    ctx->n_regions = 1;
    const size_t nh = (size_t)P.pats.size() * wpp;
    if ((rc = ctx->hits.ensure(std::max<size_t>(nh, 1)))) return rc;
    if (nh) HIP_TRY(hipMemsetAsync(ctx->hits.p, 0, nh * 8, ctx->stream));
    int l = launch_scan(ctx, 1, ctx->hits.p, wpp);
    if (l < 0) return l;
    if ((rc = check_overflow(ctx, 1, ctx->hits.p, wpp))) return rc;  // a rescan (larger lists) sets the same bits again
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

namespace tfbs {

int ensure_host_var_counts(const Batch &B) {
    std::lock_guard<std::mutex> g(B.var_mu);
    if (B.var_host) return B.var_err;
    Batch &M = const_cast<Batch &>(B);
    int rc = M.var_counts.reserve(std::max<size_t>(B.var_n * 4, 1));
    if (!rc && B.var_n) {
        int dev = -1;
        (void)hipGetDevice(&dev);
        const hipError_t e = hipSetDevice(B.var_device);
        const hipError_t c = e == hipSuccess ? hipMemcpy(M.var_counts.p, B.var_dev, B.var_n * 4, hipMemcpyDeviceToHost) : e;
        if (dev >= 0) (void)hipSetDevice(dev);
        if (c != hipSuccess) rc = fail(TFBS_E_HIP, std::string("varying counts download: ") + hipGetErrorString(c));
    }
    M.var_host = true;
    M.var_err = rc;
    M.var_dev = nullptr;
    return rc;
}

void forget_var_counts(Batch &B) {
    if (B.var_ctx && B.var_ctx->var_owner == &B) B.var_ctx->var_owner = nullptr;
    B.var_ctx = nullptr;
}

}  // namespace tfbs
