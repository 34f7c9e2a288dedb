// Device context and the device-side C-ABI (tfbs_ctx_*, tfbs_batch_upload,
// tfbs_scan, tfbs_batch_download, tfbs_matches).  The kernels live in
// scan_kernels.hip; this file owns device memory, the stream and timing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "batch.hpp"
#include "patterns.hpp"
#include "keys.hpp"
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
    hipEvent_t evk0 = nullptr, evk1 = nullptr;  // around the dominant kernel (the MFMA launches)
    // the per-depth MFMA launches run on kSide + 1 streams so that they overlap
    static constexpr int kSide = 3;
    hipStream_t side[kSide] = {};
    hipEvent_t fork = nullptr, join[kSide] = {};
    // the matrix-core scan adds into zeroed counts: the idle buffer of a pair is
    // zeroed on zero_stream beside each scan, for the next one (TFBS_PREZERO)
    hipStream_t zero_stream = nullptr;
    hipEvent_t zero_fork = nullptr, zero_ev = nullptr;
    size_t alt_zero_n = 0;  // counts_alt's elements zeroed (0: none pending)
    bool prezero = true;
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
    DevBuf<uint32_t> cands;              // matrix-core candidate lists (scan.hpp)
    DevBuf<uint32_t> ref_hits, ref_count, ref_over, ref_over_count;  // reference-window reuse (scan.hpp)
    uint32_t ref_over_cap = 1u << 16;
    DevBuf<uint32_t> cand_over;  // candidates past the waves' list regions (scan.hpp)
    uint32_t cand_over_cap = 1u << 20;
    bool debug_over = false;  // TFBS_DEBUG_OVER: print the overflow lists' fill after each scan
    uint32_t n_regions = 0;                // of the resident batch
    uint32_t *ref_count_host = nullptr;    // pinned: the overflow lists' counts (reference hits, candidates)
    uint32_t cand_cap = 1024;            // per scan workgroup (TFBS_CAND_CAP)
    DevBuf<DevMSuper> m_supers;
    bool mfma = true;             // int8 matrix-core path for eligible strands (TFBS_MFMA=0: LUT only)
    uint32_t mfma_lds = 44 * 1024;  // LDS image budget of one MFMA super tile
    uint32_t mfma_hpb = 64;         // haplotypes per MFMA workgroup
    uint32_t mfma_group_words = 0;  // packed words of the largest haplotype group (LDS staging)
    // batch image
    DevBuf<uint32_t> words, nmask, counts, counts_alt;
    DevBuf<int32_t> posrel, inner;
    DevBuf<DevHap> haps;
    DevBuf<DevRegion> regions;
    DevBuf<unsigned long long> hits;
    // key reduction (tfbs_batch_reduce)
    DevBuf<uint32_t> key_first, var_counts;
    DevBuf<uint8_t> key_flags;
    DevBuf<DevVarKey> var_keys, enc_keys;
    // per-sample encoding (tfbs_batch_encode)
    DevBuf<uint8_t> enc_memb, enc_codes, enc_packed;
    tfbs::PinnedBytes enc_memb_host;  // membership rows staged for upload (reused; no zero fill)
    DevBuf<uint64_t> enc_off;
    DevBuf<EncHdr> enc_hdr;
    DevBuf<uint32_t> enc_vals, enc_hist;
    const tfbs_batch *resident = nullptr;
    float last_ms = 0.f;
    int last_launches = 0;
    bool timing_pending = false;
};

namespace tfbs {
int PinnedBytes::reserve(size_t n) {
    if (n <= cap) return TFBS_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const hipError_t e = hipHostMalloc((void **)&p, std::max<size_t>(n, 1 << 20), hipHostMallocDefault);
    if (e != hipSuccess) {
        p = nullptr;
        return tfbs::fail(TFBS_E_HIP, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    }
    cap = std::max<size_t>(n, 1 << 20);
    return TFBS_OK;
}
PinnedBytes::~PinnedBytes() {
    if (p) (void)hipHostFree(p);
}

}  // namespace tfbs

static int env_int(const char *name, int dflt) {
    const char *v = getenv(name);
    if (!v || !*v) return dflt;
    return atoi(v);
}

static int launch_scan(tfbs_ctx *ctx, uint32_t n_haps, unsigned long long *hits, uint32_t hits_wpp) {
    const Plan &P = ctx->plan;
    if (n_haps == 0) return 0;
    ScanArgs a{};
    a.haps = ctx->haps.p;
    a.n_haps = n_haps;
    a.regions = ctx->regions.p;
    a.inner = ctx->inner.p;
    a.words = ctx->words.p;
    a.nmask = ctx->nmask.p;
    a.posrel = ctx->posrel.p;
    a.counts = ctx->counts.p;
    a.haps_per_block = ctx->haps_per_block;
    a.hits = hits;
    a.hits_wpp = hits_wpp;
    a.n_patterns_total = (uint32_t)ctx->pats->pats.size();
    int launches = 0;
    if (!P.m_supers.empty()) {  // atomic adds: zero its slots first (the other kernels store theirs)
        if (ctx->counts.n) {
            const size_t need = ctx->counts.n;
            if (ctx->alt_zero_n >= need) {  // zeroed beside the previous scan
                std::swap(ctx->counts, ctx->counts_alt);
                ctx->counts.n = need;
                HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->zero_ev, 0));
            } else {
                HIP_TRY(hipMemsetAsync(ctx->counts.p, 0, need * 4, ctx->stream));
            }
            ctx->alt_zero_n = 0;
            a.counts = ctx->counts.p;
            if (ctx->prezero) {  // the other buffer for the next scan (its last reader is already queued)
                int rc;
                if ((rc = ctx->counts_alt.ensure(need))) return rc;
                HIP_TRY(hipEventRecord(ctx->zero_fork, ctx->stream));
                HIP_TRY(hipStreamWaitEvent(ctx->zero_stream, ctx->zero_fork, 0));
                HIP_TRY(hipMemsetAsync(ctx->counts_alt.p, 0, need * 4, ctx->zero_stream));
                HIP_TRY(hipEventRecord(ctx->zero_ev, ctx->zero_stream));
                ctx->alt_zero_n = need;
            }
        }
        ScanArgs m = a;
        m.msupers = ctx->m_supers.p;
        m.n_msupers = (uint32_t)P.m_supers.size();
        m.mimage = ctx->m_image.p;
        m.mweights = ctx->m_weights.p;
        m.mmeta = ctx->m_meta.p;
        m.haps_per_block = ctx->mfma_hpb;
        // one candidate region per scan workgroup (super tile x haplotype group)
        const uint64_t n_regions = (uint64_t)P.m_supers.size() * ((n_haps + ctx->mfma_hpb - 1) / ctx->mfma_hpb);
        int rc;
        if ((rc = ctx->cands.ensure(n_regions * ctx->cand_cap * kCandWords))) return rc;
        m.cands = ctx->cands.p;
        m.cand_cap = ctx->cand_cap;
        const uint32_t nr = std::max<uint32_t>(1, ctx->n_regions);
        if ((rc = ctx->ref_count.ensure(nr)) || (rc = ctx->ref_hits.ensure((size_t)nr * kRefPerRegion * 2)) ||
            (rc = ctx->ref_over_count.ensure(2)) || (rc = ctx->ref_over.ensure((size_t)ctx->ref_over_cap * 3)) ||
            (rc = ctx->cand_over.ensure((size_t)ctx->cand_over_cap * 3)))
            return rc;
        m.dedup = 1;
        m.n_regions = ctx->n_regions;
        m.ref_hits = ctx->ref_hits.p;
        m.ref_count = ctx->ref_count.p;
        m.ref_over = ctx->ref_over.p;
        m.ref_over_count = ctx->ref_over_count.p;
        m.ref_over_cap = ctx->ref_over_cap;
        m.cand_over = ctx->cand_over.p;
        m.cand_over_cap = ctx->cand_over_cap;
        HIP_TRY(hipMemsetAsync(ctx->ref_count.p, 0, (size_t)nr * 4, ctx->stream));
        HIP_TRY(hipMemsetAsync(ctx->ref_over_count.p, 0, 8, ctx->stream));
        HIP_TRY(hipEventRecord(ctx->evk0, ctx->stream));
        HIP_TRY(hipEventRecord(ctx->fork, ctx->stream));
        hipStream_t streams[tfbs_ctx::kSide + 1] = {ctx->stream};
        for (int i = 0; i < tfbs_ctx::kSide; i++) {
            HIP_TRY(hipStreamWaitEvent(ctx->side[i], ctx->fork, 0));
            streams[i + 1] = ctx->side[i];
        }
        const int n = launch_mfma(m, P.m_supers.data(), (uint32_t)P.m_supers.size(), ctx->mfma_group_words, n_haps,
                                  streams, tfbs_ctx::kSide + 1);
        if (n < 0) return n;
        for (int i = 0; i < tfbs_ctx::kSide; i++) {
            HIP_TRY(hipEventRecord(ctx->join[i], ctx->side[i]));
            HIP_TRY(hipStreamWaitEvent(ctx->stream, ctx->join[i], 0));
        }
        HIP_TRY(hipEventRecord(ctx->evk1, ctx->stream));
        ctx->kernel_timed = true;
        launches += n;
        const int f = launch_ref_fixup(m, ctx->stream);
        if (f < 0) return f;
        launches += f;
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
    ctx->fast_units.release(); ctx->gen_pats.release(); ctx->fast_tiles.release(); ctx->gen_tiles.release();
    ctx->lut.release(); ctx->wfull.release(); ctx->gen_w.release();
    ctx->m_image.release(); ctx->m_weights.release(); ctx->m_meta.release(); ctx->m_supers.release();
    ctx->cands.release(); ctx->cand_over.release(); ctx->ref_hits.release(); ctx->ref_count.release(); ctx->ref_over.release();
    ctx->ref_over_count.release();
    if (ctx->ref_count_host) (void)hipHostFree(ctx->ref_count_host);
    ctx->words.release(); ctx->nmask.release(); ctx->counts.release(); ctx->counts_alt.release(); ctx->posrel.release();
    ctx->inner.release(); ctx->haps.release(); ctx->regions.release(); ctx->hits.release();
    ctx->key_first.release(); ctx->var_counts.release(); ctx->key_flags.release(); ctx->var_keys.release();
    ctx->enc_keys.release(); ctx->enc_memb.release(); ctx->enc_codes.release(); ctx->enc_hdr.release();
    ctx->enc_vals.release(); ctx->enc_hist.release(); ctx->enc_packed.release(); ctx->enc_off.release();
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->evk0) (void)hipEventDestroy(ctx->evk0);
    if (ctx->evk1) (void)hipEventDestroy(ctx->evk1);
    for (int i = 0; i < tfbs_ctx::kSide; i++) {
        if (ctx->side[i]) (void)hipStreamSynchronize(ctx->side[i]);
        if (ctx->side[i]) (void)hipStreamDestroy(ctx->side[i]);
        if (ctx->join[i]) (void)hipEventDestroy(ctx->join[i]);
    }
    if (ctx->fork) (void)hipEventDestroy(ctx->fork);
    if (ctx->zero_fork) (void)hipEventDestroy(ctx->zero_fork);
    if (ctx->zero_ev) (void)hipEventDestroy(ctx->zero_ev);
    if (ctx->zero_stream) (void)hipStreamDestroy(ctx->zero_stream);
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
    ctx->mfma_hpb = (uint32_t)std::min(256, std::max(4, env_int("TFBS_MFMA_HAPS_PER_BLOCK", 64)));  // 8 bits in a candidate entry
    ctx->cand_cap = (uint32_t)std::min(1 << 16, std::max(64, env_int("TFBS_CAND_CAP", 1024)));
    ctx->prezero = env_int("TFBS_PREZERO", 1) != 0;
    ctx->debug_over = env_int("TFBS_DEBUG_OVER", 0) != 0;
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
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->zero_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->zero_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->zero_ev, hipEventDisableTiming);
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
        (rc = ctx->m_supers.put(P.m_supers, ctx->stream))) {
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
            ms = 0.f;
            if (c->kernel_timed && hipEventElapsedTime(&ms, c->evk0, c->evk1) == hipSuccess) c->last_kernel_ms = ms;
        }
        c->timing_pending = false;
    }
    return c->last_ms;
}

int tfbs_ctx_last_scan_launches(const tfbs_ctx *ctx) { return ctx ? ctx->last_launches : 0; }

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
    int rc;
    if ((rc = ctx->words.put(B.words, ctx->stream)) || (rc = ctx->nmask.put(B.nmask, ctx->stream)) ||
        (rc = ctx->posrel.put(B.posrel, ctx->stream)) || (rc = ctx->haps.put(B.haps, ctx->stream)) ||
        (rc = ctx->regions.put(B.regions, ctx->stream)) || (rc = ctx->inner.put(B.inner, ctx->stream)) ||
        (rc = ctx->counts.ensure(B.n_counts)))
        return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    ctx->resident = b;
    ctx->mfma_group_words = mfma_group_words(B.haps.data(), (uint32_t)B.haps.size(), ctx->mfma_hpb);
    ctx->n_regions = (uint32_t)B.regions.size();
    return TFBS_OK;
}

int tfbs_scan(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not uploaded to this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipEventRecord(ctx->ev0, ctx->stream));
    ctx->kernel_timed = false;
    int n = launch_scan(ctx, (uint32_t)b->b.haps.size(), nullptr, 0);
    if (n < 0) return n;
    // the overflow lists (reference hits, candidates) must have held every entry:
    // otherwise grow them and scan again
    for (int round = 0; !ctx->plan.m_supers.empty(); round++) {
        if (!ctx->ref_count_host) HIP_TRY(hipHostMalloc((void **)&ctx->ref_count_host, 8, hipHostMallocDefault));
        HIP_TRY(hipMemcpyAsync(ctx->ref_count_host, ctx->ref_over_count.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        const uint32_t nref = ctx->ref_count_host[0], ncand = ctx->ref_count_host[1];
        if (ctx->debug_over)
            fprintf(stderr, "tfbs_scan overflow lists: reference hits %u/%u candidates %u/%u\n", nref,
                    ctx->ref_over_cap, ncand, ctx->cand_over_cap);
        if (nref <= ctx->ref_over_cap && ncand <= ctx->cand_over_cap) break;
        // a dropped candidate may have been a reference hit: the next scan is checked too
        if (round == 8) return tfbs::fail(TFBS_E_NOMEM, "scan overflow lists still full after 8 rescans");
        auto grow = [](uint32_t &cap, uint32_t need, uint64_t lim) {
            if (need > cap) cap = (uint32_t)std::min<uint64_t>(lim, (uint64_t)need * 5 / 4 + 1024);
        };
        grow(ctx->ref_over_cap, ncand > ctx->cand_over_cap ? 2 * std::max(nref, 1024u) : nref, UINT32_MAX / 4);
        grow(ctx->cand_over_cap, ncand, UINT32_MAX / 4);
        ctx->kernel_timed = false;
        n = launch_scan(ctx, (uint32_t)b->b.haps.size(), nullptr, 0);
        if (n < 0) return n;
    }
    HIP_TRY(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->last_launches = n;
    ctx->timing_pending = true;
    b->b.counts_valid = b->b.reduced = false;
    b->b.enc_r0 = b->b.enc_r1 = 0;
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

int tfbs_batch_reduce(tfbs_ctx *ctx, tfbs_batch *b) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    HIP_TRY(hipSetDevice(ctx->device));
    Batch &B = b->b;
    const uint64_t n_keys = (uint64_t)(B.inner.size() / 2) * B.n_slots;
    int rc;
    if ((rc = ctx->key_first.ensure(n_keys)) || (rc = ctx->key_flags.ensure(n_keys))) return rc;
    if ((rc = launch_key_reduce(ctx->haps.p, ctx->regions.p, (uint32_t)B.regions.size(), ctx->counts.p, B.n_slots,
                                ctx->key_first.p, ctx->key_flags.p, ctx->stream)))
        return rc;
    B.key_first.resize(n_keys);
    B.key_flags.resize(n_keys);
    if (n_keys) {
        HIP_TRY(hipMemcpyAsync(B.key_first.data(), ctx->key_first.p, n_keys * 4, hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipMemcpyAsync(B.key_flags.data(), ctx->key_flags.p, n_keys, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    // columns of the varying keys, one count per distinct haplotype
    std::vector<DevVarKey> vk;
    B.var_off.assign(n_keys, UINT32_MAX);
    B.var_idx.assign(n_keys, UINT32_MAX);
    uint64_t total = 0;
    for (uint32_t r = 0; r < B.regions.size(); r++) {
        const DevRegion &rg = B.regions[r];
        const uint64_t ko = (uint64_t)rg.inner_off * B.n_slots;
        const uint32_t K = B.n_slots * rg.n_inner;
        for (uint32_t j = 0; j < K; j++)
            if (B.key_flags[ko + j] & KEY_VARIES) {
                if (total + rg.hap_count >= UINT32_MAX) return tfbs::fail(TFBS_E_NOMEM, "too many varying counts");
                B.var_off[ko + j] = (uint32_t)total;
                B.var_idx[ko + j] = (uint32_t)vk.size();
                vk.push_back(DevVarKey{r, j, total});
                total += rg.hap_count;
            }
    }
    if ((rc = B.var_counts.reserve(total * 4))) return rc;
    B.var_keys = vk;
    B.enc_r0 = B.enc_r1 = 0;
    B.enc_idx.clear();
    if (!vk.empty()) {
        if ((rc = ctx->var_keys.put(vk, ctx->stream)) || (rc = ctx->var_counts.ensure(total))) return rc;
        if ((rc = launch_key_gather(ctx->haps.p, ctx->regions.p, ctx->counts.p, B.n_slots, ctx->var_keys.p,
                                    (uint32_t)vk.size(), ctx->var_counts.p, ctx->stream)))
            return rc;
        HIP_TRY(hipMemcpyAsync(B.var_counts.p, ctx->var_counts.p, total * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    B.reduced = true;
    return TFBS_OK;
}

int tfbs_batch_encode(tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1) {
    if (!ctx || !b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (ctx->resident != b) return tfbs::fail(TFBS_E_STATE, "batch not resident on this ctx");
    Batch &B = b->b;
    if (!B.reduced) return tfbs::fail(TFBS_E_STATE, "keys not reduced (tfbs_batch_reduce)");
    if (!B.keep_membership) return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    r1 = std::min(r1, B.rh.size());
    r0 = std::min(r0, r1);
    HIP_TRY(hipSetDevice(ctx->device));
    B.enc_r0 = B.enc_r1 = 0;
    B.enc_idx.assign(B.var_keys.size(), UINT32_MAX);
    B.enc_hdr.clear();
    B.enc_vals.clear();
    B.enc_hist.clear();
    B.enc_code_off.assign(1, 0);
    const uint32_t N = B.n_samples, H = 2 * N;
    if (N == 0 || r0 == r1) {
        B.enc_r0 = (uint32_t)r0;
        B.enc_r1 = (uint32_t)r1;
        return TFBS_OK;
    }
    // the keys to encode: varying keys of [r0, r1) whose region has <= 255 distinct haplotypes
    std::vector<DevVarKey> ek;
    std::vector<uint32_t> ek_var;
    for (uint32_t i = 0; i < B.var_keys.size(); i++) {
        const DevVarKey &k = B.var_keys[i];
        if (k.region < r0 || k.region >= r1 || B.regions[k.region].hap_count > kEncMaxHaps) continue;
        B.enc_idx[i] = (uint32_t)ek.size();
        ek.push_back(k);
        ek_var.push_back(i);
    }
    const size_t nk = ek.size();
    // membership rows: haplotype id -> distinct index (u8), 2 N bytes per region of
    // [r0, r1), written by the host threads into the ctx's pinned staging buffer
    // (rows of regions with no encoded keys are left unwritten: never read)
    const size_t mbytes = (r1 - r0) * (size_t)H;
    int rc;
    if ((rc = ctx->enc_memb_host.reserve(mbytes))) return rc;
    uint8_t *const memb = ctx->enc_memb_host.p;
    {
        const uint32_t T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::atomic<size_t> next(r0);
        auto work = [&]() {
            for (size_t r; (r = next.fetch_add(1)) < r1;) {
                const RegionH &R = B.rh[r];
                if (R.hap_count > kEncMaxHaps) continue;
                uint8_t *row = memb + (r - r0) * (size_t)H;
                memset(row, R.ref_local < 0 ? 0 : R.ref_local, H);
                for (size_t i = 0; i < R.nonref_id.size(); i++) row[R.nonref_id[i]] = (uint8_t)R.nonref_local[i];
            }
        };
        std::vector<std::thread> ts;
        for (uint32_t t = 1; t < T; t++) ts.emplace_back(work);
        work();
        for (auto &t : ts) t.join();
    }
    if ((rc = ctx->enc_memb.ensure(mbytes)))
        return rc;
    HIP_TRY(hipMemcpyAsync(ctx->enc_memb.p, memb, mbytes, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = ctx->enc_keys.put(ek, ctx->stream)) ||
        (rc = ctx->enc_hdr.ensure(std::max<size_t>(nk, 1))) ||
        (rc = ctx->enc_vals.ensure(std::max<size_t>(nk, 1) * (kEncMaxVals + 1))) ||
        (rc = ctx->enc_hist.ensure(std::max<size_t>(nk, 1) * (kEncMaxVals + 1))) ||
        (rc = ctx->enc_codes.ensure(std::max<size_t>(nk, 1) * N)))
        return rc;
    if ((rc = launch_key_encode(ctx->haps.p, ctx->regions.p, ctx->counts.p, B.n_slots, ctx->enc_keys.p, (uint32_t)nk,
                                ctx->enc_memb.p, (uint32_t)r0, N, ctx->enc_hdr.p, ctx->enc_vals.p, ctx->enc_hist.p,
                                ctx->enc_codes.p, ctx->stream)))
        return rc;
    B.enc_hdr.resize(nk);
    B.enc_vals.resize(nk * (kEncMaxVals + 1));
    B.enc_hist.resize(nk * (kEncMaxVals + 1));
    if (nk) {
        HIP_TRY(hipMemcpyAsync(B.enc_hdr.data(), ctx->enc_hdr.p, nk * sizeof(EncHdr), hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipMemcpyAsync(B.enc_vals.data(), ctx->enc_vals.p, B.enc_vals.size() * 4, hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipMemcpyAsync(B.enc_hist.data(), ctx->enc_hist.p, B.enc_hist.size() * 4, hipMemcpyDeviceToHost,
                               ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        // the packed codes back to back (a key's width is known only now), one download
        B.enc_code_off.resize(nk + 1);
        for (size_t k = 0; k < nk; k++) {
            const EncHdr &h = B.enc_hdr[k];
            const uint64_t bytes = h.status ? 0 : ((uint64_t)N * h.width + 7) / 8;
            B.enc_code_off[k + 1] = B.enc_code_off[k] + bytes;
        }
        const uint64_t total = B.enc_code_off[nk];
        if ((rc = ctx->enc_off.put(B.enc_code_off, ctx->stream)) ||
            (rc = ctx->enc_packed.ensure(std::max<uint64_t>(total, 1))) || (rc = B.enc_codes.reserve(total)))
            return rc;
        if ((rc = launch_code_compact(ctx->enc_codes.p, (uint32_t)nk, N, ctx->enc_off.p, ctx->enc_packed.p,
                                      ctx->stream)))
            return rc;
        if (total)
            HIP_TRY(hipMemcpyAsync(B.enc_codes.p, ctx->enc_packed.p, total, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    B.enc_r0 = (uint32_t)r0;
    B.enc_r1 = (uint32_t)r1;
    return TFBS_OK;
}

int tfbs_matches(tfbs_ctx *ctx, const uint8_t *nucs, const uint64_t *pos, size_t n, uint32_t *counts,
                 uint64_t *out_start, uint64_t *out_end, size_t cap, size_t *n_total) {
    if (!ctx || !n_total || !counts || (n && (!nucs || !pos))) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (n >= kMaxHapLen) return tfbs::fail(TFBS_E_ARG, "haplotype longer than 2^29 - 1 bases");
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
    std::vector<DevRegion> regions{DevRegion{0, 0, 0, 1, UINT32_MAX, 1, {0, 0}}};
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
    ctx->mfma_group_words = mfma_group_words(haps.data(), 1, ctx->mfma_hpb);
    ctx->n_regions = 1;
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
