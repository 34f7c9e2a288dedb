// The find-tfbs command flow (main.rs:234-393) on top of the batch + GPU scan:
// PWM load, BED load/merge, BCF + FASTA reads, distinct haplotypes per merged
// region, the scan, count aggregation and the pseudo-VCF rows through a BGZF
// writer, renamed from <out>.part at the end (or bgzip + tabix'ed).
//
// Differences from the reference that are choices, not gaps:
// regions are processed in merged-peak order in batches of `regions_per_batch`
// (the reference spreads 50-peak chunks over threads and emits rows in thread
// interleaving / HashMap order); rows within a region are sorted (D2); the
// POS counter is therefore deterministic.
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <condition_variable>
#include <mutex>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "batch.hpp"
#include "io.hpp"
#include "patterns.hpp"
#include "rows.hpp"

namespace tfbs {
int batch_row_bodies(const Batch &B, uint32_t min_maf, std::string &out, uint32_t threads);
std::string strip_chr(const std::string &c);
}

namespace {

std::vector<std::string> split(const std::string &s, char sep) {
    std::vector<std::string> out;
    size_t a = 0;
    for (;;) {
        size_t c = s.find(sep, a);
        out.push_back(s.substr(a, c == std::string::npos ? std::string::npos : c - a));
        if (c == std::string::npos) break;
        a = c + 1;
    }
    return out;
}

std::string basename_of(const std::string &p) {
    size_t k = p.find_last_of('/');
    return k == std::string::npos ? p : p.substr(k + 1);
}

bool in_path(const char *prog) {
    const char *path = getenv("PATH");
    if (!path) return false;
    for (auto &d : split(path, ':')) {
        std::string f = d + "/" + prog;
        if (access(f.c_str(), X_OK) == 0) return true;
    }
    return false;
}

// One device's share of the run: batches of merged regions (global batch g =
// regions [g per_batch, (g + 1) per_batch)), processed in a three-stage pipeline
// (one thread fetches batch g + 2's inputs -- FASTA windows, inner peaks, BCF
// records with their carriers (load_diffs) --, another builds batch g + 1's
// distinct haplotypes, grouped on the device where it can, while batch g is
// scanned, reduced and encoded on the device) with its own readers and ctx;
// out(g, ctx, batch) emits each batch's rows.
struct Shard {
    std::vector<size_t> batches;  // global batch indices, ascending
    int device = 0;
    uint32_t threads = 1;
    int rc = TFBS_OK;
    std::string err;
    size_t regions = 0;
    double t_prep = 0, t_wait = 0, t_gpu = 0, t_rows = 0;
    double t_bcf = 0, t_build = 0;  // of t_prep (fetch + build stages): BCF fetch + decode + record ids, add_regions
    double t_fasta = 0, t_ids = 0;   // of t_prep: FASTA + inner peaks; of t_bcf: make_record_ids
    // the BCF reader's own phases (of t_bcf): file reads, inflate + condense, record
    // boundary scan, record decode
    double b_read = 0, b_inflate = 0, b_scan = 0, b_wait = 0, b_decode = 0;
    double t_create = 0;                 // of t_prep: tfbs_batch_create
    double rows_plan = 0, rows_dev = 0;  // of t_rows: host row plans, device blocks + copy back + write
    double drain[3] = {0, 0, 0};         // of rows_dev: waits for the device's blocks, their copy back, the writes
    double t_setup = 0, t_boot = 0, t_end = 0;  // readers + ctx + grouper; the first batches' stages; flush + ctx release
};

struct RunSetup {
    const tfbs_run_args *a;
    std::string chrom;
    tfbs_patterns *pp;
    std::vector<std::pair<std::string, std::vector<std::pair<uint64_t, uint64_t>>>> beds;
    // per bed source: its peaks' indices by start, and the longest peak's span (the
    // inner peaks of a merged region by binary search, not a pass over every peak)
    std::vector<std::vector<uint32_t>> by_start;
    std::vector<uint64_t> max_span;
    std::vector<std::pair<uint64_t, uint64_t>> merged;
    std::vector<size_t> sel;
    size_t per_batch;
};

template <class Out>
int run_shard(const RunSetup &S, Shard &sh, Out &&out) {
    using namespace tfbs;
    const tfbs_run_args *a = S.a;
    if (sh.batches.empty()) return TFBS_OK;
    const double t_in = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    Bcf bcf;
    int rc = bcf.open(a->bcf, sh.threads);
    if (rc) return rc;
    if ((rc = bcf.select(S.sel))) return rc;  // GT decoded for these samples only
    if ((rc = bcf.set_carriers_mode(true))) return rc;  // load_diffs' carriers found while decoding
    const int rid = bcf.contig_index(S.chrom);
    Fasta fasta;
    if ((rc = fasta.open(a->reference))) return rc;
    // The device side -- the ctx (plan tables, streams) and the grouper that groups
    // SNV-only regions on this device (haplotype.rs:16-88 on the GPU; one for the
    // shard's batches, its membership rows recycled batch to batch; TFBS_RUN_BUILD_DEVICE=0:
    // every region on the host) -- is made on a helper thread while the first batch's
    // inputs are fetched.
    tfbs_ctx *ctx = nullptr;
    std::shared_ptr<DevGrouper> grouper;
    int dev_rc = TFBS_OK;
    std::string dev_err;
    std::thread dev_setup([&] {
        int r = tfbs_ctx_create(sh.device, S.pp, &ctx);
        if (!r) r = tfbs_ctx_set_host_threads(ctx, sh.threads);
        if (!r && !(getenv("TFBS_RUN_BUILD_DEVICE") && atoi(getenv("TFBS_RUN_BUILD_DEVICE")) == 0)) {
            grouper.reset(make_gpu_grouper(sh.device));
            if (!grouper) r = fail(TFBS_E_NODEVICE, "no device for the grouper");
        }
        if (r) dev_err = tfbs_last_error();
        dev_rc = r;
    });
    struct DevGuard {  // every exit: the helper joined, a ctx not handed to cguard released
        std::thread &t;
        tfbs_ctx *&c;
        bool owned = false;
        ~DevGuard() {
            if (t.joinable()) t.join();
            if (!owned && c) tfbs_ctx_destroy(c);
        }
    } dev_guard{dev_setup, ctx};
    std::unique_ptr<tfbs_ctx, void (*)(tfbs_ctx *)> cguard(nullptr, tfbs_ctx_destroy);
    auto dev_ready = [&]() -> int {
        dev_setup.join();
        if (dev_rc) return fail(dev_rc, dev_err);
        cguard.reset(ctx);
        dev_guard.owned = true;
        // one device writing straight to the output: its rows' writes go out on the ctx's
        // writer thread while the next batch runs (flushed below, joined by the ctx's destroy)
        if (out.device_rows && out.async_rows) rows_set_async(ctx, true);
        return TFBS_OK;
    };
    using BatchPtr = std::unique_ptr<tfbs_batch, void (*)(tfbs_batch *)>;
    std::vector<const BcfRecord *> recs;
    auto clock = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    struct BcfPhases {
        Bcf &b;
        Shard &sh;
        ~BcfPhases() { b.phase_seconds(sh.b_read, sh.b_inflate, sh.b_scan, sh.b_wait, sh.b_decode); }
    } bcf_phases{bcf, sh};
    // The shard's batches go through three stages at once: batch g + 2's inputs are
    // fetched (FASTA, inner peaks, the BCF's records with their carriers -- the reader
    // inflating ahead on its own thread) while batch g + 1 is built (add_regions:
    // distinct haplotypes, grouped on the device where it can) and batch g is
    // scanned, reduced and encoded on the device and its rows written here.
    struct Pending {
        BatchPtr bp{nullptr, tfbs_batch_destroy};
        std::vector<RegionInput> ins;
    };
    struct Times {
        double fetch = 0, build = 0, bcf = 0, ids = 0, fasta = 0, create = 0;
    };
    auto fetch = [&](size_t g, Pending &p, std::string &err, Times &t) -> int {
        const double t_in = clock();
        struct Done {
            double &acc, t0;
            ~Done() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() - t0; }
        } done{t.fetch, t_in};
        const size_t b0 = g * S.per_batch, b1 = std::min(S.merged.size(), b0 + S.per_batch);
        tfbs_batch *bb = nullptr;
        int rc = tfbs_batch_create(S.pp, (uint32_t)S.sel.size(), 1, &bb);
        t.create += clock() - t_in;
        if (rc) return err = tfbs_last_error(), rc;
        p.bp = BatchPtr(bb, tfbs_batch_destroy);
        Batch &B = bb->b;
        for (auto &b : S.beds) B.beds.push_back(b.first);
        p.ins.clear();
        p.ins.reserve(b1 - b0);
        for (size_t r = b0; r < b1; r++) {
            const double tf = clock();
            const auto &m = S.merged[r];
            RegionInput in;
            in.R.ms = m.first;
            in.R.me = m.second;
            rc = tfbs_batch_region_ext(bb, m.first, m.second, &in.R.es, &in.R.ee);
            if (rc) return err = tfbs_last_error(), rc;
            std::string ref;
            rc = fasta.fetch(S.chrom, in.R.es, in.R.ee + 1, ref);  // main.rs:156-161
            if (rc) return err = tfbs_last_error(), rc;
            in.ref.resize(ref.size());
            for (size_t i = 0; i < ref.size(); i++) {
                const int c = to_nuc((uint8_t)ref[i]);
                if (c < 0) {
                    err = "Unknown nucleotide " + std::to_string((int)(uint8_t)ref[i]);
                    return TFBS_E_BADBASE;
                }
                in.ref[i] = (uint8_t)c;
            }
            // select_inner_peaks (main.rs:62-72): p.overlaps(merged), in file order; only
            // peaks starting in [m.first - the longest span, m.second] can overlap
            for (size_t bi = 0; bi < S.beds.size(); bi++) {
                const auto &pk = S.beds[bi].second;
                const auto &ord = S.by_start[bi];
                const uint64_t lo = m.first >= S.max_span[bi] ? m.first - S.max_span[bi] : 0;
                auto it = std::lower_bound(ord.begin(), ord.end(), lo,
                                           [&](uint32_t i, uint64_t v) { return pk[i].first < v; });
                std::vector<uint32_t> hit;
                for (; it != ord.end() && pk[*it].first <= m.second; ++it) {
                    const auto &q = pk[*it];
                    const bool ov = (m.first >= q.first && m.first <= q.second) ||
                                    (m.second >= q.first && m.second <= q.second);
                    if (ov) hit.push_back(*it);
                }
                std::sort(hit.begin(), hit.end());
                for (uint32_t i : hit) in.inner.push_back({(uint32_t)bi, {pk[i].first, pk[i].second}});
            }
            // load_diffs (haplotype.rs:78-80): name2rid(chrom).unwrap() panics on an unknown contig
            if (rid < 0) {
                err = "chromosome " + S.chrom + " not in the BCF header";
                return TFBS_E_ARG;
            }
            const double tb = clock();
            t.fasta += tb - tf;
            if ((rc = bcf.fetch(rid, in.R.es, in.R.ee + 1, recs))) return err = tfbs_last_error(), rc;
            const double ti = clock();
            // the next region of the batch starts at beg_next: a record it cannot return
            // gives its carriers away instead of a copy
            uint64_t beg_next = 0, ee_next = 0;
            const bool has_next =
                r + 1 < b1 && tfbs_batch_region_ext(bb, S.merged[r + 1].first, S.merged[r + 1].second, &beg_next,
                                                    &ee_next) == TFBS_OK;
            for (const BcfRecord *br : recs) {
                Record rec;
                const char *alt = br->n_alleles >= 2 ? br->alt.c_str() : nullptr;
                rc = has_next && bcf.dropped_before(br, beg_next)
                         ? make_record_ids(br->pos, br->n_alleles, br->ref.c_str(), alt, bcf.take_carriers(br),
                                           br->gt_status, rec)
                         : make_record_ids(br->pos, br->n_alleles, br->ref.c_str(), alt, br->carriers, br->gt_status,
                                           rec);
                if (rc) return err = tfbs_last_error(), rc;
                in.recs.push_back(std::move(rec));
            }
            const double te = clock();
            t.ids += te - ti;
            t.bcf += te - tb;
            p.ins.push_back(std::move(in));
        }
        return TFBS_OK;
    };
    auto build = [&](Pending &p, std::string &err, Times &t) -> int {
        const double tb = clock();
        p.bp->b.grouper = grouper;
        const int rc = add_regions(p.bp->b, p.ins, sh.threads);
        std::vector<RegionInput>().swap(p.ins);
        t.build += clock() - tb;
        return rc ? (err = tfbs_last_error(), rc) : TFBS_OK;
    };
    auto account = [&](const Times &t) {
        sh.t_prep += t.fetch + t.build;
        sh.t_bcf += t.bcf;
        sh.t_build += t.build;
        sh.t_fasta += t.fasta;
        sh.t_ids += t.ids;
        sh.t_create += t.create;
    };
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const size_t nb = sh.batches.size();
    Pending cur, nxt, nxt2;
    std::string err;
    {
        Times t;
        if ((rc = fetch(sh.batches[0], cur, err, t))) return fail(rc, err);
        if ((rc = dev_ready())) return rc;
        sh.t_setup = now() - t_in;  // (readers, the first fetch, the device side: the longer)
        const double tb0 = now();
        struct Boot {
            double &acc, t0;
            ~Boot() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() - t0; }
        } boot{sh.t_boot, tb0};
        if ((rc = build(cur, err, t)) || (nb > 1 && (rc = fetch(sh.batches[1], nxt, err, t)))) return fail(rc, err);
        account(t);
    }
    for (size_t bi = 0; bi < nb; bi++) {
        const size_t g = sh.batches[bi];
        Times ta, tb;
        std::string ea, eb;
        int ra = TFBS_OK, rb = TFBS_OK;
        std::thread th_fetch, th_build;
        if (bi + 2 < nb) th_fetch = std::thread([&, bi] { ra = fetch(sh.batches[bi + 2], nxt2, ea, ta); });
        if (bi + 1 < nb) th_build = std::thread([&] { rb = build(nxt, eb, tb); });
        // join the helpers on every exit path
        struct Joiner {
            std::thread &a, &b;
            ~Joiner() {
                if (a.joinable()) a.join();
                if (b.joinable()) b.join();
            }
        } joiner{th_fetch, th_build};
        tfbs_batch *bb = cur.bp.get();
        Batch &B = bb->b;
        double t0 = now();
        if ((rc = tfbs_batch_upload(ctx, bb)) || (rc = tfbs_scan(ctx, bb)) || (rc = tfbs_batch_assemble(ctx, bb)) ||
            (rc = tfbs_batch_reduce(ctx, bb)) ||
            (rc = tfbs_batch_encode_flags(ctx, bb, 0, B.rh.size(), out.device_rows ? TFBS_ENC_DEVICE_CODES : 0)))
            return rc;
        double t1 = now();
        sh.t_gpu += t1 - t0;
        sh.regions += B.rh.size();
        if ((rc = out(g, ctx, bb))) return rc;
        sh.t_rows += now() - t1;
        if (a->verbose) {
            for (size_t r = 0; r < B.rh.size(); r++)
                fprintf(stdout, "Peak %zu/%zu\t%llu\t%llu\t%u haplotypes\t%u variants\n", g * S.per_batch + r + 1,
                        S.merged.size(), (unsigned long long)B.rh[r].ms, (unsigned long long)B.rh[r].me,
                        B.rh[r].hap_count, B.rh[r].n_variants);
        }
        t0 = now();
        if (th_fetch.joinable()) th_fetch.join();
        if (th_build.joinable()) th_build.join();
        sh.t_wait += now() - t0;
        account(ta);
        account(tb);
        if (rb) return fail(rb, eb);
        if (ra) return fail(ra, ea);
        cur = std::move(nxt);
        nxt = std::move(nxt2);
        nxt2 = Pending();
    }
    const double te = now();
    struct End {  // the flush and the ctx's release (cguard, after this)
        double &acc, t0;
        ~End() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() - t0; }
    } end_t{sh.t_end, te};
    if ((rc = rows_flush(ctx))) return rc;
    double rs[2];
    if (tfbs_ctx_rows_bgzf_seconds(ctx, rs) == TFBS_OK) sh.rows_plan = rs[0], sh.rows_dev = rs[1];
    rows_bgzf_drain_seconds(ctx, sh.drain);
    return TFBS_OK;
}

// The batches' output in batch order across the devices' threads: the POS chain
// (batch g's first POS = batch g - 1's + its rows, published as soon as g - 1 has
// counted them, before it deflates) and the ordered writer (each batch's BGZF
// blocks -- in a memory file -- or row bodies, written out in order).
struct Ordered {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int64_t> base;  // POS of batch g's first row, -1 unknown
    struct Item {
        bool ready = false;
        int fd = -1;           // BGZF blocks (memory file), or
        std::string bodies;    // row bodies (host rows)
    };
    std::vector<Item> items;
    size_t written = 0;  // batches [0, written) are written out
    // at most kAhead batches past the first unwritten one hold their blocks (memory
    // files of hundreds of MB at 50 000 samples): a shard waits before making more
    static constexpr size_t kAhead = 6;
    // device rows: batch g's blocks go to [off[g], off[g] + size[g]) of the output, known
    // once every batch before it is submitted, so the writer threads copy several
    // batches at once (positioned writes); done[g]: batch g is in the output
    std::vector<uint64_t> size;
    std::vector<int64_t> off;
    std::vector<uint8_t> done_;
    size_t sized = 0;  // off[0 .. sized] known
    bool failed = false;
    int first_rc = TFBS_OK;  // the failure that stopped the others
    std::string first_err;
    explicit Ordered(size_t n) : base(n + 1, -1), items(n), size(n, 0), off(n + 1, -1), done_(n, 0) { base[0] = 1; }
    int chain(size_t g, uint64_t n_rows, uint32_t *fake) {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return failed || base[g] >= 0; });
        if (failed) return tfbs::fail(TFBS_E_STATE, "another device's shard failed");
        *fake = (uint32_t)base[g];
        base[g + 1] = base[g] + (int64_t)n_rows;
        cv.notify_all();
        return TFBS_OK;
    }
    void submit(size_t g, Item &&it, uint64_t bytes = 0) {
        std::lock_guard<std::mutex> l(mu);
        items[g] = std::move(it);
        items[g].ready = true;
        size[g] = bytes;
        while (off[sized] >= 0 && sized < items.size() && items[sized].ready) {
            off[sized + 1] = off[sized] + (int64_t)size[sized];
            sized++;
        }
        cv.notify_all();
    }
    // the output offset of batch 0 (after the header); then offsets follow the sizes
    void start(int64_t at) {
        std::lock_guard<std::mutex> l(mu);
        off[0] = at;
        while (sized < items.size() && items[sized].ready) {
            off[sized + 1] = off[sized] + (int64_t)size[sized];
            sized++;
        }
        cv.notify_all();
    }
    // waits until batch g is submitted and placed; false if a shard failed
    bool placed(size_t g, Item &it, int64_t &at) {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return failed || (items[g].ready && off[g] >= 0); });
        if (failed) return false;
        it = std::move(items[g]);
        items[g].fd = -1;  // the writer owns (and closes) the memory file now
        at = off[g];
        return true;
    }
    void finished(size_t g) {  // batch g is in the output
        std::lock_guard<std::mutex> l(mu);
        done_[g] = 1;
        while (written < done_.size() && done_[written]) written++;
        cv.notify_all();
    }
    void abort(int rc, const std::string &err) {
        std::lock_guard<std::mutex> l(mu);
        if (!failed) {
            first_rc = rc;
            first_err = err;
        }
        failed = true;
        cv.notify_all();
    }
    bool room(size_t g) {  // waits until batch g may hold its blocks; false if a shard failed
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return failed || g < written + kAhead; });
        return !failed;
    }
    bool take(size_t g, Item &it) {  // waits for batch g; false if a shard failed
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return failed || items[g].ready; });
        if (failed) return false;
        it = std::move(items[g]);
        items[g].fd = -1;  // the writer owns (and closes) the memory file now
        return true;
    }
};

// A memory file's n bytes to dst at offset at, through the thread's 8 MiB buffer
// (a mapping's page faults made it ~0.7 GB/s per thread).
int copy_fd_at(int src, uint64_t n, int dst, uint64_t at) {
    thread_local std::vector<char> buf;
    if (buf.empty()) buf.resize(8u << 20);
    for (uint64_t k = 0; k < n;) {
        const ssize_t r = pread(src, buf.data(), (size_t)std::min<uint64_t>(n - k, buf.size()), (off_t)k);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return tfbs::fail(TFBS_E_IO, std::string("read: ") + (r < 0 ? strerror(errno) : "short read"));
        for (ssize_t q = 0; q < r;) {
            const ssize_t w = pwrite(dst, buf.data() + q, (size_t)(r - q), (off_t)(at + k + (uint64_t)q));
            if (w < 0 && errno == EINTR) continue;
            if (w <= 0) return tfbs::fail(TFBS_E_IO, std::string("write: ") + (w < 0 ? strerror(errno) : "short write"));
            q += w;
        }
        k += (uint64_t)r;
    }
    return TFBS_OK;
}

// "<chr>\t<POS>\t" before every row body, POS counted by *fake (main.rs:415-429)
int write_prefixed(tfbs::BgzfWriter &w, const std::string &chr, const char *p, size_t n, uint32_t *fake) {
    std::string out;
    out.reserve(n + 64);
    char head[32];
    for (size_t i = 0; i < n;) {
        const char *nl = (const char *)memchr(p + i, '\n', n - i);
        const size_t e = nl ? (size_t)(nl - p) + 1 : n;
        const int m = snprintf(head, sizeof head, "\t%u\t", *fake);
        out += chr;
        out.append(head, (size_t)m);
        out.append(p + i, e - i);
        (*fake)++;
        i = e;
        if (out.size() >= (8u << 20)) {
            if (int rc = w.write(out.data(), out.size())) return rc;
            out.clear();
        }
    }
    return w.write(out.data(), out.size());
}

std::vector<int> parse_devices(const tfbs_run_args *a) {
    std::vector<int> d;
    if (a->devices && *a->devices)
        for (auto &x : split(a->devices, ','))
            if (!x.empty()) d.push_back(atoi(x.c_str()));
    if (d.empty()) d.push_back(a->device);
    return d;
}

}  // namespace

extern "C" {

int tfbs_run(const tfbs_run_args *a) {
    using namespace tfbs;
    if (!a || !a->chromosome || !a->bcf || !a->bed_files || !a->reference || !a->pwm_file || !a->pwm_threshold_dir ||
        !a->pwm_names || !a->output)
        return fail(TFBS_E_ARG, "missing required argument");
    RunSetup S;
    S.a = a;
    S.chrom = a->chromosome;
    if (a->tabix && (!in_path("bgzip") || !in_path("tabix")))
        return fail(TFBS_E_IO, "bgzip/tabix cannot be found in PATH");  // main.rs:220-223
    // the HIP runtime's start-up overlaps the PWM / BED / BCF-header parsing below
    std::thread warm([a] { warm_devices(parse_devices(a)); });
    struct Joined {
        std::thread &t;
        ~Joined() {
            if (t.joinable()) t.join();
        }
    } warm_join{warm};

    // patterns (main.rs:237-250)
    int rc = tfbs_patterns_from_files(a->pwm_file, a->pwm_threshold_dir, a->pwm_threshold, a->pwm_names,
                                      a->forward_only ? 0 : 1, &S.pp);
    if (rc) return rc;
    std::unique_ptr<tfbs_patterns, void (*)(tfbs_patterns *)> pguard(S.pp, tfbs_patterns_destroy);

    // BED sources (bed.rs:25-47): keyed by path (a repeated path counts once), merged
    // over all of them, inner peaks keyed by basename (a later file with the same
    // basename replaces an earlier one).
    std::vector<std::string> paths;
    for (auto &b : split(a->bed_files, ','))
        if (std::find(paths.begin(), paths.end(), b) == paths.end()) paths.push_back(b);
    std::vector<std::pair<uint64_t, uint64_t>> all;
    for (auto &path : paths) {
        struct stat st;
        if (stat(path.c_str(), &st) != 0) return fail(TFBS_E_IO, "Bed file " + path + " does not exist");
        std::vector<std::pair<uint64_t, uint64_t>> peaks, kept;
        rc = load_bed(path, S.chrom, peaks);
        if (rc) return rc;
        for (auto &p : peaks)
            if (p.first >= a->after_position) kept.push_back(p);
        all.insert(all.end(), kept.begin(), kept.end());
        const std::string bn = basename_of(path);
        bool replaced = false;
        for (auto &b : S.beds)
            if (b.first == bn) { b.second = kept; replaced = true; }
        if (!replaced) S.beds.push_back({bn, kept});
    }
    S.merged = merge_ranges(all);
    for (auto &b : S.beds) {
        std::vector<uint32_t> ord(b.second.size());
        uint64_t span = 0;
        for (uint32_t i = 0; i < ord.size(); i++) {
            ord[i] = i;
            if (b.second[i].second >= b.second[i].first) span = std::max(span, b.second[i].second - b.second[i].first);
        }
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return b.second[x].first < b.second[y].first; });
        S.by_start.push_back(std::move(ord));
        S.max_span.push_back(span);
    }

    // BCF header + samples (main.rs:255, 293-314)
    std::vector<std::string> sample_names;
    {
        Bcf hdr;
        if ((rc = hdr.open(a->bcf, 1))) return rc;
        sample_names = hdr.samples;
    }
    if (a->samples_file && *a->samples_file) {
        std::ifstream sf(a->samples_file);
        if (!sf) return fail(TFBS_E_IO, std::string("Could not open sample file ") + a->samples_file);
        std::set<std::string> want;
        std::string l;
        while (std::getline(sf, l))
            if (l.size() > 1) want.insert(l);
        for (size_t i = 0; i < sample_names.size(); i++)
            if (want.count(sample_names[i])) S.sel.push_back(i);
    } else {
        for (size_t i = 0; i < sample_names.size(); i++) S.sel.push_back(i);
    }
    {
        Fasta fasta;  // main.rs:259: the reference opens it before any region
        if ((rc = fasta.open(a->reference))) return rc;
    }

    // output (main.rs:264-290, 320-324)
    const std::string out = a->output, part = out + ".part";
    BgzfWriter w;
    const uint32_t threads = std::max(1u, a->threads);
    rc = w.open(part, threads);
    if (rc) return rc;
    std::string header = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT";
    for (size_t i : S.sel) header += "\t" + sample_names[i];
    header += "\n";
    rc = w.write(header.data(), header.size());
    if (rc) return rc;

    // shards: batch g of merged regions on device g % n (one device:
    // every batch); rows in merged-peak order, POS counted across the devices
    S.per_batch = a->regions_per_batch ? a->regions_per_batch : 512;
    const std::vector<int> devs = parse_devices(a);
    const size_t n_batches = (S.merged.size() + S.per_batch - 1) / S.per_batch;
    const size_t n_sh = std::max<size_t>(1, std::min(devs.size(), n_batches));
    std::vector<Shard> shards(n_sh);
    for (size_t k = 0; k < n_sh; k++) {
        shards[k].device = devs[k];
        shards[k].threads = std::max<uint32_t>(1, threads / (uint32_t)n_sh);
    }
    for (size_t g = 0; g < n_batches; g++) shards[g % n_sh].batches.push_back(g);
    const std::string chr = strip_chr(S.chrom);
    uint32_t fake = 1;
    const bool timing = getenv("TFBS_RUN_TIMING") && atoi(getenv("TFBS_RUN_TIMING"));
    // TFBS_GPU_BGZF=0: rows formatted on the host and deflated by the writer's host
    // threads (zlib); default: BGZF blocks made on each device (bgzf_gpu.hip)
    const bool gpu_bgzf = !(getenv("TFBS_GPU_BGZF") && atoi(getenv("TFBS_GPU_BGZF")) == 0);
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = now();
    double t_write = 0;
    if (n_sh == 1) {  // one device: its batches in order, straight to the output
        struct One {
            bool device_rows;
            bool async_rows;  // (straight to the output file: writes may trail the call)
            const RunSetup &S;
            tfbs::BgzfWriter &w;
            const std::string &chr;
            uint32_t &fake;
            double &t_write;
            int operator()(size_t, tfbs_ctx *ctx, tfbs_batch *bb) {
                const size_t n = bb->b.rh.size();
                if (device_rows) {
                    const int fd = w.raw_fd();
                    if (fd < 0) return fd;
                    return tfbs_batch_rows_bgzf(ctx, bb, 0, n, S.chrom.c_str(), S.a->min_maf, &fake, fd, nullptr,
                                                nullptr, nullptr);
                }
                std::string bodies;
                if (int rc = tfbs::batch_row_bodies(bb->b, S.a->min_maf, bodies, std::max(1u, S.a->threads))) return rc;
                return write_prefixed(w, chr, bodies.data(), bodies.size(), &fake);
            }
        } one{gpu_bgzf, !(getenv("TFBS_RUN_ASYNC_WRITE") && atoi(getenv("TFBS_RUN_ASYNC_WRITE")) == 0), S, w, chr, fake,
              t_write};
        shards[0].rc = run_shard(S, shards[0], one);
        if (shards[0].rc) shards[0].err = tfbs_last_error();
    } else {  // several: each batch's output to the ordered writer
        Ordered ord(n_batches);
        struct Many {
            bool device_rows;
            bool async_rows;  // false: each batch's memory file is complete when submitted
            const RunSetup &S;
            Ordered &ord;
            uint32_t threads;
            int operator()(size_t g, tfbs_ctx *ctx, tfbs_batch *bb) {
                const size_t n = bb->b.rh.size();
                Ordered::Item it;
                if (device_rows) {  // BGZF blocks into a memory file; the POS base from the chain
                    if (!ord.room(g)) return tfbs::fail(TFBS_E_STATE, "another device's shard failed");
                    it.fd = memfd_create("tfbs_rows", MFD_CLOEXEC);
                    if (it.fd < 0) return tfbs::fail(TFBS_E_IO, std::string("memfd_create: ") + strerror(errno));
                    uint32_t fk = 0;
                    const int rc = tfbs::rows_bgzf_chained(
                        ctx, bb, 0, n, S.chrom.c_str(), S.a->min_maf, &fk, it.fd, nullptr, nullptr,
                        [&](uint64_t rows, uint32_t *base) { return ord.chain(g, rows, base); });
                    if (rc) {
                        close(it.fd);
                        return rc;
                    }
                    const off_t end = lseek(it.fd, 0, SEEK_END);
                    if (end < 0) {
                        close(it.fd);
                        return tfbs::fail(TFBS_E_IO, std::string("lseek: ") + strerror(errno));
                    }
                    ord.submit(g, std::move(it), (uint64_t)end);
                    return TFBS_OK;
                } else if (int rc = tfbs::batch_row_bodies(bb->b, S.a->min_maf, it.bodies, threads)) {
                    return rc;
                }
                ord.submit(g, std::move(it));
                return TFBS_OK;
            }
        };
        // device rows: kWriters threads copy the batches' memory files to their places in
        // the output (positioned writes: several batches at once); host rows: one thread
        // prefixes the bodies with POS and deflates them in batch order
        constexpr int kWriters = 4;
        int out_fd = -1;
        int64_t out_at = 0;
        if (gpu_bgzf) {
            out_fd = w.raw_fd();
            if (out_fd < 0) return out_fd;
            out_at = (int64_t)lseek(out_fd, 0, SEEK_END);
            if (out_at < 0) return fail(TFBS_E_IO, std::string("lseek: ") + strerror(errno));
            ord.start(out_at);
        }
        std::atomic<size_t> next_w(0);
        std::mutex tw_mu;
        auto writer_fn = [&] {
            for (;;) {
                const size_t g = gpu_bgzf ? next_w.fetch_add(1) : next_w.load();
                if (g >= n_batches) return;
                Ordered::Item it;
                int64_t at = 0;
                if (gpu_bgzf ? !ord.placed(g, it, at) : !ord.take(g, it)) return;
                const double t0 = now();
                int rc;
                if (it.fd >= 0) {
                    rc = copy_fd_at(it.fd, ord.size[g], out_fd, (uint64_t)at);
                    close(it.fd);
                } else {
                    rc = write_prefixed(w, chr, it.bodies.data(), it.bodies.size(), &fake);
                    next_w.store(g + 1);
                }
                {
                    std::lock_guard<std::mutex> l(tw_mu);
                    t_write += now() - t0;
                }
                if (rc) {
                    ord.abort(rc, tfbs_last_error());
                    return;
                }
                ord.finished(g);
            }
        };
        std::vector<std::thread> writers;
        for (int k = 0; k < (gpu_bgzf ? kWriters : 1); k++) writers.emplace_back(writer_fn);
        auto run_one = [&](size_t k) {
            Many m{gpu_bgzf, false, S, ord, shards[k].threads};
            shards[k].rc = run_shard(S, shards[k], m);
            if (shards[k].rc) {
                shards[k].err = tfbs_last_error();
                ord.abort(shards[k].rc, shards[k].err);
            }
        };
        std::vector<std::thread> ts;
        for (size_t k = 1; k < n_sh; k++) ts.emplace_back(run_one, k);
        run_one(0);
        for (auto &t : ts) t.join();
        for (auto &t : writers) t.join();
        if (gpu_bgzf && !ord.failed) {  // the stream continues after the last batch's blocks
            if (int rc2 = w.seek_to((uint64_t)ord.off[n_batches])) return rc2;
        }
        {  // memory files no writer took (a failed run); taken ones were handed over (fd -1 here)
            std::lock_guard<std::mutex> l(ord.mu);
            for (auto &it : ord.items)
                if (it.fd >= 0) close(it.fd);
        }
        if (ord.failed) return fail(ord.first_rc, ord.first_err);
    }
    for (auto &sh : shards)
        if (sh.rc) return fail(sh.rc, sh.err);
    // the reference flushes twice before drop (main.rs:271, 275): two empty blocks
    double t0 = now();
    if ((rc = w.flush()) || (rc = w.flush()) || (rc = w.close())) return rc;
    const double t_close = now() - t0;
    if (timing)
        for (size_t k = 0; k < n_sh; k++)
            fprintf(stderr,
                    "tfbs_run_timing {\"shard\": %zu, \"device\": %d, \"regions\": %zu, \"batches\": %zu, "
                    "\"prep_s\": %.4f, \"prep_bcf_s\": %.4f, \"prep_build_s\": %.4f, \"prep_fasta_s\": %.4f, "
                    "\"prep_ids_s\": %.4f, \"bcf_read_s\": %.4f, \"bcf_inflate_s\": %.4f, \"bcf_scan_s\": %.4f, "
                    "\"bcf_ahead_wait_s\": %.4f, \"bcf_decode_s\": %.4f, \"prep_create_s\": %.4f, \"rows_plan_s\": %.4f, \"rows_dev_s\": %.4f, "
                    "\"drain_gpu_s\": %.4f, \"drain_copy_s\": %.4f, \"drain_write_s\": %.4f, \"setup_s\": %.4f, \"boot_s\": %.4f, "
                    "\"end_s\": %.4f, \"prep_wait_s\": %.4f, "
                    "\"gpu_s\": %.4f, \"rows_s\": %.4f, \"ordered_write_s\": %.4f, \"close_s\": %.4f, \"loop_s\": %.4f}\n",
                    k, shards[k].device, shards[k].regions, shards[k].batches.size(), shards[k].t_prep,
                    shards[k].t_bcf, shards[k].t_build, shards[k].t_fasta, shards[k].t_ids, shards[k].b_read,
                    shards[k].b_inflate, shards[k].b_scan, shards[k].b_wait, shards[k].b_decode, shards[k].t_create, shards[k].rows_plan,
                    shards[k].rows_dev, shards[k].drain[0], shards[k].drain[1], shards[k].drain[2],
                    shards[k].t_setup, shards[k].t_boot, shards[k].t_end,
                    shards[k].t_wait, shards[k].t_gpu, shards[k].t_rows, t_write, t_close, now() - t_start);
    if (a->tabix) {
        const std::string cmd = "zcat '" + part + "' | bgzip > '" + out + "'; tabix -f -p vcf '" + out + "'; rm '" +
                                part + "'";
        if (system(cmd.c_str()) != 0) fprintf(stdout, "Failed to tabix file %s\n", out.c_str());
    } else if (rename(part.c_str(), out.c_str()) != 0) {
        return fail(TFBS_E_IO, "Could not rename " + part + " into " + out);
    }
    return TFBS_OK;
}

// ----------------------------------------------------------------------------
// File-format entry points (f2-f4), for tests and embedding.
// ----------------------------------------------------------------------------
struct tfbs_bcf {
    tfbs::Bcf b;
    std::vector<const tfbs::BcfRecord *> cur;
};

int tfbs_bcf_open(const char *path, tfbs_bcf **out) {
    if (!path || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    auto *b = new tfbs_bcf();
    int rc = b->b.open(path);
    if (rc) {
        delete b;
        return rc;
    }
    *out = b;
    return TFBS_OK;
}
void tfbs_bcf_close(tfbs_bcf *b) { delete b; }
int tfbs_bcf_select(tfbs_bcf *b, const size_t *idx, size_t n) {
    if (!b || (n && !idx)) return tfbs::fail(TFBS_E_ARG, "null argument");
    b->cur.clear();
    return b->b.select(std::vector<size_t>(idx, idx + n));
}
size_t tfbs_bcf_num_samples(const tfbs_bcf *b) { return b ? b->b.samples.size() : 0; }
int tfbs_bcf_indexed(const tfbs_bcf *b) { return b && b->b.indexed() ? 1 : 0; }
const char *tfbs_bcf_sample_name(const tfbs_bcf *b, size_t i) {
    return (b && i < b->b.samples.size()) ? b->b.samples[i].c_str() : nullptr;
}
int tfbs_bcf_fetch(tfbs_bcf *b, const char *chrom, uint64_t beg, uint64_t end, size_t *n) {
    if (!b || !chrom || !n) return tfbs::fail(TFBS_E_ARG, "null argument");
    const int rid = b->b.contig_index(chrom);
    if (rid < 0) return tfbs::fail(TFBS_E_ARG, std::string("unknown contig ") + chrom);
    const int rc = b->b.fetch(rid, beg, end, b->cur);
    if (rc) return rc;
    *n = b->cur.size();
    return TFBS_OK;
}
int tfbs_bcf_record(const tfbs_bcf *b, size_t i, uint64_t *pos, uint32_t *rlen, uint32_t *n_alleles, const char **ref,
                    const char **alt, const int32_t **gt) {
    if (!b || i >= b->cur.size()) return tfbs::fail(TFBS_E_ARG, "bad record index");
    const tfbs::BcfRecord *r = b->cur[i];
    if (pos) *pos = r->pos;
    if (rlen) *rlen = r->rlen;
    if (n_alleles) *n_alleles = r->n_alleles;
    if (ref) *ref = r->ref.c_str();
    if (alt) *alt = r->n_alleles >= 2 ? r->alt.c_str() : nullptr;
    if (gt) *gt = r->gt.empty() ? nullptr : r->gt.data();
    return TFBS_OK;
}

int tfbs_bcf_set_carriers_mode(tfbs_bcf *b, int on) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    b->cur.clear();
    return b->b.set_carriers_mode(on != 0);
}
int tfbs_bcf_record_carriers(const tfbs_bcf *b, size_t i, const uint32_t **ids, size_t *n, int *gt_status) {
    if (!b || i >= b->cur.size()) return tfbs::fail(TFBS_E_ARG, "bad record index");
    const tfbs::BcfRecord *r = b->cur[i];
    if (ids) *ids = r->carriers.data();
    if (n) *n = r->carriers.size();
    if (gt_status) *gt_status = r->gt_status;
    return TFBS_OK;
}

int tfbs_fasta_fetch(const char *path, const char *chrom, uint64_t start, uint64_t stop, char **out, size_t *n) {
    if (!path || !chrom || !out || !n) return tfbs::fail(TFBS_E_ARG, "null argument");
    tfbs::Fasta f;
    int rc = f.open(path);
    if (rc) return rc;
    std::string s;
    rc = f.fetch(chrom, start, stop, s);
    if (rc) return rc;
    char *p = (char *)malloc(s.size() + 1);
    memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    *out = p;
    *n = s.size();
    return TFBS_OK;
}

int tfbs_bgzf_write_file(const char *path, const char *text, size_t n, int flushes) {
    if (!path || (n && !text)) return tfbs::fail(TFBS_E_ARG, "null argument");
    tfbs::BgzfWriter w;
    int rc = w.open(path);
    if (!rc) rc = w.write(text, n);
    for (int i = 0; !rc && i < flushes; i++) rc = w.flush();
    if (!rc) rc = w.close();
    return rc;
}

int tfbs_bgzf_read_file(const char *path, char **out, size_t *n) {
    if (!path || !out || !n) return tfbs::fail(TFBS_E_ARG, "null argument");
    std::ifstream in(path, std::ios::binary);
    if (!in) return tfbs::fail(TFBS_E_IO, std::string("Could not open file ") + path);
    std::string raw((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>()), txt;
    int rc = tfbs::bgzf_inflate(raw, txt);
    if (rc) return rc;
    char *p = (char *)malloc(txt.size() + 1);
    memcpy(p, txt.data(), txt.size());
    p[txt.size()] = 0;
    *out = p;
    *n = txt.size();
    return TFBS_OK;
}

int tfbs_merge_ranges(const uint64_t *starts, const uint64_t *ends, size_t n, uint64_t *out_s, uint64_t *out_e,
                      size_t *n_out) {
    if (!n_out || (n && (!starts || !ends || !out_s || !out_e))) return tfbs::fail(TFBS_E_ARG, "null argument");
    std::vector<std::pair<uint64_t, uint64_t>> r(n);
    for (size_t i = 0; i < n; i++) r[i] = {starts[i], ends[i]};
    auto m = tfbs::merge_ranges(r);
    for (size_t i = 0; i < m.size(); i++) {
        out_s[i] = m[i].first;
        out_e[i] = m[i].second;
    }
    *n_out = m.size();
    return TFBS_OK;
}

}  // extern "C"
