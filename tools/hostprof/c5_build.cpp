// Host-side cost of the C5 region build (build_regions' device-grouped,
// host-patched path and commit_regions) without a GPU: the device grouper is
// replaced by a CPU stand-in (masks from the carrier lists, no membership rows),
// so mask_finish and the commit run exactly as in the product.  Profiling aid
// only (not built into the library): make -C tools/hostprof && ./c5_build [regions].
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>

#include "batch.hpp"
#include "tfbs_internal.hpp"
#include "tfbs_amd.h"

using namespace tfbs;

struct CpuGrouper : DevGrouper {
    std::vector<uint32_t> car;
    double secs = 0;  // in group()
    int device() const override { return 0; }
    uint32_t *carriers(size_t n) override {
        car.resize(n);
        return car.data();
    }
    int group(size_t, const std::vector<GrpRecord> &recs, const std::vector<GrpRegion> &regs, uint32_t H,
              GroupOut &out) override {
        const auto t0 = std::chrono::steady_clock::now();
        struct T {
            std::chrono::steady_clock::time_point t0;
            double &acc;
            ~T() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
        } timer{t0, secs};
        out = GroupOut();
        std::vector<uint64_t> m(H);
        for (const GrpRegion &g : regs) {
            std::fill(m.begin(), m.end(), 0);
            for (uint32_t k = 0; k < g.n_rec; k++) {
                const GrpRecord &r = recs[g.rec_off + k];
                for (uint32_t i = 0; i < r.n; i++) m[car[r.off + i]] |= 1ull << r.rank;
            }
            std::map<uint64_t, uint32_t> cnt;
            for (uint64_t x : m)
                if (x) cnt[x]++;
            out.first.push_back((uint32_t)out.masks.size());
            if (cnt.size() > kGrpMax) {
                out.n_groups.push_back(UINT32_MAX);
            } else {
                out.n_groups.push_back((uint32_t)cnt.size());
                for (auto &kv : cnt) {
                    out.masks.push_back(kv.first);
                    out.counts.push_back(kv.second);
                }
            }
            out.memb.push_back(0);
        }
        return 0;
    }
    int fetch(uint64_t, uint32_t H, uint16_t *o) override {
        for (uint32_t h = 0; h < H; h++) o[h] = 0;
        return 0;
    }
    void recycle(std::vector<void *> &) override {}
};

int main(int argc, char **argv) {
    const uint64_t regions = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2000;
    const uint32_t indel = argc > 2 ? (uint32_t)atoi(argv[2]) : 30;
    char *names = nullptr;
    system("mkdir -p /tmp/hostprof_pwms");
    if (tfbs_synth_write_pwms("/tmp/hostprof_pwms", 600, 5, 5, &names)) return 1;
    tfbs_patterns *p = nullptr;
    if (tfbs_patterns_from_files("/tmp/hostprof_pwms/pwms.txt", "/tmp/hostprof_pwms/thr", 1e-4f, names, 1, &p)) return 1;
    tfbs_batch *b = nullptr;
    if (tfbs_batch_create(p, 50000, 0, &b)) return 1;
    auto g = std::make_shared<CpuGrouper>();
    b->b.grouper = g;
    // the inputs as tfbs_synth_fill_batch makes them, then build_regions and
    // commit_regions timed apart (best of 3 fresh batches)
    const uint32_t lmax = b->b.lmax();
    std::vector<RegionInput> proto(regions);
    for (uint64_t j = 0; j < regions; j++) {
        tfbs_synth_region *R = nullptr;
        if (tfbs_synth_region_make(5, j, 50000, lmax, indel, &R)) return 1;
        uint64_t ms, me, es;
        const char *ra;
        size_t nref, nrec;
        tfbs_synth_region_info(R, &ms, &me, &es, &ra, &nref, &nrec);
        RegionInput &in = proto[j];
        in.R.ms = ms;
        in.R.me = me;
        in.R.es = es;
        in.R.ee = me + std::max<uint32_t>(lmax, 1) - 1;
        for (size_t i = 0; i < nref; i++) in.ref.push_back((uint8_t)to_nuc((uint8_t)ra[i]));
        for (size_t k = 0; k < nrec; k++) {
            uint64_t pos;
            const char *rf, *al;
            const uint32_t *car;
            size_t nc;
            tfbs_synth_region_record(R, k, &pos, &rf, &al, &car, &nc);
            Record r;
            r.pos = pos;
            for (const char *c = rf; *c; c++) r.ref.push_back((uint8_t)to_nuc((uint8_t)*c));
            for (const char *c = al; *c; c++) r.alt.push_back((uint8_t)to_nuc((uint8_t)*c));
            r.carriers.assign(car, car + nc);
            in.recs.push_back(std::move(r));
        }
        tfbs_synth_region_destroy(R);
        in.inner.push_back({0u, {ms, me}});
    }
    const char *env = getenv("TFBS_HOST_THREADS");
    const uint32_t T = env ? (uint32_t)atoi(env) : 1;
    double best_b = 1e9, best_c = 1e9, gsec = 0;
    size_t haps = 0, patched = 0;
    for (int rep = 0; rep < 3; rep++) {
        tfbs_batch *bb = nullptr;
        if (tfbs_batch_create(p, 50000, 0, &bb)) return 1;
        tfbs_batch_add_bed(bb, "synthetic.bed");
        auto gr = std::make_shared<CpuGrouper>();
        bb->b.grouper = gr;
        std::vector<RegionInput> ins = proto;
        std::vector<RegionBuilt> built;
        auto t0 = std::chrono::steady_clock::now();
        if (int rc = build_regions(bb->b, ins, T, built, nullptr)) {
            fprintf(stderr, "build: %s\n", tfbs_last_error());
            return rc;
        }
        auto t1 = std::chrono::steady_clock::now();
        commit_regions(bb->b, built, T);
        auto t2 = std::chrono::steady_clock::now();
        size_t bytes = 0;
        for (const RegionBuilt &rb : built)
            for (const Distinct &d : rb.dist) bytes += d.nuc.capacity() + d.pos.r.capacity() * sizeof(PosRun);
        printf("rep %d: build %.3f s (less the grouper), commit %.3f s, the distinct haplotypes' sequences %.1f MB\n",
               rep, std::chrono::duration<double>(t1 - t0).count() - gr->secs,
               std::chrono::duration<double>(t2 - t1).count(), bytes / 1e6);
        best_b = std::min(best_b, std::chrono::duration<double>(t1 - t0).count() - gr->secs);
        best_c = std::min(best_c, std::chrono::duration<double>(t2 - t1).count());
        gsec = gr->secs;
        if (rep == 0) {  // a digest of the committed batch image (words, N masks, positions, runs, descriptors)
            uint64_t h = 1469598103934665603ull;
            auto mixb = [&](const void *p, size_t n) {
                const uint8_t *c = (const uint8_t *)p;
                for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
            };
            mixb(bb->b.words.data(), bb->b.words.size() * 4);
            mixb(bb->b.nmask.data(), bb->b.nmask.size() * 4);
            mixb(bb->b.posrel.data(), bb->b.posrel.size() * 4);
            mixb(bb->b.druns.data(), bb->b.druns.size() * 4);
            mixb(bb->b.haps.data(), bb->b.haps.size() * sizeof(bb->b.haps[0]));
            printf("batch image digest %016llx (words %zu, posrel %zu, druns %zu)\n", (unsigned long long)h,
                   (size_t)bb->b.words.size(), (size_t)bb->b.posrel.size(), (size_t)bb->b.druns.size());
        }
        haps = bb->b.haps.size();
        patched = bb->b.patched_regions;
        tfbs_batch_destroy(bb);
    }
    printf("regions %llu threads %u: build (less the stand-in grouper's %.3f s) %.3f s, commit %.3f s; per region "
           "%.1f + %.1f us; patched on host %zu, haplotypes %zu\n",
           (unsigned long long)regions, T, gsec, best_b, best_c, best_b / regions * 1e6, best_c / regions * 1e6,
           patched, haps);
    tfbs_batch_destroy(b);
    tfbs_patterns_destroy(p);
    free(names);
    return 0;
}
