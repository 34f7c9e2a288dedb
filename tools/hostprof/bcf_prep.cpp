// The run flow's per-region BCF part (run.cpp prepare: Bcf::fetch of each merged
// region's window + make_record_ids) on a synthetic dataset, without a GPU: where
// prep_bcf_s goes.  Profiling aid only: ./bcf_prep <dir of tools/synth_dataset.py> [threads] [lmax]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "batch.hpp"
#include "io.hpp"
#include "tfbs_internal.hpp"

using namespace tfbs;

int main(int argc, char **argv) {
    if (argc < 2) return 1;
    const std::string dir = argv[1];
    const uint32_t threads = argc > 2 ? (uint32_t)atoi(argv[2]) : 8;
    const uint64_t lmax = argc > 3 ? strtoull(argv[3], nullptr, 10) : 30;
    std::vector<std::pair<uint64_t, uint64_t>> peaks;
    if (load_bed(dir + "/regions.bed", "chr1", peaks)) return 1;
    const auto merged = merge_ranges(peaks);
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = now();
    Bcf bcf;
    if (bcf.open(dir + "/genotypes.bcf", threads) || bcf.set_carriers_mode(true)) return 1;
    const int rid = bcf.contig_index("chr1");
    std::vector<const BcfRecord *> recs;
    double t_fetch = 0, t_ids = 0;
    size_t n_rec = 0, n_car = 0;
    const double t1 = now();
    for (const auto &m : merged) {
        const uint64_t es = m.first >= lmax - 1 ? m.first - (lmax - 1) : 0, ee = m.second + lmax - 1;
        const double a = now();
        if (bcf.fetch(rid, es, ee + 1, recs)) {
            fprintf(stderr, "%s\n", tfbs_last_error());
            return 1;
        }
        const double b = now();
        for (const BcfRecord *br : recs) {
            Record rec;
            if (make_record_ids(br->pos, br->n_alleles, br->ref.c_str(), br->alt.c_str(), br->carriers, br->gt_status, rec))
                return 1;
            n_car += rec.carriers.size();
        }
        n_rec += recs.size();
        t_fetch += b - a;
        t_ids += now() - b;
    }
    printf("regions %zu records %zu carriers %zu threads %u: open %.3f s, fetch %.3f s, record ids %.3f s, total %.3f s\n",
           merged.size(), n_rec, n_car, threads, t1 - t0, t_fetch, t_ids, now() - t0);
    return 0;
}
