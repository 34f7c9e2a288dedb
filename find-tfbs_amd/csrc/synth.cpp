// Synthetic workloads of SURVEY.md section 8(d): HOCOMOCO-format PWM sets with
// exact-distribution thresholds, and phased haplotype regions drawn on demand.
// Everything is a pure function of (seed, index), so ranks of a multi-GPU run
// generate disjoint shards without communicating.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "batch.hpp"
#include "patterns.hpp"

namespace tfbs {
namespace {

inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(splitmix(seed ^ 0x5DEECE66Dull)) {}
    uint64_t next() { return splitmix(s += 0x632BE59BD9B4E019ull); }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
    double gamma_lt1(double a) {  // Marsaglia-Tsang with the a < 1 boost
        double g = gamma_ge1(a + 1.0);
        double u = uniform();
        while (u <= 0.0) u = uniform();
        return g * std::pow(u, 1.0 / a);
    }
    double normal() {
        double u1 = uniform(), u2 = uniform();
        while (u1 <= 0.0) u1 = uniform();
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
    double gamma_ge1(double a) {
        const double d = a - 1.0 / 3.0, c = 1.0 / std::sqrt(9.0 * d);
        for (;;) {
            double x = normal(), v = 1.0 + c * x;
            if (v <= 0) continue;
            v = v * v * v;
            double u = uniform();
            if (u < 1.0 - 0.0331 * x * x * x * x) return d * v;
            if (std::log(u) < 0.5 * x * x + d * (1.0 - v + std::log(v))) return d * v;
        }
    }
    uint32_t poisson(double lambda) {
        const double L = std::exp(-lambda);
        uint32_t k = 0;
        double p = 1.0;
        do {
            k++;
            p *= uniform();
        } while (p > L);
        return k - 1;
    }
};

// Reference base at a synthetic chromosome position: A/T 0.295, C/G 0.205.
inline char ref_base(uint64_t seed, uint64_t x) {
    const double u = (splitmix(seed * 0x9E3779B97F4A7C15ull ^ splitmix(x)) >> 11) * (1.0 / 9007199254740992.0);
    return u < 0.295 ? 'A' : u < 0.5 ? 'C' : u < 0.705 ? 'G' : 'T';
}

uint32_t pwm_length(int config, uint32_t i, uint32_t n) {
    switch (config) {
    case 2: { static const uint32_t L2[10] = {8, 9, 10, 11, 12, 13, 14, 15, 10, 12}; return L2[i % 10]; }
    case 5: return 25 + i % 6;
    default: return (n >= 30 && i >= n - 30) ? 23 + (i - (n - 30)) % 8 : 8 + i % 15;
    }
}

}  // namespace

struct SynthRegion {
    uint64_t ms, me, es;
    std::string ref;
    struct Rec { uint64_t pos; std::string ref, alt; std::vector<uint32_t> carriers; };
    std::vector<Rec> recs;
};

// Harmonic CDF for P(k) ~ 1/k on 1..K, cached per K.
static const std::vector<double> &harmonic_cdf(uint32_t K) {
    thread_local uint32_t cached_k = 0;
    thread_local std::vector<double> cdf;
    if (cached_k != K) {
        cdf.resize(K);
        double s = 0;
        for (uint32_t k = 1; k <= K; k++) cdf[k - 1] = (s += 1.0 / k);
        cached_k = K;
    }
    return cdf;
}

void synth_region(uint64_t seed, uint64_t index, uint32_t n_samples, uint32_t lmax, uint32_t indel_pct,
                  SynthRegion &R) {
    R.ms = 1000 + 400 * index;
    R.me = 1200 + 400 * index;
    const uint64_t L = std::max<uint32_t>(lmax, 1);
    R.es = R.ms + 1 - L;
    const uint64_t ee = R.me + L - 1;
    R.ref.resize(ee - R.es + 1);
    for (uint64_t x = R.es; x <= ee; x++) R.ref[x - R.es] = ref_base(seed, x);
    R.recs.clear();
    Rng rng(splitmix(seed) ^ splitmix(index + 0x1234567ull));
    const uint32_t H = 2 * n_samples;
    const uint32_t nsites = std::min<uint32_t>(rng.poisson(20.0), (uint32_t)(ee - R.es + 1));
    std::vector<uint64_t> sites;
    while (sites.size() < nsites) {
        uint64_t p = R.es + rng.below(ee - R.es + 1);
        if (std::find(sites.begin(), sites.end(), p) == sites.end()) sites.push_back(p);
    }
    std::sort(sites.begin(), sites.end());
    static const char B[4] = {'A', 'C', 'G', 'T'};
    uint64_t blocked_until = 0;  // no site inside an earlier deletion's span
    const uint32_t K = std::max<uint32_t>(1, H / 10);
    const std::vector<double> &cdf = harmonic_cdf(K);
    thread_local std::vector<uint64_t> bitmap;
    bitmap.assign((H + 63) / 64, 0);
    for (uint64_t p : sites) {
        if (p <= blocked_until && blocked_until) continue;
        SynthRegion::Rec r;
        r.pos = p;
        const char rb = R.ref[p - R.es];
        const bool indel = rng.below(100) < indel_pct;
        if (indel) {
            const uint32_t len = 1 + (uint32_t)rng.below(10);
            if (rng.below(2) == 0) {  // insertion
                r.ref = std::string(1, rb);
                r.alt = r.ref;
                for (uint32_t i = 0; i < len; i++) r.alt.push_back(B[rng.below(4)]);
            } else {  // deletion of len bases after p (within the window)
                r.ref = std::string(1, rb);
                for (uint32_t i = 1; i <= len && p + i <= ee; i++) r.ref.push_back(R.ref[p + i - R.es]);
                r.alt = std::string(1, rb);
                if (r.ref.size() == 1) {  // at the window end: make it an insertion instead
                    r.alt.push_back(B[rng.below(4)]);
                }
                blocked_until = p + r.ref.size() - 1;
            }
        } else {
            char a;
            do a = B[rng.below(4)]; while (a == rb);
            r.ref = std::string(1, rb);
            r.alt = std::string(1, a);
        }
        // carrier count k ~ 1/k on 1..H/10, carriers uniform over haplotypes
        const double u = rng.uniform() * cdf.back();
        uint32_t k = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()) + 1;
        k = std::min(k, H);
        r.carriers.reserve(k);
        while (r.carriers.size() < k) {
            uint32_t h = (uint32_t)rng.below(H);
            uint64_t &w = bitmap[h >> 6];
            if (w & (1ull << (h & 63))) continue;
            w |= 1ull << (h & 63);
            r.carriers.push_back(h);
        }
        for (uint32_t h : r.carriers) bitmap[h >> 6] &= ~(1ull << (h & 63));
        std::sort(r.carriers.begin(), r.carriers.end());
        R.recs.push_back(std::move(r));
    }
}

}  // namespace tfbs

struct tfbs_synth_region {
    tfbs::SynthRegion r;
};

extern "C" {

int tfbs_synth_write_pwms(const char *dir, uint32_t n, int config, uint64_t seed, char **names_csv) {
    using namespace tfbs;
    if (!dir || !names_csv) return fail(TFBS_E_ARG, "null argument");
    std::string d(dir), td = d + "/thr";
    mkdir(d.c_str(), 0755);
    mkdir(td.c_str(), 0755);
    std::vector<std::string> names(n), text(n), thr(n);
    auto work = [&](uint32_t t0, uint32_t step) {
        for (uint32_t i = t0; i < n; i += step) {
            Rng rng(splitmix(seed) ^ splitmix(0xABCDEFull + i));
            const uint32_t L = pwm_length(config, i, n);
            char nb[64];
            snprintf(nb, sizeof nb, "SYN%04u_HUMAN.H11MO.0.A", i);
            names[i] = nb;
            std::string t = ">" + names[i] + "\n";
            std::vector<int32_t> w(4 * L);
            for (uint32_t j = 0; j < L; j++) {
                double g[4], s = 0;
                for (int c = 0; c < 4; c++) s += (g[c] = rng.gamma_lt1(0.5));
                for (int c = 0; c < 4; c++) {
                    const double p = s > 0 ? g[c] / s : 0.25;
                    const double x = std::log(((p + 0.01) / 1.04) / 0.25);
                    char fb[32];
                    snprintf(fb, sizeof fb, "%.3f", x);
                    int32_t v;
                    parse_weight(fb, &v);
                    w[4 * j + c] = v;
                    t += fb;
                    t += c == 3 ? "\n" : "\t";
                }
            }
            text[i] = t;
            // exact score distribution under a uniform background
            std::vector<int32_t> mn(L), mx(L);
            int64_t lo = 0, hi = 0;
            for (uint32_t j = 0; j < L; j++) {
                mn[j] = *std::min_element(&w[4 * j], &w[4 * j] + 4);
                mx[j] = *std::max_element(&w[4 * j], &w[4 * j] + 4);
                lo += mn[j];
                hi += mx[j];
            }
            std::vector<double> dist(1, 1.0), nd;
            for (uint32_t j = 0; j < L; j++) {
                const uint32_t span = (uint32_t)(mx[j] - mn[j]);
                nd.assign(dist.size() + span, 0.0);
                for (int c = 0; c < 4; c++) {
                    const uint32_t off = (uint32_t)(w[4 * j + c] - mn[j]);
                    double *o = nd.data() + off;
                    for (size_t k = 0; k < dist.size(); k++) o[k] += 0.25 * dist[k];
                }
                dist.swap(nd);
            }
            // tail[k] = P(score >= lo + k)
            std::vector<double> tail(dist.size() + 1, 0.0);
            for (size_t k = dist.size(); k-- > 0;) tail[k] = tail[k + 1] + dist[k];
            static const double targets[] = {1.0, 0.1, 0.01, 0.005, 0.001, 0.0005, 0.0001, 0.00005, 0.00001, 0.000001};
            std::vector<std::pair<int64_t, double>> lines;
            for (double tg : targets) {
                size_t k = 0;
                while (k < dist.size() && tail[k] > tg) k++;
                if (k > 0) lines.push_back({lo + (int64_t)k - 1, tail[k - 1]});
                if (k < dist.size()) lines.push_back({lo + (int64_t)k, tail[k]});
            }
            std::sort(lines.begin(), lines.end());
            lines.erase(std::unique(lines.begin(), lines.end()), lines.end());
            std::string th;
            for (auto &l : lines) {
                char lb[64];
                snprintf(lb, sizeof lb, "%.3f\t%.6g\n", l.first / 1000.0, l.second);
                th += lb;
            }
            thr[i] = th;
            (void)hi;
        }
    };
    const uint32_t T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < T; t++) ts.emplace_back(work, t, T);
    for (auto &t : ts) t.join();
    FILE *f = fopen((d + "/pwms.txt").c_str(), "wb");
    if (!f) return fail(TFBS_E_IO, "cannot write " + d + "/pwms.txt");
    for (auto &t : text) fwrite(t.data(), 1, t.size(), f);
    fclose(f);
    std::string csv;
    for (uint32_t i = 0; i < n; i++) {
        FILE *g = fopen((td + "/" + names[i] + ".thr").c_str(), "wb");
        if (!g) return fail(TFBS_E_IO, "cannot write threshold file");
        fwrite(thr[i].data(), 1, thr[i].size(), g);
        fclose(g);
        if (i) csv += ',';
        csv += names[i];
    }
    *names_csv = strdup(csv.c_str());
    return TFBS_OK;
}

int tfbs_synth_region_make(uint64_t seed, uint64_t index, uint32_t n_samples, uint32_t lmax, uint32_t indel_pct,
                           tfbs_synth_region **out) {
    if (!out) return tfbs::fail(TFBS_E_ARG, "null argument");
    auto *r = new tfbs_synth_region();
    tfbs::synth_region(seed, index, n_samples, lmax, indel_pct, r->r);
    *out = r;
    return TFBS_OK;
}

void tfbs_synth_region_destroy(tfbs_synth_region *r) { delete r; }

void tfbs_synth_region_info(const tfbs_synth_region *r, uint64_t *ms, uint64_t *me, uint64_t *es, const char **ref,
                            size_t *n_ref, size_t *n_rec) {
    *ms = r->r.ms;
    *me = r->r.me;
    *es = r->r.es;
    *ref = r->r.ref.c_str();
    *n_ref = r->r.ref.size();
    *n_rec = r->r.recs.size();
}

void tfbs_synth_region_record(const tfbs_synth_region *r, size_t i, uint64_t *pos, const char **ref, const char **alt,
                              const uint32_t **carriers, size_t *n) {
    const auto &q = r->r.recs[i];
    *pos = q.pos;
    *ref = q.ref.c_str();
    *alt = q.alt.c_str();
    *carriers = q.carriers.data();
    *n = q.carriers.size();
}

int tfbs_synth_fill_batch(tfbs_batch *b, uint64_t seed, uint64_t first, uint64_t count, uint32_t indel_pct) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    tfbs::Batch &B = b->b;
    if (B.open) return tfbs::fail(TFBS_E_STATE, "region open");
    int bed = -1;
    for (size_t i = 0; i < B.beds.size(); i++)
        if (B.beds[i] == "synthetic.bed") bed = (int)i;
    if (bed < 0) bed = tfbs_batch_add_bed(b, "synthetic.bed");
    const uint32_t lmax = B.lmax();
    const char *env = getenv("TFBS_HOST_THREADS");
    uint32_t T = env && *env ? (uint32_t)atoi(env) : std::thread::hardware_concurrency();
    T = std::max(1u, std::min(16u, T));
    B.counts_valid = false;
    const uint64_t chunk = 64ull * T;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_fill = now();
    std::vector<tfbs::RegionBuilt> prev;  // the last chunk built, committed during the next build
    bool have_prev = false, prev_first = false;
    const char *ov = getenv("TFBS_PREP_OVERLAP");  // 0: never (A/B)
    const bool overlap = !(ov && *ov && atoi(ov) == 0);
    uint64_t prev_n = 0;
    auto commit = [&] {
        tfbs::commit_regions(B, prev, T);
        if (prev_first && prev_n < count)  // the rest of the regions will look alike: room for them now
            tfbs::reserve_batch(B, 1.15 * (double)(B.rh.size() + count - prev_n) / (double)std::max<size_t>(B.rh.size(), 1));
        prev.clear();
    };
    for (uint64_t c0 = first; c0 < first + count; c0 += chunk) {
        const uint64_t n = std::min<uint64_t>(chunk, first + count - c0);
        // phase 1: the synthetic inputs (what a BCF / FASTA reader would hand over)
        std::vector<tfbs::RegionInput> ins(n);
        std::atomic<uint64_t> next(0);
        std::mutex mu;
        auto gen = [&]() {
            tfbs::SynthRegion R;
            double t_gen = 0;
            for (;;) {
                const uint64_t j = next.fetch_add(1);
                if (j >= n) break;
                const double t0 = now();
                tfbs::synth_region(seed, c0 + j, B.n_samples, lmax, indel_pct, R);
                tfbs::RegionInput &in = ins[j];
                in.R.ms = R.ms;
                in.R.me = R.me;
                in.R.es = R.es;
                in.R.ee = R.me + std::max<uint32_t>(lmax, 1) - 1;
                in.ref.resize(R.ref.size());
                for (size_t i = 0; i < R.ref.size(); i++) in.ref[i] = (uint8_t)tfbs::to_nuc((uint8_t)R.ref[i]);
                for (auto &q : R.recs) {
                    tfbs::Record r;
                    r.pos = q.pos;
                    for (char c : q.ref) r.ref.push_back((uint8_t)tfbs::to_nuc((uint8_t)c));
                    for (char c : q.alt) r.alt.push_back((uint8_t)tfbs::to_nuc((uint8_t)c));
                    r.carriers = std::move(q.carriers);
                    in.recs.push_back(std::move(r));
                }
                in.inner.push_back({(uint32_t)bed, {R.ms, R.me}});
                t_gen += now() - t0;
            }
            std::lock_guard<std::mutex> g(mu);
            B.prep_s[0] += t_gen;
        };
        {
            std::vector<std::thread> ts;
            for (uint32_t t = 0; t + 1 < T && t + 1 < n; t++) ts.emplace_back(gen);
            gen();
            for (auto &t : ts) t.join();
        }
        // phase 2: load_diffs / group / patch / dedup / pack (build_regions: on the
        // device grouper where the region qualifies), while the previous chunk's regions
        // are committed on another thread (the build waits on the device and neither
        // keeps 16 threads busy throughout: C3 0.22 -> 0.16 s, C5 0.79 -> 0.72 s on one
        // box).  build_regions and commit_regions touch disjoint batch fields; the
        // generation above ran alone, so the overlap hides only build and commit time
        // behind each other.
        const double t_build = now();
        std::thread committer;
        if (have_prev) committer = std::thread([&] { commit(); });
        std::vector<tfbs::RegionBuilt> built;
        const int rc = tfbs::build_regions(B, ins, T, built, &B.prep_s[1]);
        if (committer.joinable()) committer.join();
        if (rc) return rc;
        prev = std::move(built);
        prev_first = c0 == first;
        prev_n = n;
        have_prev = true;
        if (!overlap) {  // (TFBS_PREP_OVERLAP=0: committed as it is built)
            commit();
            have_prev = false;
        }
        B.prep_s[2] += now() - t_build;
    }
    if (have_prev) {
        const double t = now();
        commit();
        B.prep_s[2] += now() - t;
    }
    B.prep_s[3] += now() - t_fill;
    return TFBS_OK;
}

}  // extern "C"
