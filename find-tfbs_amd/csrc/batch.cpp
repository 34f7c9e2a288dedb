// Region batches: load_diffs / group_by_diffs / load_haplotypes / patch_haplotype
// (haplotype.rs:13-156) and the packing of distinct haplotypes for the GPU.
//
// Determinism where the reference iterates a HashMap (documented in DESIGN.md):
// groups are visited in ascending Vec<Diff> order, and when two groups patch to
// the same sequence the later one wins (HashMap::insert, haplotype.rs:84); the
// loser's haplotype ids stay with the reference group (main.rs:103-105, 129-137).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>
#include <unordered_map>

#include "batch.hpp"

namespace tfbs {

// derived Ord on Diff (types.rs:39-44): pos, then reference, then alternative.
static bool diff_less(const Record *a, const Record *b) {
    if (a->pos != b->pos) return a->pos < b->pos;
    if (a->ref != b->ref) return std::lexicographical_compare(a->ref.begin(), a->ref.end(), b->ref.begin(), b->ref.end());
    return std::lexicographical_compare(a->alt.begin(), a->alt.end(), b->alt.begin(), b->alt.end());
}
static bool diff_equal(const Record *a, const Record *b) {
    return a->pos == b->pos && a->ref == b->ref && a->alt == b->alt;
}

// A reference window: consecutive positions [start, start + n) (the batch case).
struct RefWindow {
    const uint8_t *nuc;
    uint64_t start;
    size_t n;
    // haplotype.rs:90-92 get(): bases with pos in [s, e]
    void get(uint64_t s, uint64_t e, std::vector<uint8_t> &nucs, PosRuns &pos) const {
        if (n == 0 || e < s) return;
        const uint64_t lo = std::max(s, start), hi = std::min(e, start + n - 1);
        if (hi < lo) return;
        nucs.insert(nucs.end(), nuc + (lo - start), nuc + (hi - start) + 1);
        pos.push_range(lo, hi);
    }
    // haplotype.rs:119-125: the base at pos, N if absent
    uint8_t at(uint64_t p) const { return (p >= start && p - start < n) ? nuc[p - start] : 4; }
};

// haplotype.rs:94-156.  The recursion of next_chunk is a loop with the same case order.
// (Diffs already inside [rs, re] and in Diff order -- a group's bits over the sorted
// distinct records -- are used as they are: no copy, no sort.)
static int patch_window(uint64_t rs, uint64_t re, const std::vector<const Record *> &diffs_in, const RefWindow &ref,
                        std::vector<uint8_t> &nucs, PosRuns &pos) {
    bool as_is = true;
    for (size_t i = 0; i < diffs_in.size() && as_is; i++)
        as_is = diffs_in[i]->pos >= rs && diffs_in[i]->pos <= re && (i == 0 || !diff_less(diffs_in[i], diffs_in[i - 1]));
    std::vector<const Record *> sorted;
    if (!as_is) {
        sorted = diffs_in;
        sorted.erase(std::remove_if(sorted.begin(), sorted.end(), [&](const Record *d) { return d->pos < rs || d->pos > re; }),
                     sorted.end());
        std::stable_sort(sorted.begin(), sorted.end(), diff_less);
    }
    const std::vector<const Record *> &diffs = as_is ? diffs_in : sorted;
    uint64_t at = rs;
    size_t k = 0;
    for (;;) {
        if (k == diffs.size()) {
            if (at <= re) ref.get(at, re, nucs, pos);
            return TFBS_OK;
        }
        const Record *d = diffs[k];
        if (d->pos > at) {
            ref.get(at, d->pos - 1, nucs, pos);
            at = d->pos;
        } else if (d->pos == at && d->ref.size() == 1) {  // SNV or insertion
            if (d->ref[0] != ref.at(at))
                return fail(TFBS_E_REFMISMATCH,
                            "First reference nucleotide of variant doesn't match reference genome at " +
                                std::to_string(at));
            for (uint8_t a : d->alt) {
                nucs.push_back(a);
                pos.push(at);
            }
            at += 1;
            k++;
        } else if (d->pos == at && d->alt.size() == 1) {  // deletion
            nucs.push_back(d->alt[0]);
            pos.push(at);
            at += d->ref.size();
            k++;
        } else if (d->pos == at) {
            return fail(TFBS_E_MNP, "Missing case in haplotype patcher at " + std::to_string(at));
        } else if (at >= re) {
            ref.get(at, at, nucs, pos);
            return TFBS_OK;
        } else {
            return TFBS_OK;  // overlapping diffs truncate the haplotype
        }
    }
}

int patch(uint64_t rs, uint64_t re, std::vector<const Record *> diffs, const uint8_t *ref, uint64_t ref_start,
          size_t n_ref, std::vector<uint8_t> &nucs, std::vector<uint64_t> &pos) {
    RefWindow w{ref, ref_start, n_ref};
    PosRuns runs;
    const int rc = patch_window(rs, re, diffs, w, nucs, runs);
    pos.resize(runs.n);
    runs.expand(pos.data(), [](uint64_t p) { return p; });
    return rc;
}

// load_haplotypes' HashMap<(nucs, pos), group> insert (haplotype.rs:84): the
// patched sequences of a region by a hash of their bases (8 at a time) and of their
// runs of consecutive positions, in a flat open-addressing table; a sequence equal
// to an earlier one gives that entry the later group (HashMap::insert replaces the
// value), else it is appended to dist.
namespace {
struct SeqTable {
    std::vector<uint64_t> key;  // hash, 0 = empty
    std::vector<uint32_t> idx;
    uint32_t mask = 0;
    explicit SeqTable(size_t n) {
        size_t c = 16;
        while (c < 2 * n) c *= 2;
        key.assign(c, 0);
        idx.assign(c, 0);
        mask = (uint32_t)c - 1;
    }
    static uint64_t hash(const Distinct &d, uint64_t es) {
        auto mix = [](uint64_t h, uint64_t v) {
            h ^= v * 0x9E3779B97F4A7C15ull;
            h ^= h >> 29;
            return h * 0xBF58476D1CE4E5B9ull;
        };
        const size_t n = d.nuc.size();
        uint64_t h = mix(0x243F6A8885A308D3ull, n);
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t x;
            memcpy(&x, d.nuc.data() + i, 8);
            h = mix(h, x);
        }
        for (; i < n; i++) h = mix(h, d.nuc[i] | 0x100u);
        // positions: their offsets from the affine ones, weighted by 2i + 1 (sum over
        // a run [a, b) of the run's constant offset x (b^2 - a^2), mod 2^64)
        uint64_t ps = 0;
        for (size_t k = 0; k < d.pos.r.size(); k++) {
            const uint64_t a = d.pos.r[k].at, b = d.pos.end(k);
            ps += (d.pos.r[k].p - es - a) * (b * b - a * a);
        }
        h = mix(h, ps);
        return h | 1;  // (never 0: the empty mark)
    }
    void insert(std::vector<Distinct> &dist, Distinct &&d, uint64_t es) {
        const uint64_t h = hash(d, es);
        for (uint32_t s = (uint32_t)(h ^ (h >> 32)) & mask;; s = (s + 1) & mask) {
            if (!key[s]) {
                key[s] = h;
                idx[s] = (uint32_t)dist.size();
                dist.push_back(std::move(d));
                return;
            }
            if (key[s] == h && dist[idx[s]].nuc == d.nuc && dist[idx[s]].pos == d.pos) {
                dist[idx[s]].group = d.group;
                return;
            }
        }
    }
};
}  // namespace

uint64_t Batch::device_bytes() const {
    return words.size() * 4ull + nmask.size() * 4ull + posrel.size() * 4ull + druns.size() * 4ull +
           haps.size() * sizeof(DevHap) + regions.size() * sizeof(DevRegion) + inner.size() * 4ull;
}

// ---------------------------------------------------------------------------
// Builds one region's distinct haplotypes from its inputs; touches no batch
// state, so regions can be built on several host threads (commit is serial).
// inner keys: unique (bed, s, e) with multiplicity; distinct non-empty ranges
static void inner_keys(std::vector<std::pair<uint32_t, std::pair<uint64_t, uint64_t>>> in, RegionH &R) {
    R.keys.clear();
    R.ranges.clear();
    std::sort(in.begin(), in.end(), [](const auto &a, const auto &b) {
        if (a.second != b.second) return a.second < b.second;
        return a.first < b.first;
    });
    for (size_t i = 0; i < in.size();) {
        size_t j = i;
        while (j < in.size() && in[j] == in[i]) j++;
        InnerKey k{in[i].first, in[i].second.first, in[i].second.second, (uint32_t)(j - i), -1};
        if (k.e >= k.s) {
            auto r = std::make_pair(k.s, k.e);
            if (R.ranges.empty() || R.ranges.back() != r) R.ranges.push_back(r);
            k.slot = (int32_t)R.ranges.size() - 1;
        }
        R.keys.push_back(k);
        i = j;
    }
}

int build_region(const Batch &B, RegionInput &&I, RegionBuilt &out) {
    out.R = std::move(I.R);
    RegionH &R = out.R;
    const uint32_t H = 2 * B.n_samples;
    R.n_variants = (uint32_t)I.recs.size();  // variant_count counts every fetched record (haplotype.rs:25)
    inner_keys(std::move(I.inner), R);

    // ---- load_diffs: (haplotype id, canonical diff rank) in record order
    std::vector<const Record *> uniq;
    for (auto &r : I.recs)
        if (r.n_alleles == 2 && !r.carriers.empty()) uniq.push_back(&r);
    std::stable_sort(uniq.begin(), uniq.end(), diff_less);
    uniq.erase(std::unique(uniq.begin(), uniq.end(), diff_equal), uniq.end());
    auto rank_of = [&](const Record *r) {
        return (uint32_t)(std::lower_bound(uniq.begin(), uniq.end(), r, diff_less) - uniq.begin());
    };
    // Result of load_diffs + group_by_diffs: hap_ids ascending, each haplotype's
    // diff ranks ascending in hd[span_b[k], span_e[k]), and the groups as runs of
    // `order` (indices into hap_ids), in ascending Vec<Diff> order.
    // (The mask path keeps no spans: a group's diffs are its mask's bits, gmask.)
    std::vector<std::pair<uint32_t, uint32_t>> hd;  // (hap, rank)
    std::vector<uint32_t> span_b, span_e, order;
    thread_local std::vector<uint32_t> hap_ids;  // reused: no page faults per region
    hap_ids.clear();
    std::vector<uint64_t> gmask;  // mask path: each group's diff mask
    struct Group { uint32_t first, last; };  // run in `order`
    std::vector<Group> groups;
    bool masks_ok = uniq.size() <= 64;
    thread_local std::vector<uint64_t> sig;
    if (masks_ok) {
        // every haplotype's diff list as a 64-bit rank mask: one pass over the
        // carrier lists, one pass over the haplotypes, a hash of the distinct masks.
        // A haplotype carrying one diff twice (duplicate records) has the list
        // [d, d], not [d] (haplotype.rs:65-75): masks cannot say so, so such a
        // region takes the sorted-list path.
        if (sig.size() < H) sig.assign(H, 0);
        bool dup = false;
        for (auto &r : I.recs) {
            if (r.n_alleles != 2 || r.carriers.empty()) continue;
            const uint64_t bit = 1ull << rank_of(&r);
            for (uint32_t h : r.carriers)
                if (h < H) {
                    dup |= (sig[h] & bit) != 0;
                    sig[h] |= bit;
                }
        }
        if (dup) {
            for (auto &r : I.recs)
                for (uint32_t h : r.carriers)
                    if (h < H) sig[h] = 0;
            masks_ok = false;
        }
    }
    if (masks_ok) {
        // mask -> distinct mask index in an open-addressed table (masks are
        // non-zero, 0 marks a free slot); each haplotype's index in gk, then the
        // members scattered per mask in ascending haplotype order (counting sort)
        thread_local std::vector<uint64_t> tkey;
        thread_local std::vector<uint32_t> tval;
        size_t cap = 1024;
        tkey.assign(cap, 0);
        tval.resize(cap);
        std::vector<uint64_t> masks;
        std::vector<uint32_t> gcount;
        thread_local std::vector<uint32_t> gk;
        gk.clear();
        auto slot_of = [&](uint64_t m) {
            size_t s = (size_t)((m * 0x9E3779B97F4A7C15ull) >> 40) & (cap - 1);
            while (tkey[s] != 0 && tkey[s] != m) s = (s + 1) & (cap - 1);
            return s;
        };
        for (uint32_t h = 0; h < H; h++) {
            const uint64_t m = sig[h];
            if (!m) continue;
            sig[h] = 0;
            hap_ids.push_back(h);
            size_t s = slot_of(m);
            if (tkey[s] == 0) {
                if (2 * (masks.size() + 1) > cap) {  // grow to keep the load under 1/2
                    cap *= 2;
                    tkey.assign(cap, 0);
                    tval.resize(cap);
                    for (uint32_t q = 0; q < masks.size(); q++) {
                        const size_t t = slot_of(masks[q]);
                        tkey[t] = masks[q];
                        tval[t] = q;
                    }
                    s = slot_of(m);
                }
                tkey[s] = m;
                tval[s] = (uint32_t)masks.size();
                masks.push_back(m);
                gcount.push_back(0);
            }
            gk.push_back(tval[s]);
            gcount[tval[s]]++;
        }
        // Vec<Diff> order of the masks' ascending rank lists
        auto lex_less = [](uint64_t a, uint64_t b) {
            const uint64_t d = a ^ b;
            if (!d) return false;
            const uint64_t low = d & (~d + 1);  // lowest rank in exactly one list
            const uint64_t above = ~((low << 1) - 1);
            return (a & low) ? (b & above) != 0 : (a & above) == 0;
        };
        std::vector<uint32_t> gs(masks.size());
        std::iota(gs.begin(), gs.end(), 0u);
        std::sort(gs.begin(), gs.end(), [&](uint32_t x, uint32_t y) { return lex_less(masks[x], masks[y]); });
        std::vector<uint32_t> start(masks.size());
        uint32_t at = 0;
        for (uint32_t g : gs) {
            start[g] = at;
            groups.push_back({at, at + gcount[g]});
            gmask.push_back(masks[g]);
            at += gcount[g];
        }
        order.resize(at);
        for (uint32_t k = 0; k < (uint32_t)gk.size(); k++) order[start[gk[k]]++] = k;
    } else {
        for (auto &r : I.recs) {
            if (r.n_alleles != 2 || r.carriers.empty()) continue;
            uint32_t rk = rank_of(&r);
            for (uint32_t h : r.carriers)
                if (h < H) hd.push_back({h, rk});
        }
        std::stable_sort(hd.begin(), hd.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        // per-hap spans
        for (size_t i = 0; i < hd.size();) {
            size_t j = i;
            while (j < hd.size() && hd[j].first == hd[i].first) j++;
            hap_ids.push_back(hd[i].first);
            span_b.push_back((uint32_t)i);
            span_e.push_back((uint32_t)j);
            i = j;
        }
        // ---- group_by_diffs: sort haplotypes by diff list (rank order == Vec<Diff> order)
        order.resize(hap_ids.size());
        std::iota(order.begin(), order.end(), 0);
        auto seq_less = [&](uint32_t a, uint32_t b) {
            return std::lexicographical_compare(
                hd.begin() + span_b[a], hd.begin() + span_e[a], hd.begin() + span_b[b], hd.begin() + span_e[b],
                [](const auto &x, const auto &y) { return x.second < y.second; });
        };
        auto seq_eq = [&](uint32_t a, uint32_t b) {
            if (span_e[a] - span_b[a] != span_e[b] - span_b[b]) return false;
            for (uint32_t t = 0; t < span_e[a] - span_b[a]; t++)
                if (hd[span_b[a] + t].second != hd[span_b[b] + t].second) return false;
            return true;
        };
        std::stable_sort(order.begin(), order.end(), seq_less);
        for (uint32_t i = 0; i < order.size();) {
            uint32_t j = i;
            while (j < order.size() && seq_eq(order[i], order[j])) j++;
            groups.push_back({i, j});
            i = j;
        }
    }

    // ---- load_haplotypes: patch each group, dedup by (nucs, pos) sequence; later group wins
    std::vector<Distinct> &dist = out.dist;
    dist.clear();
    SeqTable table(groups.size());
    RefWindow ref{I.ref.data(), R.es, I.ref.size()};
    for (uint32_t g = 0; g < groups.size(); g++) {
        uint32_t rep = order[groups[g].first];
        std::vector<const Record *> diffs;
        if (masks_ok)
            for (uint64_t x = gmask[g]; x; x &= x - 1) diffs.push_back(uniq[__builtin_ctzll(x)]);
        else
            for (uint32_t t = span_b[rep]; t < span_e[rep]; t++) diffs.push_back(uniq[hd[t].second]);
        Distinct d;
        d.nuc.reserve(R.ee - R.es + 16);
        int rc = patch_window(R.es, R.ee, diffs, ref, d.nuc, d.pos);
        if (rc) return rc;
        d.group = (int32_t)g;
        table.insert(dist, std::move(d), R.es);
    }
    // membership and carrier counts
    std::vector<uint32_t> &carriers = out.carriers;
    carriers.assign(dist.size(), 0);
    // local distinct index per entry of hap_ids (ascending haplotype ids; each
    // in at most one group, a losing group's members in none)
    std::vector<uint32_t> local_of;
    if (B.keep_membership) local_of.assign(hap_ids.size(), UINT32_MAX);
    uint64_t covered = 0;
    for (uint32_t i = 0; i < dist.size(); i++) {
        const Group &G = groups[dist[i].group];
        carriers[i] = G.last - G.first;
        covered += carriers[i];
        if (B.keep_membership)
            for (uint32_t t = G.first; t < G.last; t++) local_of[order[t]] = i;
    }
    R.ref_local = -1;
    if (covered < H) {  // haplotypes_with_reference_genome is non-empty (main.rs:129)
        Distinct d;
        d.nuc = I.ref;
        d.pos = PosRuns::affine(R.es, I.ref.size());
        d.group = -1;
        R.ref_local = (int32_t)dist.size();
        dist.push_back(std::move(d));
        carriers.push_back((uint32_t)(H - covered));
    }
    // reference-window reuse needs the reference's windows: without a reference
    // group, a helper copy is scanned after the distinct haplotypes (no carriers,
    // no keys)
    // (only when the reference's windows can be reused: it and some distinct
    // haplotype have at most kDedupMaxWindows bases)
    out.helper = false;
    auto fits = [](size_t n) { return n <= kDedupMaxWindows; };
    bool reusable = false;
    for (const Distinct &d : dist) reusable = reusable || fits(d.nuc.size());
    if (B.dedup && R.ref_local < 0 && reusable && fits(I.ref.size())) {
        Distinct d;
        d.nuc = I.ref;
        d.pos = PosRuns::affine(R.es, I.ref.size());
        d.group = -2;
        dist.push_back(std::move(d));
        carriers.push_back(0);
        out.helper = true;
    }
    // the kernels index windows with 29 bits (scan_mfma.hip queue entries)
    for (const Distinct &d : dist)
        if (d.nuc.size() >= kMaxHapLen) return fail(TFBS_E_ARG, "haplotype longer than 2^26 - 1 bases");
    if (B.keep_membership) {  // (hap id, local) in ascending hap id: hap_ids' order
        R.nonref_id.clear();
        R.nonref_local.clear();
        for (size_t k = 0; k < hap_ids.size(); k++)
            if (local_of[k] != UINT32_MAX) {
                R.nonref_id.push_back(hap_ids[k]);
                R.nonref_local.push_back(local_of[k]);
            }
    }

    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// Device grouping (tfbs_batch_set_build_device).  A region qualifies when
// load_haplotypes reduces to substitutions into the reference window: every
// applied record (bi-allelic, with carriers) is an SNV inside the window whose
// REF base is the window's and whose ALT is another of A/C/G/T; at most 64 of
// them, no two at one position; every carrier list strictly ascending below 2 *
// n_samples; no N in the window.  (A region of more than kGrpMax distinct masks
// is built on the host too.)  Then no diff list repeats a diff, no two
// lists patch to one sequence (so HashMap::insert never replaces, haplotype.rs:84)
// and no patch truncates (haplotype.rs:140-152): the distinct haplotypes are
// the distinct diff masks in Vec<Diff> order plus the reference group, exactly
// what build_region finds.  The device computes the masks, the groups and the
// membership (build_gpu.hip); the host takes the rest from the masks.  Anything
// else -- and a region of more than kGrpMax masks -- is built by build_region.
static bool snv_prepare(const Batch &B, const RegionInput &I, RegionBuilt &out, std::vector<const Record *> &uniq) {
    const uint32_t H = 2 * B.n_samples;
    const uint64_t n = I.ref.size();
    if (n == 0 || I.R.ee < I.R.es || n != I.R.ee - I.R.es + 1) return false;
    for (uint8_t c : I.ref)
        if (c > 3) return false;
    uniq.clear();
    for (const Record &r : I.recs) {
        if (r.n_alleles != 2 || r.carriers.empty()) continue;  // not applied (haplotype.rs:28-31)
        if (r.ref.size() != 1 || r.alt.size() != 1 || r.alt[0] > 3 || r.pos < I.R.es || r.pos > I.R.ee) return false;
        if (I.ref[r.pos - I.R.es] != r.ref[0] || r.alt[0] == r.ref[0]) return false;
        if (r.carriers.back() >= H) return false;
        for (size_t i = 1; i < r.carriers.size(); i++)
            if (r.carriers[i] <= r.carriers[i - 1]) return false;
        uniq.push_back(&r);
    }
    if (uniq.size() > 64) return false;
    std::sort(uniq.begin(), uniq.end(), diff_less);
    for (size_t i = 1; i < uniq.size(); i++)
        if (uniq[i]->pos == uniq[i - 1]->pos) return false;
    out = RegionBuilt();
    out.R = I.R;
    out.R.n_variants = (uint32_t)I.recs.size();
    inner_keys(I.inner, out.R);
    out.dev = true;
    for (const Record *r : uniq) {
        out.snv_rel.push_back((uint32_t)(r->pos - I.R.es));
        out.snv_alt.push_back(r->alt[0]);
    }
    out.ref = I.ref;
    return true;
}

// The device's groups of a qualifying region: G masks with their carrier counts,
// then the reference group (ids in no group) and the helper as build_region adds them.
static int snv_finish(const Batch &B, RegionBuilt &b, const uint64_t *masks, const uint32_t *counts, uint32_t G,
                      uint64_t memb) {
    const uint32_t H = 2 * B.n_samples;
    RegionH &R = b.R;
    b.masks.assign(masks, masks + G);
    b.carriers.assign(counts, counts + G);
    uint64_t covered = 0;
    for (uint32_t i = 0; i < G; i++) covered += counts[i];
    R.ref_local = -1;
    if (covered < H) {
        R.ref_local = (int32_t)G;
        b.masks.push_back(0);
        b.carriers.push_back((uint32_t)(H - covered));
    }
    const size_t n = b.ref.size();
    const bool fits = n <= kDedupMaxWindows;
    b.helper = false;
    if (B.dedup && R.ref_local < 0 && !b.masks.empty() && fits) {
        b.masks.push_back(0);
        b.carriers.push_back(0);
        b.helper = true;
    }
    if (n >= kMaxHapLen) return fail(TFBS_E_ARG, "haplotype longer than 2^26 - 1 bases");
    R.memb_dev = memb;
    R.memb_host = false;
    R.nonref_id.clear();
    R.nonref_local.clear();
    return TFBS_OK;
}

// Device grouping for the other regions whose diff lists are masks (at most 64
// applied records, all distinct diffs, carrier lists strictly ascending below 2 *
// n_samples): the device finds the distinct masks in Vec<Diff> order, their
// carrier counts and the membership (build_gpu.hip) -- load_diffs and
// group_by_diffs over every haplotype id, the region's O(H x records) part -- and
// the host patches only the distinct groups (haplotype.rs:77-88; mask_finish),
// exactly as build_region's mask path does after its grouping.
static bool mask_prepare(const Batch &B, const RegionInput &I, std::vector<const Record *> &uniq) {
    const uint32_t H = 2 * B.n_samples;
    uniq.clear();
    for (const Record &r : I.recs) {
        if (r.n_alleles != 2 || r.carriers.empty()) continue;  // not applied (haplotype.rs:28-31)
        if (r.carriers.back() >= H) return false;
        for (size_t i = 1; i < r.carriers.size(); i++)
            if (r.carriers[i] <= r.carriers[i - 1]) return false;
        uniq.push_back(&r);
    }
    if (uniq.size() > 64) return false;
    std::stable_sort(uniq.begin(), uniq.end(), diff_less);
    for (size_t i = 1; i < uniq.size(); i++)
        if (diff_equal(uniq[i], uniq[i - 1])) return false;  // [d, d] lists: build_region's list path
    return true;
}

// The device's groups of a mask_prepare region, patched (build_region's
// load_haplotypes part: dedup by (nucs, pos), the later group wins, the loser's ids
// join the reference group), then the reference group and the helper.  The
// device's membership row (group rank per id, G for ids without a diff) is the
// distinct index as it stands unless a group lost; then the row is fetched and
// remapped here.
static int mask_finish(const Batch &B, RegionInput &I, RegionBuilt &out, const std::vector<const Record *> &uniq,
                       const uint64_t *masks, const uint32_t *counts, uint32_t G, uint64_t memb) {
    const uint32_t H = 2 * B.n_samples;
    out = RegionBuilt();
    out.R = I.R;
    RegionH &R = out.R;
    R.n_variants = (uint32_t)I.recs.size();
    inner_keys(I.inner, R);
    out.dev_grouped = true;
    std::vector<Distinct> &dist = out.dist;
    dist.reserve(G + 2);
    SeqTable table(G);
    RefWindow ref{I.ref.data(), R.es, I.ref.size()};
    std::vector<const Record *> diffs;
    for (uint32_t g = 0; g < G; g++) {
        diffs.clear();
        for (uint64_t x = masks[g]; x; x &= x - 1) diffs.push_back(uniq[__builtin_ctzll(x)]);
        Distinct d;
        d.nuc.reserve(R.ee - R.es + 16);
        if (int rc = patch_window(R.es, R.ee, diffs, ref, d.nuc, d.pos)) return rc;
        d.group = (int32_t)g;
        table.insert(dist, std::move(d), R.es);
    }
    std::vector<uint32_t> &carriers = out.carriers;
    carriers.assign(dist.size(), 0);
    uint64_t covered = 0;
    for (uint32_t i = 0; i < dist.size(); i++) {
        carriers[i] = counts[dist[i].group];
        covered += carriers[i];
    }
    const bool lost = dist.size() != G;  // a group's sequence taken by a later group
    R.ref_local = -1;
    if (covered < H) {
        Distinct d;
        d.nuc = I.ref;
        d.pos = PosRuns::affine(R.es, I.ref.size());
        d.group = -1;
        R.ref_local = (int32_t)dist.size();
        dist.push_back(std::move(d));
        carriers.push_back((uint32_t)(H - covered));
    }
    out.helper = false;
    auto fits = [](size_t n) { return n <= kDedupMaxWindows; };
    bool reusable = false;
    for (const Distinct &d : dist) reusable = reusable || fits(d.nuc.size());
    if (B.dedup && R.ref_local < 0 && reusable && fits(I.ref.size())) {
        Distinct d;
        d.nuc = I.ref;
        d.pos = PosRuns::affine(R.es, I.ref.size());
        d.group = -2;
        dist.push_back(std::move(d));
        carriers.push_back(0);
        out.helper = true;
    }
    for (const Distinct &d : dist)
        if (d.nuc.size() >= kMaxHapLen) return fail(TFBS_E_ARG, "haplotype longer than 2^26 - 1 bases");
    R.nonref_id.clear();
    R.nonref_local.clear();
    if (!lost) {  // the device row holds the distinct indices (G = ref_local for ids without a diff)
        R.memb_dev = memb;
        R.memb_host = false;
        return TFBS_OK;
    }
    R.memb_dev = 0;
    R.memb_host = true;
    if (!B.keep_membership) return TFBS_OK;
    std::vector<uint32_t> local(G + 1, (uint32_t)R.ref_local);  // group rank -> distinct index
    for (uint32_t i = 0; i < dist.size(); i++)
        if (dist[i].group >= 0) local[dist[i].group] = i;
    std::vector<uint16_t> row(H);
    if (int rc = B.grouper->fetch(memb, H, row.data())) return rc;
    for (uint32_t h = 0; h < H; h++) {
        const uint32_t v = row[h] < G ? local[row[h]] : (uint32_t)R.ref_local;
        if (v != (uint32_t)R.ref_local) {
            R.nonref_id.push_back(h);
            R.nonref_local.push_back(v);
        }
    }
    return TFBS_OK;
}

int build_regions(Batch &B, std::vector<RegionInput> &ins, uint32_t threads, std::vector<RegionBuilt> &built,
                  double *build_s) {
    const size_t n = ins.size();
    built.clear();
    built.resize(n);
    std::vector<int> rcs(n, TFBS_OK);
    std::vector<std::vector<const Record *>> uniq(n);
    std::vector<uint8_t> where(n, 0);  // 1: device grouping, 2: device overflow (host build)
    const bool dev = B.grouper && B.n_samples > 0;
    std::mutex mu;
    auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    auto par = [&](size_t count, auto fn) {
        std::atomic<size_t> next(0);
        auto work = [&]() {
            const double t0 = now();
            for (size_t j; (j = next.fetch_add(1)) < count;) fn(j);
            if (build_s) {
                std::lock_guard<std::mutex> g(mu);
                *build_s += now() - t0;
            }
        };
        std::vector<std::thread> ts;
        for (uint32_t t = 1; t < threads && t < count; t++) ts.emplace_back(work);
        work();
        for (auto &t : ts) t.join();
    };
    // TFBS_BUILD_PROF: the phases' wall seconds, summed over the calls (debug)
    static const bool prof = getenv("TFBS_BUILD_PROF") != nullptr;
    double tp[6] = {0, 0, 0, 0, 0, 0};  // prepare, staging, device grouping, finish, host fallback, (calls)
    double tq = now();
    auto lap = [&](int k) {
        if (!prof) return;
        const double t = now();
        tp[k] += t - tq;
        tq = t;
    };
    struct Report {
        const double *tp;
        ~Report() {
            static std::mutex m;
            static double acc[6];
            if (!getenv("TFBS_BUILD_PROF")) return;
            std::lock_guard<std::mutex> g(m);
            for (int k = 0; k < 5; k++) acc[k] += tp[k];
            acc[5] += 1;
            fprintf(stderr, "[build prof] calls %.0f: prepare %.3f staging %.3f grouping %.3f finish %.3f host %.3f s\n",
                    acc[5], acc[0], acc[1], acc[2], acc[3], acc[4]);
        }
    } report{tp};
    // 1: SNV-only, grouped and patched from the masks; 3: grouped on the device,
    // patched on the host (mask_finish); 2: device overflow -> build_region
    par(n, [&](size_t j) {
        if (dev && snv_prepare(B, ins[j], built[j], uniq[j])) {
            where[j] = 1;
            return;
        }
        if (dev && B.dev_patch && mask_prepare(B, ins[j], uniq[j])) {
            where[j] = 3;
            return;
        }
        rcs[j] = build_region(B, std::move(ins[j]), built[j]);
    });
    if (dev) {
        std::vector<size_t> dj;
        for (size_t j = 0; j < n; j++)
            if (where[j] == 1 || where[j] == 3) dj.push_back(j);
        const uint32_t H = 2 * B.n_samples;
        // chunks: the masks scratch (8 bytes per haplotype id and region) within 1 GiB
        const size_t max_regions = std::max<size_t>(1, std::min<size_t>(1024, (1ull << 30) / (8ull * H)));
        for (size_t c0 = 0; c0 < dj.size();) {
            size_t c1 = c0;
            uint64_t ncar = 0;
            while (c1 < dj.size() && c1 - c0 < max_regions) {
                uint64_t m = 0;
                for (const Record *r : uniq[dj[c1]]) m += r->carriers.size();
                if (c1 > c0 && ncar + m > (1ull << 30)) break;
                ncar += m;
                c1++;
            }
            std::vector<GrpRecord> recs;
            std::vector<GrpRegion> regs;
            std::vector<uint32_t> rec0(c1 - c0);
            uint32_t off = 0;
            for (size_t k = c0; k < c1; k++) {
                const auto &u = uniq[dj[k]];
                rec0[k - c0] = (uint32_t)recs.size();
                regs.push_back({(uint32_t)recs.size(), (uint32_t)u.size()});
                for (uint32_t q = 0; q < u.size(); q++) {
                    recs.push_back({off, (uint32_t)u[q]->carriers.size(), q, (uint32_t)(k - c0)});
                    off += (uint32_t)u[q]->carriers.size();
                }
            }
            lap(0);
            uint32_t *car = B.grouper->carriers(ncar);
            if (!car) return fail(TFBS_E_NOMEM, "device grouping staging");
            par(c1 - c0, [&](size_t k) {
                const auto &u = uniq[dj[c0 + k]];
                for (uint32_t q = 0; q < u.size(); q++) {
                    const GrpRecord &g = recs[rec0[k] + q];
                    memcpy(car + g.off, u[q]->carriers.data(), (size_t)g.n * 4);
                }
            });
            lap(1);
            GroupOut go;
            if (int rc = B.grouper->group(ncar, recs, regs, H, go)) return rc;
            lap(2);
            if (go.memb_alloc) B.memb_allocs.push_back(go.memb_alloc);
            par(c1 - c0, [&](size_t c) {
                const size_t j = dj[c0 + c];
                if (go.n_groups[c] == UINT32_MAX) {
                    where[j] = 2;
                    return;
                }
                if (where[j] == 1)
                    rcs[j] = snv_finish(B, built[j], go.masks.data() + go.first[c], go.counts.data() + go.first[c],
                                        go.n_groups[c], go.memb[c]);
                else
                    rcs[j] = mask_finish(B, ins[j], built[j], uniq[j], go.masks.data() + go.first[c],
                                         go.counts.data() + go.first[c], go.n_groups[c], go.memb[c]);
            });
            c0 = c1;
            lap(3);
        }
        std::vector<size_t> hj;
        for (size_t j = 0; j < n; j++)
            if (where[j] == 2) hj.push_back(j);
        par(hj.size(), [&](size_t k) {
            const size_t j = hj[k];
            built[j] = RegionBuilt();
            rcs[j] = build_region(B, std::move(ins[j]), built[j]);
        });
        lap(4);
    }
    for (size_t j = 0; j < n; j++) {
        if (rcs[j]) return rcs[j];
        if (built[j].dev || built[j].dev_grouped) B.dev_regions++;
        else B.host_regions++;
        if (built[j].dev_grouped) B.patched_regions++;
    }
    return TFBS_OK;
}

int region_membership(const Batch &B, const RegionH &R) {
    if (R.memb_host) return TFBS_OK;
    if (!B.grouper) return fail(TFBS_E_STATE, "membership on a device without its grouper");
    const uint32_t H = 2 * B.n_samples;
    std::vector<uint16_t> row(H);
    if (int rc = B.grouper->fetch(R.memb_dev, H, row.data())) return rc;
    R.nonref_id.clear();
    R.nonref_local.clear();
    const uint32_t ref = R.ref_local < 0 ? UINT32_MAX : (uint32_t)R.ref_local;
    for (uint32_t h = 0; h < H; h++)
        if (row[h] != ref) {
            R.nonref_id.push_back(h);
            R.nonref_local.push_back(row[h]);
        }
    R.memb_host = true;
    return TFBS_OK;
}

// Appends built regions to the batch in order: packs their haplotypes for the
// GPU.  Offsets are laid out serially (prefix sums over the regions'
// haplotypes), the packing of bases, N masks and positions runs on `threads`
// threads.
// The windows [0, nw) of a HAP_DEDUP haplotype with diff runs `runs` that a depth
// class of span S reads: those meeting a run (tfbs_internal.hpp run_meets).
static uint64_t dirty_windows(const uint32_t *runs, size_t nruns, uint32_t S, uint32_t nw) {
    uint64_t n = 0, next = 0;  // windows below `next` are counted
    for (size_t k = 0; k < nruns; k += 2) {
        const uint64_t lo = std::max<uint64_t>(next, runs[k] >= S - 1 ? runs[k] - (S - 1) : 0);
        const uint64_t hi = std::min<uint64_t>(runs[k + 1], nw - 1);  // inclusive
        if (hi + 1 > lo) {
            n += hi + 1 - lo;
            next = hi + 1;
        }
    }
    return n;
}

// 16 base codes (0-3; N = 4 as 0) as one packed word, 2 bits each, base 0 lowest
static inline uint32_t pack16(const uint8_t *p) {
    auto half = [](uint64_t x) {
        x &= 0x0303030303030303ull;
        x = (x | (x >> 6)) & 0x000F000F000F000Full;
        x = (x | (x >> 12)) & 0x000000FF000000FFull;
        x = (x | (x >> 24)) & 0xFFFFull;
        return (uint32_t)x;
    };
    uint64_t lo, hi;
    memcpy(&lo, p, 8);
    memcpy(&hi, p + 8, 8);
    return half(lo) | (half(hi) << 16);
}

void commit_regions(Batch &B, std::vector<RegionBuilt> &built, uint32_t threads) {
    const size_t nr = built.size();
    if (!nr) return;
    // per haplotype: length, has N, affine positions (parallel scan of the sequences)
    struct HapInfo {
        uint32_t n;
        bool has_n, affine, dedup = false;
        uint32_t r0 = 0, rn = 0;  // HAP_DEDUP: its diff runs (a, b), ascending, merged: rruns[j][r0 .. r0 + rn)
        // and the same in the reference's columns (rruns[j][q0 .. q0 + qn)), q0 = r0 when
        // both are the same list (every column at its reference column: no indel)
        uint32_t q0 = 0, qn = 0;
        bool rsep = false;  // the reference-column runs are a list of their own (an indel haplotype)
    };
    std::vector<std::vector<HapInfo>> info(nr);
    std::vector<std::vector<uint32_t>> rruns(nr);  // per region, its haplotypes' diff runs
    auto par = [&](auto fn) {
        std::atomic<size_t> next(0);
        auto work = [&]() {
            for (size_t j; (j = next.fetch_add(1)) < nr;) fn(j);
        };
        std::vector<std::thread> ts;
        for (uint32_t t = 1; t < threads && t < nr; t++) ts.emplace_back(work);
        work();
        for (auto &t : ts) t.join();
    };
    par([&](size_t j) {
        const RegionBuilt &rb = built[j];
        info[j].resize(rb.n_haps());
        if (rb.dev) {  // the reference window with SNVs: its length, no N, affine positions
            for (HapInfo &h : info[j]) {
                h.n = (uint32_t)rb.ref.size();
                h.has_n = false;
                h.affine = true;
            }
        }
        for (size_t i = 0; i < rb.dist.size(); i++) {
            const Distinct &d = rb.dist[i];
            HapInfo &h = info[j][i];
            h.n = (uint32_t)d.nuc.size();
            h.has_n = h.n && memchr(d.nuc.data(), 4, h.n) != nullptr;
            h.affine = d.pos.is_affine(rb.R.es);
        }
        // reference-window reuse: a window whose bases equal those of the reference
        // window that starts at its first base's position has that window's score and
        // match range (pattern.rs:151-156: the range is [pos_i, pos_i + L - 1]), so its
        // hit (or none) is the reference's.  A haplotype's *segments* are maximal runs of
        // columns equal to the reference column at their position with consecutive
        // positions (one shift each: 0 before an indel, the indel's length after it),
        // their reference ranges ascending and disjoint; a window inside one segment is
        // the reference window shifted by the segment's shift.  The columns outside the
        // segments form the haplotype's diff runs (in its own columns: the windows the
        // scan reads, tfbs_internal.hpp), those outside the segments' reference ranges
        // the same runs in the reference's columns (the reference hits the key assembly
        // passes on); two segments that touch get a boundary run (a, a - 1), which meets
        // exactly the windows spanning both.  Haplotypes and reference of up to
        // kDedupMaxWindows bases, at most kMaxDiffRuns runs of either kind.
        const int32_t ref = rb.R.ref_local >= 0 ? rb.R.ref_local : (rb.helper ? (int32_t)rb.n_haps() - 1 : -1);
        if (!B.dedup || ref < 0) return;
        std::vector<uint32_t> &rv = rruns[j];
        auto add = [&](uint32_t r0, uint32_t p, uint32_t e) {  // columns p .. e (e = p - 1: a boundary), ascending
            if (rv.size() > r0 && (rv.back() == kRunToEnd || rv.back() + 1 >= p)) {
                rv.back() = std::max(rv.back(), e);
            } else {
                rv.push_back(p);
                rv.push_back(e);
            }
        };
        if (rb.dev) {  // every haplotype has the reference's length: its SNV columns differ
            if (rb.ref.size() > kDedupMaxWindows) return;
            for (size_t i = 0; i < rb.masks.size(); i++) {
                if ((int32_t)i == ref) continue;
                HapInfo &h = info[j][i];
                h.r0 = h.q0 = (uint32_t)rv.size();
                for (uint64_t x = rb.masks[i]; x; x &= x - 1) {
                    const uint32_t p = rb.snv_rel[__builtin_ctzll(x)];
                    add(h.r0, p, p);
                }
                h.rn = h.qn = (uint32_t)rv.size() - h.r0;
                h.dedup = h.rn / 2 <= kMaxDiffRuns;
                if (!h.dedup) rv.resize(h.r0), h.rn = h.qn = 0;
            }
            return;
        }
        const std::vector<uint8_t> &rn = rb.dist[ref].nuc;
        const uint32_t m = (uint32_t)rn.size();
        if (m > kDedupMaxWindows) return;
        struct Seg {
            uint32_t a, b, qa;  // columns [a, b) at reference columns [qa, qa + b - a)
        };
        std::vector<Seg> segs;
        std::vector<uint64_t> dpos;  // the haplotype's positions, expanded from its runs
        for (size_t i = 0; i < rb.dist.size(); i++) {
            HapInfo &h = info[j][i];
            if ((int32_t)i == ref || h.n > kDedupMaxWindows) continue;
            const Distinct &d = rb.dist[i];
            dpos.resize(h.n);
            d.pos.expand(dpos.data(), [](uint64_t p) { return p; });
            segs.clear();
            uint32_t qend = 0;  // the last segment's reference end (exclusive)
            bool open = false;
            for (uint32_t p = 0; p < h.n; p++) {
                if (open) {  // 8 columns at a time while the segment goes on (consecutive
                    // positions, bases equal to the reference's at them)
                    for (;;) {
                        const uint64_t at = dpos[p - 1] + 1, qq = at - rb.R.es;
                        if (p + 8 > h.n || qq + 8 > m) break;
                        uint64_t x, y, off = 0;
                        memcpy(&x, d.nuc.data() + p, 8);
                        memcpy(&y, rn.data() + qq, 8);
                        for (uint32_t k = 0; k < 8; k++) off |= dpos[p + k] ^ (at + k);
                        if (x != y || off) break;
                        p += 8;
                    }
                    if (p >= h.n) break;
                }
                const int64_t q = (int64_t)dpos[p] - (int64_t)rb.R.es;
                const bool ok = q >= 0 && q < (int64_t)m && d.nuc[p] == rn[(size_t)q];
                if (open && ok && dpos[p] == dpos[p - 1] + 1) continue;  // the segment goes on
                if (open) {
                    segs.back().b = p;
                    qend = segs.back().qa + (p - segs.back().a);
                    open = false;
                }
                if (ok && (segs.empty() || (uint32_t)q >= qend)) {
                    segs.push_back({p, h.n, (uint32_t)q});
                    open = true;
                }
            }
            // the haplotype's own columns: outside the segments, and where two touch
            h.r0 = (uint32_t)rv.size();
            uint32_t at = 0;
            for (size_t k = 0; k < segs.size(); k++) {
                if (segs[k].a > at) add(h.r0, at, segs[k].a - 1);
                else if (k) add(h.r0, at, at - 1);
                at = segs[k].b;
            }
            if (at < h.n || segs.empty()) add(h.r0, at, kRunToEnd);
            h.rn = (uint32_t)rv.size() - h.r0;
            bool shifted = false;  // some segment off its own column: a separate reference-column list
            for (const Seg &g : segs) shifted = shifted || g.qa != g.a;
            if (h.n != m) shifted = true;
            if (!shifted) {
                h.q0 = h.r0;
                h.qn = h.rn;
            } else {  // the reference's columns: outside the segments' ranges, and where two touch
                h.rsep = true;  // (q0 == r0 when the haplotype's own list is empty: the flag tells)
                h.q0 = (uint32_t)rv.size();
                uint32_t qa = 0;
                for (size_t k = 0; k < segs.size(); k++) {
                    if (segs[k].qa > qa) add(h.q0, qa, segs[k].qa - 1);
                    else if (k) add(h.q0, qa, qa - 1);
                    qa = segs[k].qa + (segs[k].b - segs[k].a);
                }
                if (qa < m || segs.empty()) add(h.q0, qa, kRunToEnd);
                h.qn = (uint32_t)rv.size() - h.q0;
            }
            h.dedup = h.rn / 2 <= kMaxDiffRuns && h.qn / 2 <= kMaxDiffRuns;
            if (!h.dedup) {
                rv.resize(h.r0);
                h.rn = h.qn = 0;
                h.rsep = false;
            }
        }
    });
    // serial layout: region / haplotype / word / mask / position offsets
    struct Off {
        size_t hap, inner;
        uint64_t word, nmask, pos, count, runs;
    };
    std::vector<Off> off(nr);
    Off cur{B.haps.size(), B.inner.size(), B.words.size(), B.nmask.size(), B.posrel.size(), B.n_counts,
            B.druns.size()};
    for (size_t j = 0; j < nr; j++) {
        off[j] = cur;
        const uint32_t n_inner = (uint32_t)built[j].R.ranges.size();
        cur.hap += built[j].n_haps();
        cur.inner += 2 * n_inner;
        for (const HapInfo &h : info[j]) {
            cur.word += (h.n + 15) / 16 + 3;
            if (h.has_n) cur.nmask += (h.n + 31) / 32 + 2;
            if (!h.affine) cur.pos += h.n;
            cur.count += (uint64_t)B.n_slots * n_inner;
            cur.runs += h.rn + (h.rsep ? h.qn : 0);
        }
    }
    const uint32_t region0 = (uint32_t)B.rh.size();
    B.haps.resize(cur.hap);
    B.hap_carriers.resize(cur.hap);
    B.inner.resize(cur.inner);
    B.words.resize(cur.word);  // (uninitialised: every word is written below, pads and tails zeroed)
    B.nmask.resize(cur.nmask);  // (the same)
    B.posrel.resize(cur.pos);
    B.druns.resize(cur.runs);
    B.regions.resize(region0 + nr);
    B.n_counts = cur.count;
    std::vector<uint64_t> win(nr, 0), eff(nr, 0), cells(nr, 0), swin(nr, 0), scells(nr, 0);
    // the window lists' span per depth class: its longest strand (build_window_lists)
    uint32_t class_lmax[2] = {0, 0};
    for (const auto &lc : B.pwm_len_hist)
        if (lc.first <= (uint32_t)(kMMaxChunks * kMChunkCols)) {
            uint32_t &m = class_lmax[mfma_depth_class((lc.first + kMChunkCols - 1) / kMChunkCols) > 2];
            m = std::max(m, lc.first);
        }
    par([&](size_t j) {
        RegionBuilt &rb = built[j];
        RegionH &R = rb.R;
        const Off &o = off[j];
        R.hap_begin = (uint32_t)o.hap;
        R.hap_count = (uint32_t)rb.n_haps() - (rb.helper ? 1 : 0);
        const int32_t ref = R.ref_local >= 0 ? R.ref_local : (rb.helper ? (int32_t)R.hap_count : -1);
        DevRegion dr{};
        dr.inner_off = (uint32_t)(o.inner / 2);
        dr.n_inner = (uint32_t)R.ranges.size();
        dr.hap_begin = R.hap_begin;
        dr.hap_count = R.hap_count;
        // the reference's hits are listed only when some haplotype reuses them
        bool reused = false;
        for (const HapInfo &h : info[j]) reused = reused || h.dedup;
        dr.ref_hap = ref >= 0 && B.dedup && reused ? R.hap_begin + (uint32_t)ref : UINT32_MAX;
        dr.count_stride = (uint32_t)rb.n_haps();
        R.key_off = (uint64_t)dr.inner_off * B.n_slots;
        size_t ii = o.inner;
        for (auto &r : R.ranges) {
            // positions relative to ext_start, clamped: only containment of small
            // non-negative positions is ever tested, which clamping preserves.
            auto rel = [&](uint64_t x) -> int32_t {
                if (x < R.es) { uint64_t d = R.es - x; return d > (1u << 30) ? -(1 << 30) : -(int32_t)d; }
                uint64_t d = x - R.es;
                return d > (1u << 30) ? (1 << 30) : (int32_t)d;
            };
            B.inner[ii++] = rel(r.first);
            B.inner[ii++] = rel(r.second);
        }
        B.regions[region0 + j] = dr;
        uint64_t word = o.word, nmask = o.nmask, pos = o.pos, count = o.count, runs = o.runs;
        // per-region sums in registers (the arrays are shared by the threads)
        uint64_t r_win = 0, r_eff = 0, r_cells = 0, r_swin = 0, r_scells = 0;
        std::vector<uint32_t> refw;  // device-grouped: the reference window packed once
        if (rb.dev) {
            refw.assign((rb.ref.size() + 15) / 16, 0u);
            for (size_t p = 0; p < rb.ref.size(); p++) refw[p / 16] |= (uint32_t)rb.ref[p] << (2 * (p % 16));
        }
        for (uint32_t i = 0; i < rb.n_haps(); i++) {
            const HapInfo &h = info[j][i];
            const uint32_t n = h.n;
            DevHap hm{};
            hm.word_off = (uint32_t)word;
            hm.len = n;
            hm.region = region0 + (uint32_t)j;
            uint32_t *w = B.words.data() + word;
            std::fill(w + n / 16, w + (n + 15) / 16 + 3, 0u);  // the partial last word and the 3 pads
            if (rb.dev) {  // the reference's words, the SNVs' bases written over
                std::copy(refw.begin(), refw.end(), w);
                for (uint64_t x = rb.masks[i]; x; x &= x - 1) {
                    const uint32_t k = __builtin_ctzll(x), p = rb.snv_rel[k];
                    w[p / 16] = (w[p / 16] & ~(3u << (2 * (p % 16)))) | ((uint32_t)rb.snv_alt[k] << (2 * (p % 16)));
                }
            } else {
                const Distinct &d = rb.dist[i];
                uint32_t p = 0;  // N (4) packs as A (masked by the N bits): the low two bits
                for (; p + 16 <= n; p += 16) w[p / 16] = pack16(d.nuc.data() + p);
                for (; p < n; p++) w[p / 16] |= (uint32_t)(d.nuc[p] & 3u) << (2 * (p % 16));
            }
            word += (n + 15) / 16 + 3;
            if (h.has_n) {
                const Distinct &d = rb.dist[i];
                hm.flags |= HAP_HAS_N;
                hm.nmask_off = (uint32_t)nmask;
                uint32_t *m = B.nmask.data() + nmask;
                std::fill(m, m + (n + 31) / 32 + 2, 0u);
                for (uint32_t p = 0; p < n; p++)
                    if (d.nuc[p] == 4) m[p / 32] |= 1u << (p % 32);
                nmask += (n + 31) / 32 + 2;
            }
            if (!h.affine) {
                const Distinct &d = rb.dist[i];
                hm.flags |= HAP_HAS_POS;
                hm.pos_off = (uint32_t)pos;
                const uint64_t es = R.es;
                d.pos.expand(B.posrel.data() + pos, [es](uint64_t p) { return (int32_t)(p - es); });
                pos += n;
            }
            hm.count_off = count + i;  // key-major: [key][haplotype]
            if (dr.ref_hap == o.hap + i) hm.flags |= HAP_REF;
            if (h.dedup) {
                hm.flags |= HAP_DEDUP;
                hm.drun_off = (uint32_t)(runs / 2);
                hm.n_druns = h.rn / 2;
                std::copy(rruns[j].begin() + h.r0, rruns[j].begin() + h.r0 + h.rn, B.druns.begin() + runs);
                runs += h.rn;
                hm.rrun_off = hm.drun_off;
                hm.n_rruns = h.qn / 2;
                if (h.rsep) {  // (an indel haplotype) its runs in the reference's columns follow
                    hm.rrun_off = (uint32_t)(runs / 2);
                    std::copy(rruns[j].begin() + h.q0, rruns[j].begin() + h.q0 + h.qn, B.druns.begin() + runs);
                    runs += h.qn;
                }
            }
            B.haps[o.hap + i] = hm;
            B.hap_carriers[o.hap + i] = rb.carriers[i];
            const bool helper = rb.helper && i + 1 == rb.n_haps();
            uint64_t wn = 0;
            for (const auto &lc : B.pwm_len_hist)
                if (n >= lc.first) {
                    const uint64_t nw = n - lc.first + 1;
                    uint64_t sw = nw;  // windows the scan reads
                    if (h.dedup && lc.first <= (uint32_t)(kMMaxChunks * kMChunkCols)) {
                        const uint32_t span = class_lmax[mfma_depth_class((lc.first + kMChunkCols - 1) / kMChunkCols) > 2];
                        sw = dirty_windows(rruns[j].data() + h.r0, h.rn, span, (uint32_t)nw);
                    }
                    r_swin += sw * lc.second;
                    r_scells += sw * lc.first * lc.second;
                    if (helper) continue;
                    wn += nw * lc.second;
                    r_cells += nw * lc.first * lc.second;
                }
            r_win += wn;
            r_eff += wn * rb.carriers[i];
        }
        win[j] = r_win;
        eff[j] = r_eff;
        cells[j] = r_cells;
        swin[j] = r_swin;
        scells[j] = r_scells;
    });
    for (size_t j = 0; j < nr; j++) {
        B.windows += win[j];
        B.eff_windows += eff[j];
        B.cell_ops += cells[j];
        B.scan_windows += swin[j];
        B.scan_cell_ops += scells[j];
        B.rh.push_back(std::move(built[j].R));
    }
}

void reserve_batch(Batch &B, double factor) {
    auto grow = [factor](auto &v) {
        const size_t want = (size_t)((double)v.size() * factor) + 16;
        if (want > v.capacity()) v.reserve(want);
    };
    grow(B.words);
    grow(B.nmask);
    grow(B.posrel);
    grow(B.druns);
    grow(B.haps);
    grow(B.hap_carriers);
    grow(B.regions);
    grow(B.inner);
    grow(B.rh);
}

void commit_region(Batch &B, RegionBuilt &&built) {
    std::vector<RegionBuilt> one(1);
    one[0] = std::move(built);
    commit_regions(B, one, 1);
}

}  // namespace tfbs

using tfbs::Batch;

extern "C" {

int tfbs_batch_create(const tfbs_patterns *p, uint32_t n_samples, int keep_membership, tfbs_batch **out) {
    if (!p || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    const tfbs::Patterns &P = tfbs::patterns_of(p);
    if (P.pats.empty()) return tfbs::fail(TFBS_E_NOPATTERN, "no pattern");  // main.rs:238
    if ((uint64_t)n_samples * 2 > 0xFFFFFFF0ull) return tfbs::fail(TFBS_E_ARG, "too many samples");
    std::vector<uint16_t> slot_pid;
    bool zero_len_panics = false;
    int rc = P.slot_order(slot_pid, zero_len_panics);
    if (rc) return rc;
    if (zero_len_panics)
        return tfbs::fail(TFBS_E_ZEROLEN, "length-0 PWM with negative min_score (pattern.rs:150-156)");
    auto *b = new tfbs_batch();
    Batch &B = b->b;
    B.pats = &P;
    B.n_samples = n_samples;
    B.keep_membership = keep_membership != 0;
    {
        const char *v = getenv("TFBS_DEDUP");
        B.dedup = !(v && *v && atoi(v) == 0);
        const char *w = getenv("TFBS_DEV_PATCH");  // 0: only SNV-only regions are grouped on the device
        B.dev_patch = !(w && *w && atoi(w) == 0);
    }
    B.slot_pid = std::move(slot_pid);
    B.slots_by_pid.resize(B.slot_pid.size());
    std::iota(B.slots_by_pid.begin(), B.slots_by_pid.end(), 0u);
    std::sort(B.slots_by_pid.begin(), B.slots_by_pid.end(),
              [&](uint32_t a, uint32_t b) { return B.slot_pid[a] < B.slot_pid[b]; });
    B.n_slots = (uint32_t)B.slot_pid.size();
    std::map<uint32_t, uint32_t> lens;
    for (auto &q : P.pats)
        if (q.kind == TFBS_KIND_PWM && q.len > 0) lens[q.len]++;
    B.pwm_len_hist.assign(lens.begin(), lens.end());
    *out = b;
    return TFBS_OK;
}

void tfbs_batch_destroy(tfbs_batch *b) {
    if (b) tfbs::forget_var_counts(b->b);
    delete b;
}

int tfbs_batch_add_bed(tfbs_batch *b, const char *basename) {
    if (!b || !basename) return tfbs::fail(TFBS_E_ARG, "null argument");
    b->b.beds.push_back(basename);
    return (int)b->b.beds.size() - 1;
}

int tfbs_batch_set_window_lmax(tfbs_batch *b, uint32_t lmax) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (lmax < b->b.pats->max_length()) return tfbs::fail(TFBS_E_ARG, "window L_max below the longest pattern");
    if (!b->b.rh.empty() || b->b.open) return tfbs::fail(TFBS_E_STATE, "regions already added");
    b->b.window_lmax = lmax;
    return TFBS_OK;
}

int tfbs_batch_set_build_device(tfbs_batch *b, int device) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    Batch &B = b->b;
    if (!B.rh.empty() || B.open) return tfbs::fail(TFBS_E_STATE, "regions already added");
    B.grouper.reset();
    if (device < 0) return TFBS_OK;
    tfbs::DevGrouper *g = tfbs::make_gpu_grouper(device);
    if (!g) return TFBS_E_NODEVICE;
    B.grouper.reset(g);
    return TFBS_OK;
}

int tfbs_batch_build_stats(const tfbs_batch *b, uint64_t *dev_regions, uint64_t *host_regions) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (dev_regions) *dev_regions = b->b.dev_regions;
    if (host_regions) *host_regions = b->b.host_regions;
    return TFBS_OK;
}

int tfbs_batch_patch_stats(const tfbs_batch *b, uint64_t *patched_regions) {
    if (!b) return tfbs::fail(TFBS_E_ARG, "null argument");
    if (patched_regions) *patched_regions = b->b.patched_regions;
    return TFBS_OK;
}

int tfbs_batch_region_ext(const tfbs_batch *b, uint64_t ms, uint64_t me, uint64_t *es, uint64_t *ee) {
    if (!b || !es || !ee) return tfbs::fail(TFBS_E_ARG, "null argument");
    uint64_t L = b->b.lmax();
    if (ms + 1 < L) return tfbs::fail(TFBS_E_RANGE, "region start closer than the PWM length to 0 (main.rs:407)");
    *es = ms + 1 - L;  // u64 wrapping as in --release (L = 0 gives [s+1, e-1])
    *ee = me + L - 1;
    return TFBS_OK;
}

int tfbs_batch_region_begin(tfbs_batch *b, uint64_t ms, uint64_t me, const char *ref_ascii, size_t n_ref) {
    if (!b || (n_ref && !ref_ascii)) return tfbs::fail(TFBS_E_ARG, "null argument");
    Batch &B = b->b;
    if (B.open) return tfbs::fail(TFBS_E_STATE, "region already open");
    B.cur = tfbs::RegionH();
    B.cur_rec.clear();
    B.cur_inner.clear();
    B.status = TFBS_OK;
    B.cur.ms = ms;
    B.cur.me = me;
    int rc = tfbs_batch_region_ext(b, ms, me, &B.cur.es, &B.cur.ee);
    if (rc) return rc;
    B.cur_ref.resize(n_ref);
    for (size_t i = 0; i < n_ref; i++) {
        int c = tfbs::to_nuc((uint8_t)ref_ascii[i]);
        if (c < 0) return tfbs::fail(TFBS_E_BADBASE, std::string("Unknown nucleotide ") + std::to_string((int)(uint8_t)ref_ascii[i]));
        B.cur_ref[i] = (uint8_t)c;
    }
    B.open = true;
    return TFBS_OK;
}

int tfbs_batch_region_add_inner(tfbs_batch *b, uint32_t bed, uint64_t s, uint64_t e) {
    if (!b || !b->b.open) return tfbs::fail(TFBS_E_STATE, "no open region");
    if (bed >= b->b.beds.size()) return tfbs::fail(TFBS_E_ARG, "unknown bed index");
    b->b.cur_inner.push_back({bed, {s, e}});
    return TFBS_OK;
}

static int to_codes(const char *s, std::vector<uint8_t> &out) {
    out.clear();
    for (const char *p = s; *p; p++) {
        int c = tfbs::to_nuc((uint8_t)*p);
        if (c < 0) return tfbs::fail(TFBS_E_BADBASE, std::string("Unknown nucleotide ") + std::to_string((int)(uint8_t)*p));
        out.push_back((uint8_t)c);
    }
    return TFBS_OK;
}

}  // extern "C"

namespace tfbs {
// haplotype.rs:16-60 for one record: alleles[0]/[1] decode (may panic on a bad
// base even for multi-allelic records, line 20-22); for bi-allelic records the
// ploidy assert (line 32) and Left = Unphased(1) = raw 4, Right = Phased(1) = raw 5.
int make_record_gt(uint32_t n_samples, uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                   const int32_t *gt, Record &r) {
    if (n_alleles < 2 || !alt) return fail(TFBS_E_ALLELES, "record with one allele (haplotype.rs:22)");
    if (!ref || (n_alleles == 2 && n_samples && !gt)) return fail(TFBS_E_ARG, "null argument");
    r = Record();
    r.pos = pos;
    r.n_alleles = n_alleles;
    int rc = to_codes(ref, r.ref);
    if (!rc) rc = to_codes(alt, r.alt);
    if (rc) return rc;
    if (n_alleles == 2) {
        const int32_t VE = INT32_MIN + 1;
        for (uint32_t s = 0; s < n_samples; s++) {
            const int32_t g0 = gt[2 * s], g1 = gt[2 * s + 1];
            const uint32_t glen = g0 == VE ? 0 : (g1 == VE ? 1 : 2);
            if (glen != n_alleles) return fail(TFBS_E_PLOIDY, "Inconsistent number of alleles");
            if (g0 == 4) r.carriers.push_back(2 * s);      // GenotypeAllele::Unphased(1)
            if (g1 == 5) r.carriers.push_back(2 * s + 1);  // GenotypeAllele::Phased(1)
        }
    }
    return TFBS_OK;
}

template <class V>
static int record_ids(uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt, V &&carriers, int gt_status,
                      Record &r) {
    if (n_alleles < 2 || !alt) return fail(TFBS_E_ALLELES, "record with one allele (haplotype.rs:22)");
    if (!ref) return fail(TFBS_E_ARG, "null argument");
    r = Record();
    r.pos = pos;
    r.n_alleles = n_alleles;
    int rc = to_codes(ref, r.ref);
    if (!rc) rc = to_codes(alt, r.alt);
    if (rc) return rc;
    if (n_alleles == 2) {
        if (gt_status) return fail(gt_status, "Inconsistent number of alleles");
        r.carriers = std::forward<V>(carriers);
    }
    return TFBS_OK;
}
int make_record_ids(uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                    const std::vector<uint32_t> &carriers, int gt_status, Record &r) {
    return record_ids(pos, n_alleles, ref, alt, carriers, gt_status, r);
}
int make_record_ids(uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                    std::vector<uint32_t> &&carriers, int gt_status, Record &r) {
    return record_ids(pos, n_alleles, ref, alt, std::move(carriers), gt_status, r);
}

// Builds regions on up to `threads` host threads, commits them in order.
int add_regions(Batch &B, std::vector<RegionInput> &ins, uint32_t threads) {
    std::vector<RegionBuilt> built;
    B.counts_valid = B.reduced = false;
    if (int rc = build_regions(B, ins, threads, built, nullptr)) return rc;
    commit_regions(B, built, threads);
    return TFBS_OK;
}
}  // namespace tfbs

extern "C" {

int tfbs_batch_region_add_record_gt(tfbs_batch *b, uint64_t pos, uint32_t n_alleles, const char *ref, const char *alt,
                                    const int32_t *gt) {
    if (!b || !b->b.open) return tfbs::fail(TFBS_E_STATE, "no open region");
    Batch &B = b->b;
    if (B.status) return B.status;
    tfbs::Record r;
    int rc = tfbs::make_record_gt(B.n_samples, pos, n_alleles, ref, alt, gt, r);
    if (rc) return B.status = rc;
    B.cur_rec.push_back(std::move(r));
    return TFBS_OK;
}

int tfbs_batch_region_add_record_carriers(tfbs_batch *b, uint64_t pos, const char *ref, const char *alt,
                                          const uint32_t *ids, size_t n) {
    if (!b || !b->b.open) return tfbs::fail(TFBS_E_STATE, "no open region");
    Batch &B = b->b;
    if (B.status) return B.status;
    if (!ref || !alt || (n && !ids)) return tfbs::fail(TFBS_E_ARG, "null argument");
    tfbs::Record r;
    r.pos = pos;
    int rc = to_codes(ref, r.ref);
    if (!rc) rc = to_codes(alt, r.alt);
    if (rc) return B.status = rc;
    r.carriers.assign(ids, ids + n);
    B.cur_rec.push_back(std::move(r));
    return TFBS_OK;
}

int tfbs_batch_region_end(tfbs_batch *b) {
    if (!b || !b->b.open) return tfbs::fail(TFBS_E_STATE, "no open region");
    Batch &B = b->b;
    B.open = false;
    if (B.status) return B.status;
    B.counts_valid = B.reduced = false;
    tfbs::RegionInput in;
    in.R = std::move(B.cur);
    in.ref = std::move(B.cur_ref);
    in.recs = std::move(B.cur_rec);
    in.inner = std::move(B.cur_inner);
    B.cur_rec.clear();
    B.cur_inner.clear();
    std::vector<tfbs::RegionInput> ins(1);
    ins[0] = std::move(in);
    return tfbs::add_regions(B, ins, 1);
}

size_t tfbs_batch_num_regions(const tfbs_batch *b) { return b ? b->b.rh.size() : 0; }
size_t tfbs_batch_num_haplotypes(const tfbs_batch *b) {  // helper reference copies excluded
    if (!b) return 0;
    size_t n = 0;
    for (const auto &R : b->b.rh) n += R.hap_count;
    return n;
}
uint64_t tfbs_batch_num_windows(const tfbs_batch *b) { return b ? b->b.windows : 0; }
uint64_t tfbs_batch_num_effective_windows(const tfbs_batch *b) { return b ? b->b.eff_windows : 0; }
uint64_t tfbs_batch_num_cell_ops(const tfbs_batch *b) { return b ? b->b.cell_ops : 0; }
uint64_t tfbs_batch_num_scan_windows(const tfbs_batch *b) { return b ? b->b.scan_windows : 0; }
uint64_t tfbs_batch_num_scan_cell_ops(const tfbs_batch *b) { return b ? b->b.scan_cell_ops : 0; }
uint64_t tfbs_batch_input_bytes(const tfbs_batch *b) { return b ? b->b.device_bytes() : 0; }
uint64_t tfbs_batch_output_bytes(const tfbs_batch *b) { return b ? b->b.n_counts * 4ull : 0; }

int tfbs_batch_region_stats(const tfbs_batch *b, size_t region, uint32_t *nh, uint32_t *nv) {
    if (!b || region >= b->b.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    if (nh) *nh = b->b.rh[region].hap_count;
    if (nv) *nv = b->b.rh[region].n_variants;
    return TFBS_OK;
}

int tfbs_patch_haplotype(uint64_t rs, uint64_t re, size_t nd, const uint64_t *dpos, const uint8_t *dref,
                         const uint32_t *dnref, const uint8_t *dalt, const uint32_t *dnalt, const uint8_t *ref_nucs,
                         const uint64_t *ref_pos, size_t n_ref, uint8_t *out_nucs, uint64_t *out_pos, size_t cap,
                         size_t *n_out) {
    if (!n_out || (nd && (!dpos || !dnref || !dnalt)) || (n_ref && (!ref_nucs || !ref_pos)))
        return tfbs::fail(TFBS_E_ARG, "null argument");
    std::vector<tfbs::Record> recs(nd);
    size_t ro = 0, ao = 0;
    for (size_t i = 0; i < nd; i++) {
        recs[i].pos = dpos[i];
        recs[i].ref.assign(dref + ro, dref + ro + dnref[i]);
        recs[i].alt.assign(dalt + ao, dalt + ao + dnalt[i]);
        ro += dnref[i];
        ao += dnalt[i];
    }
    std::vector<const tfbs::Record *> ptrs;
    for (auto &r : recs) ptrs.push_back(&r);
    std::vector<uint8_t> nuc;
    std::vector<uint64_t> pos;
    int rc;
    bool consecutive = true;
    for (size_t i = 1; i < n_ref; i++)
        if (ref_pos[i] != ref_pos[0] + i) consecutive = false;
    if (consecutive) {
        rc = tfbs::patch(rs, re, ptrs, ref_nucs, n_ref ? ref_pos[0] : 0, n_ref, nuc, pos);
    } else {
        // arbitrary reference vectors: materialise a dense window over [min, max]
        uint64_t lo = UINT64_MAX, hi = 0;
        for (size_t i = 0; i < n_ref; i++) { lo = std::min(lo, ref_pos[i]); hi = std::max(hi, ref_pos[i]); }
        if (hi - lo > (1u << 26)) return tfbs::fail(TFBS_E_ARG, "reference positions too sparse");
        (void)lo;
        return tfbs::fail(TFBS_E_ARG, "reference positions must be consecutive");
    }
    if (rc) return rc;
    *n_out = nuc.size();
    if (nuc.size() > cap) return tfbs::fail(TFBS_E_ARG, "output capacity too small");
    if (!nuc.empty()) {
        memcpy(out_nucs, nuc.data(), nuc.size());
        memcpy(out_pos, pos.data(), pos.size() * 8);
    }
    return TFBS_OK;
}

}  // extern "C"
