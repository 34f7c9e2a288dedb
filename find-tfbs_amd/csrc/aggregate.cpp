// Count aggregation and VCF row emission from the scan's per-haplotype counts.
//
// count_matches_by_sample (main.rs:500-534) adds, for every match and every
// inner peak it overlaps, +1 to each carrying haplotype's side.  Here the scan
// already summed hits per (distinct haplotype, pattern_id, inner range), so a
// key's per-sample vectors are gathers: L[s] = C[hap(2s)], R[s] = C[hap(2s+1)],
// times the multiplicity of the range in that bed list.  counts_as_genotypes
// (main.rs:439-498) and the row format (main.rs:415-429) follow.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "batch.hpp"
#include "rows.hpp"

namespace tfbs {

namespace {

struct KeyRef {
    const InnerKey *ik;
    uint32_t slot;  // pattern_id slot
};

// hap id -> local distinct index for region R (a device-grouped region's row is
// fetched from the device; a failed copy there is fatal)
struct Membership {
    const RegionH &R;
    std::vector<uint32_t> local;  // dense, built once per region
    Membership(const Batch &B, const RegionH &r, uint32_t H)
        : R(r), local(H, r.ref_local < 0 ? 0u : (uint32_t)r.ref_local) {
        if (!r.memb_host) {
            std::vector<uint16_t> row(H);
            if (!B.grouper || B.grouper->fetch(r.memb_dev, H, row.data())) {
                fprintf(stderr, "tfbs: membership fetch from the device failed: %s\n", tfbs_last_error());
                abort();
            }
            for (uint32_t h = 0; h < H; h++) local[h] = row[h];
            return;
        }
        for (size_t i = 0; i < r.nonref_id.size(); i++) local[r.nonref_id[i]] = r.nonref_local[i];
    }
};

inline uint64_t key_of(const Batch &B, const RegionH &R, uint32_t slot, int32_t range_slot) {
    return R.key_off + (uint64_t)slot * R.ranges.size() + (uint32_t)range_slot;
}

// Readers of the varying counts (count_of) on the host: the device key reduction's
// counts are downloaded on first use (ensure_host_var_counts).
inline int host_counts(const Batch &B) { return B.counts_valid ? 0 : ensure_host_var_counts(B); }

// Count of distinct haplotype `local` for a key, from the dense download or
// from the device key reduction (tfbs_batch_reduce).
inline uint32_t count_of(const Batch &B, const RegionH &R, uint32_t local, uint32_t slot, int32_t range_slot) {
    if (B.counts_valid) {
        const DevHap &h = B.haps[R.hap_begin + local];
        const uint32_t n_inner = (uint32_t)R.ranges.size();
        return B.counts[h.count_off + ((uint64_t)slot * n_inner + (uint32_t)range_slot) * B.regions[h.region].count_stride];
    }
    const uint64_t k = key_of(B, R, slot, range_slot);
    const uint32_t off = B.var_off[k];
    return off == UINT32_MAX ? B.key_first[k] : reinterpret_cast<const uint32_t *>(B.var_counts.data())[off + local];
}

// Some distinct haplotype matched (the key exists in the reference's HashMap).
inline bool key_any(const Batch &B, const RegionH &R, uint32_t slot, int32_t range_slot) {
    if (!B.counts_valid) return (B.key_flags[key_of(B, R, slot, range_slot)] & KEY_ANY) != 0;
    bool any = false;
    for (uint32_t l = 0; l < R.hap_count && !any; l++) any = count_of(B, R, l, slot, range_slot) != 0;
    return any;
}

// Distinct haplotypes disagree (otherwise every sample has the same total: no row).
inline bool key_varies(const Batch &B, const RegionH &R, uint32_t slot, int32_t range_slot) {
    if (!B.counts_valid) return (B.key_flags[key_of(B, R, slot, range_slot)] & KEY_VARIES) != 0;
    const uint32_t c0 = count_of(B, R, 0, slot, range_slot);
    for (uint32_t h = 1; h < R.hap_count; h++)
        if (count_of(B, R, h, slot, range_slot) != c0) return true;
    return false;
}

inline bool have_counts(const Batch &B) { return B.counts_valid || B.reduced; }

// Keys of a region in row order (inner.start, inner.end, bed index, pattern_id)
// that exist in the reference's HashMap, i.e. got at least one match.
std::vector<KeyRef> region_keys(const Batch &B, const RegionH &R) {
    std::vector<KeyRef> out;
    for (const InnerKey &k : R.keys) {
        if (k.slot < 0) continue;  // empty range: no match can overlap it
        for (uint32_t s : B.slots_by_pid)
            if (key_any(B, R, s, k.slot)) out.push_back({&k, s});
    }
    return out;  // R.keys is sorted by (s, e, bed); slots_by_pid ascends with pattern_id
}

}  // namespace

// main.rs:439-498.  Returns true and appends to info/gts if the counts vary.
bool counts_as_genotypes(const uint32_t *v1, const uint32_t *v2, size_t n, uint32_t *maf, std::string &info,
                         std::string &gts) {
    if (n == 0) return false;
    uint32_t lo = v1[0] + v2[0], hi = lo;
    for (size_t i = 1; i < n; i++) {
        uint32_t v = v1[i] + v2[i];
        lo = std::min(lo, v);
        hi = std::max(hi, v);
    }
    if (lo == hi) return false;
    const uint32_t i1 = (lo * 1000u * 3u + hi * 1000u) / 4u;  // u32, wrapping as --release
    const uint32_t i3 = (lo * 1000u + hi * 1000u * 3u) / 4u;
    std::vector<uint32_t> all{lo, hi};
    uint32_t zero = 0, one = 0, two = 0;
    const float lof = (float)lo;
    const float spread = (float)hi - lof;
    char buf[48];
    gts.reserve(gts.size() + n * 9);
    for (size_t i = 0; i < n; i++) {
        const uint32_t x = v1[i] + v2[i];
        if (x == lo) { gts += "\t0|0:0.0"; zero++; }
        else if (x == hi) { gts += "\t1|1:2.0"; two++; }
        else {
            if (std::find(all.begin(), all.end(), x) == all.end()) all.push_back(x);
            const uint32_t x1000 = x * 1000u;
            if (x1000 < i1) { gts += "\t0|0"; zero++; }
            else if (x1000 < i3) { gts += "\t0|1"; one++; }
            else { gts += "\t1|1"; two++; }
            const float ds = (((float)x - lof) * 2.0f) / spread;  // f32 throughout
            int m = snprintf(buf, sizeof buf, ":%.4f", (double)ds);
            gts.append(buf, (size_t)m);
        }
    }
    if (zero >= one && zero >= two) *maf = one + two;
    else if (two >= zero && two >= one) *maf = zero + one;
    else *maf = zero + two;
    std::sort(all.begin(), all.end());
    info += "COUNTS=";
    for (size_t j = 0; j < all.size(); j++) {
        int m = snprintf(buf, sizeof buf, j ? ",%u" : "%u", all[j]);
        info.append(buf, (size_t)m);
    }
    int m = snprintf(buf, sizeof buf, ";freqs=%u/%u/%u", zero, one, two);
    info.append(buf, (size_t)m);
    return true;
}

// chromosome.replace("chr", "") (main.rs:402)
std::string strip_chr(const std::string &c) {
    std::string o;
    for (size_t i = 0; i < c.size();) {
        if (c.compare(i, 3, "chr") == 0) i += 3;
        else o.push_back(c[i++]);
    }
    return o;
}

// The device encoding of a key (tfbs_batch_encode) of region r, or UINT32_MAX;
// host_codes: the caller formats from the codes on the host (they were downloaded).
static uint32_t encoded_key(const Batch &B, size_t r, uint64_t key, bool host_codes = true) {
    if (!B.reduced || B.counts_valid || r < B.enc_r0 || r >= B.enc_r1) return UINT32_MAX;
    if (host_codes && !B.enc_codes_host) return UINT32_MAX;
    const uint32_t vi = B.var_idx[key];
    if (vi == UINT32_MAX) return UINT32_MAX;
    const uint32_t e = B.enc_idx[vi];
    return (e != UINT32_MAX && B.enc_hdr[e].status == 0) ? e : UINT32_MAX;
}

// A key's per-value sample texts (16-byte slots, len bytes used) and the
// length of its genotype text.
struct EncText {
    char tab[kEncMaxVals + 1][16];
    uint8_t len[kEncMaxVals + 1];
    uint64_t total;
};

// counts_as_genotypes (main.rs:439-498) from a device encoding: the text of
// each distinct total is built once (with the range multiplicity applied,
// u32 arithmetic as counts_as_genotypes), a sample's text is the table entry
// of its code (encoded_write).  Returns 1 (row), 0 (the totals do not vary) or
// -1 (the multiplicity would wrap the totals: use the host path).
static int encoded_genotypes(const Batch &B, uint32_t e, uint32_t mult, uint32_t *maf, std::string &info,
                             EncText &t) {
    const EncHdr &h = B.enc_hdr[e];
    if ((uint64_t)h.hi * mult > UINT32_MAX) return -1;
    if (h.n_vals < 2) return 0;
    const uint32_t *vals = B.enc_vals.data() + B.enc_val_off[e];
    const uint32_t *hist = B.enc_hist.data() + B.enc_val_off[e];
    const uint32_t nv = h.n_vals, lo = vals[0] * mult, hi = vals[nv - 1] * mult;
    const uint32_t i1 = (lo * 1000u * 3u + hi * 1000u) / 4u;  // u32, wrapping as --release
    const uint32_t i3 = (lo * 1000u + hi * 1000u * 3u) / 4u;
    const float lof = (float)lo;
    const float spread = (float)hi - lof;
    char(&tab)[kEncMaxVals + 1][16] = t.tab;
    uint8_t(&len)[kEncMaxVals + 1] = t.len;
    uint64_t cls[3] = {0, 0, 0}, total = 0;
    for (uint32_t k = 0; k < nv; k++) {
        const uint32_t x = vals[k] * mult;
        int c;
        memset(tab[k], 0, 16);
        if (x == lo) { memcpy(tab[k], "\t0|0:0.0", 8); len[k] = 8; c = 0; }
        else if (x == hi) { memcpy(tab[k], "\t1|1:2.0", 8); len[k] = 8; c = 2; }
        else {
            const uint32_t x1000 = x * 1000u;
            c = x1000 < i1 ? 0 : (x1000 < i3 ? 1 : 2);
            const float ds = (((float)x - lof) * 2.0f) / spread;  // f32 throughout
            char buf[32];
            const int m = snprintf(buf, sizeof buf, "%s:%.4f", c == 0 ? "\t0|0" : (c == 1 ? "\t0|1" : "\t1|1"),
                                   (double)ds);
            memcpy(tab[k], buf, 16);
            len[k] = (uint8_t)m;
        }
        cls[c] += hist[k];
        total += (uint64_t)hist[k] * len[k];
    }
    const uint32_t zero = (uint32_t)cls[0], one = (uint32_t)cls[1], two = (uint32_t)cls[2];
    if (zero >= one && zero >= two) *maf = one + two;
    else if (two >= zero && two >= one) *maf = zero + one;
    else *maf = zero + two;
    char buf[48];
    info += "COUNTS=";
    for (uint32_t k = 0; k < nv; k++) {
        const int m = snprintf(buf, sizeof buf, k ? ",%u" : "%u", vals[k] * mult);
        info.append(buf, (size_t)m);
    }
    const int m = snprintf(buf, sizeof buf, ";freqs=%u/%u/%u", zero, one, two);
    info.append(buf, (size_t)m);
    t.total = total;
    return 1;
}

// The genotype text of key e into dst (t.total bytes; up to kEncPad written
// past it).  Codes of 2 or 4 bits go a whole byte at a time through a table of
// the byte's concatenated sample texts (16 bytes per sample slot).
constexpr size_t kEncPad = 64;
__attribute__((target_clones("avx2", "default"))) static void encoded_write(const Batch &B, uint32_t e, const EncText &t, char *dst) {
    const EncHdr &h = B.enc_hdr[e];
    const uint8_t *codes = B.enc_codes.data() + B.enc_code_off[e];
    const uint32_t width = h.width, per = 8 / width, mask = (1u << width) - 1u;
    uint32_t s = 0;
    if (per > 1) {
        const uint32_t slot = 16 * per;  // 64 or 32 bytes
        thread_local char bt[256 * 64];
        uint8_t bl[256];
        for (uint32_t v = 0; v < 256; v++) {
            char *q = bt + v * slot;
            uint32_t n = 0;
            for (uint32_t k = 0, x = v; k < per; k++, x >>= width) {
                const uint32_t c = x & mask;
                if (c >= h.n_vals) {  // a byte the codes never hold
                    n = 0;
                    break;
                }
                memcpy(q + n, t.tab[c], t.len[c]);
                n += t.len[c];
            }
            bl[v] = (uint8_t)n;
        }
        const uint32_t full = B.n_samples / per;
        // a sample's text is at most 11 bytes: 4 of them fit 48, 2 of them 24
        if (slot == 64) {
            for (uint32_t i = 0; i < full; i++) {
                const uint32_t v = codes[i];
                memcpy(dst, bt + v * 64, 48);
                dst += bl[v];
            }
        } else {
            for (uint32_t i = 0; i < full; i++) {
                const uint32_t v = codes[i];
                memcpy(dst, bt + v * 32, 24);
                dst += bl[v];
            }
        }
        s = full * per;
    }
    for (; s < B.n_samples; s += per) {
        uint32_t byte = codes[s / per];
        for (uint32_t q = 0; q < per && s + q < B.n_samples; q++, byte >>= width) {
            const uint32_t c = byte & mask;
            memcpy(dst, t.tab[c], 16);
            dst += t.len[c];
        }
    }
}

// Rows of one region appended to out, each without its "<chr>\t<POS>\t" prefix
// (the POS counter is assigned in order afterwards) and '\n'-terminated; returns
// the number of rows.  Keys the device encoded (tfbs_batch_encode) are
// formatted from their value tables and codes straight into out; the others
// from the per-haplotype counts through the membership.  kStream: each row goes
// to per_row(head, gts, n) as soon as it is complete, the row being head + the
// n bytes at gts + '\n'; the genotype text of an encoded key is then written
// into a reused raw buffer (cache-resident, never zero-filled) and head is the
// consumer's to clear.
template <bool kStream, class PerRow>
size_t region_rows_each(const Batch &B, const RegionH &R, uint32_t min_maf, std::string &out, PerRow &&per_row) {
    const uint32_t H = 2 * B.n_samples;
    const size_t ri = (size_t)(&R - B.rh.data());
    std::vector<uint32_t> l, r;
    std::unique_ptr<Membership> M;
    std::string info, gts;
    EncText et;
    size_t n_rows = 0;
    for (const KeyRef &k : region_keys(B, R)) {
        if (!key_varies(B, R, k.slot, k.ik->slot)) continue;
        uint32_t maf = 0;
        info.clear();
        gts.clear();
        const uint32_t e = encoded_key(B, ri, key_of(B, R, k.slot, k.ik->slot));
        int made = e == UINT32_MAX ? -1 : encoded_genotypes(B, e, k.ik->mult, &maf, info, et);
        const bool direct = made > 0;
        if (made < 0) {
            info.clear();
            gts.clear();
            if (!M) {
                M.reset(new Membership(B, R, H));
                l.resize(B.n_samples);
                r.resize(B.n_samples);
            }
            for (uint32_t s = 0; s < B.n_samples; s++) {
                l[s] = count_of(B, R, M->local[2 * s], k.slot, k.ik->slot) * k.ik->mult;
                r[s] = count_of(B, R, M->local[2 * s + 1], k.slot, k.ik->slot) * k.ik->mult;
            }
            made = counts_as_genotypes(l.data(), r.data(), B.n_samples, &maf, info, gts) ? 1 : 0;
        }
        if (!made) continue;
        if (maf < min_maf) continue;
        const uint16_t pid = B.slot_pid[k.slot];
        auto it = B.pats->names.find(pid);
        const std::string &pname = it == B.pats->names.end() ? std::string() : it->second;
        const uint64_t body = direct ? et.total : gts.size();
        if (out.capacity() < out.size() + body + 4096)
            out.reserve(std::max<size_t>(2 * out.capacity(), out.size() + body + 4096));
        out += B.beds[k.ik->bed];
        out += ',';
        out += pname;
        char head[96];
        snprintf(head, sizeof head, ",%llu-%llu\t.\t.\t.\tPASS\t", (unsigned long long)k.ik->s,
                 (unsigned long long)k.ik->e);
        out += head;
        out += info;
        out += "\tGT:DS";
        if (kStream) {
            thread_local std::unique_ptr<char[]> gbuf;
            thread_local size_t gcap = 0;
            const char *tail = gts.data();
            if (direct) {
                if (gcap < body + kEncPad) {
                    gcap = body + kEncPad;
                    gbuf.reset(new char[gcap]);
                }
                encoded_write(B, e, et, gbuf.get());
                tail = gbuf.get();
            }
            n_rows++;
            per_row(out, tail, (size_t)body);
            continue;
        }
        if (direct) {
            const size_t at = out.size();
            out.resize(at + body + kEncPad);
            encoded_write(B, e, et, &out[at]);
            out.resize(at + body);
        } else {
            out += gts;
        }
        out += '\n';
        n_rows++;
    }
    return n_rows;
}

// One row of build_row_plan before its POS: the head after "<chr>\t<POS>\t"
// (the whole row text but its '\n' when the device did not encode the key), and
// for an encoded key its index, value texts and genotype text length.
struct RowPart {
    std::string head;
    uint32_t e = UINT32_MAX;
    uint32_t nv = 0;
    uint64_t total = 0;
    std::vector<char> tok;     // kRowTokBytes per value
    std::vector<uint8_t> len;
};

// region_rows_each's rows of one region as RowParts (no genotype text for the
// keys the device encoded).
static void region_row_parts(const Batch &B, const RegionH &R, uint32_t min_maf, std::vector<RowPart> &parts) {
    const uint32_t H = 2 * B.n_samples;
    const size_t ri = (size_t)(&R - B.rh.data());
    std::vector<uint32_t> l, r;
    std::unique_ptr<Membership> M;
    std::string info, gts;
    EncText et;
    for (const KeyRef &k : region_keys(B, R)) {
        if (!key_varies(B, R, k.slot, k.ik->slot)) continue;
        uint32_t maf = 0;
        info.clear();
        gts.clear();
        const uint32_t e = encoded_key(B, ri, key_of(B, R, k.slot, k.ik->slot), false);
        int made = e == UINT32_MAX ? -1 : encoded_genotypes(B, e, k.ik->mult, &maf, info, et);
        const bool direct = made > 0;
        if (made < 0) {
            info.clear();
            gts.clear();
            if (!M) {
                M.reset(new Membership(B, R, H));
                l.resize(B.n_samples);
                r.resize(B.n_samples);
            }
            if (host_counts(B)) return;  // (build_row_plan returns the error)
            for (uint32_t s = 0; s < B.n_samples; s++) {
                l[s] = count_of(B, R, M->local[2 * s], k.slot, k.ik->slot) * k.ik->mult;
                r[s] = count_of(B, R, M->local[2 * s + 1], k.slot, k.ik->slot) * k.ik->mult;
            }
            made = counts_as_genotypes(l.data(), r.data(), B.n_samples, &maf, info, gts) ? 1 : 0;
        }
        if (!made) continue;
        if (maf < min_maf) continue;
        const uint16_t pid = B.slot_pid[k.slot];
        auto it = B.pats->names.find(pid);
        const std::string &pname = it == B.pats->names.end() ? std::string() : it->second;
        parts.emplace_back();
        RowPart &p = parts.back();
        p.head += B.beds[k.ik->bed];
        p.head += ',';
        p.head += pname;
        char head[96];
        snprintf(head, sizeof head, ",%llu-%llu\t.\t.\t.\tPASS\t", (unsigned long long)k.ik->s,
                 (unsigned long long)k.ik->e);
        p.head += head;
        p.head += info;
        p.head += "\tGT:DS";
        if (direct) {
            p.e = e;
            p.nv = B.enc_hdr[e].n_vals;
            p.total = et.total;
            p.tok.assign((size_t)p.nv * kRowTokBytes, 0);
            p.len.assign(et.len, et.len + p.nv);
            for (uint32_t v = 0; v < p.nv; v++) memcpy(&p.tok[(size_t)v * kRowTokBytes], et.tab[v], kRowTokBytes);
        } else {
            p.head += gts;
        }
    }
}

struct RowParts {
    size_t r0 = 0;
    std::vector<std::vector<RowPart>> parts;  // per region of [r0, r0 + parts.size())
};

int build_row_parts(const Batch &B, size_t r0, size_t r1, uint32_t min_maf, uint32_t threads,
                    std::shared_ptr<RowParts> &out, uint64_t *n_rows) {
    if (!have_counts(B)) return fail(TFBS_E_STATE, "counts not downloaded");
    if (!B.keep_membership && B.n_samples) return fail(TFBS_E_STATE, "batch created without membership");
    r1 = std::min(r1, B.rh.size());
    r0 = std::min(r0, r1);
    const size_t n = r1 - r0;
    out = std::make_shared<RowParts>();
    out->r0 = r0;
    std::vector<std::vector<RowPart>> &parts = out->parts;
    parts.resize(n);
    std::atomic<size_t> next(0);
    auto work = [&]() {
        for (size_t j; (j = next.fetch_add(1)) < n;)
            if (B.rh[r0 + j].hap_count) region_row_parts(B, B.rh[r0 + j], min_maf, parts[j]);
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads && t < n; t++) ts.emplace_back(work);
    work();
    for (auto &t : ts) t.join();
    if (!B.counts_valid && B.var_host && B.var_err) return B.var_err;  // a lazy count download failed
    uint64_t rows = 0;
    for (auto &v : parts) rows += v.size();
    if (n_rows) *n_rows = rows;
    return TFBS_OK;
}

int plan_from_parts(const Batch &B, RowParts &P, size_t r0, size_t r1, const std::string &chrom, uint32_t *fake,
                    RowPlan &plan) {
    // serially: POS, offsets in the stream, token slots (sized first: one allocation each)
    plan = RowPlan();
    const std::string chr = strip_chr(chrom);
    const size_t q0 = std::max(r0, P.r0), q1 = std::min(r1, P.r0 + P.parts.size());
    size_t n_rows = 0, head_bytes = 0, n_tok = 0;
    for (size_t r = q0; r < q1; r++)
        for (const RowPart &p : P.parts[r - P.r0]) {
            n_rows++;
            head_bytes += chr.size() + 12 + p.head.size();  // ("\t<POS>\t": at most 12 bytes)
            if (p.e != UINT32_MAX) n_tok += p.nv;
        }
    plan.rows.reserve(n_rows);
    plan.heads.reserve(head_bytes);
    plan.tok_len.reserve(n_tok);
    plan.tok_text.reserve(n_tok * kRowTokBytes);
    uint64_t at = 0;
    char pos[16];
    for (size_t r = q0; r < q1; r++) {
        for (RowPart &p : P.parts[r - P.r0]) {
            DevRow d{};
            d.head_off = (uint32_t)plan.heads.size();
            // "\t<POS>\t" (the fake position, decimal)
            char *e = pos + sizeof pos;
            *--e = '\t';
            uint32_t v = (*fake)++;
            do {
                *--e = (char)('0' + v % 10);
                v /= 10;
            } while (v);
            *--e = '\t';
            plan.heads += chr;
            plan.heads.append(e, (size_t)(pos + sizeof pos - e));
            plan.heads += p.head;
            if (plan.heads.size() >= UINT32_MAX) return fail(TFBS_E_NOMEM, "row heads past 4 GiB in one call");
            d.head_len = (uint32_t)(plan.heads.size() - d.head_off);
            d.text_off = at;
            if (p.e != UINT32_MAX) {
                d.geno_len = p.total;
                d.code_off = B.enc_code_off[p.e];
                d.width = B.enc_hdr[p.e].width;
                d.tok = (uint32_t)plan.tok_len.size();
                d.nv = p.nv;
                plan.tok_len.insert(plan.tok_len.end(), p.len.begin(), p.len.end());
                plan.tok_text.insert(plan.tok_text.end(), p.tok.begin(), p.tok.end());
            }
            at += d.head_len + d.geno_len + 1;
            plan.rows.push_back(d);
        }
        std::vector<RowPart>().swap(P.parts[r - P.r0]);  // (the region's parts are done)
    }
    plan.text_bytes = at;
    plan.n_rows = plan.rows.size();
    return TFBS_OK;
}

int build_row_plan(const Batch &B, size_t r0, size_t r1, const std::string &chrom, uint32_t min_maf,
                   uint32_t *fake, uint32_t threads, RowPlan &plan) {
    static const bool prof = getenv("TFBS_PLAN_PROF") != nullptr;  // (debug: the two halves' seconds)
    static std::atomic<uint64_t> t_parts(0), t_plan(0), calls(0);
    auto now = [] { return std::chrono::steady_clock::now(); };
    const auto t0 = now();
    std::shared_ptr<RowParts> P;
    if (int rc = build_row_parts(B, r0, r1, min_maf, threads, P, nullptr)) return rc;
    const auto t1 = now();
    const int rc = plan_from_parts(B, *P, r0, r1, chrom, fake, plan);
    if (prof) {
        t_parts += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
        t_plan += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(now() - t1).count();
        if (++calls % 40 == 0)
            fprintf(stderr, "[plan prof] %llu plans: parts %.3f s, from parts %.3f s\n", (unsigned long long)calls.load(),
                    t_parts.load() * 1e-6, t_plan.load() * 1e-6);
    }
    return rc;
}

size_t region_rows(const Batch &B, const RegionH &R, uint32_t min_maf, std::string &out) {
    return region_rows_each<false>(B, R, min_maf, out, [](std::string &, const char *, size_t) {});
}

// Row bodies (each row without its "<chr>\t<POS>\t" prefix, '\n'-terminated)
// of every region in batch order, regions formatted in parallel on `threads`
// threads (main.rs:395-432).
int batch_row_bodies(const Batch &B, uint32_t min_maf, std::string &out, uint32_t threads) {
    if (!have_counts(B)) return fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = host_counts(B)) return rc;  // the varying counts on the host
    if (!B.keep_membership && B.n_samples) return fail(TFBS_E_STATE, "batch created without membership");
    const size_t n = B.rh.size();
    std::vector<std::string> rows(n);  // each region's rows
    std::atomic<size_t> next(0);
    auto work = [&]() {
        for (size_t j; (j = next.fetch_add(1)) < n;)
            if (B.rh[j].hap_count) region_rows(B, B.rh[j], min_maf, rows[j]);
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads && t < n; t++) ts.emplace_back(work);
    work();
    for (auto &t : ts) t.join();
    size_t bytes = out.size();
    for (auto &v : rows) bytes += v.size();
    out.reserve(bytes);
    for (auto &v : rows) {
        out += v;
        std::string().swap(v);
    }
    return TFBS_OK;
}

// The same rows with the prefix, POS counter `fake` in row order.
int batch_rows(const Batch &B, const std::string &chrom, uint32_t min_maf, uint32_t *fake, std::string &out,
               uint32_t threads) {
    std::string bodies;
    if (int rc = batch_row_bodies(B, min_maf, bodies, threads)) return rc;
    const std::string chr = strip_chr(chrom);
    char head[32];
    out.reserve(out.size() + bodies.size() + 64);
    for (size_t i = 0; i < bodies.size();) {
        size_t e = bodies.find('\n', i);
        e = e == std::string::npos ? bodies.size() : e + 1;
        const int m = snprintf(head, sizeof head, "\t%u\t", *fake);
        out += chr;
        out.append(head, (size_t)m);
        out.append(bodies, i, e - i);
        (*fake)++;
        i = e;
    }
    return TFBS_OK;
}

}  // namespace tfbs

using tfbs::Batch;

extern "C" {

int tfbs_batch_region_num_keys(const tfbs_batch *b, size_t region, size_t *n) {
    if (!b || !n || region >= b->b.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    if (!tfbs::have_counts(b->b)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    *n = tfbs::region_keys(b->b, b->b.rh[region]).size();
    return TFBS_OK;
}

int tfbs_batch_region_key(const tfbs_batch *b, size_t region, size_t k, uint32_t *bed, uint64_t *start, uint64_t *end,
                          uint16_t *pid, uint32_t *left, uint32_t *right) {
    if (!b || region >= b->b.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    const Batch &B = b->b;
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    if (!B.keep_membership && B.n_samples && (left || right))
        return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    const tfbs::RegionH &R = B.rh[region];
    auto keys = tfbs::region_keys(B, R);
    if (k >= keys.size()) return tfbs::fail(TFBS_E_ARG, "bad key index");
    const auto &q = keys[k];
    if (bed) *bed = q.ik->bed;
    if (start) *start = q.ik->s;
    if (end) *end = q.ik->e;
    if (pid) *pid = B.slot_pid[q.slot];
    if (left || right) {
        if (int rc = tfbs::region_membership(B, R)) return rc;
        tfbs::Membership M(B, R, 2 * B.n_samples);
        for (uint32_t s = 0; s < B.n_samples; s++) {
            if (left) left[s] = tfbs::count_of(B, R, M.local[2 * s], q.slot, q.ik->slot) * q.ik->mult;
            if (right) right[s] = tfbs::count_of(B, R, M.local[2 * s + 1], q.slot, q.ik->slot) * q.ik->mult;
        }
    }
    return TFBS_OK;
}

int tfbs_batch_region_rows(const tfbs_batch *b, size_t region, const char *chromosome, uint32_t min_maf,
                           uint32_t *fake, char **text, size_t *len) {
    if (!b || !chromosome || !fake || !text || !len) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (region >= B.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    if (!B.keep_membership && B.n_samples) return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    std::string bodies;
    if (B.rh[region].hap_count) tfbs::region_rows(B, B.rh[region], min_maf, bodies);
    const std::string chr = tfbs::strip_chr(chromosome);
    std::string out;
    char head[32];
    for (size_t i = 0; i < bodies.size();) {
        size_t e = bodies.find('\n', i);
        e = e == std::string::npos ? bodies.size() : e + 1;
        const int m = snprintf(head, sizeof head, "\t%u\t", *fake);
        out += chr;
        out.append(head, (size_t)m);
        out.append(bodies, i, e - i);
        (*fake)++;
        i = e;
    }
    char *p = (char *)malloc(out.size() + 1);
    if (!p) return tfbs::fail(TFBS_E_NOMEM, "malloc");
    memcpy(p, out.data(), out.size());
    p[out.size()] = 0;
    *text = p;
    *len = out.size();
    return TFBS_OK;
}

// A 64-bit digest of a region's keys at the distinct-haplotype level: for every
// key in row order its (bed, range, pattern_id) and every distinct haplotype's
// count.  Per-sample vectors follow from these and the membership, so equal
// digests from the dense download and the device reduction (or from two shards
// of one workload) mean equal keys.
int tfbs_batch_region_digest(const tfbs_batch *b, size_t region, uint64_t *digest) {
    if (!b || !digest) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (region >= B.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    const tfbs::RegionH &R = B.rh[region];
    uint64_t h = 0x9E3779B97F4A7C15ull;
    auto mix = [&h](uint64_t x) {
        h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
        h *= 0xFF51AFD7ED558CCDull;
        h ^= h >> 33;
    };
    const auto keys = tfbs::region_keys(B, R);
    mix(keys.size());
    for (const auto &k : keys) {
        mix(k.ik->bed);
        mix(k.ik->s);
        mix(k.ik->e);
        mix(k.ik->mult);
        mix(B.slot_pid[k.slot]);
        for (uint32_t l = 0; l < R.hap_count; l++) mix(tfbs::count_of(B, R, l, k.slot, k.ik->slot));
    }
    *digest = h;
    return TFBS_OK;
}

namespace {
uint64_t mix64(uint64_t h, uint64_t x) {
    h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}
}  // namespace

int tfbs_batch_region_key_digest_sum(const tfbs_batch *b, size_t region, uint64_t *digest) {
    if (!b || !digest) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (region >= B.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    const tfbs::RegionH &R = B.rh[region];
    uint64_t sum = 0;
    for (const auto &k : tfbs::region_keys(B, R)) {  // one hash per key, added: order-free
        uint64_t h = 0x2545F4914F6CDD1Dull;
        h = mix64(h, k.ik->bed);
        h = mix64(h, k.ik->s);
        h = mix64(h, k.ik->e);
        h = mix64(h, k.ik->mult);
        h = mix64(h, B.slot_pid[k.slot]);
        for (uint32_t l = 0; l < R.hap_count; l++) h = mix64(h, tfbs::count_of(B, R, l, k.slot, k.ik->slot));
        sum += h;
    }
    *digest = sum;
    return TFBS_OK;
}

int tfbs_batch_region_input_digest(const tfbs_batch *b, size_t region, uint64_t *digest) {
    if (!b || !digest) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (region >= B.rh.size()) return tfbs::fail(TFBS_E_ARG, "bad region");
    const tfbs::RegionH &R = B.rh[region];
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (uint64_t x : {R.ms, R.me, R.es, R.ee, (uint64_t)R.hap_count, (uint64_t)(int64_t)R.ref_local,
                       (uint64_t)R.n_variants})
        h = mix64(h, x);
    for (const auto &k : R.keys) {
        h = mix64(h, k.bed);
        h = mix64(h, k.s);
        h = mix64(h, k.e);
        h = mix64(h, k.mult);
    }
    if (int rc = tfbs::region_membership(B, R)) return rc;
    for (size_t i = 0; i < R.nonref_id.size(); i++) h = mix64(h, ((uint64_t)R.nonref_id[i] << 32) | R.nonref_local[i]);
    for (uint32_t l = 0; l < R.hap_count; l++) {  // the packed bases, N masks and positions of each distinct haplotype
        const tfbs::DevHap &d = B.haps[R.hap_begin + l];
        h = mix64(h, d.len);
        h = mix64(h, d.flags & (tfbs::HAP_HAS_N | tfbs::HAP_HAS_POS));
        h = mix64(h, B.hap_carriers[R.hap_begin + l]);
        for (uint32_t w = 0; w < (d.len + 15) / 16; w++) {
            uint32_t x = B.words[d.word_off + w];
            if (16 * w + 16 > d.len) x &= (1u << (2 * (d.len - 16 * w))) - 1;  // bits past the end are padding
            h = mix64(h, x);
        }
        if (d.flags & tfbs::HAP_HAS_N)
            for (uint32_t w = 0; w < (d.len + 31) / 32; w++) h = mix64(h, B.nmask[d.nmask_off + w]);
        if (d.flags & tfbs::HAP_HAS_POS)
            for (uint32_t i = 0; i < d.len; i++) h = mix64(h, (uint32_t)B.posrel[d.pos_off + i]);
    }
    *digest = h;
    return TFBS_OK;
}

namespace {
// XXH64 (the published xxHash 64-bit algorithm), streaming: the row digest of
// tfbs_batch_region_digests.
struct Xxh64 {
    static constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                              P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
    uint64_t v[4] = {P1 + P2, P2, 0, 0 - P1}, total = 0;
    uint8_t buf[32];
    size_t nbuf = 0;
    static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
    static uint64_t rd64(const uint8_t *p) {
        uint64_t x;
        memcpy(&x, p, 8);
        return x;
    }
    static uint64_t round(uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; }
    void stripe(const uint8_t *p) {
        for (int k = 0; k < 4; k++) v[k] = round(v[k], rd64(p + 8 * k));
    }
    void update(const void *data, size_t n) {
        const uint8_t *p = static_cast<const uint8_t *>(data);
        total += n;
        if (nbuf) {
            const size_t take = std::min(32 - nbuf, n);
            memcpy(buf + nbuf, p, take);
            nbuf += take;
            p += take;
            n -= take;
            if (nbuf < 32) return;
            stripe(buf);
            nbuf = 0;
        }
        for (; n >= 32; p += 32, n -= 32) stripe(p);
        memcpy(buf, p, n);
        nbuf = n;
    }
    uint64_t digest() const {
        uint64_t h = total >= 32 ? rotl(v[0], 1) + rotl(v[1], 7) + rotl(v[2], 12) + rotl(v[3], 18) : P5;
        if (total >= 32)
            for (int k = 0; k < 4; k++) h = (h ^ round(0, v[k])) * P1 + P4;
        h += total;
        const uint8_t *p = buf;
        size_t n = nbuf;
        for (; n >= 8; p += 8, n -= 8) h = rotl(h ^ round(0, rd64(p)), 27) * P1 + P4;
        if (n >= 4) {
            uint32_t x;
            memcpy(&x, p, 4);
            h = rotl(h ^ (uint64_t)x * P1, 23) * P2 + P3;
            p += 4;
            n -= 4;
        }
        for (; n > 0; p++, n--) h = rotl(h ^ (uint64_t)*p * P5, 11) * P1;
        h ^= h >> 33;
        h *= P2;
        h ^= h >> 29;
        h *= P3;
        return h ^ (h >> 32);
    }
};

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
}  // namespace

int tfbs_batch_region_digests(const tfbs_batch *b, size_t r0, size_t r1, uint32_t min_maf, uint32_t threads,
                              uint64_t *keys, uint64_t *rows, uint64_t *n_rows) {
    if (!b || (!keys && !rows)) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (r1 > B.rh.size() || r0 > r1) return tfbs::fail(TFBS_E_ARG, "bad region range");
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    if (!B.keep_membership && B.n_samples) return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    const uint32_t H = 2 * B.n_samples;
    std::vector<uint64_t> w(H);
    for (uint32_t h = 0; h < H; h++) w[h] = splitmix64(h);
    std::atomic<size_t> next(r0);
    auto work = [&]() {
        std::string rr;
        std::vector<uint64_t> W;
        for (size_t j; (j = next.fetch_add(1)) < r1;) {
            const tfbs::RegionH &R = B.rh[j];
            uint64_t sum = 0;
            Xxh64 x;
            uint64_t nr = 0;
            if (R.hap_count && keys) {
                const auto ks = tfbs::region_keys(B, R);
                if (!ks.empty()) {  // W[l]: the sketch weights of distinct haplotype l's carriers
                    tfbs::Membership M(B, R, H);
                    W.assign(R.hap_count, 0);
                    for (uint32_t h = 0; h < H; h++) W[M.local[h]] += w[h];
                }
                for (const auto &k : ks) {
                    uint64_t S = 0;
                    for (uint32_t l = 0; l < R.hap_count; l++)
                        S += (uint64_t)tfbs::count_of(B, R, l, k.slot, k.ik->slot) * k.ik->mult * W[l];
                    uint64_t h = 0x2545F4914F6CDD1Dull;
                    h = mix64(h, k.ik->bed);
                    h = mix64(h, k.ik->s);
                    h = mix64(h, k.ik->e);
                    h = mix64(h, B.slot_pid[k.slot]);
                    h = mix64(h, S);
                    sum += h;
                }
            }
            if (R.hap_count && rows) {
                auto take = [&](std::string &head, const char *tail, size_t n) {
                    x.update(head.data(), head.size());
                    x.update(tail, n);
                    x.update("\n", 1);
                    head.clear();
                };
                nr = tfbs::region_rows_each<true>(B, R, min_maf, rr, take);
            }
            if (keys) keys[j - r0] = sum;
            if (rows) rows[j - r0] = x.digest();
            if (n_rows) n_rows[j - r0] = nr;
        }
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads && t < r1 - r0; t++) ts.emplace_back(work);
    work();
    for (auto &t : ts) t.join();
    return TFBS_OK;
}

int tfbs_batch_rows(const tfbs_batch *b, const char *chromosome, uint32_t min_maf, uint32_t *fake, char **text,
                    size_t *len) {
    if (!b || !chromosome || !fake || !text || !len) return tfbs::fail(TFBS_E_ARG, "null argument");
    std::string out;
    int rc = tfbs::batch_rows(b->b, chromosome, min_maf, fake, out, 1);
    if (rc) return rc;
    char *p = (char *)malloc(out.size() + 1);
    if (!p) return tfbs::fail(TFBS_E_NOMEM, "malloc");
    memcpy(p, out.data(), out.size());
    p[out.size()] = 0;
    *text = p;
    *len = out.size();
    return TFBS_OK;
}

int tfbs_batch_format_rows(const tfbs_batch *b, const char *chromosome, uint32_t min_maf, uint32_t threads,
                           size_t r0, size_t r1, uint64_t *n_rows, uint64_t *n_bytes) {
    if (!b || !chromosome || !n_rows || !n_bytes) return tfbs::fail(TFBS_E_ARG, "null argument");
    const Batch &B = b->b;
    if (!tfbs::have_counts(B)) return tfbs::fail(TFBS_E_STATE, "counts not downloaded");
    if (int rc = tfbs::host_counts(B)) return rc;  // the varying counts on the host
    if (!B.keep_membership && B.n_samples) return tfbs::fail(TFBS_E_STATE, "batch created without membership");
    const size_t n = std::min(r1, B.rh.size());
    const size_t prefix = tfbs::strip_chr(chromosome).size() + 2;
    std::atomic<size_t> next(std::min(r0, n));
    std::atomic<uint64_t> rows(0), bytes(0);
    auto work = [&]() {
        std::string rr;  // reused: one row's text at a time
        uint64_t r = 0, by = 0;
        auto take = [&](std::string &head, const char *, size_t n) {
            by += head.size() + n + 1 + prefix;
            head.clear();
        };
        for (size_t j; (j = next.fetch_add(1)) < n;)
            if (B.rh[j].hap_count) r += tfbs::region_rows_each<true>(B, B.rh[j], min_maf, rr, take);
        rows += r;
        bytes += by;
    };
    std::vector<std::thread> ts;
    for (uint32_t t = 1; t < threads && t < n; t++) ts.emplace_back(work);
    work();
    for (auto &t : ts) t.join();
    *n_rows = rows;
    *n_bytes = bytes;  // + the POS digits, which depend on the run's counter
    return TFBS_OK;
}

int tfbs_batch_prep_seconds(const tfbs_batch *b, double *out) {
    if (!b || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    memcpy(out, b->b.prep_s, sizeof b->b.prep_s);
    return TFBS_OK;
}

void tfbs_free(void *p) { free(p); }

int tfbs_counts_as_genotypes(const uint32_t *left, const uint32_t *right, size_t n, uint32_t *maf, char *info,
                             size_t info_cap, char *genotypes, size_t gt_cap) {
    if (!maf || (n && (!left || !right))) return tfbs::fail(TFBS_E_ARG, "null argument");
    std::string a, g;
    if (!tfbs::counts_as_genotypes(left, right, n, maf, a, g)) return 0;
    if (a.size() + 1 > info_cap || g.size() + 1 > gt_cap) return tfbs::fail(TFBS_E_ARG, "output capacity too small");
    memcpy(info, a.c_str(), a.size() + 1);
    memcpy(genotypes, g.c_str(), g.size() + 1);
    return 1;
}

}  // extern "C"
