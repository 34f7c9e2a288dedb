// Pattern parsing and the device pattern plan.
//
// Parsing restates pattern.rs:13-112 (parse_weight, parse_threshold_file,
// parse_pwm_files, parse_pwm_definition, reverse_complement).  The plan turns
// the pattern list into what the scan kernels consume: pattern_id slots, tiles
// of strands whose 4-mer lookup tables fit the LDS budget, the tables
// themselves and the per-column A weights used for N correction.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// Rust f32::from_str accepts [+-]digits[.digits][(e|E)[+-]digits], ".5", "5.",
// and inf/infinity/nan in any case; nothing else (no hex, no spaces).
static bool parse_f32_rust(const std::string &s, float *out) {
    size_t i = 0;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
    std::string rest = s.substr(i);
    std::string low;
    for (char c : rest) low.push_back((char)std::tolower((unsigned char)c));
    if (low == "inf" || low == "infinity" || low == "nan") {
        *out = std::strtof(s.c_str(), nullptr);
        return true;
    }
    size_t digits = 0;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) { i++; digits++; }
    if (i < s.size() && s[i] == '.') {
        i++;
        while (i < s.size() && std::isdigit((unsigned char)s[i])) { i++; digits++; }
    }
    if (!digits) return false;
    if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
        i++;
        if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
        if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return false;
        while (i < s.size() && std::isdigit((unsigned char)s[i])) i++;
    }
    if (i != s.size()) return false;
    *out = std::strtof(s.c_str(), nullptr);
    return true;
}

// pattern.rs:13-16.  The multiply is f32; round() is half away from zero; the
// `as i32` cast saturates and maps NaN to 0.
static int32_t milli(float x) {
    volatile float y = x * 1000.0f;
    float r = std::round((float)y);
    if (std::isnan(r)) return 0;
    if (r >= 2147483647.0f) return INT32_MAX;
    if (r <= -2147483648.0f) return INT32_MIN;
    return (int32_t)r;
}

static std::vector<std::string> split_ws(const std::string &line) {
    std::vector<std::string> out;
    std::istringstream is(line);
    std::string f;
    while (is >> f) out.push_back(f);
    return out;
}

int parse_weight(const std::string &s, int32_t *out) {
    float x;
    if (!parse_f32_rust(s, &x)) return fail(TFBS_E_PARSE, "cannot parse weight '" + s + "'");
    *out = milli(x);
    return TFBS_OK;
}

int parse_threshold_file(const std::string &path, float thr, int32_t *out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(TFBS_E_IO, "Could not open file " + path);  // pattern.rs:116 expect
    std::string line;
    int found = 0;
    while (std::getline(in, line)) {
        auto f = split_ws(line);
        if (f.size() != 2) continue;
        int32_t w;
        float pv;
        int rc = parse_weight(f[0], &w);
        if (rc) return rc;
        if (!parse_f32_rust(f[1], &pv)) return fail(TFBS_E_PARSE, "Can't parse pvalue in file " + path);
        if (pv > thr) {  // the last qualifying line wins
            *out = w;
            found = 1;
        }
    }
    return found;
}

void Patterns::add(const Pat &p) {
    pats.push_back(p);
    names[p.pattern_id] = p.name;  // main.rs:239-250 HashMap insert: last wins
    slot_cache = std::make_shared<SlotCache>();  // (a copy keeps the old set's)
}

int Patterns::slot_order(std::vector<uint16_t> &slot_pid, bool &zero_len_panics) const {
    std::lock_guard<std::mutex> l(slot_cache->mu);
    SlotCache &c = *slot_cache;
    if (!c.built) {
        Plan plan;  // only its slot order is used (independent of the tile options)
        PlanOptions opt;
        opt.tile_blocks = 1u << 30;
        c.rc = build_plan(opt, &plan);
        c.slot_pid = std::move(plan.slot_pid);
        c.zero_len_panics = plan.zero_len_panics;
        c.built = true;
    }
    if (c.rc) return c.rc;
    slot_pid = c.slot_pid;
    zero_len_panics = c.zero_len_panics;
    return 0;
}

uint32_t Patterns::max_length() const {
    uint32_t m = 0;
    for (auto &p : pats) m = std::max<uint32_t>(m, p.kind == TFBS_KIND_PWM ? p.len : 0);
    return m;
}

static std::vector<int32_t> revcomp(const std::vector<int32_t> &w5, uint32_t L) {
    std::vector<int32_t> o(5 * (size_t)L);
    for (uint32_t j = 0; j < L; j++) {
        const int32_t *x = &w5[5 * (size_t)(L - 1 - j)];
        int32_t *y = &o[5 * (size_t)j];
        y[0] = x[3]; y[1] = x[2]; y[2] = x[1]; y[3] = x[0]; y[4] = 0;
    }
    return o;
}

int parse_pwm_files(const std::string &pwm_file, const std::string &thr_dir, float thr,
                    const std::vector<std::string> &wanted, bool add_reverse, Patterns *out) {
    std::map<std::string, int32_t> thresholds;
    std::string dir = thr_dir;
    while (!dir.empty() && dir.back() == '/') dir.pop_back();
    for (auto &name : wanted) {
        int32_t v;
        int r = parse_threshold_file(dir + "/" + name + ".thr", thr, &v);
        if (r < 0) return r;
        if (r == 1) thresholds[name] = v;
    }
    std::ifstream in(pwm_file, std::ios::binary);
    if (!in) return fail(TFBS_E_IO, "Could not open file " + pwm_file);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string content = ss.str();
    uint16_t pattern_id = 0;
    size_t start = 0;
    while (start <= content.size()) {
        size_t gt = content.find('>', start);
        std::string chunk = content.substr(start, gt == std::string::npos ? std::string::npos : gt - start);
        start = gt == std::string::npos ? content.size() + 1 : gt + 1;
        if (chunk.empty()) continue;
        // parse_pwm_definition (pattern.rs:89-101)
        std::vector<std::string> lines;
        size_t a = 0;
        while (a <= chunk.size()) {
            size_t nl = chunk.find('\n', a);
            std::string l = chunk.substr(a, nl == std::string::npos ? std::string::npos : nl - a);
            if (!l.empty()) lines.push_back(l);
            if (nl == std::string::npos) break;
            a = nl + 1;
        }
        if (lines.empty()) return fail(TFBS_E_PARSE, "empty PWM definition");
        const std::string name = lines[0];
        std::vector<int32_t> w5;
        for (size_t i = 1; i < lines.size(); i++) {
            auto f = split_ws(lines[i]);
            if (f.size() != 4) continue;
            int32_t v[4];
            for (int k = 0; k < 4; k++) {
                int rc = parse_weight(f[k], &v[k]);
                if (rc) return rc;
            }
            w5.insert(w5.end(), {v[0], v[1], v[2], v[3], 0});
        }
        if (std::find(wanted.begin(), wanted.end(), name) == wanted.end()) continue;
        auto it = thresholds.find(name);
        if (it != thresholds.end()) {
            Pat p;
            p.kind = TFBS_KIND_PWM;
            p.direction = TFBS_DIR_P;
            p.pattern_id = pattern_id;
            p.min_score = it->second;
            p.len = (uint32_t)(w5.size() / 5);
            p.w5 = w5;
            p.name = name;
            out->add(p);
            if (add_reverse) {
                p.direction = TFBS_DIR_N;
                p.w5 = revcomp(w5, p.len);
                out->add(p);
            }
        }
        pattern_id = (uint16_t)(pattern_id + 1);  // pattern.rs:81
    }
    if (out->pats.empty()) return fail(TFBS_E_NOPATTERN, "no pattern loaded");  // main.rs:238
    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// Device plan
// ---------------------------------------------------------------------------
struct Group { uint16_t pid; bool generic; uint32_t maxlen; std::vector<int> strands; };
static std::vector<SlotGroup> groups_fast(const std::vector<Group> &groups) {
    std::vector<SlotGroup> out;
    for (uint32_t gi = 0; gi < groups.size(); gi++)
        if (!groups[gi].generic) out.push_back({gi, groups[gi].strands});
    return out;
}
// Strands are grouped by pattern_id (both strands of a PWM share it and their
// hits add into one count, main.rs:505).  Groups are ordered by (needs the
// generic kernel, longest strand, pattern_id) -- this order defines the count
// slots -- so neighbouring strands have similar lengths and pack into units
// with little padding.  Fast tiles are runs of whole groups whose table blocks
// fit the LDS budget and span at most 64 slots.
// With opt.mfma, groups whose strands all pass mfma_eligible are scored on the
// matrix cores instead (32-strand tiles, any slot mix: that kernel adds its
// counts atomically).
int Patterns::build_plan(const PlanOptions &opt, Plan *plan) const {
    *plan = Plan();
    // Scannable strands: PWM with length >= 1.  A length-0 PWM with a negative
    // min_score panics in the reference at the first region (pattern.rs:150-156
    // reads haplotype[len]); with min_score >= 0 it never matches.
    std::map<uint16_t, std::vector<int>> by_pid;
    for (size_t i = 0; i < pats.size(); i++) {
        const Pat &p = pats[i];
        if (p.kind != TFBS_KIND_PWM) continue;
        if (p.len == 0) {
            if (p.min_score < 0) plan->zero_len_panics = true;
            continue;
        }
        by_pid[p.pattern_id].push_back((int)i);
    }
    if (pats.size() > 65535) return fail(TFBS_E_ARG, "more than 65535 patterns");
    std::vector<Group> groups;
    for (auto &kv : by_pid) {
        Group g{kv.first, false, 0, kv.second};
        for (int i : g.strands) {
            g.maxlen = std::max(g.maxlen, pats[i].len);
            if (pats[i].len > (uint32_t)kFastMaxLen) g.generic = true;
        }
        groups.push_back(std::move(g));
    }
    std::stable_sort(groups.begin(), groups.end(), [](const Group &a, const Group &b) {
        if (a.generic != b.generic) return !a.generic;
        if (a.maxlen != b.maxlen) return a.maxlen < b.maxlen;
        return a.pid < b.pid;
    });
    for (auto &g : groups) plan->slot_pid.push_back(g.pid);
    std::vector<SlotGroup> fast = groups_fast(groups), lut, mat;
    for (SlotGroup &g : fast) {
        bool m = opt.mfma;
        for (int i : g.strands) m = m && mfma_eligible(pats[i]);
        (m ? mat : lut).push_back(std::move(g));
    }
    plan->slot_mfma.assign(groups.size(), 0);
    for (const SlotGroup &g : mat) plan->slot_mfma[g.slot] = 1;
    build_fast_tiles(*this, lut, opt.tile_blocks, plan);
    build_mfma_tiles(*this, mat, opt, plan);
    // --- generic (long) strands: one tile per pattern_id group, weights x5
    for (uint32_t gi = 0; gi < groups.size(); gi++) {
        const Group &g = groups[gi];
        if (!g.generic) continue;
        DevTile t{};
        t.first = (uint32_t)plan->gen_pats.size();
        t.slot_begin = gi;
        t.nslots = 1;
        t.lmin = UINT32_MAX;
        for (int i : g.strands) {
            const Pat &p = pats[i];
            if (p.len > 65535) return fail(TFBS_E_ARG, "pattern longer than 65535 columns");
            DevPattern d{};
            d.col_off = (uint32_t)(plan->gen_w.size() / 5);
            d.min_score = p.min_score;
            d.len = p.len;
            d.slot_local = 0;
            d.orig_index = (uint32_t)i;
            t.lmin = std::min<uint32_t>(t.lmin, p.len);
            plan->gen_pats.push_back(d);
            for (uint32_t j = 0; j < p.len; j++)
                for (int c = 0; c < 5; c++) plan->gen_w.push_back(c == 4 ? 0 : p.w5[5 * j + c]);
        }
        t.last = (uint32_t)plan->gen_pats.size();
        plan->gen_tiles.push_back(t);
    }
    for (auto &t : plan->fast_tiles) plan->max_tile_blocks = std::max(plan->max_tile_blocks, t.nblocks);
    return TFBS_OK;
}

}  // namespace tfbs

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
using tfbs::Patterns;

extern "C" {

struct tfbs_patterns {
    Patterns p;
};

const char *tfbs_last_error(void) { return tfbs::g_last_error.c_str(); }

const char *tfbs_version(void) { return "find-tfbs_amd 0.1 (gfx950)"; }

const char *tfbs_strerror(int code) {
    switch (code) {
    case TFBS_OK: return "ok";
    case TFBS_E_ARG: return "bad argument";
    case TFBS_E_BADBASE: return "unknown nucleotide";
    case TFBS_E_REFMISMATCH: return "variant REF does not match the reference genome";
    case TFBS_E_MNP: return "missing case in haplotype patcher (MNP)";
    case TFBS_E_PLOIDY: return "inconsistent number of alleles";
    case TFBS_E_RANGE: return "region out of range";
    case TFBS_E_PARSE: return "parse error";
    case TFBS_E_IO: return "I/O error";
    case TFBS_E_HIP: return "HIP error";
    case TFBS_E_NODEVICE: return "no HIP device";
    case TFBS_E_ALLELES: return "record has a single allele";
    case TFBS_E_ZEROLEN: return "length-0 PWM with a negative min_score";
    case TFBS_E_NOPATTERN: return "no pattern";
    case TFBS_E_STATE: return "bad call order";
    case TFBS_E_NOMEM: return "out of memory";
    default: return "unknown error";
    }
}

int tfbs_parse_weight(const char *s, int32_t *out) {
    if (!s || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    return tfbs::parse_weight(s, out);
}

int tfbs_parse_threshold_file(const char *path, float thr, int32_t *out) {
    if (!path || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    return tfbs::parse_threshold_file(path, thr, out);
}

int tfbs_patterns_create(const tfbs_pattern_desc *d, size_t n, tfbs_patterns **out) {
    if (!out || (n && !d)) return tfbs::fail(TFBS_E_ARG, "null argument");
    auto *ps = new tfbs_patterns();
    for (size_t i = 0; i < n; i++) {
        tfbs::Pat p;
        p.kind = d[i].kind;
        p.direction = d[i].direction;
        p.pattern_id = d[i].pattern_id;
        p.min_score = d[i].min_score;
        p.len = d[i].kind == TFBS_KIND_PWM ? d[i].length : 0;
        p.name = d[i].name ? d[i].name : "";
        if (p.kind != TFBS_KIND_PWM && p.kind != TFBS_KIND_OTHER) {
            delete ps;
            return tfbs::fail(TFBS_E_ARG, "unknown pattern kind");
        }
        if (p.len && !d[i].weights) {
            delete ps;
            return tfbs::fail(TFBS_E_ARG, "PWM without weights");
        }
        p.w5.resize(5 * (size_t)p.len);
        for (size_t j = 0; j < p.len; j++) {
            for (int c = 0; c < 4; c++) p.w5[5 * j + c] = d[i].weights[5 * j + c];
            p.w5[5 * j + 4] = 0;  // Weight::new forces N = 0 (types.rs:109-113)
        }
        ps->p.add(p);
    }
    *out = ps;
    return TFBS_OK;
}

int tfbs_patterns_from_files(const char *pwm_file, const char *thr_dir, float thr, const char *names_csv,
                             int add_reverse, tfbs_patterns **out) {
    if (!pwm_file || !thr_dir || !names_csv || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    std::vector<std::string> wanted;
    std::string s(names_csv);
    size_t a = 0;
    for (;;) {  // split(',') keeps empty pieces (main.rs:197)
        size_t c = s.find(',', a);
        wanted.push_back(s.substr(a, c == std::string::npos ? std::string::npos : c - a));
        if (c == std::string::npos) break;
        a = c + 1;
    }
    auto *ps = new tfbs_patterns();
    int rc = tfbs::parse_pwm_files(pwm_file, thr_dir, thr, wanted, add_reverse != 0, &ps->p);
    if (rc) {
        delete ps;
        return rc;
    }
    *out = ps;
    return TFBS_OK;
}

size_t tfbs_patterns_count(const tfbs_patterns *p) { return p ? p->p.pats.size() : 0; }

int tfbs_patterns_get(const tfbs_patterns *p, size_t i, tfbs_pattern_desc *out) {
    if (!p || !out || i >= p->p.pats.size()) return tfbs::fail(TFBS_E_ARG, "bad pattern index");
    const tfbs::Pat &q = p->p.pats[i];
    out->pattern_id = q.pattern_id;
    out->direction = (uint8_t)q.direction;
    out->kind = (uint8_t)q.kind;
    out->length = q.len;
    out->weights = q.w5.empty() ? nullptr : q.w5.data();
    out->min_score = q.min_score;
    out->name = q.name.c_str();
    return TFBS_OK;
}

const char *tfbs_patterns_name_of(const tfbs_patterns *p, uint16_t pid) {
    if (!p) return nullptr;
    auto it = p->p.names.find(pid);
    return it == p->p.names.end() ? nullptr : it->second.c_str();
}

uint32_t tfbs_patterns_max_length(const tfbs_patterns *p) { return p ? p->p.max_length() : 0; }

void tfbs_patterns_destroy(tfbs_patterns *p) { delete p; }

int tfbs_patterns_plan_stats(const tfbs_patterns *p, uint32_t tile_blocks, int mfma, tfbs_plan_stats *out) {
    if (!p || !out) return tfbs::fail(TFBS_E_ARG, "null argument");
    tfbs::Plan plan;
    tfbs::PlanOptions opt;
    opt.tile_blocks = tile_blocks;
    opt.mfma = mfma != 0;
    int rc = p->p.build_plan(opt, &plan);
    if (rc) return rc;
    *out = tfbs_plan_stats{};
    out->n_octet_strands = plan.n_octet_strands;
    out->n_quad_strands = plan.n_quad_strands;
    out->n_generic_strands = (uint32_t)plan.gen_pats.size();
    out->n_fast_tiles = (uint32_t)plan.fast_tiles.size();
    out->n_fast_units = (uint32_t)plan.fast_units.size();
    out->n_generic_tiles = (uint32_t)plan.gen_tiles.size();
    out->max_tile_blocks = plan.max_tile_blocks;
    out->lut_bytes = (uint64_t)plan.lut.size() * 4;
    out->n_mfma_strands = plan.n_mfma_strands;
    out->n_mfma_tiles = plan.n_mfma_tiles;
    out->n_mfma_supers = (uint32_t)plan.m_supers.size();
    return TFBS_OK;
}

int tfbs_patterns_mfma_bound(const tfbs_patterns *p, size_t i, const uint8_t *bases, tfbs_mfma_bound *out) {
    if (!p || !out || (!bases && i < p->p.pats.size() && p->p.pats[i].len))
        return tfbs::fail(TFBS_E_ARG, "null argument");
    if (i >= p->p.pats.size()) return tfbs::fail(TFBS_E_ARG, "pattern index out of range");
    const tfbs::Pat &pat = p->p.pats[i];
    *out = tfbs_mfma_bound{};
    for (uint32_t j = 0; j < pat.len; j++)
        if (bases[j] > 4) return tfbs::fail(TFBS_E_ARG, "base code above 4");
    if (!tfbs::mfma_eligible(pat)) return TFBS_OK;
    out->eligible = 1;
    tfbs::mfma_window_bound(pat, bases, &out->q8, &out->t8, &out->scale, &out->c);
    return TFBS_OK;
}

}  // extern "C"

namespace tfbs {
const Patterns &patterns_of(const tfbs_patterns *p) { return p->p; }
}  // namespace tfbs
