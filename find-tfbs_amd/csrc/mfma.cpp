// Matrix-core plan: pack PWM strands into 32-strand tiles of FP6 B fragments
// for scan_mfma_kernel (scan_mfma.hip).
//
// apply_pwm (pattern.rs:125-135) is score(i) = sum_j w[j][nuc(i + j)], N = 0.
// With the window's bases one-hot encoded (4 entries per column, all zero for
// N), that is a dot product of a 0/1 vector with the strand's weights.  The
// kernel computes an upper bound of it on the matrix cores at the FP4/FP6
// rate: per column c_j = max(0, max_base w_j), w' = w - c_j <= 0, and each w'
// is replaced by s q with q an FP6 (e2m3) value, q >= w' / s (magnitude
// rounded down onto the FP6 grid), s = ceil(2 max |w'| / 15) so that
// |w'| / s <= 7.5.  Then score <= C + s Q, C = sum c_j, Q = sum q over the
// window's non-N columns (an N column adds 0 <= c_j), and Q is an exact f32
// sum of multiples of 1/8.  A window can hit (score > min_score,
// pattern.rs:151) only if Q > thr = floor(8 (min_score - C) / s) / 8; those
// candidates are rescored exactly (i32 sum of the weights, m_weights), so the
// FP6 digits only ever select work.  Weights whose sum could wrap i32 go to
// the LUT path (the reference wraps; the bound would not).
#include <algorithm>
#include <climits>
#include <cstring>
#include <thread>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

namespace {

struct Split {
    float thr = 1e9f;
    int64_t t8 = 0, scale = 1, c = 0;
    std::vector<uint8_t> code;  // len x 4 (A, C, G, T) FP6 e2m3 codes
};

int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// The FP6 e2m3 magnitudes x 8: 0..7 (subnormal), 8..15, 16..30 step 2, 32..60 step 4
constexpr int kF6Grid8[32] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                              16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48, 52, 56, 60};

// Digits and threshold of the bound for one scale.  Magnitudes beyond the
// grid clip to 7.5 (still q >= w' / s: the bound only loosens).
Split split_at(const Pat &p, const std::vector<int64_t> &c, int64_t cs, int64_t scale) {
    Split s;
    s.code.resize(4 * p.len);
    for (uint32_t j = 0; j < p.len; j++)
        for (int b = 0; b < 4; b++) {
            const int64_t mag8 = 8 * (c[j] - p.w5[5 * j + b]);  // 8 |w'|
            int g = 0;  // the largest grid magnitude with s g <= |w'|
            while (g + 1 < 32 && kF6Grid8[g + 1] * scale <= mag8) g++;
            s.code[4 * j + b] = (uint8_t)(g ? 0x20 | g : 0);  // negative: sign bit 5; code g encodes kF6Grid8[g] / 8
        }
    // |Q| <= 7.5 x 32, so clamping changes no outcome
    const int64_t t8 = floor_div(8 * ((int64_t)p.min_score - cs), scale);
    s.t8 = std::max<int64_t>(-(1 << 14), std::min<int64_t>(1 << 14, t8));
    s.thr = (float)s.t8 / 8.0f;
    s.scale = scale;
    s.c = cs;
    return s;
}

// P(a window is a candidate) under uniform bases: the distribution of
// G = -8 Q = sum of the columns' grid magnitudes x 8, by convolution.
double candidate_rate(const Pat &p, const Split &s) {
    std::vector<double> d(1, 1.0), e;
    for (uint32_t j = 0; j < p.len; j++) {
        e.assign(d.size() + 60, 0.0);
        for (int b = 0; b < 4; b++) {
            const int g8 = kF6Grid8[s.code[4 * j + b] & 31];
            for (size_t x = 0; x < d.size(); x++) e[x + g8] += 0.25 * d[x];
        }
        d.swap(e);
    }
    // candidate iff Q8 = -G > t8, i.e. G < -t8
    double r = 0;
    for (size_t x = 0; x < d.size() && (int64_t)x < -s.t8; x++) r += d[x];
    return r;
}

// The bound's scale: s0 = ceil(2 max|w'| / 15) keeps every digit on the grid;
// smaller scales resolve the small |w'| (the near-best bases that decide the
// windows near the threshold) more finely and clip the large ones.  The scale
// with the fewest candidates under uniform bases is kept.
Split split_weights(const Pat &p) {
    std::vector<int64_t> c(p.len);
    int64_t mx = 0, cs = 0;
    for (uint32_t j = 0; j < p.len; j++) {
        int64_t m = 0;  // N weighs 0
        for (int b = 0; b < 4; b++) m = std::max<int64_t>(m, p.w5[5 * j + b]);
        c[j] = m;
        cs += m;
        for (int b = 0; b < 4; b++) mx = std::max<int64_t>(mx, m - p.w5[5 * j + b]);
    }
    const int64_t s0 = std::max<int64_t>(1, (2 * mx + 14) / 15);
    Split best = split_at(p, c, cs, s0);
    double best_rate = candidate_rate(p, best);
    for (const double f : {0.85, 0.72, 0.6, 0.5, 0.42, 0.35, 0.3, 0.25}) {
        const int64_t sc = std::max<int64_t>(1, (int64_t)(s0 * f));
        if (sc == s0) continue;
        Split t = split_at(p, c, cs, sc);
        const double r = candidate_rate(p, t);
        if (r < best_rate) {
            best_rate = r;
            best = std::move(t);
        }
    }
    return best;
}

// FP6 bits of element e (column 4 t + base) of a lane's 192-bit B vector
void put6(uint8_t *frag_lo, uint8_t *frag_hi, int e, uint8_t code) {
    uint32_t bit = 6 * e;
    for (int k = 0; k < 6; k++, bit++) {
        if (!((code >> k) & 1)) continue;
        uint8_t *byte = bit < 128 ? frag_lo + bit / 8 : frag_hi + (bit - 128) / 8;
        *byte |= (uint8_t)(1u << (bit % 8));
    }
}

}  // namespace

void mfma_window_bound(const Pat &p, const uint8_t *bases, int64_t *q8, int64_t *t8, int64_t *scale, int64_t *c) {
    const Split s = split_weights(p);
    int64_t g = 0;
    for (uint32_t j = 0; j < p.len; j++)
        if (bases[j] < 4) g += kF6Grid8[s.code[4 * j + bases[j]] & 31];  // an N column adds 0
    *q8 = -g;
    *t8 = s.t8;
    *scale = s.scale;
    *c = s.c;
}

bool mfma_eligible(const Pat &p) {
    if (p.kind != TFBS_KIND_PWM || p.len == 0 || p.len > (uint32_t)(kMMaxChunks * kMChunkCols)) return false;
    int64_t span = 0;  // the largest |sum| any window can reach: below 2^31, no i32 wrap
    for (uint32_t j = 0; j < p.len; j++) {
        int64_t m = 0;
        for (int c = 0; c < 4; c++) m = std::max<int64_t>(m, std::abs((int64_t)p.w5[5 * j + c]));
        span += m;
    }
    return span < INT32_MAX;
}

void build_mfma_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, const PlanOptions &opt, Plan *plan) {
    // strands in slot order (slots are sorted by length, so tiles pack similar lengths)
    std::vector<std::pair<int, uint32_t>> strands;  // (pattern index, slot)
    for (const SlotGroup &g : groups)
        for (int i : g.strands) strands.push_back({i, g.slot});
    if (strands.empty()) return;
    std::vector<Split> split(strands.size());
    std::vector<uint32_t> woff(strands.size());
    {  // the scale search convolves score distributions: spread strands over threads
        const size_t nt = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
        std::vector<std::thread> pool;
        for (size_t t = 0; t < nt; t++)
            pool.emplace_back([&, t] {
                for (size_t s = t; s < strands.size(); s += nt) split[s] = split_weights(P.pats[strands[s].first]);
            });
        for (auto &th : pool) th.join();
    }
    for (size_t s = 0; s < strands.size(); s++) {
        const Pat &p = P.pats[strands[s].first];
        woff[s] = (uint32_t)plan->m_weights.size();
        for (uint32_t j = 0; j < p.len; j++)
            for (int c = 0; c < 4; c++) plan->m_weights.push_back(p.w5[5 * j + c]);
        // zero columns up to a multiple of 8: the rescoring loop reads whole blocks
        plan->m_weights.resize(plan->m_weights.size() + 4 * ((8 - p.len % 8) % 8), 0);
    }

    struct TileSrc { size_t first, count; uint32_t nk, lmin; };
    std::vector<TileSrc> tiles;
    for (size_t s = 0; s < strands.size(); s += kMStrands) {
        TileSrc t{s, std::min<size_t>(kMStrands, strands.size() - s), 0, UINT32_MAX};
        for (size_t k = 0; k < t.count; k++) {
            const Pat &p = P.pats[strands[s + k].first];
            t.nk = std::max<uint32_t>(t.nk, (p.len + kMChunkCols - 1) / kMChunkCols);
            t.lmin = std::min(t.lmin, p.len);
        }
        tiles.push_back(t);
    }
    size_t ti = 0;
    while (ti < tiles.size()) {
        // a super tile: consecutive tiles of the same K depth within the LDS budget
        const uint32_t nk = tiles[ti].nk;
        const uint32_t per = nk * kMFragBytes + kMMetaBytes;
        const uint32_t lds_bytes = std::max(per, opt.mfma_lds_by_nk[nk] ? opt.mfma_lds_by_nk[nk] : opt.mfma_lds_bytes);
        // the run of tiles with this depth, split into equal super tiles
        size_t run = ti;
        while (run < tiles.size() && tiles[run].nk == nk) run++;
        const size_t max_per_super = std::min<size_t>(kMSuperMaxTiles, std::max<size_t>(1, lds_bytes / per));
        const size_t n_super = (run - ti + max_per_super - 1) / max_per_super;
        const size_t tj = ti + (run - ti + n_super - 1) / n_super;
        const uint32_t count = (uint32_t)(tj - ti);
        DevMSuper S{};
        S.tile_count = count;
        S.nk = nk;
        S.img_off = (uint32_t)(plan->m_image.size() * 4);
        S.img_bytes = count * per;
        S.meta_off = count * nk * kMFragBytes;
        S.lmin = UINT32_MAX;
        S.tile0 = plan->n_mfma_tiles;
        std::vector<uint8_t> img(S.img_bytes, 0);
        for (uint32_t k = 0; k < count; k++) {
            const TileSrc &t = tiles[ti + k];
            const uint32_t b_off = k * nk * kMFragBytes, meta_off = S.meta_off + k * kMMetaBytes;
            S.lmin = std::min(S.lmin, t.lmin);
            float *thr = reinterpret_cast<float *>(&img[meta_off]);
            const size_t g0 = plan->m_meta.size();
            plan->m_meta.resize(g0 + kGMetaInts, 0);
            int32_t *gm = &plan->m_meta[g0];
            for (int n = 0; n < kMStrands; n++) {
                if ((size_t)n < t.count) {
                    const auto &st = strands[t.first + n];
                    const Pat &p = P.pats[st.first];
                    thr[n] = split[t.first + n].thr;
                    gm[kGMin + n] = p.min_score;
                    gm[kGWoff + n] = (int32_t)woff[t.first + n];
                    gm[kGLen + n] = (int32_t)p.len;
                    gm[kGSlot + n] = (int32_t)st.second;
                    gm[kGOrig + n] = st.first;
                    plan->n_mfma_strands++;
                } else {  // padding column: never a candidate
                    thr[n] = 1e9f;
                    gm[kGMin + n] = INT32_MAX;
                    gm[kGOrig + n] = -1;
                }
            }
            // B fragments: lane l holds column n = l & 31 and k = 32 h + 4 t + c,
            // h = l >> 5, <-> strand column 16 kc + 8 h + t, base c: element e =
            // 4 t + c at bits 6 e of the lane's 192 bits, dwords 0-3 at lane * 16,
            // dwords 4-5 at 1024 + lane * 8
            for (uint32_t kc = 0; kc < nk; kc++)
                for (int l = 0; l < 64; l++) {
                    const int n = l & 31, h = l >> 5;
                    if ((size_t)n >= t.count) continue;
                    const Pat &p = P.pats[strands[t.first + n].first];
                    const Split &sp = split[t.first + n];
                    uint8_t *lo = &img[b_off + kc * kMFragBytes + l * 16];
                    uint8_t *hi = &img[b_off + kc * kMFragBytes + 1024 + l * 8];
                    for (int tt = 0; tt < 8; tt++) {
                        const uint32_t col = kc * kMChunkCols + 8 * h + tt;
                        if (col >= p.len) continue;
                        for (int c = 0; c < 4; c++) put6(lo, hi, 4 * tt + c, sp.code[4 * col + c]);
                    }
                }
        }
        const size_t at = plan->m_image.size();
        plan->m_image.resize(at + (S.img_bytes + 3) / 4, 0);
        std::memcpy(&plan->m_image[at], img.data(), S.img_bytes);
        plan->max_super_bytes = std::max(plan->max_super_bytes, S.img_bytes);
        plan->n_mfma_tiles += count;
        plan->m_supers.push_back(S);
        ti = tj;
    }
}

}  // namespace tfbs
