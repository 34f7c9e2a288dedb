// Matrix-core plan: pack PWM strands into 64-strand tiles of FP6 B fragments
// (two strands per GEMM column) for scan_mfma_kernel (scan_mfma.hip).
//
// apply_pwm (pattern.rs:125-135) is score(i) = sum_j w[j][nuc(i + j)], N = 0.
// With the window's bases one-hot encoded (4 entries per column, all zero for
// N), that is a dot product of a 0/1 vector with the strand's weights.  The
// kernel computes an upper bound of it on the matrix cores at the FP4/FP6
// rate: per column c_j = max(0, max_base w_j), w' = w - c_j <= 0, and each w'
// is replaced by s q with q an FP6 (e2m3) value, q >= w' / s (magnitude
// rounded down onto the FP6 grid, clipped at 7.5).  Then score <= C + s Q,
// C = sum c_j, Q = sum q over the window's non-N columns (an N column adds
// 0 <= c_j), and U = 8 Q is an integer.  A window can hit (score > min_score,
// pattern.rs:151) only if U > t8 = floor(8 (min_score - C) / s).
//
// Two strands share one output of the GEMM as two 11-bit fields (scan_mfma.hip),
// tested against one threshold T0 common to the super tile: each strand's
// scale is s = ceil(8 D / |T0|), D = C - min_score, so that t8 >= T0 and
// "U > T0" keeps every hit; its digits are clipped (still >= w' / s) until
// every window's U >= T0 - 1023, so that no field borrows from its neighbour.
// Candidates are rescored exactly (i32 sum of the weights, m_weights), so the
// FP6 digits only ever select work.  Weights whose sum could wrap i32 go to the
// LUT path (the reference wraps; the bound would not).
#include <algorithm>
#include <climits>
#include <cstring>
#include <thread>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

namespace {

// The FP6 e2m3 magnitudes x 8: 0..7 (subnormal), 8..15, 16..30 step 2, 32..60 step 4
constexpr int kF6Grid8[32] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                              16, 18, 20, 22, 24, 26, 28, 30, 32, 36, 40, 44, 48, 52, 56, 60};
// Candidate common thresholds T0 (units of 1/8 digit): coarser bounds for
// short strands, finer for long ones; the super tile keeps the best.
constexpr int kT0Choices[] = {-32, -48, -64, -96, -128, -160, -192, -256};

struct Split {
    int64_t t0 = -32, t8 = 0, scale = 1, c = 0;
    bool never = false;         // score > min_score is impossible: padding digits
    std::vector<uint8_t> gi;    // len x 4 (A, C, G, T): index into kF6Grid8 (the digit is -grid / 8)
};

int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// Digits of one strand for the common threshold t0 (see the file comment).
Split split_for(const Pat &p, int64_t t0) {
    Split s;
    s.t0 = t0;
    s.gi.assign(4 * p.len, 0);
    std::vector<int64_t> c(p.len);
    int64_t cs = 0;
    for (uint32_t j = 0; j < p.len; j++) {
        int64_t m = 0;  // N weighs 0
        for (int b = 0; b < 4; b++) m = std::max<int64_t>(m, p.w5[5 * j + b]);
        c[j] = m;
        cs += m;
    }
    s.c = cs;
    const int64_t D = cs - (int64_t)p.min_score;
    if (D <= 0) {  // score <= C <= min_score everywhere: no candidate is needed (the plan
        s.never = true;  // pads it); the digits below are still a sound bound
        int64_t mx = 0;
        for (uint32_t j = 0; j < p.len; j++)
            for (int b = 0; b < 4; b++) mx = std::max<int64_t>(mx, c[j] - p.w5[5 * j + b]);
        s.scale = std::max<int64_t>(1, (2 * mx + 14) / 15);
    } else {
        s.scale = std::max<int64_t>(1, (8 * D + (-t0) - 1) / (-t0));
    }
    s.t8 = floor_div(8 * ((int64_t)p.min_score - cs), s.scale);  // >= t0 unless never
    for (uint32_t j = 0; j < p.len; j++)
        for (int b = 0; b < 4; b++) {
            const int64_t mag8 = 8 * (c[j] - p.w5[5 * j + b]);  // 8 |w'|
            int g = 0;  // the largest grid magnitude with s g <= |w'|
            while (g + 1 < 32 && kF6Grid8[g + 1] * s.scale <= mag8) g++;
            s.gi[4 * j + b] = (uint8_t)g;
        }
    // field range: sum of the column maxima <= 1023 - t0 (cap the largest digits)
    const int64_t budget = kMFieldBias - t0;
    for (;;) {
        int64_t sum = 0;
        int top = 0;
        for (uint32_t j = 0; j < p.len; j++) {
            int m = 0;
            for (int b = 0; b < 4; b++) m = std::max<int>(m, s.gi[4 * j + b]);
            sum += kF6Grid8[m];
            top = std::max(top, m);
        }
        if (sum <= budget || top == 0) break;
        for (auto &g : s.gi) g = (uint8_t)std::min<int>(g, top - 1);
    }
    return s;
}

// P(U > t0) under uniform bases: the distribution of G = -U = sum of the
// columns' grid magnitudes x 8, truncated at -t0.
double candidate_rate(const Pat &p, const Split &s) {
    if (s.never) return 0.0;
    const size_t lim = (size_t)(-s.t0);
    std::vector<double> d(lim, 0.0), e(lim);
    d[0] = 1.0;
    for (uint32_t j = 0; j < p.len; j++) {
        std::fill(e.begin(), e.end(), 0.0);
        for (int b = 0; b < 4; b++) {
            const size_t g8 = (size_t)kF6Grid8[s.gi[4 * j + b]];
            for (size_t x = 0; x + g8 < lim; x++) e[x + g8] += 0.25 * d[x];
        }
        d.swap(e);
    }
    double r = 0;
    for (double x : d) r += x;
    return r;
}

// The T0 that minimises one strand's candidate rate (the diagnostic bound).
Split best_split(const Pat &p) {
    Split best;
    double br = 2.0;
    for (int t0 : kT0Choices) {
        Split s = split_for(p, t0);
        const double r = candidate_rate(p, s);
        if (r < br) {
            br = r;
            best = std::move(s);
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

uint32_t f32_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

}  // namespace

void mfma_window_bound(const Pat &p, const uint8_t *bases, int64_t *q8, int64_t *t8, int64_t *scale, int64_t *c) {
    const Split s = best_split(p);
    int64_t g = 0;
    for (uint32_t j = 0; j < p.len; j++)
        if (bases[j] < 4) g += kF6Grid8[s.gi[4 * j + bases[j]]];  // an N column adds 0
    *q8 = -g;
    *t8 = s.t0;
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
    constexpr size_t kNT0 = sizeof(kT0Choices) / sizeof(kT0Choices[0]);
    // every strand's candidate rate at every common threshold (convolutions over threads)
    std::vector<double> rate(strands.size() * kNT0);
    {
        const size_t nt = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
        std::vector<std::thread> pool;
        for (size_t t = 0; t < nt; t++)
            pool.emplace_back([&, t] {
                for (size_t s = t; s < strands.size(); s += nt) {
                    const Pat &p = P.pats[strands[s].first];
                    for (size_t k = 0; k < kNT0; k++) rate[s * kNT0 + k] = candidate_rate(p, split_for(p, kT0Choices[k]));
                }
            });
        for (auto &th : pool) th.join();
    }
    std::vector<uint32_t> woff(strands.size());
    for (size_t s = 0; s < strands.size(); s++) {
        const Pat &p = P.pats[strands[s].first];
        woff[s] = (uint32_t)plan->m_weights.size();
        for (uint32_t j = 0; j < p.len; j++)
            for (int c = 0; c < 4; c++) plan->m_weights.push_back(p.w5[5 * j + c]);
        // zero columns up to a multiple of 8: the rescoring loop reads whole blocks
        plan->m_weights.resize(plan->m_weights.size() + 4 * ((8 - p.len % 8) % 8), 0);
    }
    // the rescoring loads every block of 8 columns up to 32 (masked): the last
    // strand's reads stay in the buffer
    plan->m_weights.resize(plan->m_weights.size() + 4 * 32, 0);

    struct TileSrc { size_t first, count; uint32_t nk, lmin, lmax; };
    std::vector<TileSrc> tiles;
    for (size_t s = 0; s < strands.size(); s += kMStrands) {
        TileSrc t{s, std::min<size_t>(kMStrands, strands.size() - s), 0, UINT32_MAX, 0};
        for (size_t k = 0; k < t.count; k++) {
            const Pat &p = P.pats[strands[s + k].first];
            t.nk = std::max<uint32_t>(t.nk, (p.len + kMChunkCols - 1) / kMChunkCols);
            t.lmin = std::min(t.lmin, p.len);
            t.lmax = std::max(t.lmax, p.len);
        }
        tiles.push_back(t);
    }
    size_t ti = 0;
    while (ti < tiles.size()) {
        // a super tile: consecutive tiles of one depth class within the LDS budget
        const uint32_t nk = mfma_depth_class(tiles[ti].nk);
        const uint32_t lds_bytes = opt.mfma_lds_by_nk[nk] ? opt.mfma_lds_by_nk[nk] : opt.mfma_lds_bytes;
        // the run of tiles of this class, split into equal-sized super tiles
        size_t run = ti;
        uint64_t run_bytes = 0;
        while (run < tiles.size() && mfma_depth_class(tiles[run].nk) == nk) run_bytes += mfma_tile_bytes(tiles[run++].nk);
        const size_t n_super = std::max<size_t>((run - ti + kMSuperMaxTiles - 1) / kMSuperMaxTiles,
                                                (run_bytes + lds_bytes - 1) / std::max<uint32_t>(1, lds_bytes));
        const size_t per_super = (run - ti + n_super - 1) / n_super;
        size_t tj = ti;
        uint32_t img_bytes = 0;
        while (tj < run && tj - ti < per_super) img_bytes += mfma_tile_bytes(tiles[tj++].nk);
        const uint32_t count = (uint32_t)(tj - ti);
        // the common threshold with the fewest candidates over the super tile's strands
        size_t bk = 0;
        double br = -1;
        for (size_t k = 0; k < kNT0; k++) {
            double r = 0;
            for (size_t s = tiles[ti].first; s < tiles[tj - 1].first + tiles[tj - 1].count; s++) r += rate[s * kNT0 + k];
            if (br < 0 || r < br) {
                br = r;
                bk = k;
            }
        }
        const int64_t t0 = kT0Choices[bk];
        DevMSuper S{};
        S.tile_count = count;
        S.nk = nk;
        S.img_off = (uint32_t)(plan->m_image.size() * 4);
        S.img_bytes = img_bytes;
        for (uint32_t d = 1; d <= 4; d++) {  // tiles are sorted by depth (strands by length)
            uint32_t e = 0;
            while (e < count && tiles[ti + e].nk <= d) e++;
            S.seg |= e << (8 * (d - 1));
        }
        S.t0 = (int32_t)t0;
        S.acc0 = f32_bits((float)((1 << 23) + (kMFieldBias - t0) * (1 + (1 << kMFieldBits))));
        S.lmin = UINT32_MAX;
        S.tile0 = plan->n_mfma_tiles;
        // padding digits (tile padding, strands that cannot hit): 7.5 at every base of
        // the first columns, so U <= t0 for windows without N there
        const uint32_t pad_cols = (uint32_t)((-t0) / 60 + 1);
        std::vector<uint8_t> img(S.img_bytes, 0);
        uint32_t b_off = 0;
        for (uint32_t k = 0; k < count; b_off += mfma_tile_bytes(tiles[ti + k].nk), k++) {
            const TileSrc &t = tiles[ti + k];
            S.lmin = std::min(S.lmin, t.lmin);
            S.lmax = std::max(S.lmax, t.lmax);
            const size_t g0 = plan->m_meta.size();
            plan->m_meta.resize(g0 + kGMetaInts, 0);
            int32_t *gm = &plan->m_meta[g0];
            gm[kGDepth] = (int32_t)nk;
            std::vector<Split> split(kMStrands);
            for (int n = 0; n < kMStrands; n++) {
                if ((size_t)n < t.count) {
                    const auto &st = strands[t.first + n];
                    const Pat &p = P.pats[st.first];
                    split[n] = split_for(p, t0);
                    gm[kGStrandInts * n + kGMin] = p.min_score;
                    gm[kGStrandInts * n + kGWoff] = (int32_t)woff[t.first + n];
                    gm[kGStrandInts * n + kGLen] = (int32_t)p.len;
                    gm[kGStrandInts * n + kGSlot] = (int32_t)st.second;
                    gm[kGOrig + n] = st.first;
                    plan->n_mfma_strands++;
                } else {  // padding strand: never a hit (L = 0 scores 0, not > INT32_MAX)
                    split[n].never = true;
                    gm[kGStrandInts * n + kGMin] = INT32_MAX;
                    gm[kGOrig + n] = -1;
                }
            }
            // B fragments: lane l holds column n = l & 31 (strands 2n, 2n+1) and
            // k = 32 h + 4 t + c, h = l >> 5, <-> strand 2 n + h, column
            // 8 kc + t, base c: element e = 4 t + c at bits 6 e of the lane's 192
            // bits, dwords 0-3 at kc * 1536 + lane * 16, dwords 4-5 at kc * 1536 +
            // 1024 + lane * 8 (mfma_tile_bytes)
            for (uint32_t kc = 0; kc < t.nk; kc++)
                for (int l = 0; l < 64; l++) {
                    const int sn = 2 * (l & 31) + (l >> 5);
                    const Split &sp = split[sn];
                    const uint32_t len = (size_t)sn < t.count ? P.pats[strands[t.first + sn].first].len : 0;
                    uint8_t *lo = &img[b_off + kc * 1536 + l * 16];
                    uint8_t *hi = &img[b_off + kc * 1536 + 1024 + l * 8];
                    for (int tt = 0; tt < kMChunkCols; tt++) {
                        const uint32_t col = kc * kMChunkCols + tt;
                        for (int c = 0; c < 4; c++) {
                            int g = 0;
                            if (sp.never) g = col < pad_cols ? 31 : 0;
                            else if (col < len) g = sp.gi[4 * col + c];
                            if (g) put6(lo, hi, 4 * tt + c, (uint8_t)(0x20 | g));  // negative: sign bit 5
                        }
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
