// Matrix-core plan: pack PWM strands into 32-strand tiles of int8 B fragments
// for scan_mfma_kernel (scan_mfma.hip).
//
// apply_pwm (pattern.rs:125-135) is score(i) = sum_j w[j][nuc(i + j)], N = 0.
// With the window's bases one-hot encoded (4 entries per column, all zero for
// N), that is a dot product of a 0/1 vector with the strand's weights.  Each
// strand gets a scale s = ceil(max |w| / 127) (1..255) and every weight splits
// exactly as w = s q + r, q = round(w / s) (halves away from zero) in
// [-127, 127], |r| <= s / 2.  The kernel sums Q = sum q over a window with one
// MFMA per 8 columns; since score = s Q + R and R <= E = sum over columns of
// max(0, max_base r), a window can only pass `score > min_score`
// (pattern.rs:151) when Q > thr_q = floor((min_score - E) / s).  Those
// candidates are rescored exactly (i32 sum of the weights, kept here in
// m_weights), so the coarse digits only ever select work.
#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

namespace {

struct Split {
    int32_t scale = 1, thr_q = INT32_MAX;
    std::vector<int8_t> q;  // len x 4 (A, C, G, T)
};

int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

Split split_weights(const Pat &p) {
    Split s;
    int32_t mx = 0;
    for (uint32_t j = 0; j < p.len; j++)
        for (int c = 0; c < 4; c++) mx = std::max<int32_t>(mx, std::abs(p.w5[5 * j + c]));
    s.scale = std::max<int32_t>(1, (mx + 126) / 127);
    s.q.resize(4 * p.len);
    int64_t e = 0;  // the largest residual a window can add (N adds 0)
    for (uint32_t j = 0; j < p.len; j++) {
        int32_t emax = 0;
        for (int c = 0; c < 4; c++) {
            const int32_t w = p.w5[5 * j + c], a = std::abs(w);
            const int32_t q = (w < 0 ? -1 : 1) * ((a + s.scale / 2) / s.scale);
            const int32_t r = w - s.scale * q;
            s.q[4 * j + c] = (int8_t)q;
            emax = std::max(emax, r);
        }
        e += emax;
    }
    // |Q| <= 127 x 32, so clamping to +-2^24 changes no outcome and keeps the
    // kernel's thr_q - Q from wrapping
    const int64_t t = floor_div((int64_t)p.min_score - e, s.scale);
    s.thr_q = (int32_t)std::max<int64_t>(-(1 << 24), std::min<int64_t>(1 << 24, t));
    return s;
}

}  // namespace

bool mfma_eligible(const Pat &p) {
    if (p.kind != TFBS_KIND_PWM || p.len == 0 || p.len > (uint32_t)(kMMaxChunks * kMChunkCols)) return false;
    for (uint32_t j = 0; j < p.len; j++)
        for (int c = 0; c < 4; c++) {
            const int64_t w = p.w5[5 * j + c];
            if (w < -127 * kMMaxScale || w > 127 * kMMaxScale) return false;  // s <= 255
        }
    return true;
}

void build_mfma_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, const PlanOptions &opt, Plan *plan) {
    // strands in slot order (slots are sorted by length, so tiles pack similar lengths)
    std::vector<std::pair<int, uint32_t>> strands;  // (pattern index, slot)
    for (const SlotGroup &g : groups)
        for (int i : g.strands) strands.push_back({i, g.slot});
    if (strands.empty()) return;
    std::vector<Split> split(strands.size());
    std::vector<uint32_t> woff(strands.size());
    for (size_t s = 0; s < strands.size(); s++) {
        const Pat &p = P.pats[strands[s].first];
        split[s] = split_weights(p);
        woff[s] = (uint32_t)plan->m_weights.size();
        for (uint32_t j = 0; j < p.len; j++)
            for (int c = 0; c < 4; c++) plan->m_weights.push_back(p.w5[5 * j + c]);
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
        std::vector<uint8_t> img(S.img_bytes, 0);
        for (uint32_t k = 0; k < count; k++) {
            const TileSrc &t = tiles[ti + k];
            const uint32_t b_off = k * nk * kMFragBytes, meta_off = S.meta_off + k * kMMetaBytes;
            S.lmin = std::min(S.lmin, t.lmin);
            int32_t *meta = reinterpret_cast<int32_t *>(&img[meta_off]);
            for (int n = 0; n < kMStrands; n++) {
                if ((size_t)n < t.count) {
                    const auto &st = strands[t.first + n];
                    const Pat &p = P.pats[st.first];
                    const Split &sp = split[t.first + n];
                    meta[kMetaThrQ + n] = sp.thr_q;
                    meta[kMetaMin + n] = p.min_score;
                    meta[kMetaWoff + n] = (int32_t)woff[t.first + n];
                    meta[kMetaLen + n] = (int32_t)p.len;
                    meta[kMetaSlot + n] = (int32_t)st.second;
                    meta[kMetaOrig + n] = st.first;
                    plan->n_mfma_strands++;
                } else {  // padding column: never a candidate
                    meta[kMetaThrQ + n] = 1 << 24;
                    meta[kMetaMin + n] = INT32_MAX;
                    meta[kMetaWoff + n] = 0;
                    meta[kMetaLen + n] = 0;
                    meta[kMetaSlot + n] = 0;
                    meta[kMetaOrig + n] = -1;
                }
            }
            // B fragments: lane l holds column n = l & 31 and k = 16 h + 4 t + c,
            // h = l >> 5, <-> strand column 8 kc + 4 h + t, base c
            for (uint32_t kc = 0; kc < nk; kc++)
                for (int l = 0; l < 64; l++) {
                    const int n = l & 31, h = l >> 5;
                    if ((size_t)n >= t.count) continue;
                    const Pat &p = P.pats[strands[t.first + n].first];
                    const Split &sp = split[t.first + n];
                    int8_t *fq = reinterpret_cast<int8_t *>(&img[b_off + kc * kMFragBytes + l * 16]);
                    for (int tt = 0; tt < 4; tt++) {
                        const uint32_t col = kc * kMChunkCols + 4 * h + tt;
                        if (col >= p.len) continue;
                        for (int c = 0; c < 4; c++) fq[4 * tt + c] = sp.q[4 * col + c];
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
