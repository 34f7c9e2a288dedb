// Matrix-core plan: pack PWM strands into 32-strand tiles of int8 B fragments
// for scan_mfma_kernel (scan_mfma.hip).
//
// apply_pwm (pattern.rs:125-135) is score(i) = sum_j w[j][nuc(i + j)], N = 0.
// With the window's bases one-hot encoded (4 entries per column, all zero for
// N), that is a dot product of a 0/1 vector with the strand's weights.  The
// weights are split exactly as w = 64 a + b, b = ((w + 32) mod 64) - 32 in
// [-32, 31], a in [-128, 127]; each K chunk of 32 covers 4 columns twice, the
// one-hot with entries 1 against b and with entries 64 against a, so one MFMA
// per 4 columns accumulates the exact int32 score.  |score| <= 32 * 8224, so no
// intermediate wraps and the sum equals the reference's i32 sum.
#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

namespace {

inline int32_t lo_digit(int32_t w) { return ((w + 32) & 63) - 32; }
inline int32_t hi_digit(int32_t w) { return (w - lo_digit(w)) / 64; }

}  // namespace

bool mfma_eligible(const Pat &p) {
    if (p.kind != TFBS_KIND_PWM || p.len == 0 || p.len > (uint32_t)(kMMaxChunks * kMChunkCols)) return false;
    for (uint32_t j = 0; j < p.len; j++)
        for (int c = 0; c < 4; c++) {
            const int64_t w = p.w5[5 * j + c];
            if (w < -8224 || w > 8159) return false;  // 64 * [-128, 127] + [-32, 31]
        }
    return true;
}

void build_mfma_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, const PlanOptions &opt, Plan *plan) {
    // strands in slot order (slots are sorted by length, so tiles pack similar lengths)
    std::vector<std::pair<int, uint32_t>> strands;  // (pattern index, slot)
    for (const SlotGroup &g : groups)
        for (int i : g.strands) strands.push_back({i, g.slot});
    if (strands.empty()) return;

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
            int32_t *thr = reinterpret_cast<int32_t *>(&img[meta_off]);
            uint32_t *len = reinterpret_cast<uint32_t *>(&img[meta_off + 128]);
            uint32_t *slot = reinterpret_cast<uint32_t *>(&img[meta_off + 256]);
            uint32_t *orig = reinterpret_cast<uint32_t *>(&img[meta_off + 384]);
            for (int n = 0; n < kMStrands; n++) {
                if ((size_t)n < t.count) {
                    const auto &st = strands[t.first + n];
                    const Pat &p = P.pats[st.first];
                    thr[n] = p.min_score;
                    len[n] = p.len;
                    slot[n] = st.second;
                    orig[n] = (uint32_t)st.first;
                    plan->n_mfma_strands++;
                } else {  // padding column: never a hit
                    thr[n] = INT32_MAX;
                    len[n] = 0;
                    slot[n] = 0;
                    orig[n] = 0xFFFFFFFFu;
                }
            }
            // B fragments: lane l holds column n = l & 31, k = 16 d + j with
            // d = l >> 5 the digit (0: b, 1: a), j = 4 t + c <-> strand column
            // 4 kc + t, base c
            for (uint32_t kc = 0; kc < nk; kc++)
                for (int l = 0; l < 64; l++) {
                    const int n = l & 31, digit = l >> 5;
                    int8_t *frag = reinterpret_cast<int8_t *>(&img[b_off + kc * kMFragBytes + l * 16]);
                    if ((size_t)n >= t.count) continue;
                    const Pat &p = P.pats[strands[t.first + n].first];
                    for (int tt = 0; tt < 4; tt++) {
                        const uint32_t col = kc * kMChunkCols + tt;
                        if (col >= p.len) continue;
                        for (int c = 0; c < 4; c++) {
                            const int32_t w = p.w5[5 * col + c];
                            frag[4 * tt + c] = (int8_t)(digit == 0 ? lo_digit(w) : hi_digit(w));
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
