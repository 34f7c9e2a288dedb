// Fast-path tiles: pack PWM strands (L <= 32) into units of interleaved 4-mer
// tables for scan_fast_kernel.
//
// A strand of length L has ceil(L/4) blocks; block b maps a 4-mer code (bases
// i+4b..i+4b+3, first base in the low bits) to the sum of the 4 column weights.
// Two unit kinds:
//  * OCTET16 (8 strands, 16-bit entries): each block is biased by its maximum,
//    e = sum - max_b <= 0, so the window sum S' = score - sum_b(max_b) <= 0 and a
//    saturating signed 16-bit accumulation returns max(S', -32768) exactly (all
//    terms are <= 0).  The reference's test score > min_score becomes
//    S' > thr with thr = min_score - sum_b(max_b), exact whenever thr >= -32768
//    (and every block's range fits 16 bits).  The kernel starts each half at
//    -(thr + 1) in [-1, 32767] instead of 0: the partial sums only decrease, so
//    the final half is >= 0 exactly when S' > thr (no clamp can have happened
//    on the way), and clamped results stay negative.  Typical HOCOMOCO strands qualify:
//    the 1e-4 threshold sits a few thousand milli-units below the maximum.
//  * QUAD32 (4 strands, 32-bit entries, wrapping sums): every other strand.
// Both kinds use 4 KiB blocks (256 codes x 16 bytes), read with one
// ds_read_b128 per lookup.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <vector>

#include "patterns.hpp"
#include "tfbs_internal.hpp"

namespace tfbs {

namespace {

struct StrandTab {
    bool oct = false;
    uint32_t nblk = 0;
    std::vector<int32_t> sum;   // nblk x 256, wrapping i32 sums (QUAD32 entries)
    std::vector<int16_t> e16;   // nblk x 256, biased entries (OCTET16)
    int32_t thr16 = 0;
};

StrandTab make_tab(const Pat &p) {
    StrandTab t;
    t.nblk = (p.len + 3) / 4;
    t.sum.resize((size_t)t.nblk * kLutEntries);
    std::vector<int64_t> exact((size_t)t.nblk * kLutEntries);
    int64_t sum_max = 0, mag = 0;
    bool fits = true;
    for (uint32_t b = 0; b < t.nblk; b++) {
        int64_t bmax = INT64_MIN, bmin = INT64_MAX;
        for (int code = 0; code < kLutEntries; code++) {
            uint32_t w = 0;
            int64_t x = 0;
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t col = 4 * b + j;
                if (col >= p.len) break;
                const int32_t v = p.w5[5 * col + ((code >> (2 * j)) & 3)];
                w += (uint32_t)v;
                x += v;
            }
            t.sum[(size_t)b * kLutEntries + code] = (int32_t)w;
            exact[(size_t)b * kLutEntries + code] = x;
            bmax = std::max(bmax, x);
            bmin = std::min(bmin, x);
        }
        if (bmax - bmin > 32767) fits = false;
        sum_max += bmax;
        mag += std::max(std::llabs(bmax), std::llabs(bmin));
    }
    const int64_t thr = (int64_t)p.min_score - sum_max;
    // no i32 wrap anywhere (the reference sums in i32) and a representable threshold
    if (fits && mag < (1ll << 30) && thr >= -32768) {
        t.oct = true;
        t.thr16 = (int32_t)std::min<int64_t>(thr, 0);  // thr >= 0: S' <= 0 never exceeds it
        t.e16.resize(exact.size());
        for (uint32_t b = 0; b < t.nblk; b++) {
            int64_t bmax = INT64_MIN;
            for (int code = 0; code < kLutEntries; code++) bmax = std::max(bmax, exact[(size_t)b * kLutEntries + code]);
            for (int code = 0; code < kLutEntries; code++)
                t.e16[(size_t)b * kLutEntries + code] = (int16_t)(exact[(size_t)b * kLutEntries + code] - bmax);
        }
    }
    return t;
}

}  // namespace

void build_fast_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, uint32_t tile_blocks, Plan *plan) {
    std::vector<StrandTab> tabs(P.pats.size());
    for (auto &g : groups)
        for (int i : g.strands) {
            tabs[i] = make_tab(P.pats[i]);
        }
    // blocks a tile needs: octet-eligible strands in chunks of 8, the rest in chunks of 4
    auto need = [&](const std::vector<int> &strands) {
        uint32_t total = 0;
        for (int pass = 0; pass < 2; pass++) {
            const size_t per = pass == 0 ? 8 : 4;
            std::vector<int> v;
            for (int i : strands)
                if (tabs[i].oct == (pass == 0)) v.push_back(i);
            for (size_t u = 0; u < v.size(); u += per) {
                uint32_t m = 0;
                for (size_t s = u; s < std::min(v.size(), u + per); s++) m = std::max(m, tabs[v[s]].nblk);
                total += m;
            }
        }
        return total;
    };
    std::vector<int> cur;
    std::vector<uint32_t> cur_slot;
    uint32_t slot_begin = 0;
    auto close_tile = [&]() {
        if (cur.empty()) return;
        DevTile t{};
        t.first = (uint32_t)plan->fast_units.size();
        t.lut_begin = (uint32_t)(plan->lut.size() / kBlockInts);
        t.slot_begin = slot_begin;
        t.lmin = UINT32_MAX;
        uint32_t maxslot = 0;
        for (int pass = 0; pass < 2; pass++) {
            const bool oct = pass == 0;
            const size_t per = oct ? 8 : 4;
            std::vector<size_t> idx;
            for (size_t k = 0; k < cur.size(); k++)
                if (tabs[cur[k]].oct == oct) idx.push_back(k);
            for (size_t u0 = 0; u0 < idx.size(); u0 += per) {
                DevUnit U{};
                U.kind = oct ? UNIT_OCTET16 : UNIT_QUAD32;
                U.lut_off = (uint32_t)(plan->lut.size() / kBlockInts) - t.lut_begin;
                const size_t n = std::min(per, idx.size() - u0);
                U.nstrand = (uint32_t)n;
                for (size_t s = 0; s < (size_t)kUnitMax; s++) {
                    if (s < n) {
                        const int i = cur[idx[u0 + s]];
                        const Pat &p = P.pats[i];
                        U.nblk = std::max(U.nblk, tabs[i].nblk);
                        U.thr[s] = oct ? tabs[i].thr16 : p.min_score;
                        U.min_score[s] = p.min_score;
                        U.len[s] = p.len;
                        U.slot_local[s] = cur_slot[idx[u0 + s]] - slot_begin;
                        U.orig_index[s] = (uint32_t)i;
                        U.wofs[s] = (uint32_t)(plan->wfull.size() / 4);
                        for (uint32_t j = 0; j < p.len; j++)
                            for (int c = 0; c < 4; c++) plan->wfull.push_back(p.w5[5 * j + c]);
                        t.lmin = std::min(t.lmin, p.len);
                        maxslot = std::max(maxslot, cur_slot[idx[u0 + s]]);
                        if (oct) plan->n_octet_strands++;
                        else plan->n_quad_strands++;
                    } else {  // padding strand: never matches
                        U.thr[s] = oct ? 0 : INT32_MAX;
                        U.min_score[s] = INT32_MAX;
                        U.len[s] = 0;
                        U.slot_local[s] = 0;
                        U.orig_index[s] = 0xFFFFFFFFu;
                        U.wofs[s] = 0;
                    }
                }
                if (oct)  // accumulator start -(thr + 1): a strand hits iff its final half is >= 0
                    for (int d = 0; d < 4; d++)
                        U.init[d] = (uint32_t)(uint16_t)(int16_t)(-(U.thr[2 * d] + 1)) |
                                    ((uint32_t)(uint16_t)(int16_t)(-(U.thr[2 * d + 1] + 1)) << 16);
                for (uint32_t b = 0; b < U.nblk; b++) {
                    for (int code = 0; code < kLutEntries; code++) {
                        if (oct) {
                            uint16_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                            for (size_t s = 0; s < n; s++) {
                                const StrandTab &T = tabs[cur[idx[u0 + s]]];
                                if (b < T.nblk) h[s] = (uint16_t)T.e16[(size_t)b * kLutEntries + code];
                            }
                            for (int d = 0; d < 4; d++)
                                plan->lut.push_back((int32_t)((uint32_t)h[2 * d] | ((uint32_t)h[2 * d + 1] << 16)));
                        } else {
                            for (size_t s = 0; s < 4; s++) {
                                int32_t v = 0;
                                if (s < n) {
                                    const StrandTab &T = tabs[cur[idx[u0 + s]]];
                                    if (b < T.nblk) v = T.sum[(size_t)b * kLutEntries + code];
                                }
                                plan->lut.push_back(v);
                            }
                        }
                    }
                }
                plan->fast_units.push_back(U);
            }
        }
        t.last = (uint32_t)plan->fast_units.size();
        t.nblocks = (uint32_t)(plan->lut.size() / kBlockInts) - t.lut_begin;
        t.nslots = maxslot - slot_begin + 1;
        plan->fast_tiles.push_back(t);
        cur.clear();
        cur_slot.clear();
    };
    for (const SlotGroup &g : groups) {
        if (!cur.empty()) {
            std::vector<int> trial = cur;
            trial.insert(trial.end(), g.strands.begin(), g.strands.end());
            if (need(trial) > tile_blocks || g.slot - slot_begin + 1 > (uint32_t)kMaxTileSlots) close_tile();
        }
        if (cur.empty()) slot_begin = g.slot;
        for (int i : g.strands) {
            cur.push_back(i);
            cur_slot.push_back(g.slot);
        }
    }
    close_tile();
}

}  // namespace tfbs
