// Host pattern list and the device plan derived from it.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "tfbs_internal.hpp"

namespace tfbs {

struct Pat {  // Pattern (types.rs:86-90)
    int kind = TFBS_KIND_PWM;
    int direction = TFBS_DIR_P;
    uint16_t pattern_id = 0;
    int32_t min_score = 0;
    uint32_t len = 0;
    std::vector<int32_t> w5;  // len x [A,C,G,T,N=0]
    std::string name;
};

struct Plan {
    std::vector<uint16_t> slot_pid;  // slot -> pattern_id
    std::vector<uint8_t> slot_mfma;  // slot -> 1 if the matrix-core kernel scores it (sparse hits), 0: LUT/generic
    std::vector<DevUnit> fast_units;
    std::vector<DevTile> fast_tiles;
    std::vector<int32_t> lut;        // blocks x 256 codes x 16 bytes (8 x int16 or 4 x int32)
    std::vector<int32_t> wfull;      // per fast-strand column: [A,C,G,T] weights (windows containing N)
    std::vector<DevPattern> gen_pats;
    std::vector<DevTile> gen_tiles;
    std::vector<int32_t> gen_w;      // per generic column: 5 weights
    uint32_t max_tile_blocks = 0;
    uint32_t n_octet_strands = 0;
    uint32_t n_quad_strands = 0;
    // matrix-core path (mfma.cpp, scan_mfma.hip)
    std::vector<DevMSuper> m_supers;
    uint32_t n_mfma_tiles = 0;
    std::vector<int32_t> m_image;    // per super tile: B fragments + strand metadata (LDS image)
    std::vector<int32_t> m_weights;  // per MFMA strand: exact [A,C,G,T] weights per column (candidate rescoring)
    std::vector<int32_t> m_meta;     // per MFMA tile: kGMetaInts rescoring fields (tfbs_internal.hpp)
    uint32_t max_super_bytes = 0;
    uint32_t n_mfma_strands = 0;
    bool zero_len_panics = false;
};

struct PlanOptions {
    uint32_t tile_blocks = 20;          // LUT tile: 4 KiB table blocks per workgroup
    bool mfma = false;                  // score eligible strands on the matrix cores
    uint32_t mfma_lds_bytes = 64 * 1024;  // LDS image budget of one MFMA super tile
    uint32_t mfma_lds_by_nk[9] = {};      // per K depth (chunks 1-4), overrides mfma_lds_bytes when set
};

struct Patterns {
    std::vector<Pat> pats;
    std::map<uint16_t, std::string> names;
    void add(const Pat &p);
    uint32_t max_length() const;
    int build_plan(const PlanOptions &opt, Plan *plan) const;
    // the plan's slot order (slot -> pattern id) and zero_len_panics, built once per
    // pattern set and shared by every batch made from it (tfbs_batch_create)
    int slot_order(std::vector<uint16_t> &slot_pid, bool &zero_len_panics) const;

  private:
    struct SlotCache {
        std::mutex mu;
        bool built = false;
        int rc = 0;
        std::vector<uint16_t> slot_pid;
        bool zero_len_panics = false;
    };
    std::shared_ptr<SlotCache> slot_cache = std::make_shared<SlotCache>();
};

struct SlotGroup {  // the strands of one pattern_id and its count slot
    uint32_t slot;
    std::vector<int> strands;
};
void build_fast_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, uint32_t tile_blocks, Plan *plan);
// Strands the int8 one-hot formulation scores exactly (L <= 32, every weight
// splits as 64 a + b with a, b int8).
bool mfma_eligible(const Pat &p);
// The bound of one window (bases 0-4, 4 = N): 8 Q, t8, scale, C (mfma.cpp)
void mfma_window_bound(const Pat &p, const uint8_t *bases, int64_t *q8, int64_t *t8, int64_t *scale, int64_t *c);
void build_mfma_tiles(const Patterns &P, const std::vector<SlotGroup> &groups, const PlanOptions &opt, Plan *plan);

int parse_weight(const std::string &s, int32_t *out);
int parse_threshold_file(const std::string &path, float thr, int32_t *out);
int parse_pwm_files(const std::string &pwm_file, const std::string &thr_dir, float thr,
                    const std::vector<std::string> &wanted, bool add_reverse, Patterns *out);
const Patterns &patterns_of(const tfbs_patterns *p);

}  // namespace tfbs
