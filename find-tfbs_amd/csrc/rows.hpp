// Row text of the VCF out (main.rs:415-429) as the device builds it: the host
// formats each row's head (everything before the per-sample genotype text) and
// each device-encoded key's per-value sample texts; the device writes the
// genotype text from the per-sample codes of tfbs_batch_encode and deflates
// the whole stream into BGZF blocks (bgzf_gpu.hip).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "batch.hpp"

namespace tfbs {

constexpr uint32_t kBgzfRaw = 65280;      // uncompressed bytes per BGZF block (bgzip's)
constexpr uint32_t kBgzfMax = 65536;      // bytes of a block, header and trailer included
constexpr uint32_t kRowTokBytes = 16;     // one sample text: at most 11 bytes, 16-byte slots

// One row: head bytes [head_off, head_off + head_len) of RowPlan::heads, then
// (enc != UINT32_MAX) geno_len bytes of genotype text -- sample s's text is slot
// code(s) of the row's token table (tok: its first slot, token_len its
// lengths) -- then '\n'.  A row the device did not encode carries its whole
// text in the head.
struct DevRow {
    uint64_t text_off;   // offset of the row in the stream
    uint64_t geno_len;
    uint64_t code_off;   // its key's packed codes (tfbs_batch_encode's compact buffer)
    uint32_t head_off, head_len;
    uint32_t tok;        // first token slot (RowPlan::tok_text / tok_len)
    uint32_t width;      // bits per code (2, 4, 8); 0: no genotype part on the device
    uint32_t cum_off;    // its per-64-sample byte offsets (bgzf_gpu.hip)
    uint32_t nv;         // token slots (distinct totals) of the key
};

struct RowPlan {
    std::string heads;                 // every row's head, back to back
    std::vector<DevRow> rows;
    std::vector<char> tok_text;        // kRowTokBytes per slot
    std::vector<uint8_t> tok_len;      // per slot
    uint64_t text_bytes = 0;           // of the whole stream
    uint64_t n_rows = 0;
};

// The rows of regions [r0, r1) after tfbs_batch_encode over them: heads (with
// "<chr>\t<POS>\t", POS from *fake, advanced per row), token tables and row
// metadata, regions formatted on `threads` host threads.
int build_row_plan(const Batch &B, size_t r0, size_t r1, const std::string &chrom, uint32_t min_maf,
                   uint32_t *fake, uint32_t threads, RowPlan &plan);
// build_row_plan in two steps: the rows of [r0, r1) without their POS (parallel;
// *n_rows of them), then the plan of a sub-range [r0, r1) of them with POS from
// *fake (serial, cheap) -- a caller that must know a call's row count before its
// POS base (the multi-device run flow's POS chain) builds the parts first.
struct RowParts;
int build_row_parts(const Batch &B, size_t r0, size_t r1, uint32_t min_maf, uint32_t threads,
                    std::shared_ptr<RowParts> &out, uint64_t *n_rows);
int plan_from_parts(const Batch &B, RowParts &P, size_t r0, size_t r1, const std::string &chrom, uint32_t *fake,
                    RowPlan &plan);
// tfbs_batch_rows_bgzf (device.hip) whose POS base is asked for once the call's rows
// are counted: pos_base(n_rows, &base) -- it may block -- sets *fake_position.
int rows_bgzf_chained(::tfbs_ctx *ctx, tfbs_batch *b, size_t r0, size_t r1, const char *chromosome,
                      uint32_t min_maf, uint32_t *fake_position, int fd, uint64_t *bytes, uint64_t *n_rows,
                      const std::function<int(uint64_t, uint32_t *)> &pos_base);
// Seconds the ctx's BGZF row calls spent draining: waiting for the device's blocks,
// for their copy back, and writing them out.
void rows_bgzf_drain_seconds(const ::tfbs_ctx *ctx, double out[3]);
// on: the ctx's BGZF row calls return before their last blocks are written (a writer
// thread writes them in order; the fd must stay open and untouched until rows_flush,
// which waits for every write and returns the first failure)
void rows_set_async(::tfbs_ctx *ctx, bool on);
int rows_flush(::tfbs_ctx *ctx);

}  // namespace tfbs
