// Launch interface of the device BGZF row writer (bgzf_gpu.hip), used by device.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "rows.hpp"

namespace tfbs {

constexpr uint32_t kCumGroup = 64;  // samples per entry of a row's genotype text offsets
constexpr uint32_t kBgzfOps = 32;   // CRC32 shift operators of 2^k zero bytes, k < 32

struct BgArgs {
    const DevRow *rows;
    uint32_t n_rows;
    const char *heads;
    const char *tok_text;       // kRowTokBytes per token slot (bytes past the length zeroed: launch_tok_lit)
    const uint8_t *tok_len;
    uint4 *tok_lit;             // per token its literal codes (launch_tok_lit)
    uint8_t *tok_litn;          // and their bit count
    const uint8_t *codes;       // the encoded keys' packed codes (tfbs_batch_encode's compact buffer)
    uint32_t *cum;              // per row (DevRow::cum_off): (n_samples + 63) / 64 + 1 genotype text offsets
    uint32_t n_samples;
    uint64_t text_bytes;        // of the rows' stream
    uint64_t block0;            // first block of the launch
    uint8_t *out;               // kBgzfMax bytes per block of the launch
    uint32_t *out_len;          // the blocks' sizes
    const uint32_t *crc_tab;    // CRC32 byte table
    const uint32_t *crc_ops;    // kBgzfOps x 32 columns
    const uint32_t *crc_slice;  // slice-by-4 tables 1-3 (3 x 256; table 0 is crc_tab)
    const uint32_t *crc_lane;   // bgzf_wave_kernel's lane and wave shift operators (bgzf_crc_tables)
    uint32_t crc_full;          // x^(8 kBgzfRaw) applied to 0xFFFFFFFF (a full block's CRC init term)
    void *plans;                // per block of the launch: bgzf_plan_bytes() of scratch
    uint64_t *prof;             // optional (TFBS_BGZF_PROF): per block 32 words of phase clocks and counts
    uint32_t stored;            // TFBS_BGZF_STORED=1 (debug): bgzf_wave_kernel's blocks stored, its text as it is
    // TFBS_BGZF_CHECK=1 (debug): the checked bgzf_wave_kernel, which counts here every
    // block-text write that meets bits already set (the text is zeroed per block and
    // every byte written once, by an LDS OR: the invariant behind its race fix)
    uint32_t *check;
};
size_t bgzf_plan_bytes();

// CRC32 table, the x^(8 * 2^k) operators, the slice-by-4 tables 1-3 and the wave
// kernel's lane and wave operators (host side, uploaded once: 256 + 32 kBgzfOps + 768 +
// 32 x 64 + 32 x 16 words); returns crc_full.
constexpr size_t kBgzfCrcWords = 256 + 32 * kBgzfOps + 768 + 32 * 64 + 32 * 16;
uint32_t bgzf_crc_tables(uint32_t *tab, uint32_t *ops, uint32_t *slice, uint32_t *lane);
// Per token: the text's bytes past its length zeroed, its literal codes (tok_lit, tok_litn).
int launch_tok_lit(const BgArgs &a, uint32_t n_tok, hipStream_t stream);
// Per row: its genotype text offsets every 64 samples.
int launch_row_cum(const BgArgs &a, hipStream_t stream);
// Blocks [a.block0, a.block0 + n_blocks) of the stream, one workgroup each (after a
// planning kernel, one thread per block).
int launch_bgzf_blocks(const BgArgs &a, uint32_t n_blocks, hipStream_t stream);
// The blocks back to back: off[i] = the sizes len[] of the blocks before i (off[n_blocks] =
// their total), block i's bytes at off[i] of out.
int launch_bgzf_compact(const uint8_t *in, const uint32_t *len, uint64_t *off, uint32_t n_blocks, uint8_t *out,
                        hipStream_t stream);

}  // namespace tfbs
