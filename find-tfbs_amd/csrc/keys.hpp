// Launch interface of the count-gather kernels (key_kernels.hip), used by device.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "batch.hpp"

namespace tfbs {

int launch_key_reduce(const DevHap *haps, const DevRegion *regions, uint32_t n_regions, const uint32_t *counts,
                      uint32_t n_slots, uint32_t *first, uint8_t *flags, hipStream_t stream);
// One workgroup per key: v[s] = C[memb[2s]] + C[memb[2s+1]] for s < n_samples,
// where memb (u8, one row of 2 n_samples per region of the chunk, at
// memb_row[key's region - region0]) maps haplotype ids to distinct indices.
// Writes hdr[k], vals[k * 256 ..] (sorted distinct values), hist[k * 256 ..]
// (samples per value) and codes[k * n_samples ..].
int launch_key_encode(const DevHap *haps, const DevRegion *regions, const uint32_t *counts, uint32_t n_slots,
                      const DevVarKey *keys, uint32_t n_keys, const uint8_t *memb, uint32_t region0,
                      uint32_t n_samples, EncHdr *hdr, uint32_t *vals, uint32_t *hist, uint8_t *codes,
                      hipStream_t stream);
int launch_code_compact(const uint8_t *codes, uint32_t n_keys, uint32_t n_samples, const uint64_t *off, uint8_t *dst,
                        hipStream_t stream);
int launch_key_gather(const DevHap *haps, const DevRegion *regions, const uint32_t *counts, uint32_t n_slots,
                      const DevVarKey *keys, uint32_t n_keys, uint32_t *out, hipStream_t stream);

}  // namespace tfbs
