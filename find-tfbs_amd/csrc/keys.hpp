// Launch interface of the count-gather kernels (key_kernels.hip), used by device.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "batch.hpp"

namespace tfbs {

int launch_key_reduce(const DevHap *haps, const DevRegion *regions, uint32_t n_regions, const uint32_t *counts,
                      uint32_t n_slots, uint32_t *first, uint8_t *flags, hipStream_t stream);
int launch_key_gather(const DevHap *haps, const DevRegion *regions, const uint32_t *counts, uint32_t n_slots,
                      const DevVarKey *keys, uint32_t n_keys, uint32_t *out, hipStream_t stream);

}  // namespace tfbs
