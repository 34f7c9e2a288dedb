// Count gather on the device.
//
// count_matches_by_sample (main.rs:500-534) builds, per key (bed, inner range,
// pattern_id), the per-sample L/R vectors; counts_as_genotypes (main.rs:439-498)
// emits a row only when the per-sample totals differ.  The scan leaves, per
// region, a [distinct haplotype][slot * n_inner + range] count matrix in HBM.
// Every sample's total is a sum of two of its rows, so a key can only produce a
// row if its column is not constant.  key_reduce_kernel classifies every column
// (any count != 0 -> the key exists in the reference's HashMap; counts differ ->
// the key may emit a row) in one pass over the matrix, and
// key_gather_kernel compacts the columns of the varying keys, so the host
// downloads flags + first values + a few columns instead of the dense matrix.
#include <hip/hip_runtime.h>

#include <string>

#include "keys.hpp"

namespace tfbs {
namespace {

constexpr int kReduceBlock = 256;

// One workgroup per region; threads stride over the region's key columns and
// walk the distinct-haplotype rows (coalesced across the columns).
__global__ __launch_bounds__(kReduceBlock) void key_reduce_kernel(const DevHap *__restrict__ haps,
                                                                   const DevRegion *__restrict__ regions,
                                                                   const uint32_t *__restrict__ counts,
                                                                   uint32_t n_slots, uint32_t *__restrict__ first,
                                                                   uint8_t *__restrict__ flags) {
    const DevRegion rg = regions[blockIdx.x];
    const uint32_t K = n_slots * rg.n_inner;
    const uint64_t ko = (uint64_t)rg.inner_off * n_slots;
    if (rg.hap_count == 0) {  // no samples: no haplotype, no match, no key
        for (uint32_t j = threadIdx.x; j < K; j += kReduceBlock) {
            first[ko + j] = 0;
            flags[ko + j] = 0;
        }
        return;
    }
    const uint64_t base = haps[rg.hap_begin].count_off;
    for (uint32_t j = threadIdx.x; j < K; j += kReduceBlock) {
        const uint32_t c0 = counts[base + j];
        uint32_t any = c0, diff = 0;
        for (uint32_t l = 1; l < rg.hap_count; l++) {
            const uint32_t c = counts[base + (uint64_t)l * K + j];
            any |= c;
            diff |= c ^ c0;
        }
        first[ko + j] = c0;
        flags[ko + j] = (uint8_t)((any ? KEY_ANY : 0) | (diff ? KEY_VARIES : 0));
    }
}

// One wave per varying key: copy its column (one count per distinct haplotype).
__global__ __launch_bounds__(256) void key_gather_kernel(const DevHap *__restrict__ haps,
                                                         const DevRegion *__restrict__ regions,
                                                         const uint32_t *__restrict__ counts, uint32_t n_slots,
                                                         const DevVarKey *__restrict__ keys, uint32_t n_keys,
                                                         uint32_t *__restrict__ out) {
    const uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= n_keys) return;
    const DevVarKey vk = keys[k];
    const DevRegion rg = regions[vk.region];
    const uint32_t K = n_slots * rg.n_inner;
    const uint64_t base = haps[rg.hap_begin].count_off;
    for (uint32_t l = threadIdx.x & 63; l < rg.hap_count; l += 64) out[vk.out_off + l] = counts[base + (uint64_t)l * K + vk.j];
}

}  // namespace

int launch_key_reduce(const DevHap *haps, const DevRegion *regions, uint32_t n_regions, const uint32_t *counts,
                      uint32_t n_slots, uint32_t *first, uint8_t *flags, hipStream_t stream) {
    if (n_regions == 0) return TFBS_OK;
    hipLaunchKernelGGL(key_reduce_kernel, dim3(n_regions), dim3(kReduceBlock), 0, stream, haps, regions, counts,
                       n_slots, first, flags);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_reduce_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_key_gather(const DevHap *haps, const DevRegion *regions, const uint32_t *counts, uint32_t n_slots,
                      const DevVarKey *keys, uint32_t n_keys, uint32_t *out, hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(key_gather_kernel, dim3((n_keys + 3) / 4), dim3(256), 0, stream, haps, regions, counts, n_slots,
                       keys, n_keys, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_gather_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

}  // namespace tfbs
