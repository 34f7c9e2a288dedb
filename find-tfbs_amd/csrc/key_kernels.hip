// Count gather on the device.
//
// count_matches_by_sample (main.rs:500-534) builds, per key (bed, inner range,
// pattern_id), the per-sample L/R vectors; counts_as_genotypes (main.rs:439-498)
// emits a row only when the per-sample totals differ.  The scan leaves, per
// region, a [slot * n_inner + range][distinct haplotype] count matrix in HBM
// (key-major: a key's counts are adjacent, DevRegion::count_stride apart).
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

// One workgroup per region, one thread per key: the key's counts of every
// distinct haplotype are adjacent (key-major layout, DevRegion), read in order
// (unrolled: several loads in flight per lane; each cache line serves 32
// iterations).
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
        const uint32_t *col = counts + base + (uint64_t)j * rg.count_stride;
        const uint32_t c0 = col[0];
        uint32_t any = c0, diff = 0;
#pragma unroll 8
        for (uint32_t l = 1; l < rg.hap_count; l++) {
            const uint32_t c = col[l];
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
    const uint64_t base = haps[rg.hap_begin].count_off;
    const uint32_t *col = counts + base + (uint64_t)vk.j * rg.count_stride;
    for (uint32_t l = threadIdx.x & 63; l < rg.hap_count; l += 64) out[vk.out_off + l] = col[l];
}

// counts_as_genotypes' per-sample half (main.rs:439-498) for one varying key:
// the sample totals, their min / max, the distinct values (a bitmap of
// hi - lo + 1 bits in LDS, ranks from per-word prefix counts) and one code per
// sample.  Three passes over the region's membership row (L2-resident: every
// key of the region reads it); the key's column of distinct-haplotype counts
// sits in LDS.  The range multiplicity and the text stay on the host, which
// formats a row from the value table and the codes (aggregate.cpp).
constexpr int kEncBlock = 256;
constexpr uint32_t kEncWords = kEncMaxRange / 32;

__global__ __launch_bounds__(kEncBlock) void key_encode_kernel(const DevHap *__restrict__ haps,
                                                                 const DevRegion *__restrict__ regions,
                                                                 const uint32_t *__restrict__ counts, uint32_t n_slots,
                                                                 const DevVarKey *__restrict__ keys,
                                                                 const uint8_t *__restrict__ memb, uint32_t region0,
                                                                 uint32_t n_samples, EncHdr *__restrict__ hdr,
                                                                 uint32_t *__restrict__ vals,
                                                                 uint32_t *__restrict__ hist,
                                                                 uint8_t *__restrict__ codes) {
    __shared__ uint32_t s_c[kEncMaxHaps + 1];
    __shared__ uint32_t s_bits[kEncWords];
    __shared__ uint16_t s_rank[kEncWords];  // distinct values in the words before
    __shared__ uint32_t s_hist[kEncMaxVals + 1];
    __shared__ uint32_t s_red[2 * kEncBlock / 64];
    __shared__ uint32_t s_nv;
    const uint32_t k = blockIdx.x;
    const DevVarKey vk = keys[k];
    const DevRegion rg = regions[vk.region];
    const uint64_t base = haps[rg.hap_begin].count_off;
    for (uint32_t l = threadIdx.x; l < rg.hap_count; l += kEncBlock)
        s_c[l] = counts[base + (uint64_t)vk.j * rg.count_stride + l];
    __syncthreads();
    const uint16_t *m = reinterpret_cast<const uint16_t *>(memb + (size_t)(vk.region - region0) * 2 * n_samples);
    auto total = [&](uint32_t s) {
        const uint32_t pr = m[s];
        return s_c[pr & 0xFF] + s_c[pr >> 8];  // u32 wrapping, as the reference's additions
    };
    // pass 1: min / max
    uint32_t lo = UINT32_MAX, hi = 0;
    for (uint32_t s = threadIdx.x; s < n_samples; s += kEncBlock) {
        const uint32_t v = total(s);
        lo = min(lo, v);
        hi = max(hi, v);
    }
    for (int o = 32; o; o >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    const uint32_t wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_red[wave] = lo;
        s_red[kEncBlock / 64 + wave] = hi;
    }
    __syncthreads();
    lo = s_red[0];
    hi = s_red[kEncBlock / 64];
    for (int w = 1; w < kEncBlock / 64; w++) {
        lo = min(lo, s_red[w]);
        hi = max(hi, s_red[kEncBlock / 64 + w]);
    }
    if (hi - lo >= kEncMaxRange) {
        if (threadIdx.x == 0) hdr[k] = EncHdr{lo, hi, 0, 1, 0};
        return;
    }
    // pass 2: which values occur
    const uint32_t nw = (hi - lo) / 32 + 1;
    for (uint32_t w = threadIdx.x; w < nw; w += kEncBlock) s_bits[w] = 0;
    __syncthreads();
    for (uint32_t s = threadIdx.x; s < n_samples; s += kEncBlock) {
        const uint32_t d = total(s) - lo;
        atomicOr(&s_bits[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // ranks: a serial prefix over <= 2048 words
        uint32_t r = 0;
        for (uint32_t w = 0; w < nw; w++) {
            s_rank[w] = (uint16_t)min(r, 0xFFFFu);
            r += __popc(s_bits[w]);
        }
        s_nv = r;
    }
    for (uint32_t i = threadIdx.x; i <= kEncMaxVals; i += kEncBlock) s_hist[i] = 0;
    __syncthreads();
    const uint32_t nv = s_nv;
    if (nv > kEncMaxVals) {
        if (threadIdx.x == 0) hdr[k] = EncHdr{lo, hi, nv, 1, 0};
        return;
    }
    for (uint32_t w = threadIdx.x; w < nw; w += kEncBlock) {  // the sorted value table
        uint32_t b = s_bits[w], r = s_rank[w];
        while (b) {
            const uint32_t t = __ffs(b) - 1;
            b &= b - 1;
            vals[(size_t)k * (kEncMaxVals + 1) + r++] = lo + 32 * w + t;
        }
    }
    // pass 3: codes (packed: each thread writes whole bytes) and per-value sample counts
    const uint32_t width = nv <= 4 ? 2 : (nv <= 16 ? 4 : 8), per = 8 / width;
    uint8_t *out = codes + (size_t)k * n_samples;
    const uint32_t nbytes = (n_samples + per - 1) / per;
    for (uint32_t byte = threadIdx.x; byte < nbytes; byte += kEncBlock) {
        uint32_t packed = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t s = byte * per + q;
            if (s >= n_samples) break;
            const uint32_t d = total(s) - lo, w = d >> 5;
            const uint32_t c = s_rank[w] + __popc(s_bits[w] & ((1u << (d & 31)) - 1u));
            packed |= c << (q * width);
            atomicAdd(&s_hist[c], 1u);
        }
        out[byte] = (uint8_t)packed;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nv; i += kEncBlock) hist[(size_t)k * (kEncMaxVals + 1) + i] = s_hist[i];
    if (threadIdx.x == 0) hdr[k] = EncHdr{lo, hi, nv, 0, width};
}

// Copies each key's packed codes (at k * n_samples) to off[k] of a contiguous buffer.
__global__ __launch_bounds__(256) void code_compact_kernel(const uint8_t *__restrict__ codes, uint32_t n_samples,
                                                           const uint64_t *__restrict__ off, uint8_t *__restrict__ dst) {
    const uint32_t k = blockIdx.x;
    const uint64_t o = off[k], n = off[k + 1] - o;
    const uint8_t *src = codes + (size_t)k * n_samples;
    for (uint64_t i = threadIdx.x; i < n; i += 256) dst[o + i] = src[i];
}

}  // namespace

int launch_key_encode(const DevHap *haps, const DevRegion *regions, const uint32_t *counts, uint32_t n_slots,
                      const DevVarKey *keys, uint32_t n_keys, const uint8_t *memb, uint32_t region0,
                      uint32_t n_samples, EncHdr *hdr, uint32_t *vals, uint32_t *hist, uint8_t *codes,
                      hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(key_encode_kernel, dim3(n_keys), dim3(kEncBlock), 0, stream, haps, regions, counts, n_slots,
                       keys, memb, region0, n_samples, hdr, vals, hist, codes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("key_encode_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_code_compact(const uint8_t *codes, uint32_t n_keys, uint32_t n_samples, const uint64_t *off, uint8_t *dst,
                        hipStream_t stream) {
    if (n_keys == 0) return TFBS_OK;
    hipLaunchKernelGGL(code_compact_kernel, dim3(n_keys), dim3(256), 0, stream, codes, n_samples, off, dst);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("code_compact_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

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
