// Device grouping of SNV-only regions (haplotype.rs:16-88 for the regions
// batch.cpp's snv_prepare admits): every haplotype id's diff mask, the
// distinct masks in Vec<Diff> order with their carrier counts, and one u16 of
// membership per haplotype id (its distinct index; the reference group's index
// for ids carrying no diff).
//
//   mask_scatter_kernel  one workgroup per record: each carrier id ORs the
//                        record's rank bit into its mask (a chunk-wide scratch of
//                        8 bytes per id and region, zero between chunks)
//   mask_group_kernel    one workgroup per region: the ids whose lowest mask bit
//                        is the record being read (so each id once) insert their
//                        mask into an LDS hash table; the distinct masks are
//                        ranked in Vec<Diff> order; the membership row is filled
//                        with the reference group's index, then every id with a
//                        mask writes its group's; the masks are zeroed again
//
// Both passes read only carrier lists: ~20 000 ids per C3 region, not the
// 100 000 haplotype ids (build_region's loop over every id).
#include <hip/hip_runtime.h>

#include <mutex>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "batch.hpp"

#define HIP_OK(expr)                                                                                       \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) return fail(TFBS_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));  \
    } while (0)

namespace tfbs {
namespace {

constexpr int kGrpBlock = 512;
constexpr uint32_t kGrpSlots = 8192;  // LDS hash slots: kGrpMax masks + one claim per thread stay below half

__device__ __forceinline__ uint32_t mask_slot(uint64_t m) {
    return (uint32_t)((m * 0x9E3779B97F4A7C15ull) >> 51) & (kGrpSlots - 1);
}

// Vec<Diff> order of two masks' ascending rank lists (batch.cpp's lex_less)
__device__ __forceinline__ bool lex_less(uint64_t a, uint64_t b) {
    const uint64_t d = a ^ b;
    if (!d) return false;
    const uint64_t low = d & (~d + 1);
    const uint64_t above = ~((low << 1) - 1);
    return (a & low) ? (b & above) != 0 : (a & above) == 0;
}

__global__ __launch_bounds__(256) void mask_scatter_kernel(const GrpRecord *__restrict__ recs,
                                                           const uint32_t *__restrict__ car,
                                                           unsigned long long *__restrict__ sig, uint32_t H) {
    const GrpRecord r = recs[blockIdx.x];
    const unsigned long long bit = 1ull << r.rank;
    unsigned long long *row = sig + (size_t)r.region * H;
    for (uint32_t i = threadIdx.x; i < r.n; i += 256) atomicOr(&row[car[r.off + i]], bit);
}

__global__ __launch_bounds__(kGrpBlock) void mask_group_kernel(const GrpRegion *__restrict__ regs,
                                                               const GrpRecord *__restrict__ recs,
                                                               const uint32_t *__restrict__ car,
                                                               unsigned long long *__restrict__ sig, uint32_t H,
                                                               uint16_t *__restrict__ memb, size_t memb_stride,
                                                               uint32_t *__restrict__ n_groups,
                                                               uint32_t *__restrict__ first, uint32_t *__restrict__ total,
                                                               unsigned long long *__restrict__ masks,
                                                               uint32_t *__restrict__ counts) {
    __shared__ unsigned long long s_key[kGrpSlots];
    __shared__ uint32_t s_cnt[kGrpSlots];
    __shared__ uint16_t s_idx[kGrpSlots];
    __shared__ unsigned long long s_m[kGrpMax];
    __shared__ uint32_t s_c[kGrpMax], s_slot[kGrpMax];
    __shared__ uint32_t s_n, s_over, s_pos, s_first;
    const uint32_t j = blockIdx.x, tid = threadIdx.x;
    const GrpRegion R = regs[j];
    unsigned long long *row = sig + (size_t)j * H;
    for (uint32_t t = tid; t < kGrpSlots; t += kGrpBlock) {
        s_key[t] = 0;
        s_cnt[t] = 0;
    }
    if (tid == 0) {
        s_n = 0;
        s_over = 0;
        s_pos = 0;
    }
    __syncthreads();
    // pass 1: each id with a mask once (at the record of its lowest bit) into the table
    for (uint32_t q = 0; q < R.n_rec; q++) {
        const GrpRecord r = recs[R.rec_off + q];
        for (uint32_t i = tid; i < r.n; i += kGrpBlock) {
            const unsigned long long m = row[car[r.off + i]];
            if ((uint32_t)__builtin_ctzll(m) != r.rank) continue;
            uint32_t s = mask_slot(m);
            while (!*(volatile uint32_t *)&s_over) {
                const unsigned long long old = atomicCAS(&s_key[s], 0ull, m);
                if (old == 0ull) {
                    if (atomicAdd(&s_n, 1u) >= kGrpMax) atomicOr(&s_over, 1u);
                    atomicAdd(&s_cnt[s], 1u);
                    break;
                }
                if (old == m) {
                    atomicAdd(&s_cnt[s], 1u);
                    break;
                }
                s = (s + 1) & (kGrpSlots - 1);
            }
        }
    }
    __syncthreads();
    const bool over = s_over != 0;
    const uint32_t G = s_n;
    if (!over) {
        if (tid == 0) s_first = atomicAdd(total, G);  // the region's masks at [first, first + G)
        for (uint32_t t = tid; t < kGrpSlots; t += kGrpBlock)
            if (s_key[t]) {
                const uint32_t at = atomicAdd(&s_pos, 1u);
                s_m[at] = s_key[t];
                s_c[at] = s_cnt[t];
                s_slot[at] = t;
            }
    }
    __syncthreads();
    if (!over) {
        // each mask's rank in Vec<Diff> order is its distinct index
        for (uint32_t t = tid; t < G; t += kGrpBlock) {
            const unsigned long long m = s_m[t];
            uint32_t rk = 0;
            for (uint32_t u = 0; u < G; u++) rk += lex_less(s_m[u], m) ? 1u : 0u;
            masks[s_first + rk] = m;
            counts[s_first + rk] = s_c[t];
            s_idx[s_slot[t]] = (uint16_t)rk;
        }
        // the membership row: the reference group's index (G) for every id ...
        uint16_t *mrow = memb + (size_t)j * memb_stride;
        const uint32_t fill = G * 0x00010001u;
        const uint4 f4 = make_uint4(fill, fill, fill, fill);
        for (uint32_t i = tid; i < (uint32_t)(memb_stride / 8); i += kGrpBlock)
            reinterpret_cast<uint4 *>(mrow)[i] = f4;
    }
    __syncthreads();
    for (uint32_t q = 0; q < R.n_rec; q++) {
        const GrpRecord r = recs[R.rec_off + q];
        for (uint32_t i = tid; i < r.n; i += kGrpBlock) {
            const uint32_t h = car[r.off + i];
            if (!over) {  // ... then its group's for every id with a mask
                const unsigned long long m = row[h];
                if ((uint32_t)__builtin_ctzll(m) == r.rank) {
                    uint32_t s = mask_slot(m);
                    while (s_key[s] != m) s = (s + 1) & (kGrpSlots - 1);
                    memb[(size_t)j * memb_stride + h] = s_idx[s];
                }
            }
        }
    }
    __syncthreads();
    // the masks back to zero for the next chunk
    for (uint32_t q = 0; q < R.n_rec; q++) {
        const GrpRecord r = recs[R.rec_off + q];
        for (uint32_t i = tid; i < r.n; i += kGrpBlock) row[car[r.off + i]] = 0ull;
    }
    if (tid == 0) {
        n_groups[j] = over ? UINT32_MAX : G;
        first[j] = over ? 0 : s_first;
    }
}

template <typename T>
struct Buf {
    T *p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return TFBS_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t c = std::max<size_t>(n, 64);
        HIP_OK(hipMalloc(&p, c * sizeof(T)));
        cap = c;
        return TFBS_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct GpuGrouper final : DevGrouper {
    int dev = 0;
    hipStream_t stream = nullptr;
    Buf<unsigned long long> sig;  // zero between chunks
    bool sig_zero = false;        // sig holds zeros up to its capacity
    Buf<uint32_t> car, n_groups, first, counts;
    uint32_t *total_host = nullptr;  // pinned: the chunk's masks
    Buf<unsigned long long> masks;
    Buf<GrpRecord> recs;
    Buf<GrpRegion> regs;
    PinnedBytes car_host;
    // membership rows: one allocation per chunk, held by its batch until it goes
    // (recycle), then reused by a later chunk that fits
    std::mutex memb_mu;
    std::vector<std::pair<uint16_t *, size_t>> memb_all;   // every allocation (bytes)
    std::vector<std::pair<uint16_t *, size_t>> memb_free;  // returned ones

    ~GpuGrouper() override {
        (void)hipSetDevice(dev);
        if (stream) (void)hipStreamSynchronize(stream);
        sig.release();
        car.release();
        n_groups.release();
        first.release();
        counts.release();
        if (total_host) (void)hipHostFree(total_host);
        masks.release();
        recs.release();
        regs.release();
        for (auto &m : memb_all) (void)hipFree(m.first);
        if (stream) (void)hipStreamDestroy(stream);
    }
    void recycle(std::vector<void *> &allocs) override {
        std::lock_guard<std::mutex> g(memb_mu);
        for (void *p : allocs)
            for (auto &m : memb_all)
                if (m.first == p) memb_free.push_back(m);
        allocs.clear();
    }
    uint16_t *memb_alloc(size_t bytes) {  // the smallest returned allocation that fits, else a new one
        {
            std::lock_guard<std::mutex> g(memb_mu);
            size_t best = memb_free.size();
            for (size_t i = 0; i < memb_free.size(); i++)
                if (memb_free[i].second >= bytes && (best == memb_free.size() || memb_free[i].second < memb_free[best].second))
                    best = i;
            if (best < memb_free.size()) {
                uint16_t *p = memb_free[best].first;
                memb_free.erase(memb_free.begin() + best);
                return p;
            }
        }
        uint16_t *p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        std::lock_guard<std::mutex> g(memb_mu);
        memb_all.push_back({p, bytes});
        return p;
    }
    int device() const override { return dev; }
    uint32_t *carriers(size_t n) override {
        if (car_host.reserve(std::max<size_t>(n, 1) * 4)) return nullptr;
        return reinterpret_cast<uint32_t *>(car_host.p);
    }
    int group(size_t n_car, const std::vector<GrpRecord> &rv, const std::vector<GrpRegion> &rg, uint32_t H,
              GroupOut &out) override {
        HIP_OK(hipSetDevice(dev));
        const size_t nr = rg.size();
        out.n_groups.assign(nr, 0);
        out.first.assign(nr, 0);
        out.memb.assign(nr, 0);
        if (!nr) return TFBS_OK;
        const size_t stride = ((size_t)H + 7) / 8 * 8;  // u16 per id, rows 16-byte aligned
        uint16_t *mb = memb_alloc(std::max<size_t>(nr * stride * 2, 16));
        if (!mb) return fail(TFBS_E_HIP, "device grouping: membership rows");
        out.memb_alloc = mb;
        int rc;
        const size_t sig_n = nr * (size_t)H;
        if (sig_n > sig.cap) sig_zero = false;
        if ((rc = sig.ensure(sig_n)) || (rc = car.ensure(std::max<size_t>(n_car, 1))) ||
            (rc = recs.ensure(std::max<size_t>(rv.size(), 1))) || (rc = regs.ensure(nr)) ||
            (rc = n_groups.ensure(nr + 1)) || (rc = first.ensure(nr)) || (rc = masks.ensure(nr * kGrpMax)) ||
            (rc = counts.ensure(nr * kGrpMax)))
            return rc;
        if (!total_host) HIP_OK(hipHostMalloc((void **)&total_host, 4, hipHostMallocDefault));
        HIP_OK(hipMemsetAsync(n_groups.p + nr, 0, 4, stream));  // the masks' counter
        if (!sig_zero) {
            HIP_OK(hipMemsetAsync(sig.p, 0, sig.cap * sizeof(unsigned long long), stream));
            sig_zero = true;
        }
        if (n_car) HIP_OK(hipMemcpyAsync(car.p, car_host.p, n_car * 4, hipMemcpyHostToDevice, stream));
        if (!rv.empty())
            HIP_OK(hipMemcpyAsync(recs.p, rv.data(), rv.size() * sizeof(GrpRecord), hipMemcpyHostToDevice, stream));
        HIP_OK(hipMemcpyAsync(regs.p, rg.data(), nr * sizeof(GrpRegion), hipMemcpyHostToDevice, stream));
        if (!rv.empty())
            hipLaunchKernelGGL(mask_scatter_kernel, dim3((uint32_t)rv.size()), dim3(256), 0, stream, recs.p, car.p,
                               sig.p, H);
        hipLaunchKernelGGL(mask_group_kernel, dim3((uint32_t)nr), dim3(kGrpBlock), 0, stream, regs.p, recs.p, car.p,
                           sig.p, H, mb, stride, n_groups.p, first.p, n_groups.p + nr, masks.p, counts.p);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(out.n_groups.data(), n_groups.p, nr * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipMemcpyAsync(out.first.data(), first.p, nr * 4, hipMemcpyDeviceToHost, stream));
        HIP_OK(hipMemcpyAsync(total_host, n_groups.p + nr, 4, hipMemcpyDeviceToHost, stream));
        hipError_t e = hipStreamSynchronize(stream);
        if (e == hipSuccess) {
            const uint32_t tot = *total_host;
            out.masks.resize(tot);
            out.counts.resize(tot);
            if (tot) {
                e = hipMemcpyAsync(out.masks.data(), masks.p, (size_t)tot * 8, hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(out.counts.data(), counts.p, (size_t)tot * 4, hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess) e = hipStreamSynchronize(stream);
            }
        }
        if (e != hipSuccess) {
            sig_zero = false;
            return fail(TFBS_E_HIP, std::string("device grouping: ") + hipGetErrorString(e));
        }
        for (size_t j = 0; j < nr; j++) out.memb[j] = (uint64_t)(uintptr_t)(mb + j * stride);
        return TFBS_OK;
    }
    int fetch(uint64_t m, uint32_t H, uint16_t *out) override {
        HIP_OK(hipSetDevice(dev));
        HIP_OK(hipMemcpy(out, (const void *)(uintptr_t)m, (size_t)H * 2, hipMemcpyDeviceToHost));
        return TFBS_OK;
    }
};

}  // namespace

void warm_devices(const std::vector<int> &devices) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return;
    for (int d : devices)
        if (d >= 0 && d < n && hipSetDevice(d) == hipSuccess) (void)hipFree(nullptr);  // (creates the device's context)
    (void)hipGetLastError();
}

DevGrouper *make_gpu_grouper(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        fail(TFBS_E_NODEVICE, "no such HIP device for the device grouping");
        return nullptr;
    }
    auto *g = new GpuGrouper();
    g->dev = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        fail(TFBS_E_HIP, "device grouping stream");
        return nullptr;
    }
    return g;
}

}  // namespace tfbs
