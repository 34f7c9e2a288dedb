// The VCF rows of device-encoded keys as BGZF blocks, built on the GPU
// (the writer of main.rs:258-290).
//
// A row's text is its head (formatted on the host: "<chr>\t<POS>\t<id>\t.\t.\t.
// \tPASS\t<COUNTS/freqs>\tGT:DS"), then one sample text per sample -- the
// key's value text of the sample's code (tfbs_batch_encode) -- then '\n'.  At
// 50 000 samples that is ~0.4 MB per row, most of it runs of one text, so the
// text is never materialised: every BGZF block (65 280 bytes of the stream, one
// workgroup) generates its bytes from the codes and deflates them with the
// fixed Huffman code (RFC 1951 3.2.6) and matches the text's structure gives
// for free, no search: a sample text equal to the one before continues a run
// (distance = its length, one match per up to 258 bytes), otherwise it refers
// to the same text among the 8 samples before it (one match), else it is
// literals.  Each thread encodes 255 bytes of the block (bit counts, a block
// scan, then the bits at their offsets); the block's CRC32 is the XOR of the
// threads' CRCs shifted by x^(8 n) operators (powers of two precomputed).  A
// block that would not shrink is stored (BTYPE 00).
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

#include "bgzf_gpu.hpp"

namespace tfbs {
namespace {

constexpr int kBgBlock = 256;
constexpr uint32_t kBgPer = (kBgzfRaw + kBgBlock - 1) / kBgBlock;  // bytes per thread
constexpr uint32_t kBgWords = (kBgzfMax - 26) / 4;                  // deflate data words a block can hold
// the LDS bit buffer: blocks that compress to at most half are deflated (32 KiB,
// two workgroups per CU), the others stored
constexpr uint32_t kBitWords = kBgWords / 2;
constexpr uint32_t kLookback = 8;                                   // sample texts searched for a match

__device__ __forceinline__ uint32_t rev(uint32_t code, uint32_t n) { return __builtin_bitreverse32(code) >> (32 - n); }

// The bit stream of one thread: counts bits (write = false) or ORs them into the
// block's LDS buffer at their offset (neighbouring threads share edge words).
struct BitOut {
    uint32_t *buf;
    uint32_t off;
    bool write;
    __device__ void put(uint32_t v, uint32_t n) {
        if (write && n) {
            const uint32_t w = off >> 5, sh = off & 31;
            atomicOr(&buf[w], v << sh);
            if (sh + n > 32) atomicOr(&buf[w + 1], v >> (32 - sh));
        }
        off += n;
    }
    __device__ void lit(uint32_t b) {  // literal/length codes 0-143: 8 bits, 144-255: 9 bits
        if (b < 144) put(rev(0x30 + b, 8), 8);
        else put(rev(0x190 + b - 144, 9), 9);
    }
    // RFC 1951 3.2.5's length and distance codes, from the values' bit lengths:
    // lengths 3-10 and distances 1-4 have codes of their own, then each code covers
    // 2^extra values, four length codes (two distance codes) per extra bit count
    __device__ void match(uint32_t len, uint32_t dist) {  // 3 <= len <= 258, dist <= 32768
        uint32_t sym, xb = 0, xv = 0;
        if (len == 258) {
            sym = 285;
        } else if (len <= 10) {
            sym = 254 + len;
        } else {
            const uint32_t x = len - 3, nb = 31 - __builtin_clz(x);  // nb >= 3
            sym = 257 + 4 * (nb - 1) + ((x >> (nb - 2)) & 3u);
            xb = nb - 2;
            xv = x & ((1u << xb) - 1u);
        }
        if (sym < 280) put(rev(sym - 256, 7), 7);
        else put(rev(0xC0 + sym - 280, 8), 8);
        put(xv, xb);
        uint32_t dc, db = 0, dv = 0;
        if (dist <= 4) {
            dc = dist - 1;
        } else {
            const uint32_t x = dist - 1, nb = 31 - __builtin_clz(x);  // nb >= 2
            dc = 2 * nb + ((x >> (nb - 1)) & 1u);
            db = nb - 1;
            dv = x & ((1u << db) - 1u);
        }
        put(rev(dc, 5), 5);
        put(dv, db);
    }
};

// What a block stages in LDS: the descriptors of its rows (up to kStRowDesc),
// and for each of its (up to kStRows) rows with genotype text in the block the
// token lengths and texts, the group offsets (cum) of the 64-sample groups the
// block touches and those samples' packed codes (one group more before, for the
// look-backs).  bgzf_plan_kernel decides (one thread per block, so the binary
// searches of many blocks overlap); a block whose rows do not all fit (rows of a
// few samples) reads everything from global memory instead.
constexpr uint32_t kStRows = 8;
constexpr uint32_t kStRowDesc = 96;
constexpr uint32_t kStCodes = 18432;  // >= the codes of 65280 bytes of 4-byte sample texts + 3 groups per row
constexpr uint32_t kStTok = 512;      // token slots (kRowTokBytes of text each)
constexpr uint32_t kStCum = 512;
constexpr uint32_t kCrcOps = 16;      // shift operators of 2^k bytes, k < 16 (shifts below 64 KiB)

struct StRow {
    uint32_t row;          // row index
    uint32_t s_lo, s_hi;   // samples whose codes are staged (a group before the block's first, for look-backs)
    uint32_t cfirst;       // the row's code byte of sample s_lo (s_lo * width / 8)
    uint32_t code_at;      // its place in Stage::codes
    uint32_t tok_at;       // Stage::tlen / text slot of token 0
    uint32_t g_lo, ncum;   // cum entries [g_lo, g_lo + ncum) at cum_at
    uint32_t cum_at;
    uint32_t tok, nv, width, cum_off;  // the row's (DevRow): its staging reads them from the plan
    uint64_t code_off;
};

struct BlockPlan {
    uint32_t r_first, n_rows;  // the rows overlapping the block
    uint32_t n_st;
    uint32_t all;              // every row's descriptor and genotype data are staged
    StRow st[kStRows];
};

struct Stage {
    BlockPlan P;
    DevRow rows[kStRowDesc];  // rows r_first ..
    alignas(16) uint8_t codes[kStCodes];  // (dword reads: wv_item's look-back)
    uint8_t tlen[kStTok];
    alignas(16) uint8_t text[kStTok * kRowTokBytes];
    uint32_t cum[kStCum];
    uint32_t crc_tab[256];
    uint32_t crc_ops[kCrcOps * 32];
    uint32_t crc_slice[768];  // slice-by-4 tables 1-3 (bgzf_wave_kernel)
};

// the block kernel's stage, at file scope so that every access compiles to LDS
// instructions (through a generic reference the selects between staged and global
// data become flat loads that wait on both counters)
__shared__ Stage g_st;

__device__ __forceinline__ uint32_t crc_byte(const uint32_t *tab, uint32_t crc, uint32_t b) {
    return tab[(crc ^ b) & 0xFFu] ^ (crc >> 8);
}

// x^(8 n) applied to a CRC register (n < 2^kCrcOps)
__device__ __forceinline__ uint32_t crc_shift_lds(const uint32_t *ops, uint32_t v, uint32_t n) {
    for (uint32_t k = 0; n; k++, n >>= 1) {
        if (!(n & 1)) continue;
        const uint32_t *M = ops + 32 * k;
        uint32_t r = 0;
        for (uint32_t i = 0; i < 32; i++) r ^= ((v >> i) & 1u) ? M[i] : 0u;
        v = r;
    }
    return v;
}

// One row as a thread reads it.  kSt: the block staged everything (the plan's
// `all`), so every access is an LDS access; otherwise every access goes to global
// memory (blocks of many short rows).  The two never mix in one load: a select
// between LDS and global data compiles to a flat load that waits on both counters.
struct RowView {
    DevRow R;
    int32_t cbase;            // kSt: Stage::codes index of the row's code byte 0 (may be negative)
    uint32_t tok_at, cum_at, g_lo, ncum;
    uint32_t mask;
};

template <bool kSt>
struct Ctx {
    const BgArgs &A;
    uint64_t b0;
    __device__ uint64_t row_off(uint32_t r) const {
        if constexpr (kSt) return g_st.rows[r - g_st.P.r_first].text_off;
        else return A.rows[r].text_off;
    }
    // the last row starting at or before p (p inside the block)
    __device__ uint32_t find_row(uint64_t p) const {
        uint32_t lo = g_st.P.r_first, hi = g_st.P.r_first + g_st.P.n_rows - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (row_off(mid) <= p) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    }
    __device__ RowView view(uint32_t r) const {
        RowView v{};
        if constexpr (kSt) {
            v.R = g_st.rows[r - g_st.P.r_first];
            for (uint32_t k = 0; k < g_st.P.n_st; k++)
                if (g_st.P.st[k].row == r) {
                    const StRow T = g_st.P.st[k];
                    v.cbase = (int32_t)T.code_at - (int32_t)T.cfirst;
                    v.tok_at = T.tok_at;
                    v.cum_at = T.cum_at;
                    v.g_lo = T.g_lo;
                    v.ncum = T.ncum;
                }
        } else {
            v.R = A.rows[r];
        }
        v.mask = (1u << v.R.width) - 1u;
        return v;
    }
    __device__ uint32_t code(const RowView &v, uint32_t s) const {
        const uint32_t bit = s * v.R.width;
        uint32_t b;
        if constexpr (kSt) b = g_st.codes[v.cbase + (int32_t)(bit >> 3)];
        else b = A.codes[v.R.code_off + (bit >> 3)];
        return (b >> (bit & 7)) & v.mask;
    }
    __device__ uint32_t tlen(const RowView &v, uint32_t c) const {
        if constexpr (kSt) return g_st.tlen[v.tok_at + c];
        else return A.tok_len[v.R.tok + c];
    }
    __device__ uint4 ttext(const RowView &v, uint32_t c) const {  // the token's 16 bytes
        if constexpr (kSt) return reinterpret_cast<const uint4 *>(g_st.text)[v.tok_at + c];
        else return reinterpret_cast<const uint4 *>(A.tok_text)[v.R.tok + c];
    }
    static __device__ __forceinline__ uint32_t byte_of(const uint4 &t, uint32_t o) {
        const uint64_t lo = (uint64_t)t.x | ((uint64_t)t.y << 32), hi = (uint64_t)t.z | ((uint64_t)t.w << 32);
        return (uint32_t)((o < 8 ? lo : hi) >> (8 * (o & 7))) & 0xFFu;
    }
    // sample s and offset o of byte g of the row's genotype text
    __device__ void locate(const RowView &v, uint64_t g, uint32_t &s, uint32_t &o) const {
        uint32_t q, pos;
        if constexpr (kSt) {
            const uint32_t *cum = g_st.cum + v.cum_at;  // the staged groups
            uint32_t lo = 0, hi = v.ncum - 2;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (cum[mid] <= g) lo = mid;
                else hi = mid - 1;
            }
            q = v.g_lo + lo;
            pos = cum[lo];
        } else {
            const uint32_t ng = (A.n_samples + kCumGroup - 1) / kCumGroup;
            const uint32_t *cum = A.cum + v.R.cum_off;
            uint32_t lo = 0, hi = ng - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (cum[mid] <= g) lo = mid;
                else hi = mid - 1;
            }
            q = lo;
            pos = cum[lo];
        }
        s = q * kCumGroup;
        for (; s + 1 < A.n_samples; s++) {  // bounded: g lies inside the row's genotype text
            const uint32_t t = tlen(v, code(v, s));
            if (g < (uint64_t)pos + t) break;
            pos += t;
        }
        o = (uint32_t)(g - pos);
    }
    // every byte of [p, e), in order
    template <class F>
    __device__ void bytes(uint64_t p, uint64_t e, F &&f) const {
        if (p >= e) return;
        uint32_t r = find_row(p);
        while (p < e) {
            while (r + 1 < g_st.P.r_first + g_st.P.n_rows && row_off(r + 1) <= p) r++;  // (the block's rows)
            const RowView v = view(r);
            const uint64_t local = p - v.R.text_off;
            if (local < v.R.head_len) {
                const uint64_t n = min((uint64_t)v.R.head_len - local, e - p);
                for (uint64_t i = 0; i < n; i++) f((uint8_t)A.heads[v.R.head_off + local + i]);
                p += n;
                continue;
            }
            uint64_t g = local - v.R.head_len;
            if (g >= v.R.geno_len) {
                f((uint8_t)'\n');
                p++;
                continue;
            }
            uint32_t s, o;
            locate(v, g, s, o);
            while (p < e && g < v.R.geno_len) {
                const uint32_t c = code(v, s), t = tlen(v, c);
                const uint4 tx = ttext(v, c);
                const uint32_t n = (uint32_t)min((uint64_t)(t - o), e - p);
                for (uint32_t i = 0; i < n; i++) f((uint8_t)byte_of(tx, o + i));
                p += n;
                g += n;
                o += n;
                if (o == t) {
                    s++;
                    o = 0;
                }
            }
        }
    }
    // the deflate symbols of [p, e) into out; with crc, every byte into *crc too
    template <bool kCrc>
    __device__ void encode(uint64_t p, uint64_t e, BitOut &out, uint32_t *crc) const {
        if (p >= e) return;
        uint32_t r = find_row(p);
        uint32_t x = kCrc ? *crc : 0u;
        while (p < e) {
            while (r + 1 < g_st.P.r_first + g_st.P.n_rows && row_off(r + 1) <= p) r++;  // (the block's rows)
            const RowView v = view(r);
            const uint64_t local = p - v.R.text_off;
            if (local < v.R.head_len) {
                const uint64_t n = min((uint64_t)v.R.head_len - local, e - p);
                for (uint64_t i = 0; i < n; i++) {
                    const uint32_t b = (uint8_t)A.heads[v.R.head_off + local + i];
                    out.lit(b);
                    if (kCrc) x = crc_byte(g_st.crc_tab, x, b);
                }
                p += n;
                continue;
            }
            uint64_t g = local - v.R.head_len;
            if (g >= v.R.geno_len) {
                out.lit('\n');
                if (kCrc) x = crc_byte(g_st.crc_tab, x, '\n');
                p++;
                continue;
            }
            uint32_t s, o;
            locate(v, g, s, o);
            uint32_t prev = s > 0 ? code(v, s - 1) : UINT32_MAX;
            while (p < e && g < v.R.geno_len) {
                const uint32_t c = code(v, s), t = tlen(v, c);
                const uint4 tx = ttext(v, c);
                const uint64_t tok0 = p - o;  // this sample text's first byte
                if (prev == c && tok0 >= b0 + t) {
                    // a run: every byte equals the one t before it, to the run's end
                    uint64_t end = tok0 + t;
                    uint32_t s2 = s + 1;
                    while (end < e && s2 < A.n_samples && code(v, s2) == c) {
                        end += t;
                        s2++;
                    }
                    end = min(end, e);
                    uint32_t left = (uint32_t)(end - p), oo = o;
                    if (kCrc)
                        for (uint32_t i = 0, q = o; i < left; i++) {
                            x = crc_byte(g_st.crc_tab, x, byte_of(tx, q));
                            q = q + 1 == t ? 0 : q + 1;
                        }
                    while (left) {
                        if (left < 3) {  // too short for a match: literals
                            out.lit(byte_of(tx, oo));
                            oo = oo + 1 == t ? 0 : oo + 1;
                            left--;
                            continue;
                        }
                        const uint32_t m = left > 258 ? (left - 258 < 3 ? left - 3 : 258) : left;
                        out.match(m, t);
                        oo = (oo + m) % t;
                        left -= m;
                    }
                    const uint32_t adv = (uint32_t)(end - p);
                    g += adv;
                    p = end;
                    const uint32_t q = o + adv;
                    s += q / t;
                    o = q % t;
                    prev = c;
                    continue;
                }
                const uint32_t n = (uint32_t)min((uint64_t)(t - o), e - p);
                uint32_t dist = 0, acc = 0;
                for (uint32_t kk = 1; kk <= kLookback && kk <= s; kk++) {  // the same text among the samples before
                    const uint32_t cc = kk == 1 ? prev : code(v, s - kk);
                    acc += tlen(v, cc);
                    if (tok0 < b0 + acc) break;
                    if (cc == c) {
                        dist = acc;
                        break;
                    }
                }
                if (dist && n >= 3) {
                    out.match(n, dist);
                    if (kCrc)
                        for (uint32_t i = 0; i < n; i++) x = crc_byte(g_st.crc_tab, x, byte_of(tx, o + i));
                } else {
                    for (uint32_t i = 0; i < n; i++) {
                        const uint32_t b = byte_of(tx, o + i);
                        out.lit(b);
                        if (kCrc) x = crc_byte(g_st.crc_tab, x, b);
                    }
                }
                p += n;
                g += n;
                o += n;
                if (o == t) {
                    s++;
                    o = 0;
                    prev = c;
                }
            }
        }
        if (kCrc) *crc = x;
    }
};

// Row r's genotype text offsets of samples 0, 64, 128, ... (and its end): the
// packed codes a byte at a time through a table of the byte's summed text lengths.
__global__ __launch_bounds__(256) void row_cum_kernel(BgArgs A) {
    __shared__ uint32_t s_scan[256];
    __shared__ uint16_t s_blen[256];  // code byte -> bytes of text of its samples
    const uint32_t r = blockIdx.x;
    const DevRow R = A.rows[r];
    if (!R.width) return;
    const uint32_t ng = (A.n_samples + kCumGroup - 1) / kCumGroup;
    uint32_t *cum = A.cum + R.cum_off;
    const uint32_t per = 8 / R.width, mask = (1u << R.width) - 1u;
    auto tlen = [&](uint32_t c) { return (uint32_t)A.tok_len[R.tok + c]; };
    auto code = [&](uint32_t s) {
        const uint32_t bit = s * R.width;
        return (A.codes[R.code_off + (bit >> 3)] >> (bit & 7)) & mask;
    };
    {
        const uint32_t v = threadIdx.x;
        uint32_t n = 0;
        for (uint32_t k = 0; k < per; k++) {
            const uint32_t c = (v >> (k * R.width)) & mask;
            if (c < R.nv) n += tlen(c);  // (other codes never occur)
        }
        s_blen[v] = (uint16_t)n;
    }
    __syncthreads();
    const uint32_t gbytes = kCumGroup / per;  // whole bytes per group of 64 samples
    uint32_t carry = 0;
    for (uint32_t q0 = 0; q0 < ng; q0 += 256) {
        const uint32_t q = q0 + threadIdx.x;
        uint32_t sum = 0;
        if (q + 1 < ng || (q + 1 == ng && A.n_samples % kCumGroup == 0)) {  // a full group
            const uint8_t *b = A.codes + R.code_off + (size_t)q * gbytes;
            for (uint32_t i = 0; i < gbytes; i++) sum += s_blen[b[i]];
        } else if (q < ng) {  // the last, partial group: sample by sample
            for (uint32_t s = q * kCumGroup; s < A.n_samples; s++) sum += tlen(code(s));
        }
        s_scan[threadIdx.x] = sum;
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t t = threadIdx.x >= o ? s_scan[threadIdx.x - o] : 0;
            __syncthreads();
            s_scan[threadIdx.x] += t;
            __syncthreads();
        }
        if (q < ng) cum[q] = carry + s_scan[threadIdx.x] - sum;
        carry += s_scan[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) cum[ng] = carry;
}

// One thread per block of a launch: the rows overlapping it and which of their
// token tables, group offsets and codes it stages (Stage).
__global__ __launch_bounds__(256) void bgzf_plan_kernel(BgArgs A, uint32_t n_blocks) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_blocks) return;
    const uint64_t b0 = (A.block0 + i) * kBgzfRaw;
    const uint64_t e = b0 + min((uint64_t)kBgzfRaw, A.text_bytes - b0);
    auto find_row = [&](uint64_t p) {
        uint32_t lo = 0, hi = A.n_rows - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (A.rows[mid].text_off <= p) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    BlockPlan P{};
    P.r_first = find_row(b0);
    const uint32_t r_last = find_row(e - 1);
    P.n_rows = r_last - P.r_first + 1;
    const uint32_t ng = (A.n_samples + kCumGroup - 1) / kCumGroup;
    auto group_of = [&](const DevRow &R, uint64_t g) {  // the group holding genotype byte g
        const uint32_t *cum = A.cum + R.cum_off;
        uint32_t lo = 0, hi = ng - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (cum[mid] <= g) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    uint32_t n = 0, code_used = 0, tok_used = 0, cum_used = 0;
    bool all = P.n_rows <= kStRowDesc;
    for (uint32_t r = P.r_first; r <= r_last && all; r++) {
        const DevRow R = A.rows[r];
        if (!R.width) continue;
        const uint64_t gs = R.text_off + R.head_len, ge = gs + R.geno_len;
        const uint64_t lo = max(b0, gs), hi = min(e, ge);
        if (lo >= hi) continue;
        const uint32_t g_lo = lo == gs ? 0 : group_of(R, lo - gs);
        const uint32_t g_hi = hi == ge ? ng - 1 : group_of(R, hi - 1 - gs);
        const uint32_t s_lo = (g_lo ? g_lo - 1 : 0) * kCumGroup, s_hi = min(A.n_samples, (g_hi + 1) * kCumGroup);
        const uint32_t cb0 = s_lo * R.width / 8, cb1 = (s_hi * R.width + 7) / 8;
        const uint32_t ncum = g_hi - g_lo + 2;
        // (the codes at the source's offset mod 4: bgzf_wave_kernel copies dwords)
        const uint32_t code_at = ((code_used + 3) & ~3u) + (uint32_t)((R.code_off + cb0) & 3u);
        if (n == kStRows || code_at + (cb1 - cb0) > kStCodes || tok_used + R.nv > kStTok ||
            cum_used + ncum > kStCum) {
            all = false;
            break;
        }
        P.st[n] = StRow{r, s_lo, s_hi, cb0, code_at, tok_used, g_lo, ncum, cum_used, R.tok, R.nv, R.width, R.cum_off,
                        R.code_off};
        code_used = code_at + (cb1 - cb0);
        tok_used += R.nv;
        cum_used += ncum;
        n++;
    }
    P.n_st = n;
    P.all = all ? 1u : 0u;
    reinterpret_cast<BlockPlan *>(A.plans)[i] = P;
}

__global__ __launch_bounds__(kBgBlock) void bgzf_block_kernel(BgArgs A) {
    __shared__ uint32_t s_bits[kBitWords + 1];
    __shared__ uint32_t s_scan[kBgBlock];
    __shared__ uint32_t s_crc[kBgBlock];
    Stage &S = g_st;
    const uint32_t tid = threadIdx.x;
    const uint64_t blk = A.block0 + blockIdx.x;
    const uint64_t b0 = blk * kBgzfRaw;
    const uint32_t n = (uint32_t)min((uint64_t)kBgzfRaw, A.text_bytes - b0);
    // the block's plan, rows, token tables, group offsets and codes into LDS
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(reinterpret_cast<const BlockPlan *>(A.plans) + blockIdx.x);
        for (uint32_t i = tid; i < sizeof(BlockPlan) / 4; i += kBgBlock) reinterpret_cast<uint32_t *>(&S.P)[i] = src[i];
        for (uint32_t i = tid; i < 256; i += kBgBlock) S.crc_tab[i] = A.crc_tab[i];
        for (uint32_t i = tid; i < kCrcOps * 32; i += kBgBlock) S.crc_ops[i] = A.crc_ops[i];
        for (uint32_t i = tid; i <= kBitWords; i += kBgBlock) s_bits[i] = 0;
    }
    __syncthreads();
    if (S.P.all) return;  // (uniform) bgzf_wave_kernel's block
    if (S.P.all) {  // (uniform: the whole block stages or none of it)
        const uint32_t nd = S.P.n_rows * (uint32_t)(sizeof(DevRow) / 4);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(A.rows + S.P.r_first);
        for (uint32_t i = tid; i < nd; i += kBgBlock) reinterpret_cast<uint32_t *>(S.rows)[i] = src[i];
        for (uint32_t k = 0; k < S.P.n_st; k++) {
            const StRow T = S.P.st[k];
            const DevRow R = A.rows[T.row];
            const uint32_t nb = (T.s_hi * R.width + 7) / 8 - T.cfirst;
            for (uint32_t i = tid; i < nb; i += kBgBlock) S.codes[T.code_at + i] = A.codes[R.code_off + T.cfirst + i];
            for (uint32_t i = tid; i < R.nv; i += kBgBlock) S.tlen[T.tok_at + i] = A.tok_len[R.tok + i];
            for (uint32_t i = tid; i < R.nv * kRowTokBytes; i += kBgBlock)
                S.text[T.tok_at * kRowTokBytes + i] = (uint8_t)A.tok_text[(size_t)R.tok * kRowTokBytes + i];
            for (uint32_t i = tid; i < T.ncum; i += kBgBlock) S.cum[T.cum_at + i] = A.cum[R.cum_off + T.g_lo + i];
        }
    }
    __syncthreads();
    const bool all = S.P.all != 0;
    const Ctx<true> CS{A, b0};
    const Ctx<false> CG{A, b0};
    const uint64_t p = b0 + min(n, tid * kBgPer), e = b0 + min(n, (tid + 1) * kBgPer);
    // pass 1: the thread's bits, and the CRC32 (reflected 0xEDB88320, zero start) of
    // its bytes shifted to the block end
    BitOut cnt{s_bits, 0, false};
    uint32_t crc = 0;
    if (all) CS.template encode<true>(p, e, cnt, &crc);
    else CG.template encode<true>(p, e, cnt, &crc);
    s_crc[tid] = crc_shift_lds(S.crc_ops, crc, (uint32_t)(b0 + n - e));
    s_scan[tid] = cnt.off;
    __syncthreads();
    for (uint32_t o = 1; o < kBgBlock; o <<= 1) {
        const uint32_t t = tid >= o ? s_scan[tid - o] : 0;
        __syncthreads();
        s_scan[tid] += t;
        __syncthreads();
    }
    const uint32_t total_bits = 3 + s_scan[kBgBlock - 1] + 7;  // BFINAL + BTYPE, symbols, end of block
    const uint32_t dbytes = (total_bits + 7) / 8;
    const bool stored = dbytes > 4 * kBitWords;  // (also when deflate would not fit the BGZF block)
    if (!stored) {  // pass 2: the bits at their offsets
        if (tid == 0) s_bits[0] = 0x3u;  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
        __syncthreads();
        BitOut w{s_bits, 3 + s_scan[tid] - cnt.off, true};
        if (all) CS.template encode<false>(p, e, w, nullptr);
        else CG.template encode<false>(p, e, w, nullptr);
    }
    // the block's CRC: XOR of the shifted parts, then the start value and final XOR
    for (uint32_t o = kBgBlock / 2; o; o >>= 1) {
        __syncthreads();
        if (tid < o) s_crc[tid] ^= s_crc[tid + o];
    }
    if (tid == 0) s_crc[0] ^= crc_shift_lds(S.crc_ops, 0xFFFFFFFFu, n) ^ 0xFFFFFFFFu;
    __syncthreads();
    uint8_t *out = A.out + (size_t)blockIdx.x * kBgzfMax;
    const uint32_t clen = stored ? 5 + n : dbytes;
    const uint32_t bsize = 18 + clen + 8;
    if (stored) {  // BFINAL = 1, BTYPE = 00, LEN, NLEN, the bytes
        uint32_t k = 0;
        CG.bytes(p, e, [&](uint8_t b) { out[18 + 5 + (p - b0) + k++] = b; });
        if (tid == 0) {
            out[18] = 1;
            out[19] = (uint8_t)n;
            out[20] = (uint8_t)(n >> 8);
            out[21] = (uint8_t)~n;
            out[22] = (uint8_t)(~n >> 8);
        }
    } else {
        const uint8_t *src = reinterpret_cast<const uint8_t *>(s_bits);
        for (uint32_t i = tid; i < dbytes; i += kBgBlock) out[18 + i] = src[i];
    }
    if (tid == 0) {
        const uint8_t hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43, 2, 0,
                                 (uint8_t)((bsize - 1) & 0xff), (uint8_t)((bsize - 1) >> 8)};
        for (int i = 0; i < 18; i++) out[i] = hdr[i];
        const uint32_t crc32 = s_crc[0];
        for (int i = 0; i < 4; i++) out[18 + clen + i] = (uint8_t)(crc32 >> (8 * i));
        for (int i = 0; i < 4; i++) out[18 + clen + 4 + i] = (uint8_t)(n >> (8 * i));
        A.out_len[blockIdx.x] = bsize;
    }
}

// ---------------------------------------------------------------------------
// The wave-parallel encoder of blocks whose rows are all staged (BlockPlan::all):
// one wave per 64-sample group of a row -- lane = sample -- so that every lane
// does the same work (bgzf_block_kernel's thread-serial loop diverges per byte).
// A group's sample texts get their offsets from a wave prefix sum of their
// lengths; a text equal to the one before it (inside the block) belongs to a
// run, the wave's runs are cut into matches of up to 258 bytes at distance =
// the text's length (a run continuing into the next group starts a new match
// there: one more symbol per 64 texts); another text is a match against the same
// text among the 8 before it, or literals; texts cut by the block's edges are
// literals.  Heads and newlines are literals.  Pass 1 counts each group's bits
// and writes the block's bytes to LDS (for the CRC), a block scan gives every
// group its bit offset, pass 2 writes the bits.
constexpr int kWv = 1024;             // threads
constexpr uint32_t kWvItems = 768;    // heads, groups, newlines of a block (<= 2 kStRowDesc + kStCum)
static_assert(kWvItems >= 2 * kStRowDesc + kStCum, "a block's items");
// items: a row's head, a 64-sample group, a newline, or a run of 1-15 groups (item
// bits: kind 30-31, row 23-29, staged row 20-22, run groups 16-19, group 0-15)
enum : uint32_t { IT_HEAD = 0u, IT_GROUP = 1u, IT_NL = 2u, IT_RUN = 3u };
constexpr uint32_t kRunGroups = 15;

__shared__ uint32_t g_bits[kBitWords + 1];
// the block's bytes, 4 bytes of padding after every 64 (so that the CRC's 64-byte
// slices, one per lane, start in different banks): byte q at txt_at(q)
alignas(16) __shared__ uint8_t g_text[kBgzfRaw + kBgzfRaw / 16 + 16];
__device__ __forceinline__ uint32_t txt_at(uint32_t q) { return q + ((q >> 6) << 2); }
__shared__ uint32_t g_item[kWvItems];
// per staged token slot: the fixed-Huffman literal codes of its text, LSB first,
// and their bit count (kNoTokLit: more than 128 bits, the per-byte path), so that
// a whole text of literals is a few 32-bit puts, not one per byte
__shared__ uint4 g_tlit[kStTok];
__shared__ uint8_t g_tlitn[kStTok];
constexpr uint32_t kNoTokLit = 255;
__shared__ uint32_t g_ioff[kWvItems + 1];
__shared__ uint32_t g_red[kWv / 64];
__shared__ uint32_t g_pub[kWvItems];  // item i's end bit + 1 (0: not yet known; wv_place)
__shared__ uint32_t g_agg[kWvItems];  // item i's bit count + 1 (0: not yet known; wv_place)
// TFBS_BGZF_PROF counts: wv_place's waits; items all-run, with look-back matches,
// with whole-token literals, with byte literals; heads; newlines; other groups; then
// wave-cycles of run groups' counts, of deferred emits, -, of other groups' counts, of
// byte-literal groups, -; other groups on the serial look-back
__shared__ uint32_t g_pstat[16];
__device__ __forceinline__ void wv_pcycles(const BgArgs &A, uint32_t lane, uint32_t k, uint64_t t0) {
    if (A.prof && lane == 0) atomicAdd(&g_pstat[k], (uint32_t)(clock64() - t0));
}

// A lane's bit stream: symbols gathered in a register, ORed into g_bits 32 bits at
// a time (two LDS atomics at most per 32 bits, not per symbol)
struct LaneBits {
    uint64_t acc;
    uint32_t n, off;  // bits held; the stream offset of the first
    __device__ void out(uint32_t v, uint32_t nb) {  // (bits past the buffer: the block is stored)
        const uint32_t w = off >> 5, sh = off & 31;
        if (w <= kBitWords) atomicOr(&g_bits[w], v << sh);
        if (sh + nb > 32 && w < kBitWords) atomicOr(&g_bits[w + 1], v >> (32 - sh));
    }
    __device__ void put(uint32_t v, uint32_t nb) {  // nb <= 32, v < 2^nb
        acc |= (uint64_t)v << n;
        n += nb;
        if (n >= 32) {
            out((uint32_t)acc, 32);
            off += 32;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ void finish() {
        if (n) out((uint32_t)acc & (n == 32 ? ~0u : ((1u << n) - 1u)), n);
        off += n;
        acc = 0;
        n = 0;
    }
};

__device__ __forceinline__ void wv_put(LaneBits &o, uint32_t v, uint32_t n) {
    if (n) o.put(v, n);
}
__device__ __forceinline__ uint32_t lit_bits(uint32_t b) { return b < 144 ? 8u : 9u; }
__device__ __forceinline__ void wv_lit(LaneBits &o, uint32_t b) {
    if (b < 144) wv_put(o, rev(0x30 + b, 8), 8);
    else wv_put(o, rev(0x190 + b - 144, 9), 9);
}
// RFC 1951 3.2.5: a match's codes as they go into the stream (LSB first) and
// their bit count (<= 8 + 5 + 5 + 13 = 31), one put
__device__ __forceinline__ uint2 match_code(uint32_t len, uint32_t dist) {
    uint32_t sym, xv = 0, xb = 0;
    if (len == 258) {
        sym = 285;
    } else if (len <= 10) {
        sym = 254 + len;
    } else {
        const uint32_t x = len - 3, nb = 31 - __builtin_clz(x);
        sym = 257 + 4 * (nb - 1) + ((x >> (nb - 2)) & 3u);
        xb = nb - 2;
        xv = x & ((1u << xb) - 1u);
    }
    uint32_t dc, dv = 0, db = 0;
    if (dist <= 4) {
        dc = dist - 1;
    } else {
        const uint32_t x = dist - 1, nb = 31 - __builtin_clz(x);
        dc = 2 * nb + ((x >> (nb - 1)) & 1u);
        db = nb - 1;
        dv = x & ((1u << db) - 1u);
    }
    uint32_t v, at;
    if (sym < 280) {
        v = rev(sym - 256, 7);
        at = 7;
    } else {
        v = rev(0xC0 + sym - 280, 8);
        at = 8;
    }
    v |= xv << at;
    at += xb;
    v |= rev(dc, 5) << at;
    at += 5;
    v |= dv << at;
    return uint2{v, at + db};
}

// wave64 inclusive prefix sum with DPP (GFX9 row shifts within 16 lanes, then the
// row_bcast:15 / row_bcast:31 carries across rows): no LDS permutes
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t) { return wave_incl_sum(v) - v; }
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(v), 63);
}

// Item i's first bit by decoupled look-back (no chain through the waves): the
// item's bit count is published first (g_agg); then the wave's lanes read the
// 64 items before it at once -- lane k item i - 1 - k -- and the first bit is
// the end of the nearest one whose end is known (g_pub) plus the bit counts of
// the items between (a wave sum), further windows of 64 while none is known.
// Every item publishes its count before it looks back and waits only on lower
// items, so all counts arrive (items go to the waves round-robin, in order).
// Then item i's end is published.
__device__ __forceinline__ void wv_publish(uint32_t i, uint32_t total, uint32_t lane) {
    if (lane == 0) __hip_atomic_store(&g_agg[i], total + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t wv_lookback(uint32_t i, uint32_t total, uint32_t lane) {
#ifdef BG_PROBE_NOPLACE  // (timing probe: no look-back, wrong offsets)
    if (total != 0xFFFFFFFFu) return 64 * 128 * (i & 3);
#endif
    uint32_t acc = 3;  // BFINAL + BTYPE before item 0
    for (int32_t hi = (int32_t)i; hi > 0;) {
        const int32_t j = hi - 1 - (int32_t)lane;
        uint32_t inc = 0, agg = 1;
        if (j >= 0) {
            inc = __hip_atomic_load(&g_pub[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            agg = __hip_atomic_load(&g_agg[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const uint64_t have = __ballot(j >= 0 && inc != 0);
        const uint32_t ks = have ? (uint32_t)__builtin_ctzll(have) : 64u;  // nearest known end
        const bool need = j >= 0 && lane < ks;
        if (__ballot(need && agg == 0)) {  // a count between not published yet: look again
            if (lane == 0) atomicAdd(&g_pstat[0], 1u);
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        acc += wave_sum(need ? agg - 1 : 0u);
        if (have) {
            acc += (uint32_t)__builtin_amdgcn_readlane((int)inc, (int)ks) - 1 - 3;  // (its end includes the 3)
            break;
        }
        hi -= 64;
    }
    if (lane == 0) __hip_atomic_store(&g_pub[i], acc + total + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return acc;
}
__device__ __forceinline__ uint32_t wv_place(uint32_t i, uint32_t total, uint32_t lane) {
    wv_publish(i, total, lane);
    return wv_lookback(i, total, lane);
}

// A lane's symbols as up to 4 words (LSB first, bn bits) at stream bit off: at most
// two LDS ORs each (bits past the buffer: the block is stored)
__device__ __forceinline__ void wv_words(uint32_t off, const uint32_t (&bw)[4], uint32_t bn) {
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        if (!__ballot(bn > 32 * k)) break;
        if (bn > 32 * k) {
            const uint32_t o = off + 32 * k, w = o >> 5, sh = o & 31, nk = min(bn - 32 * k, 32u);
            if (w <= kBitWords) atomicOr(&g_bits[w], bw[k] << sh);
            if (sh + nk > 32 && w < kBitWords) atomicOr(&g_bits[w + 1], bw[k] >> (32 - sh));
        }
    }
}

// A group item whose symbols wait for their place: its bit count (wave-uniform) and
// each lane's symbol words.  A wave counts its next item before it places this one,
// so that the look-back's wait overlaps that work (wv_emit).
struct Pend {
    uint32_t i;  // the item (~0u: none)
    uint32_t total;
    uint32_t bw[4], bn;
};
__device__ __forceinline__ void wv_emit(const BgArgs &A, const Pend &p, uint32_t lane) {
    const uint64_t pt0 = A.prof ? clock64() : 0;
    const uint32_t base = wv_lookback(p.i, p.total, lane);
#ifdef BG_PROBE_NOBITS
    if (base == 0xFFFFFFFFu)
#endif
    wv_words(base + wave_excl_sum(p.bn, lane), p.bw, p.bn);
    wv_pcycles(A, lane, 9, pt0);
}

// One byte of the block at q into g_text: ORed into its dword (a byte store racing
// another wave's OR of a neighbouring text's edge dword loses one of them: every
// g_text write is an OR)
// CHECK (TFBS_BGZF_CHECK, debug): the OR returns the dword's old value, and a write
// meeting bits already set -- a byte written twice, or a text's zero padding that is
// not zero -- is counted in A.check (the host fails the call).
template <bool CHECK>
__device__ __forceinline__ void wv_text_put(const BgArgs &A, uint32_t a4, uint32_t v) {
    uint32_t *w = reinterpret_cast<uint32_t *>(g_text + a4);
    if (CHECK) {
        if (atomicOr(w, v) & v) atomicAdd(A.check, 1u);
    } else {
        atomicOr(w, v);
    }
}
template <bool CHECK>
__device__ __forceinline__ void wv_text_byte(const BgArgs &A, uint32_t q, uint32_t b) {
    const uint32_t a = txt_at(q);
    wv_text_put<CHECK>(A, a & ~3u, b << (8 * (a & 3u)));
}

// A whole text at block byte rel (>= 0, inside the block) into g_text: its dwords,
// ORed (neighbouring texts share edge dwords; the staged text's bytes past its length
// are zero)
template <bool CHECK>
__device__ __forceinline__ void wv_text_or(const BgArgs &A, int32_t rel, uint32_t t, const uint4 &tx) {
    const uint32_t a8 = 8 * ((uint32_t)rel & 3u), k0 = (uint32_t)rel >> 2, k1 = (uint32_t)(rel + (int32_t)t - 1) >> 2;
    const uint32_t T[5] = {tx.x, tx.y, tx.z, tx.w, 0u};
    uint32_t prev = 0;
#pragma unroll
    for (uint32_t j = 0; j < 5; j++) {
        const uint32_t dw = (uint32_t)(((((uint64_t)T[j]) << 32) | prev) >> (32 - a8));
        prev = T[j];
        if (k0 + j <= k1) wv_text_put<CHECK>(A, txt_at(4 * (k0 + j)), dw);
    }
}

// Item i of the block (all lanes of a wave together): its bytes into g_text, its bit
// count; then a group's symbols go to *out (placed by wv_emit), the other items' (and
// groups with byte literals) are placed (wv_place) and written at once (out->i = ~0u).
// v / vkey: the wave's last item's row view and its key (item bits 20-31), kept
// across the wave's items (consecutive ones are mostly groups of one row).
template <bool CHECK>
__device__ void wv_item(const BgArgs &A, const Ctx<true> &C, uint64_t b0, uint64_t e, uint32_t i, uint32_t lane,
                        RowView &v, uint32_t &vkey, Pend &out) {
    const uint64_t pt0 = A.prof ? clock64() : 0;
    out.i = ~0u;
    const uint32_t item = (uint32_t)__builtin_amdgcn_readfirstlane((int)g_item[i]);
    const uint32_t kind = item >> 30, d = (item >> 23) & 0x7Fu;
    // the item's row as wave-uniform values (SGPRs: its arithmetic is scalar)
    // (the key: row, staged row, and whether the item reads the row's staged groups --
    // runs and groups of one row share it)
    if ((((item >> 20) & 0x3FFu) | ((kind & 1u) << 10)) != vkey) {
        vkey = ((item >> 20) & 0x3FFu) | ((kind & 1u) << 10);
        const DevRow &R = g_st.rows[d];
        auto u32 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
        auto u64 = [&](uint64_t x) { return (uint64_t)u32((uint32_t)x) | ((uint64_t)u32((uint32_t)(x >> 32)) << 32); };
        v.R.text_off = u64(R.text_off);
        v.R.geno_len = u64(R.geno_len);
        v.R.code_off = u64(R.code_off);
        v.R.head_off = u32(R.head_off);
        v.R.head_len = u32(R.head_len);
        v.R.tok = u32(R.tok);
        v.R.width = u32(R.width);
        v.R.cum_off = u32(R.cum_off);
        v.R.nv = u32(R.nv);
        v.mask = (1u << v.R.width) - 1u;
        if (kind & 1u) {  // IT_GROUP, IT_RUN: its staged codes, tokens and group offsets (item bits 20-22)
            const StRow &T = g_st.P.st[(item >> 20) & 7u];
            v.cbase = (int32_t)u32(T.code_at) - (int32_t)u32(T.cfirst);
            v.tok_at = u32(T.tok_at);
            v.cum_at = u32(T.cum_at);
            v.g_lo = u32(T.g_lo);
            v.ncum = u32(T.ncum);
        } else {
            v.cbase = 0;
            v.tok_at = v.cum_at = v.g_lo = v.ncum = 0;
        }
    }
    if (A.prof && lane == 0) atomicAdd(&g_pstat[kind == IT_NL ? 6 : 5], kind != IT_GROUP ? 1u : 0u);
    if (kind == IT_NL) {
        const uint32_t base = wv_place(i, 8, lane);
        if (lane == 0) {
            wv_text_byte<CHECK>(A, (uint32_t)(v.R.text_off + v.R.head_len + v.R.geno_len - b0), '\n');
            LaneBits o{0, 0, base};
            wv_lit(o, '\n');
            o.finish();
        }
        return;
    }
    if (kind == IT_HEAD) {
        const uint64_t hs = max(b0, v.R.text_off), he = min(e, v.R.text_off + v.R.head_len);
        uint32_t total = 0;
        for (uint64_t q0 = hs; q0 < he; q0 += 64) {
            const uint64_t q = q0 + lane;
            const bool in = q < he;
            const uint32_t b = in ? (uint8_t)A.heads[v.R.head_off + (q - v.R.text_off)] : 0u;
            if (in) wv_text_byte<CHECK>(A, (uint32_t)(q - b0), b);
            total += wave_sum(in ? lit_bits(b) : 0u);
        }
        uint32_t at = wv_place(i, total, lane);
        for (uint64_t q0 = hs; q0 < he; q0 += 64) {
            const uint64_t q = q0 + lane;
            const bool in = q < he;
            const uint32_t b = in ? (uint8_t)A.heads[v.R.head_off + (q - v.R.text_off)] : 0u;
            const uint32_t nb = in ? lit_bits(b) : 0u;
            LaneBits o{0, 0, at + wave_excl_sum(nb, lane)};
            if (in) wv_lit(o, b);
            o.finish();
            at += wave_sum(nb);
        }
        return;
    }
    if (kind == IT_RUN) {
        // G groups of 64 samples of one text that the sample before them also has, inside
        // the block (bgzf_wave_kernel's listing): one run of 64 G texts, so its symbols
        // follow from the run's length alone: 258-byte matches at distance t, then the
        // remainder r (r = 1, 2: the last whole match gives 3 - r bytes to a final 3-byte
        // match); at most 59 + 2 symbols (G <= 15, t <= 16), a lane each
        const uint32_t g = item & 0xFFFFu, G = (item >> 16) & 15u;
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)C.code(v, g * kCumGroup));
        const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)C.tlen(v, c0));
        const uint4 tx = C.ttext(v, c0);
        const uint32_t cum_g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g_st.cum[v.cum_at + g - v.g_lo]);
        const int32_t rel0 = (int32_t)((int64_t)(v.R.text_off + v.R.head_len + cum_g) - (int64_t)b0);
        for (uint32_t j = 0; j < G; j++) wv_text_or<CHECK>(A, rel0 + (int32_t)((kCumGroup * j + lane) * t0), t0, tx);
        const uint32_t Lr = kCumGroup * G * t0, nfull = Lr / 258, r = Lr % 258;
        const bool split = r == 1 || r == 2;
        const uint32_t n258 = split ? nfull - 1 : nfull;
        const uint2 M = match_code(258, t0);
        const uint2 X = split ? match_code(255 + r, t0) : (r ? match_code(r, t0) : uint2{0, 0});
        const uint2 Y = split ? match_code(3, t0) : uint2{0, 0};
        if (A.prof && lane == 0) atomicAdd(&g_pstat[1], G);
        const uint2 sym = lane < n258 ? M : (lane == n258 ? X : (lane == n258 + 1 ? Y : uint2{0, 0}));
        out.total = n258 * M.y + X.y + Y.y;
        out.bw[0] = sym.x;
        out.bw[1] = out.bw[2] = out.bw[3] = 0;
        out.bn = sym.y;  // (lane k's symbol starts after lanes 0 .. k - 1's)
        wv_publish(i, out.total, lane);
        out.i = i;
        wv_pcycles(A, lane, 8, pt0);
        return;
    }
    // a 64-sample group
    const uint32_t g = item & 0xFFFFu, N = A.n_samples;
    const uint32_t s = g * kCumGroup + lane;
    const bool valid = s < N;
    // the sample's code and the one before's, then its text (one round of LDS reads each)
    uint32_t c = 0, t = 0;
    const uint32_t prevc = valid && s > 0 ? C.code(v, s - 1) : 0xFFFFFFFFu;
    if (valid) c = C.code(v, s);
    const uint32_t cum_g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g_st.cum[v.cum_at + g - v.g_lo]);
    const int32_t n = (int32_t)(e - b0);
    if (valid) t = C.tlen(v, c);
    const uint4 tx = C.ttext(v, c);
    const uint32_t tlitn = g_tlitn[v.tok_at + c];  // (loaded with the text)
    const uint4 tlit = g_tlit[v.tok_at + c];
    // the text's first byte relative to the block start (may be negative at its edge)
    const int32_t rel = (int32_t)((int64_t)(v.R.text_off + v.R.head_len + cum_g) - (int64_t)b0) +
                        (int32_t)wave_excl_sum(t, lane);
    const int32_t lo = max(rel, 0), hi = min(rel + (int32_t)t, n);
    const bool in = valid && hi > lo;
    const bool full = in && rel >= 0 && rel + (int32_t)t <= n;
    const bool run = full && prevc == c && rel >= (int32_t)t && t >= 1;
    // the wave's runs: a run's first and last texts
    const uint64_t rm = __ballot(run);
    const uint64_t starts = rm & ~(rm << 1), ends = rm & ~(rm >> 1);
    const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t sb = starts & below, ea = ends & ~((1ull << lane) - 1ull);
    const uint32_t sl = sb ? 63u - (uint32_t)__builtin_clzll(sb) : lane;
    const uint32_t el = ea ? (uint32_t)__builtin_ctzll(ea) : lane;
    const int32_t S0 = __shfl(rel, sl), S1 = __shfl(rel + (int32_t)t, el);
    // the same text among the 8 before it, inside the block: the nearest, from the
    // 8 packed codes before the sample (a zero-field test of codes ^ c), its distance
    // from the texts' offsets (a lane of this item, or the token lengths between);
    // 8-bit codes and a row's first 8 samples: sample by sample
    uint32_t dist = 0;
    const bool want = full && !run && t >= 3;
#ifdef BG_PROBE_NOLB
    const bool packed = false && want;
#else
    const bool packed = want && v.R.width <= 4 && s >= kLookback;
#endif
    uint32_t kk = 0, P = 0;
    if (packed) {
        const uint32_t w = v.R.width, bit0 = (s - kLookback) * w, a = (uint32_t)(v.cbase + (int32_t)(bit0 >> 3));
        const uint32_t *dw = reinterpret_cast<const uint32_t *>(g_st.codes) + (a >> 2);
        const uint64_t x = (uint64_t)dw[0] | ((uint64_t)dw[1] << 32);
        P = (uint32_t)(x >> (8 * (a & 3u) + (bit0 & 7u)));  // field k: sample s - 8 + k
        const uint32_t R = w == 2 ? 0x5555u : 0x11111111u, H = R << (w - 1), M = H - R;
        if (w == 2) P &= 0xFFFFu;
        const uint32_t X = P ^ (c * R), Z = ~(((X & M) + M) | X | M) & H;
        if (Z) kk = kLookback - ((31u - __builtin_clz(Z)) >> (w == 2 ? 1 : 2));
    }
    const int32_t rsrc = __shfl(rel, (int)(lane - min(kk, lane)));
    if (kk) {
        uint32_t acc;
        if (kk <= lane) {
            acc = (uint32_t)(rel - rsrc);
        } else {  // sample s - kk is in the group before
            acc = 0;
#pragma unroll
            for (uint32_t k = 1; k <= kLookback; k++)  // (all loads at once)
                acc += k <= kk ? C.tlen(v, (P >> ((kLookback - k) * v.R.width)) & v.mask) : 0u;
        }
        if (rel >= (int32_t)acc) dist = acc;
    } else if (want && !packed) {
        uint32_t acc = 0;
        for (uint32_t k = 1; k <= kLookback && k <= s; k++) {
            const uint32_t cc = C.code(v, s - k);
            acc += C.tlen(v, cc);
            if (rel < (int32_t)acc) break;
            if (cc == c) {
                dist = acc;
                break;
            }
        }
    }
    // the run's matches that start in this text: 258 bytes each from the run's first
    // byte; a remainder of 1-2 bytes moves 3 - r bytes of the last whole match into a
    // final 3-byte match
    uint32_t m1 = 0, m2 = 0;
    const bool runm = run && S1 - S0 >= 3;  // (texts are >= 4 bytes: every run is)
    if (runm) {
        const uint32_t a = (uint32_t)(rel - S0), b = a + t, Lr = (uint32_t)(S1 - S0);
        const uint32_t nfull = Lr / 258, r = Lr % 258;
        const uint32_t j = (a + 257) / 258;
        if (258 * j < b) {
            if (r == 0 || r >= 3) m1 = j < nfull ? 258u : (j == nfull ? r : 0u);
            else m1 = j + 1 < nfull ? 258u : (j + 1 == nfull ? 255u + r : 0u);
        }
        if ((r == 1 || r == 2) && Lr >= 3 && a <= Lr - 3 && Lr - 3 < b) m2 = 3;
    }
    // the text's bytes (for the CRC)
#ifdef BG_PROBE_NOTEXT
    if (false) {
#else
    if (full) {
#endif
        wv_text_or<CHECK>(A, rel, t, tx);
    } else if (in) {
        for (int32_t q = lo; q < hi; q++) wv_text_byte<CHECK>(A, (uint32_t)q, Ctx<true>::byte_of(tx, (uint32_t)(q - rel)));
    }
    // its bits, its place in the block's stream, its symbols: a match or two, or a
    // whole token's literal codes, as up to 4 words (LSB first) that go into the
    // stream with at most two LDS ORs each; texts cut by the block's edges and tokens
    // of more than 128 bits of literals go byte by byte (rare)
    const uint32_t tn = in ? tlitn : 0u;
    const bool whole_lit = full && tn != kNoTokLit;
    const bool by_byte = in && !runm && !dist && !whole_lit;
    uint32_t bw[4] = {0, 0, 0, 0}, bn = 0;
    if (runm || dist) {
        const uint2 a = runm ? (m1 ? match_code(m1, t) : uint2{0, 0}) : match_code(t, dist);
        const uint2 b = runm && m2 ? match_code(m2, t) : uint2{0, 0};
        const uint64_t x = (uint64_t)a.x | ((uint64_t)b.x << a.y);
        bw[0] = (uint32_t)x;
        bw[1] = (uint32_t)(x >> 32);
        bn = a.y + b.y;
    } else if (whole_lit) {
        const uint4 L = tlit;
        bw[0] = L.x;
        bw[1] = L.y;
        bw[2] = L.z;
        bw[3] = L.w;
        bn = tn;
    }
    uint32_t nb = bn;
    const bool any_bytes = __ballot(by_byte) != 0;
    if (any_bytes && by_byte)
        for (int32_t q = lo; q < hi; q++) nb += lit_bits(Ctx<true>::byte_of(tx, (uint32_t)(q - rel)));
    if (A.prof) {
        const bool all_run = __ballot(run) == ~0ull, lb = __ballot(dist != 0) != 0,
                   wl = __ballot(!runm && !dist && whole_lit) != 0, ser = __ballot(want && !packed) != 0;
        if (lane == 0) {
            atomicAdd(&g_pstat[7], 1u);
            if (ser) atomicAdd(&g_pstat[14], 1u);
            if (all_run) atomicAdd(&g_pstat[1], 1u);
            if (lb) atomicAdd(&g_pstat[2], 1u);
            if (wl) atomicAdd(&g_pstat[3], 1u);
            if (any_bytes) atomicAdd(&g_pstat[4], 1u);
        }
    }
    const uint32_t total = wave_sum(nb);
    if (!any_bytes) {  // (nb == bn)
        wv_publish(i, total, lane);
        out.total = total;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) out.bw[k] = bw[k];
        out.bn = bn;
        out.i = i;
        wv_pcycles(A, lane, 11, pt0);
        return;
    }
    const uint32_t off = wv_place(i, total, lane) + wave_excl_sum(nb, lane);
    wv_words(off, bw, bn);
    if (by_byte) {
        LaneBits o{0, 0, off};
        for (int32_t q = lo; q < hi; q++) wv_lit(o, Ctx<true>::byte_of(tx, (uint32_t)(q - rel)));
        o.finish();
    }
    wv_pcycles(A, lane, 12, pt0);
}

template <bool CHECK>
__global__ __launch_bounds__(kWv) void bgzf_wave_kernel(BgArgs A) {
    Stage &S = g_st;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t b0 = (A.block0 + blockIdx.x) * kBgzfRaw;
    const uint32_t n = (uint32_t)min((uint64_t)kBgzfRaw, A.text_bytes - b0);
    const uint64_t e = b0 + n;
    // phase clocks (TFBS_BGZF_PROF): start, staged, items listed, items done, CRC, end
    uint64_t *const pf = A.prof ? A.prof + 32 * (size_t)blockIdx.x : nullptr;
    auto stamp = [&](int k) {
        if (pf && tid == 0) pf[k] = clock64();
    };
    stamp(0);
    if (tid < 16) g_pstat[tid] = 0;
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(reinterpret_cast<const BlockPlan *>(A.plans) + blockIdx.x);
        for (uint32_t i = tid; i < sizeof(BlockPlan) / 4; i += kWv) reinterpret_cast<uint32_t *>(&S.P)[i] = src[i];
    }
    __syncthreads();
    if (!S.P.all) return;  // (uniform) bgzf_block_kernel's block
    // the block's reads as one flat list of segments -- the CRC tables, the rows'
    // descriptors, per staged row its codes (dwords from the aligned-down source: the
    // plan put code_at at the same offset mod 4), token texts, token lengths (bytes),
    // group offsets and the tokens' literal codes and bit counts (bytes; tok_lit_kernel)
    // --, every thread issuing its loads before its stores (a loop per segment waited on
    // one load per segment).  The list lives in g_item (listed later): [0, 64) source
    // low words, [64, 128) high words, [128, 192) destination: byte offset into g_st /
    // g_tlit / g_tlitn (bits 29-30), bit 31: a byte segment; [192, 256) the segments'
    // inclusive end in units.
    for (uint32_t i = tid; i <= kBitWords; i += kWv) g_bits[i] = i ? 0u : 0x3u;  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
    for (uint32_t i = tid; i < kWvItems; i += kWv) g_pub[i] = g_agg[i] = 0;
    for (uint32_t i = tid; i < sizeof(g_text) / 16; i += kWv) reinterpret_cast<uint4 *>(g_text)[i] = uint4{0, 0, 0, 0};
    if (wave == 0) {
        static_assert(4 + 6 * kStRows <= 64 && 256 <= kWvItems, "the segment list");
        uint64_t src = 0;
        uint32_t dst = 0, nu = 0;
        if (lane == 0) {
            src = (uint64_t)A.crc_tab;
            dst = offsetof(Stage, crc_tab);
            nu = 256;
        } else if (lane == 1) {
            src = (uint64_t)A.crc_ops;
            dst = offsetof(Stage, crc_ops);
            nu = kCrcOps * 32;
        } else if (lane == 2) {
            src = (uint64_t)A.crc_slice;
            dst = offsetof(Stage, crc_slice);
            nu = 768;
        } else if (lane == 3) {
            src = (uint64_t)(A.rows + S.P.r_first);
            dst = offsetof(Stage, rows);
            nu = S.P.n_rows * (uint32_t)(sizeof(DevRow) / 4);
        } else if (lane < 4 + 6 * S.P.n_st) {
            const uint32_t k = (lane - 4) / 6, m = (lane - 4) % 6;
            const StRow &T = S.P.st[k];
            if (m == 0) {
                const uint64_t a = T.code_off + T.cfirst;
                const uint32_t lead = (uint32_t)(a & 3u), nb = (T.s_hi * T.width + 7) / 8 - T.cfirst;
                src = (uint64_t)(A.codes + (a - lead));
                dst = (uint32_t)offsetof(Stage, codes) + T.code_at - lead;
                nu = (lead + nb + 3) / 4;
            } else if (m == 1) {
                src = (uint64_t)(A.tok_text + (size_t)T.tok * kRowTokBytes);
                dst = (uint32_t)offsetof(Stage, text) + T.tok_at * kRowTokBytes;
                nu = T.nv * (kRowTokBytes / 4);
            } else if (m == 2) {
                src = (uint64_t)(A.tok_len + T.tok);
                dst = ((uint32_t)offsetof(Stage, tlen) + T.tok_at) | 0x80000000u;
                nu = T.nv;
            } else if (m == 3) {
                src = (uint64_t)(A.cum + T.cum_off + T.g_lo);
                dst = (uint32_t)offsetof(Stage, cum) + 4 * T.cum_at;
                nu = T.ncum;
            } else if (m == 4) {
                src = (uint64_t)(A.tok_lit + T.tok);
                dst = (1u << 29) | (16 * T.tok_at);
                nu = T.nv * 4;
            } else {
                src = (uint64_t)(A.tok_litn + T.tok);
                dst = 0x80000000u | (2u << 29) | T.tok_at;
                nu = T.nv;
            }
        }
        g_item[lane] = (uint32_t)src;
        g_item[64 + lane] = (uint32_t)(src >> 32);
        g_item[128 + lane] = dst;
        g_item[192 + lane] = wave_incl_sum(nu);  // (lanes past the list: the total)
    }
    __syncthreads();
    {
        uint8_t *const sb = reinterpret_cast<uint8_t *>(&g_st);
        uint8_t *const sl = reinterpret_cast<uint8_t *>(g_tlit);
        const uint32_t total = g_item[192 + 63];
        for (uint32_t u0 = tid; u0 < total; u0 += 4 * kWv) {
            uint32_t val[4], at[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t u = u0 + j * kWv;
                at[j] = ~0u;
                val[j] = 0;
                if (u < total) {
                    uint32_t k = 0;  // the first segment ending past u
#pragma unroll
                    for (uint32_t b = 32; b; b >>= 1)
                        if (g_item[192 + k + b - 1] <= u) k += b;
                    const uint32_t idx = u - (k ? g_item[192 + k - 1] : 0u), d = g_item[128 + k];
                    const uint64_t src = (uint64_t)g_item[k] | ((uint64_t)g_item[64 + k] << 32);
                    if (d >> 31) {
                        val[j] = *reinterpret_cast<const uint8_t *>(src + idx);
                        at[j] = d + idx;
                    } else {
                        val[j] = *reinterpret_cast<const uint32_t *>(src + 4 * (uint64_t)idx);
                        at[j] = d + 4 * idx;
                    }
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                if (at[j] == ~0u) continue;
                const uint32_t o = at[j] & 0x1FFFFFFFu, base = (at[j] >> 29) & 3u;
                if (at[j] >> 31) (base == 2 ? g_tlitn : sb)[o] = (uint8_t)val[j];
                else *reinterpret_cast<uint32_t *>((base == 1 ? sl : sb) + o) = val[j];
            }
        }
    }
    __syncthreads();
    stamp(1);
    // the block's items in stream order: per row its head, its groups, its newline;
    // counted per row, offsets by a wave scan, then one wave per row writes them (its
    // lanes the groups: a row holds up to kStCum of them)
    const Ctx<true> C{A, b0};
    auto row_items = [&](uint32_t r, bool &head, bool &nl, uint32_t &groups, uint32_t &k_st) {
        const DevRow &R = S.rows[r];
        head = R.head_len && R.text_off < e && R.text_off + R.head_len > b0;
        const uint64_t q = R.text_off + R.head_len + R.geno_len;
        nl = q >= b0 && q < e;
        groups = 0;
        k_st = 0;
        for (uint32_t k = 0; k < S.P.n_st; k++)
            if (S.P.st[k].row == S.P.r_first + r) {
                groups = S.P.st[k].ncum - 1;
                k_st = k;
            }
    };
    // a group is part of a run when its 64 samples and the one before have one code and
    // its texts lie inside the block with the text before; up to kRunGroups consecutive
    // run groups of a row make one IT_RUN item (each starting a new run: the symbols
    // depend on the run's length only).  A thread per staged group (Stage::cum's index,
    // the lower waves; the upper ones make the literal codes) tests its packed codes as
    // whole dwords against the code's byte pattern; then each wave takes a contiguous
    // share of the rows, turns their groups' flags into items and counts them, and after
    // one barrier writes them from its share's offset (the waves' counts before it).
    // The flags live in g_ioff[kFlags + Stage::cum index]: bit 0 an item starts here,
    // bit 1 a run, bits 2-5 the run's groups; g_ioff[0, 16) the waves' counts.
    constexpr uint32_t kFlags = kWv / 64;
    static_assert(kFlags + kStCum <= kWvItems, "the listing's flags");
    if (tid < kStCum) {
        bool run = false;
        for (uint32_t k = 0; k < S.P.n_st; k++) {
            const StRow &T = S.P.st[k];
            if (tid < T.cum_at || tid + 1 >= T.cum_at + T.ncum) continue;  // (ncum - 1 groups)
            const uint32_t g = T.g_lo + tid - T.cum_at, w = T.width;
            if (g == 0 || g * kCumGroup + kCumGroup > A.n_samples) break;
            const uint32_t a = T.code_at - T.cfirst + ((g * kCumGroup * w) >> 3);  // (a whole byte)
            const uint32_t *dw = reinterpret_cast<const uint32_t *>(S.codes) + (a >> 2), sh = 8 * (a & 3u);
            const uint32_t c = S.codes[a] & ((1u << w) - 1u);
            const uint32_t pat = (w == 8 ? c : (w == 4 ? c * 0x11u : (w == 2 ? c * 0x55u : (c ? 0xFFu : 0u)))) * 0x01010101u;
            bool same = ((uint32_t)S.codes[a - 1] >> (8 - w)) == c;  // the sample before
#pragma unroll
            for (uint32_t j = 0; j < 16; j++)  // the 2 w dwords of the group's codes
                if (j < 2 * w) same = same && (uint32_t)((((uint64_t)dw[j + 1] << 32) | dw[j]) >> sh) == pat;
            const DevRow &R = S.rows[T.row - S.P.r_first];
            const uint32_t t = S.tlen[T.tok_at + c];
            const int64_t rel0 = (int64_t)(R.text_off + R.head_len + S.cum[tid]) - (int64_t)b0;
            run = same && t >= 1 && rel0 >= (int64_t)t && rel0 + kCumGroup * t <= (int64_t)(e - b0);
            break;
        }
        g_ioff[kFlags + tid] = run ? 1u : 0u;
    }
    __syncthreads();
    stamp(7);
    const uint32_t r_lo = wave * S.P.n_rows / (kWv / 64), r_hi = (wave + 1) * S.P.n_rows / (kWv / 64);
    {
        uint32_t cnt = 0;
        for (uint32_t r = r_lo; r < r_hi; r++) {
            bool head, nl;
            uint32_t groups, k_st;
            row_items(r, head, nl, groups, k_st);
            cnt += (head ? 1u : 0u) + (nl ? 1u : 0u);
            const uint32_t *const fl = g_ioff + kFlags + S.P.st[k_st].cum_at;
            for (uint32_t q0 = 0; q0 < groups; q0 += 64) {
                const uint32_t q = q0 + lane;
                const bool in = q < groups;
                const bool run = in && fl[q] != 0;
                const uint64_t rb = __ballot(run);
                const bool link = run && lane > 0 && ((rb >> (lane - 1)) & 1u);  // (a window starts its own item)
                const uint64_t nl_mask = ~__ballot(link) | 1ull, below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
                const uint32_t first = 63u - (uint32_t)__builtin_clzll(nl_mask & below);  // the chain's start lane
                const bool start = in && (!link || (lane - first) % kRunGroups == 0);
                const uint64_t sm = __ballot(start);
                const uint64_t after = lane == 63 ? 0ull : (sm & ~below);
                const uint32_t next = min(after ? (uint32_t)__builtin_ctzll(after) : 64u, groups - q0);
                if (in) const_cast<uint32_t *>(fl)[q] = start ? (1u | (run ? 2u : 0u) | ((next - lane) << 2)) : 0u;
                cnt += (uint32_t)__builtin_popcountll(sm);
            }
        }
        if (lane == 0) g_ioff[wave] = cnt;
    }
    __syncthreads();
    {
        const uint32_t x = lane < kWv / 64 ? g_ioff[lane] : 0u;
        uint32_t at = wave_sum(lane < wave ? x : 0u);  // the waves' items before this one's rows
        if (wave == 0) {
            const uint32_t total = wave_sum(x);
            if (lane == 0) g_ioff[kWvItems] = total;
        }
        for (uint32_t r = r_lo; r < r_hi; r++) {
            bool head, nl;
            uint32_t groups, k_st;
            row_items(r, head, nl, groups, k_st);
            if (head && lane == 0) g_item[at] = (IT_HEAD << 30) | (r << 23);
            at += head ? 1u : 0u;
            const StRow &T = S.P.st[k_st];
            for (uint32_t q0 = 0; q0 < groups; q0 += 64) {
                const uint32_t q = q0 + lane;
                const uint32_t f = q < groups ? g_ioff[kFlags + T.cum_at + q] : 0u;
                const uint64_t sm = __ballot(f & 1u);
                if (f & 1u) {
                    const uint32_t k = at + (uint32_t)__builtin_popcountll(sm & ((1ull << lane) - 1ull));
                    g_item[k] = ((f & 2u) ? (IT_RUN << 30) | (((f >> 2) & 15u) << 16) : (IT_GROUP << 30)) | (r << 23) |
                                (k_st << 20) | (T.g_lo + q);
                }
                at += (uint32_t)__builtin_popcountll(sm);
            }
            if (nl && lane == 0) g_item[at] = (IT_NL << 30) | (r << 23);
            at += nl ? 1u : 0u;
        }
    }
    __syncthreads();
    const uint32_t n_items = g_ioff[kWvItems];
    stamp(2);
    // the items in one pass (wv_item: the bytes, the bit count, the chained offset, the
    // bits); a block that does not shrink to the bit buffer is stored instead
    {
        RowView v{};
        uint32_t vkey = ~0u;
        Pend pend{~0u, 0, {0, 0, 0, 0}, 0};
        for (uint32_t i = wave; i < n_items; i += kWv / 64) {
            Pend cur;
            wv_item<CHECK>(A, C, b0, e, i, lane, v, vkey, cur);
#ifdef BG_NO_DEFER  // (timing probe: each group placed at once)
            if (cur.i != ~0u) wv_emit(A, cur, lane);
            continue;
#endif
            if (pend.i != ~0u) wv_emit(A, pend, lane);
            pend = cur;
        }
        if (pend.i != ~0u) wv_emit(A, pend, lane);
    }
    __syncthreads();
    stamp(3);
    const uint32_t total_bits = g_pub[n_items - 1] - 1 + 7;  // BFINAL + BTYPE, symbols, end of block
    const uint32_t dbytes = (total_bits + 7) / 8;
    const bool stored = dbytes > 4 * kBitWords || A.stored;
    // the CRC32 of the block's bytes: 64 per thread counted from the block's end, so
    // that thread t's CRC shifts by 64 (kWv - 1 - t) = 64 (63 - lane) + 4096 (15 - wave)
    // bytes: each lane applies its lane operator (x^(8 * 64 (63 - lane)), a column per
    // register from the table, coalesced), the wave XORs and applies its wave operator
    // (x^(8 * 4096 (15 - wave)); the tables' reads issued before the slice), then wave 0
    // XORs the waves' (CRC(a b) = x^(8 |b|) CRC(a) ^ CRC(b)) and the init term (a full
    // block's precomputed)
    {
        // (the lane table, 2 048 words, goes to LDS over the codes -- dead: the items are
        // done -- two words per thread; the wave's columns are wave-uniform: scalar loads)
        const uint32_t lt0 = A.crc_lane[tid], lt1 = A.crc_lane[kWv + tid];
        typedef const __attribute__((address_space(4))) uint32_t *ConstPtr;
        const ConstPtr W = (ConstPtr)(uintptr_t)(A.crc_lane + 64 * 32 + 32 * __builtin_amdgcn_readfirstlane((int)wave));
        uint32_t wcol[32];
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) wcol[i] = W[i];
        const int32_t q1 = (int32_t)n - 64 * (kWv - 1 - (int32_t)tid), q0 = max(0, q1 - 64);
        uint32_t crc = 0;
        if (q1 - q0 == 64 && (q0 & 63) == 0) {  // a whole padded slice: dword reads, no bank conflicts
            const uint32_t *w = reinterpret_cast<const uint32_t *>(g_text) + (txt_at((uint32_t)q0) >> 2);
            for (uint32_t i = 0; i < 16; i++) {  // slice-by-4: four independent table reads per dword
                const uint32_t x = w[i] ^ crc;
                crc = S.crc_slice[512 + (x & 0xFFu)] ^ S.crc_slice[256 + ((x >> 8) & 0xFFu)] ^
                      S.crc_slice[(x >> 16) & 0xFFu] ^ S.crc_tab[x >> 24];
            }
        } else {
            for (int32_t q = q0; q < q1; q++) crc = crc_byte(S.crc_tab, crc, g_text[txt_at((uint32_t)q)]);
        }
        uint32_t *const lt = reinterpret_cast<uint32_t *>(S.codes);
        lt[tid] = lt0;
        lt[kWv + tid] = lt1;
        __syncthreads();
        uint32_t r = 0;
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) r ^= ((crc >> i) & 1u) ? lt[i * 64 + lane] : 0u;
#pragma unroll
        for (uint32_t o = 32; o; o >>= 1) r ^= (uint32_t)__shfl_xor((int)r, (int)o);
        uint32_t rw = 0;
#pragma unroll
        for (uint32_t i = 0; i < 32; i++) rw ^= ((r >> i) & 1u) ? wcol[i] : 0u;
        if (lane == 0) g_red[wave] = rw;
        __syncthreads();
        if (wave == 0) {
            r = lane < kWv / 64 ? g_red[lane] : 0u;
#pragma unroll
            for (uint32_t o = 8; o; o >>= 1) r ^= (uint32_t)__shfl_xor((int)r, (int)o);
            if (lane == 0)
                g_red[0] = r ^ (n == kBgzfRaw ? A.crc_full : crc_shift_lds(S.crc_ops, 0xFFFFFFFFu, n)) ^ 0xFFFFFFFFu;
        }
        __syncthreads();
    }
    stamp(4);
    // the block (header, deflate data, CRC32, ISIZE) in aligned 16-byte stores, every
    // thread its share: inside the deflate data a dword is two bit-buffer words
    // funnelled (block byte 18 = bit-buffer byte 0), the few dwords around it byte by byte
    uint8_t *out = A.out + (size_t)blockIdx.x * kBgzfMax;
    const uint32_t clen = stored ? 5 + n : dbytes;
    const uint32_t bsize = 18 + clen + 8;
    const uint32_t crc32 = g_red[0];
    auto byte_at = [&](uint32_t p) -> uint32_t {
        if (p < 16) {
            constexpr uint32_t h0 = 0x04088b1fu, h2 = 0x0006ff00u, h3 = 0x00024342u;
            const uint32_t w = (p >> 2) == 0 ? h0 : (p >> 2) == 2 ? h2 : (p >> 2) == 3 ? h3 : 0u;
            return (w >> (8 * (p & 3))) & 0xFFu;
        }
        if (p < 18) return ((bsize - 1) >> (8 * (p - 16))) & 0xFFu;
        if (p < 18 + clen) {
            if (!stored) return (g_bits[(p - 18) >> 2] >> (8 * ((p - 18) & 3))) & 0xFFu;
            if (p >= 23) return g_text[txt_at(p - 23)];
            const uint32_t len = n | ((~n & 0xFFFFu) << 16);  // LEN, NLEN after BFINAL = 1, BTYPE = 00
            return p == 18 ? 1u : (len >> (8 * (p - 19))) & 0xFFu;
        }
        if (p < 22 + clen) return (crc32 >> (8 * (p - 18 - clen))) & 0xFFu;
        if (p < bsize) return (n >> (8 * (p - 22 - clen))) & 0xFFu;
        return 0u;
    };
    const uint32_t n16 = (bsize + 15) / 16;
    for (uint32_t c = tid; c < n16; c += kWv) {
        uint32_t w[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t p = 16 * c + 4 * k;
            if (!stored && p >= 20 && p + 4 <= 18 + clen) {
                const uint32_t j = (p - 18) >> 2;  // p - 18 = 4 j + 2
                w[k] = (g_bits[j] >> 16) | (g_bits[j + 1] << 16);
            } else {
                w[k] = byte_at(p) | byte_at(p + 1) << 8 | byte_at(p + 2) << 16 | byte_at(p + 3) << 24;
            }
        }
        reinterpret_cast<uint4 *>(out)[c] = uint4{w[0], w[1], w[2], w[3]};
    }
    if (tid == 0) A.out_len[blockIdx.x] = bsize;
    stamp(5);
    if (pf && tid == 0) {
        pf[6] = n_items;
        for (int k = 0; k < 16; k++) pf[8 + k] = g_pstat[k];
    }
}

// Per token of the launch's rows: its text's bytes past its length zeroed (the wave
// kernel ORs whole text dwords into the block's bytes) and its fixed-Huffman literal
// codes, LSB first, with their bit count (kNoTokLit: more than 128 bits), which the
// wave kernel stages with the texts.
__global__ __launch_bounds__(256) void tok_lit_kernel(uint32_t *__restrict__ text, const uint8_t *__restrict__ len,
                                                      uint32_t n_tok, uint4 *__restrict__ lit, uint8_t *__restrict__ litn) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n_tok) return;
    const uint32_t t = len[k];
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int32_t keep = (int32_t)t - 4 * j;  // bytes of dword j inside the text
        w[j] = text[4 * k + j] & (keep >= 4 ? ~0u : (keep <= 0 ? 0u : (1u << (8 * keep)) - 1u));
        text[4 * k + j] = w[j];
    }
    uint64_t lo = 0, hi = 0;
    uint32_t nb = 0;
    for (uint32_t i = 0; i < t && nb <= 128; i++) {
        const uint32_t b = (w[(i >> 2) & 3u] >> (8 * (i & 3))) & 0xFFu;
        const uint32_t code = b < 144 ? rev(0x30 + b, 8) : rev(0x190 + b - 144, 9), n = b < 144 ? 8u : 9u;
        if (nb < 64) {
            lo |= (uint64_t)code << nb;
            if (nb + n > 64) hi |= (uint64_t)code >> (64 - nb);
        } else {
            hi |= (uint64_t)code << (nb - 64);
        }
        nb += n;
    }
    lit[k] = uint4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    litn[k] = (uint8_t)(nb <= 128 ? nb : kNoTokLit);
}

// off[i] = the sizes of blocks before i, off[nb] = their total (one workgroup).
__global__ __launch_bounds__(1024) void bgzf_offsets_kernel(const uint32_t *__restrict__ len, uint32_t nb,
                                                            uint64_t *__restrict__ off) {
    __shared__ uint64_t s_sum[1024];
    const uint32_t tid = threadIdx.x, per = (nb + 1023) / 1024;
    const uint32_t i0 = min(nb, tid * per), i1 = min(nb, i0 + per);
    uint64_t mine = 0;
    for (uint32_t i = i0; i < i1; i++) mine += len[i];
    s_sum[tid] = mine;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint64_t t = tid >= o ? s_sum[tid - o] : 0;
        __syncthreads();
        s_sum[tid] += t;
        __syncthreads();
    }
    uint64_t at = s_sum[tid] - mine;
    for (uint32_t i = i0; i < i1; i++) {
        off[i] = at;
        at += len[i];
    }
    if (tid == 1023) off[nb] = s_sum[1023];
}

// Copies each block to its offset of one contiguous buffer.
__global__ __launch_bounds__(256) void bgzf_compact_kernel(const uint8_t *__restrict__ in,
                                                           const uint64_t *__restrict__ off,
                                                           uint8_t *__restrict__ out) {
    const uint64_t o = off[blockIdx.x], n = off[blockIdx.x + 1] - o;
    const uint8_t *src = in + (size_t)blockIdx.x * kBgzfMax;
    for (uint64_t i = threadIdx.x; i < n; i += 256) out[o + i] = src[i];
}

}  // namespace

uint32_t bgzf_crc_tables(uint32_t *tab, uint32_t *ops, uint32_t *slice, uint32_t *lane) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        tab[i] = c;
    }
    // one zero byte: v -> tab[v & 0xff] ^ (v >> 8); 2^(k+1) bytes = 2^k bytes twice
    for (uint32_t i = 0; i < 32; i++) {
        const uint32_t v = 1u << i;
        ops[i] = tab[v & 0xFF] ^ (v >> 8);
    }
    for (uint32_t k = 1; k < kBgzfOps; k++)
        for (uint32_t i = 0; i < 32; i++) {
            uint32_t v = ops[32 * (k - 1) + i], r = 0;
            for (uint32_t j = 0; j < 32; j++)
                if ((v >> j) & 1u) r ^= ops[32 * (k - 1) + j];
            ops[32 * k + i] = r;
        }
    // slice-by-4: table k gives the CRC of a byte followed by k zero bytes
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = tab[i];
        for (uint32_t k = 0; k < 3; k++) {
            c = tab[c & 0xFFu] ^ (c >> 8);
            slice[256 * k + i] = c;
        }
    }
    // x^(8 n) on v: the operators of n's set bits in turn
    auto shift = [&](uint32_t v, uint32_t n) {
        for (uint32_t k = 0; n; k++, n >>= 1)
            if (n & 1u) {
                uint32_t r = 0;
                for (uint32_t j = 0; j < 32; j++)
                    if ((v >> j) & 1u) r ^= ops[32 * k + j];
                v = r;
            }
        return v;
    };
    // bgzf_wave_kernel's lane operators x^(8 * 64 (63 - l)), column i of lane l at
    // [64 i + l], then its wave operators x^(8 * 4096 (15 - w)), column i at [2048 + 32 w + i]
    for (uint32_t l = 0; l < 64; l++)
        for (uint32_t i = 0; i < 32; i++) lane[64 * i + l] = shift(1u << i, 64 * (63 - l));
    for (uint32_t w = 0; w < 16; w++)
        for (uint32_t i = 0; i < 32; i++) lane[64 * 32 + 32 * w + i] = shift(1u << i, 4096 * (15 - w));
    return shift(0xFFFFFFFFu, kBgzfRaw);  // (on 0xFFFFFFFF: a full block's init term)
}

int launch_tok_lit(const BgArgs &a, uint32_t n_tok, hipStream_t stream) {
    if (n_tok == 0) return TFBS_OK;
    hipLaunchKernelGGL(tok_lit_kernel, dim3((n_tok + 255) / 256), dim3(256), 0, stream,
                       reinterpret_cast<uint32_t *>(const_cast<char *>(a.tok_text)), a.tok_len, n_tok, a.tok_lit,
                       a.tok_litn);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("tok_lit_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_row_cum(const BgArgs &a, hipStream_t stream) {
    if (a.n_rows == 0) return TFBS_OK;
    hipLaunchKernelGGL(row_cum_kernel, dim3(a.n_rows), dim3(256), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("row_cum_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

size_t bgzf_plan_bytes() { return sizeof(BlockPlan); }

int launch_bgzf_blocks(const BgArgs &a, uint32_t n_blocks, hipStream_t stream) {
    if (n_blocks == 0) return TFBS_OK;
    hipLaunchKernelGGL(bgzf_plan_kernel, dim3((n_blocks + 255) / 256), dim3(256), 0, stream, a, n_blocks);
    if (a.check)
        hipLaunchKernelGGL(bgzf_wave_kernel<true>, dim3(n_blocks), dim3(kWv), 0, stream, a);
    else
        hipLaunchKernelGGL(bgzf_wave_kernel<false>, dim3(n_blocks), dim3(kWv), 0, stream, a);
    hipLaunchKernelGGL(bgzf_block_kernel, dim3(n_blocks), dim3(kBgBlock), 0, stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("bgzf_block_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

int launch_bgzf_compact(const uint8_t *in, const uint32_t *len, uint64_t *off, uint32_t n_blocks, uint8_t *out,
                        hipStream_t stream) {
    if (n_blocks == 0) return TFBS_OK;
    hipLaunchKernelGGL(bgzf_offsets_kernel, dim3(1), dim3(1024), 0, stream, len, n_blocks, off);
    hipLaunchKernelGGL(bgzf_compact_kernel, dim3(n_blocks), dim3(256), 0, stream, in, off, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(TFBS_E_HIP, std::string("bgzf_compact_kernel: ") + hipGetErrorString(e));
    return TFBS_OK;
}

}  // namespace tfbs
