// Raw DEFLATE decoder (RFC 1951) for the BGZF reader's blocks (io.cpp).
//
// The BCF's GT columns are long runs of one genotype pair ("0|0" as bytes 02 03),
// which deflate writes as chains of distance-2, length-258 matches: zlib copies
// those byte by byte.  This decoder reads the bit stream 64 bits at a time,
// decodes with one table lookup per symbol (canonical Huffman, 2-level tables),
// and copies matches 8 or 16 bytes per step (a period of 1, 2, 4 or 8 bytes as
// one 16-byte pattern stored repeatedly; other short periods unrolled first).  A block it cannot decode exactly (malformed data) returns an error and
// the caller inflates it with zlib instead.
#include <cstdint>
#include <cstring>

#include "io.hpp"
#include "../../include/tfbs_amd.h"

namespace tfbs {
namespace {

constexpr int kLitBits = 10, kDistBits = 8;  // main table index bits
constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

// Table entry: bits 0-3 code length (main entries) or sub-table index bits (links),
// bit 4 link, bits 16-31 the symbol or the sub-table's offset.
struct Table {
    uint32_t e[2048 + 2 * 2048];  // main table + sub-tables (worst case well inside)
    int bits = 0;
};

struct Rev8 {
    uint8_t r[256];
    Rev8() {
        for (int x = 0; x < 256; x++) {
            int y = 0;
            for (int i = 0; i < 8; i++) y |= ((x >> i) & 1) << (7 - i);
            r[x] = (uint8_t)y;
        }
    }
};
const Rev8 kRev8;
// the low n (<= 16) bits of x reversed
inline uint32_t rev_bits(uint32_t x, int n) {
    return (((uint32_t)kRev8.r[x & 0xFF] << 8) | kRev8.r[(x >> 8) & 0xFF]) >> (16 - n);
}

// How build() treats an incomplete code (fewer codes than its lengths allow), as
// zlib's inflate_table does: a dynamic block's code-length code must be complete,
// its literal/length and distance codes too unless they hold a single code of
// length 1 (or none at all); the fixed distance code (30 of 32) is incomplete.
enum Incomplete { kRejectIncomplete, kSingleCode, kAllowIncomplete };

// Entry payloads (bits 8-31) of the literal/length and distance codes: a literal's
// byte, a length's or distance's base with its extra-bit count, end of block, or a
// symbol the format reserves (286-287, 30-31).  One lookup then gives the whole
// length or distance: base + the extra bits that follow the code.
constexpr uint32_t kLit = 1u << 12, kEob = 1u << 13, kBad = 1u << 14;
struct Payloads {
    uint32_t lit[288], dist[32];
    Payloads() {
        for (int s = 0; s < 288; s++)
            lit[s] = s < 256    ? ((uint32_t)s << 16) | kLit
                     : s == 256 ? kEob
                     : s < 286  ? ((uint32_t)kLenBase[s - 257] << 16) | ((uint32_t)kLenExtra[s - 257] << 8)
                                : kBad;
        for (int s = 0; s < 32; s++)
            dist[s] = s < 30 ? ((uint32_t)kDistBase[s] << 16) | ((uint32_t)kDistExtra[s] << 8) : kBad;
    }
};
const Payloads kPay;

// Canonical Huffman code of lens[0..n) (0: unused) into t; false if over-subscribed
// or incomplete where `inc` forbids it.  Entries carry pay[s] (nullptr: the symbol).
bool build(Table &t, const uint8_t *lens, int n, int main_bits, Incomplete inc, const uint32_t *pay = nullptr) {
    int count[16] = {0};
    for (int i = 0; i < n; i++) count[lens[i]]++;
    count[0] = 0;
    int left = 1, max_len = 0;
    for (int l = 1; l < 16; l++) {
        left = (left << 1) - count[l];
        if (left < 0) return false;
        if (count[l]) max_len = l;
    }
    if (left > 0 && max_len > 0 && inc != kAllowIncomplete && (inc == kRejectIncomplete || max_len != 1))
        return false;  // zlib: "invalid code lengths set" / "invalid literal/lengths set"
    int next[16] = {0};
    for (int l = 1, code = 0; l < 16; l++) {
        code = (code + count[l - 1]) << 1;
        next[l] = code;
    }
    t.bits = main_bits;
    const uint32_t msize = 1u << main_bits;
    for (uint32_t i = 0; i < msize; i++) t.e[i] = 0;  // len 0: invalid code
    uint32_t sub_at = msize;
    // longest code among the codes sharing each main-table prefix (for sub-table sizes;
    // only when some code is longer than the main table's index)
    bool longer = false;
    for (int l = main_bits + 1; l < 16; l++) longer = longer || count[l];
    if (longer) {
        uint8_t sub_len[1 << kLitBits];
        memset(sub_len, 0, msize);
        int nx[16];
        memcpy(nx, next, sizeof nx);
        for (int s = 0; s < n; s++) {
            const int l = lens[s];
            if (l > main_bits) {
                const uint32_t r = rev_bits((uint32_t)nx[l], l);
                const uint32_t pre = r & (msize - 1);
                if (l - main_bits > sub_len[pre]) sub_len[pre] = (uint8_t)(l - main_bits);
            }
            if (l) nx[l]++;
        }
        for (uint32_t pre = 0; pre < msize; pre++)
            if (sub_len[pre]) {
                if (sub_at + (1u << sub_len[pre]) > sizeof(t.e) / sizeof(t.e[0])) return false;
                t.e[pre] = (sub_at << 16) | 16u | (uint32_t)sub_len[pre];
                for (uint32_t k = 0; k < (1u << sub_len[pre]); k++) t.e[sub_at + k] = 0;
                sub_at += 1u << sub_len[pre];
            }
    }
    for (int s = 0; s < n; s++) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t r = rev_bits((uint32_t)next[l]++, l);
        const uint32_t ent = (pay ? pay[s] : (uint32_t)s << 16) | (uint32_t)l;
        if (l <= main_bits) {
            for (uint32_t k = r; k < msize; k += 1u << l) t.e[k] = ent;
        } else {
            const uint32_t link = t.e[r & (msize - 1)];
            const uint32_t base = link >> 16, sb = link & 15u;
            const int rest = l - main_bits;
            for (uint32_t k = r >> main_bits; k < (1u << sb); k += 1u << rest) t.e[base + k] = ent;
        }
    }
    return true;
}

struct Bits {
    const uint8_t *p, *end;
    uint64_t buf = 0;
    int n = 0;
    uint32_t pad = 0;  // zero bytes appended past the input's end (must stay unconsumed)
    inline void refill() {
        if (end - p >= 8) {
            uint64_t x;
            memcpy(&x, p, 8);
            buf |= x << n;
            p += (63 - n) >> 3;
            n |= 56;
        } else {
            while (n <= 56) {
                if (p < end) buf |= (uint64_t)*p++ << n;
                else pad++;
                n += 8;
            }
        }
    }
    inline uint32_t peek(int k) const { return (uint32_t)(buf & ((1ull << k) - 1)); }
    inline void drop(int k) {
        buf >>= k;
        n -= k;
    }
    inline uint32_t get(int k) {
        if (n < k) refill();
        const uint32_t v = peek(k);
        drop(k);
        return v;
    }
    bool overrun() const { return (uint64_t)n < 8ull * pad; }  // padding bits consumed
};

// Decodes one symbol with t (the bit buffer holds >= 15 bits); -1: invalid code.
inline int decode(const Table &t, Bits &b) {
    uint32_t e = t.e[b.peek(t.bits)];
    if (e & 16u) {
        const uint32_t sub = (e >> 16) + ((uint32_t)(b.buf >> t.bits) & ((1u << (e & 15u)) - 1u));
        e = t.e[sub];
    }
    const int l = (int)(e & 15u);
    if (!l) return -1;
    b.drop(l);
    return (int)(e >> 16);
}

// t's entry for the code at the bottom of buf (>= 15 bits there), the sub-table
// link followed; bits 0-3 the code's length (0: no such code)
inline uint32_t lookup(const Table &t, uint64_t buf) {
    uint32_t e = t.e[buf & ((1u << t.bits) - 1u)];
    if (__builtin_expect(e & 16u, 0)) e = t.e[(e >> 16) + ((uint32_t)(buf >> t.bits) & ((1u << (e & 15u)) - 1u))];
    return e;
}

struct FixedTables {
    Table lit, dist;
    FixedTables() {
        uint8_t l[288];
        for (int i = 0; i < 144; i++) l[i] = 8;
        for (int i = 144; i < 256; i++) l[i] = 9;
        for (int i = 256; i < 280; i++) l[i] = 7;
        for (int i = 280; i < 288; i++) l[i] = 8;
        build(lit, l, 288, kLitBits, kAllowIncomplete, kPay.lit);
        uint8_t d[30];
        for (int i = 0; i < 30; i++) d[i] = 5;
        build(dist, d, 30, kDistBits, kAllowIncomplete, kPay.dist);
    }
};

}  // namespace

int inflate_raw_fast(const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len) {
    static const FixedTables fixed;
    Bits b{in, in + in_len};
    size_t o = 0;
    Table dyn_lit, dyn_dist;
    for (;;) {
        b.refill();
        const uint32_t final = b.get(1), type = b.get(2);
        if (type == 0) {  // stored
            b.drop(b.n & 7);
            if (b.n < 32) b.refill();
            const uint32_t len = b.get(16), nlen = b.get(16);
            if ((len ^ 0xFFFFu) != nlen || b.overrun()) return -1;
            uint32_t k = 0;  // the bytes already in the bit buffer come first
            for (; k < len && b.n >= 8; k++) {
                if (o >= out_len) return -1;
                out[o++] = (uint8_t)b.get(8);
            }
            if (b.overrun()) return -1;
            const size_t rest = len - k;
            if (rest) {  // (the buffer is empty: the rest follows at p)
                b.buf = 0;   // (a fast refill leaves the unconsumed byte at p above the count)
                if ((size_t)(b.end - b.p) < rest || o + rest > out_len) return -1;
                memcpy(out + o, b.p, rest);
                o += rest;
                b.p += rest;
            }
        } else if (type == 1 || type == 2) {
            const Table *lt = &fixed.lit, *dt = &fixed.dist;
            if (type == 2) {
                const int hlit = (int)b.get(5) + 257, hdist = (int)b.get(5) + 1, hclen = (int)b.get(4) + 4;
                static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
                uint8_t cl[19] = {0};
                for (int i = 0; i < hclen; i++) cl[ord[i]] = (uint8_t)b.get(3);
                Table ct;
                if (!build(ct, cl, 19, 7, kRejectIncomplete)) return -1;
                uint8_t lens[288 + 32];
                int n = 0;
                while (n < hlit + hdist) {
                    if (b.n < 16) b.refill();
                    const int sym = decode(ct, b);
                    if (sym < 0) return -1;
                    if (sym < 16) {
                        lens[n++] = (uint8_t)sym;
                    } else {
                        int rep;
                        uint8_t v = 0;
                        if (sym == 16) {
                            if (!n) return -1;
                            v = lens[n - 1];
                            rep = 3 + (int)b.get(2);
                        } else if (sym == 17) {
                            rep = 3 + (int)b.get(3);
                        } else {
                            rep = 11 + (int)b.get(7);
                        }
                        if (n + rep > hlit + hdist) return -1;
                        while (rep--) lens[n++] = v;
                    }
                }
                if (!lens[256]) return -1;
                if (!build(dyn_lit, lens, hlit, kLitBits, kSingleCode, kPay.lit) ||
                    !build(dyn_dist, lens + hlit, hdist, kDistBits, kSingleCode, kPay.dist))
                    return -1;
                lt = &dyn_lit;
                dt = &dyn_dist;
            }
            for (;;) {
                // one refill per symbol (>= 56 bits): a length code with its extra bits
                // (<= 20) and a distance code with its (<= 28) fit
                b.refill();
                const uint32_t e = lookup(*lt, b.buf);
                const int l = (int)(e & 15u);
                if (!l) return -1;
                if (e & kLit) {
                    if (o >= out_len) return -1;
                    b.drop(l);
                    out[o++] = (uint8_t)(e >> 16);
                    continue;
                }
                if (e & (kEob | kBad)) {
                    if (e & kBad) return -1;
                    b.drop(l);
                    break;
                }
                const int lx = (int)((e >> 8) & 15u);
                const uint32_t len = (e >> 16) + ((uint32_t)(b.buf >> l) & ((1u << lx) - 1u));
                b.drop(l + lx);
                const uint32_t de = lookup(*dt, b.buf);
                const int dl = (int)(de & 15u);
                if (!dl || (de & kBad)) return -1;
                const int dx = (int)((de >> 8) & 15u);
                const uint32_t dist = (de >> 16) + ((uint32_t)(b.buf >> dl) & ((1u << dx) - 1u));
                b.drop(dl + dx);
                if (dist > o || o + len > out_len) return -1;
                uint8_t *dst = out + o;
                const uint8_t *src = dst - dist;
                if (o + len + 16 <= out_len) {  // 8- / 16-byte steps (may write up to 15 bytes past: slack)
                    uint32_t k = 0;
                    if (dist == 1 || dist == 2 || dist == 4 || dist == 8) {
                        // a period dividing 16: one 16-byte pattern, stored over and over
                        // (no load depends on the store before it)
                        uint64_t v;
                        if (dist == 1) {
                            v = src[0] * 0x0101010101010101ull;
                        } else if (dist == 2) {
                            uint16_t x;
                            memcpy(&x, src, 2);
                            v = x * 0x0001000100010001ull;
                        } else if (dist == 4) {
                            uint32_t x;
                            memcpy(&x, src, 4);
                            v = x * 0x0000000100000001ull;
                        } else {
                            memcpy(&v, src, 8);
                        }
                        for (; k < len; k += 16) {
                            memcpy(dst + k, &v, 8);
                            memcpy(dst + k + 8, &v, 8);
                        }
                    } else if (dist < 8) {
                        // the match repeats its first dist bytes: once d (a multiple of dist,
                        // >= 8) bytes of it are out, copy from d back 8 bytes at a time
                        const uint32_t d = dist * ((8 + dist - 1) / dist);
                        const uint32_t head = len < d ? len : d;
                        for (; k < head; k++) dst[k] = src[k];
                        for (; k < len; k += 8) memcpy(dst + k, dst + k - d, 8);
                    } else if (dist < 16) {
                        for (; k < len; k += 8) memcpy(dst + k, src + k, 8);
                    } else {
                        for (; k < len; k += 16) memcpy(dst + k, src + k, 16);
                    }
                } else {
                    for (uint32_t k = 0; k < len; k++) dst[k] = src[k];
                }
                o += len;
            }
        } else {
            return -1;
        }
        if (b.overrun()) return -1;
        if (final) break;
    }
    return o == out_len ? 0 : -1;
}

}  // namespace tfbs

extern "C" int tfbs_inflate_raw(const void *in, size_t in_len, void *out, size_t out_len) {
    if ((!in && in_len) || (!out && out_len)) return TFBS_E_ARG;
    return tfbs::inflate_raw_fast(static_cast<const uint8_t *>(in), in_len, static_cast<uint8_t *>(out), out_len) == 0
               ? TFBS_OK
               : TFBS_E_PARSE;
}
