// Inputs and outputs around the scoring path:
// a BGZF/BCF2 reader with region fetch (replaces rust-htslib 0.26.1 IndexedReader,
// haplotype.rs:16-24, 78-79), a FASTA/.fai reader (bio 0.28.2, main.rs:156-161),
// a BED reader (bed.rs:9-19) and a BGZF writer (bgzip 0.0.3, main.rs:264-276).
//
// The BCF reader decodes the whole file once and keeps each contig's records in
// file order; fetch(contig, beg, end) returns the records overlapping the
// 0-based half-open [beg, end) the way htslib's region iterator does
// (pos < end && pos + rlen > beg).  GT values are kept raw (BCF2 encoding
// (allele + 1) << 1 | phased) with vector_end normalised to INT32_MIN + 1.
#include <immintrin.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "tfbs_internal.hpp"
#include "io.hpp"

namespace tfbs {

// run fn(t) for t in [0, n) on up to `threads` threads
template <class F> static void par_for(size_t n, uint32_t threads, F fn) {
    const size_t T = std::min<size_t>(std::max<uint32_t>(threads, 1), n);
    if (T <= 1) {
        for (size_t i = 0; i < n; i++) fn(i);
        return;
    }
    // items taken in small grains from a shared counter: a thread the scheduler holds
    // back (the run flow's other stages share the cores) leaves its share to the others
    const size_t grain = std::max<size_t>(1, n / (T * 16));
    std::atomic<size_t> next(0);
    auto work = [&] {
        for (size_t i0; (i0 = next.fetch_add(grain)) < n;)
            for (size_t i = i0; i < std::min(n, i0 + grain); i++) fn(i);
    };
    std::vector<std::thread> ts;
    for (size_t t = 1; t < T; t++) ts.emplace_back(work);
    work();
    for (auto &x : ts) x.join();
}

static int read_file(const std::string &path, std::string &out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(TFBS_E_IO, "Could not open file " + path);
    std::stringstream ss;
    ss << in.rdbuf();
    out = ss.str();
    return TFBS_OK;
}

// Inflate a concatenation of gzip members (BGZF blocks are gzip members).
int bgzf_inflate(const std::string &in, std::string &out) {
    out.clear();
    size_t off = 0;
    std::vector<char> buf(1 << 16);
    while (off < in.size()) {
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return fail(TFBS_E_IO, "inflateInit2 failed");
        zs.next_in = (Bytef *)(in.data() + off);
        zs.avail_in = (uInt)std::min<size_t>(in.size() - off, 0x7FFFFFFF);
        int rc;
        do {
            zs.next_out = (Bytef *)buf.data();
            zs.avail_out = (uInt)buf.size();
            rc = inflate(&zs, Z_NO_FLUSH);
            if (rc != Z_OK && rc != Z_STREAM_END) {
                inflateEnd(&zs);
                return fail(TFBS_E_IO, "corrupt gzip/BGZF data");
            }
            out.append(buf.data(), buf.size() - zs.avail_out);
        } while (rc != Z_STREAM_END);
        off += zs.total_in;
        inflateEnd(&zs);
        if (zs.total_in == 0) break;
    }
    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// BGZF writer: <= 65280 input bytes per block, raw deflate, BC extra field,
// CRC32 + ISIZE trailer; flush() ends the current block; close() appends the
// standard 28-byte EOF block (the layout expected_output_*.vcf.gz shows).
// ---------------------------------------------------------------------------
static const unsigned char kBgzfEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                           2,    0,    0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

int bgzf_block(const char *data, size_t n, std::string &out) {
    std::vector<unsigned char> comp(compressBound((uLong)n) + 64);
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, Z_DEFAULT_COMPRESSION, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
        return fail(TFBS_E_IO, "deflateInit2 failed");
    zs.next_in = (Bytef *)data;
    zs.avail_in = (uInt)n;
    zs.next_out = comp.data();
    zs.avail_out = (uInt)comp.size();
    int rc = deflate(&zs, Z_FINISH);
    deflateEnd(&zs);
    if (rc != Z_STREAM_END) return fail(TFBS_E_IO, "deflate failed");
    const size_t clen = zs.total_out;
    const size_t bsize = 18 + clen + 8;  // header + data + trailer
    if (bsize > 65536) return fail(TFBS_E_IO, "BGZF block too large");
    unsigned char hdr[18] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43, 2, 0, 0, 0};
    hdr[16] = (unsigned char)((bsize - 1) & 0xff);
    hdr[17] = (unsigned char)((bsize - 1) >> 8);
    out.append((const char *)hdr, 18);
    out.append((const char *)comp.data(), clen);
    uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), (const Bytef *)data, (uInt)n);
    unsigned char tr[8];
    for (int i = 0; i < 4; i++) tr[i] = (unsigned char)(crc >> (8 * i));
    for (int i = 0; i < 4; i++) tr[4 + i] = (unsigned char)(((uint32_t)n) >> (8 * i));
    out.append((const char *)tr, 8);
    return TFBS_OK;
}

int BgzfWriter::open(const std::string &path, uint32_t nthreads) {
    f = fopen(path.c_str(), "wb");
    if (!f) return fail(TFBS_E_IO, "Could not create output file " + path);
    threads = std::max(1u, nthreads);
    return TFBS_OK;
}
int BgzfWriter::write(const char *p, size_t n) {
    while (n) {
        const size_t open_at = ends.empty() ? 0 : ends.back();
        const size_t take = std::min(n, kBlock - (raw.size() - open_at));
        raw.append(p, take);
        p += take;
        n -= take;
        if (raw.size() - open_at == kBlock) {
            ends.push_back(raw.size());
            if (ends.size() >= 8 * (size_t)threads)
                if (int rc = drain()) return rc;
        }
    }
    return TFBS_OK;
}
// deflate the queued blocks in parallel, write them in order, keep the open block
int BgzfWriter::drain() {
    const size_t nb = ends.size();
    if (!nb) return TFBS_OK;
    std::vector<std::string> out(nb);
    std::vector<int> rcs(nb, TFBS_OK);
    par_for(nb, threads, [&](size_t i) {
        const size_t b = i ? ends[i - 1] : 0;
        rcs[i] = bgzf_block(raw.data() + b, ends[i] - b, out[i]);
    });
    for (size_t i = 0; i < nb; i++) {
        if (rcs[i]) return fail(TFBS_E_IO, "deflate failed");
        if (fwrite(out[i].data(), 1, out[i].size(), f) != out[i].size()) return fail(TFBS_E_IO, "write failed");
    }
    raw.erase(0, ends.back());
    ends.clear();
    return TFBS_OK;
}
int BgzfWriter::raw_fd() {
    if (raw.size() > (ends.empty() ? 0 : ends.back())) ends.push_back(raw.size());
    if (int rc = drain()) return rc;
    if (fflush(f) != 0) return fail(TFBS_E_IO, "write failed");
    return fileno(f);
}
int BgzfWriter::seek_to(uint64_t at) {
    if (fflush(f) != 0 || fseeko(f, (off_t)at, SEEK_SET) != 0) return fail(TFBS_E_IO, "seek failed");
    return TFBS_OK;
}
// like BGzWriter::flush: ends the block (an empty block if nothing is buffered)
int BgzfWriter::flush() {
    ends.push_back(raw.size());
    return ends.size() >= 8 * (size_t)threads ? drain() : TFBS_OK;
}
int BgzfWriter::close() {
    if (!f) return TFBS_OK;
    int rc = TFBS_OK;
    if (raw.size() > (ends.empty() ? 0 : ends.back())) ends.push_back(raw.size());
    rc = drain();
    if (!rc && fwrite(kBgzfEof, 1, sizeof kBgzfEof, f) != sizeof kBgzfEof) rc = fail(TFBS_E_IO, "write failed");
    fclose(f);
    f = nullptr;
    return rc;
}
BgzfWriter::~BgzfWriter() {
    if (f) fclose(f);
}

// ---------------------------------------------------------------------------
// BCF2
// ---------------------------------------------------------------------------
namespace {
struct Cur {
    const unsigned char *p, *e;
    bool ok = true;
    bool need(size_t n) {
        if ((size_t)(e - p) < n) ok = false;
        return ok;
    }
};
// typed value descriptor: returns (type, count)
bool typed(Cur &c, int &type, uint32_t &count);
bool read_int(Cur &c, int type, int64_t &v) {
    switch (type) {
    case 1: if (!c.need(1)) return false; v = (int8_t)c.p[0]; c.p += 1; return true;
    case 2: if (!c.need(2)) return false; { int16_t x; memcpy(&x, c.p, 2); v = x; } c.p += 2; return true;
    case 3: if (!c.need(4)) return false; { int32_t x; memcpy(&x, c.p, 4); v = x; } c.p += 4; return true;
    default: return false;
    }
}
bool typed(Cur &c, int &type, uint32_t &count) {
    if (!c.need(1)) return false;
    const unsigned char d = *c.p++;
    type = d & 0x0F;
    count = d >> 4;
    if (count == 15) {
        int t2;
        uint32_t n2;
        if (!typed(c, t2, n2) || n2 != 1) return false;
        int64_t v;
        if (!read_int(c, t2, v) || v < 0) return false;
        count = (uint32_t)v;
    }
    return true;
}
size_t type_size(int t) {
    switch (t) {
    case 0: return 0;
    case 1: case 7: return 1;
    case 2: return 2;
    case 3: case 5: return 4;
    default: return 0;
    }
}
}  // namespace

// Header dictionaries (VCF 4.3 / BCF2): strings PASS + FILTER/INFO/FORMAT (IDX= wins), contigs.
static void parse_bcf_header(const std::string &text, std::vector<std::string> &samples,
                             std::vector<std::string> &contigs, int &gt_key) {
    std::map<int, std::string> sdict;
    sdict[0] = "PASS";
    int next = 1, cnext = 0;
    std::istringstream hs(text);
    std::string line;
    auto field = [](const std::string &l, const std::string &key) -> std::string {
        size_t a = l.find(key + "=");
        if (a == std::string::npos) return "";
        a += key.size() + 1;
        size_t b = a;
        while (b < l.size() && l[b] != ',' && l[b] != '>') b++;
        return l.substr(a, b - a);
    };
    while (std::getline(hs, line)) {
        if (!line.empty() && line.back() == '\0') line.pop_back();
        if (line.rfind("##contig=<", 0) == 0) {
            std::string id = field(line, "ID"), idx = field(line, "IDX");
            int i = idx.empty() ? cnext : atoi(idx.c_str());
            if ((int)contigs.size() <= i) contigs.resize(i + 1);
            contigs[i] = id;
            cnext = i + 1;
        } else if (line.rfind("##FILTER=<", 0) == 0 || line.rfind("##INFO=<", 0) == 0 ||
                   line.rfind("##FORMAT=<", 0) == 0) {
            std::string id = field(line, "ID"), idx = field(line, "IDX");
            if (id == "PASS") continue;
            int i = idx.empty() ? next : atoi(idx.c_str());
            if (!sdict.count(i)) sdict[i] = id;
            next = std::max(next, i + 1);
        } else if (line.rfind("#CHROM", 0) == 0) {
            std::vector<std::string> cols;
            std::string col;
            std::istringstream ls(line);
            while (std::getline(ls, col, '\t')) cols.push_back(col);
            for (size_t i = 9; i < cols.size(); i++) samples.push_back(cols[i]);
        }
    }
    gt_key = -1;
    for (auto &kv : sdict)
        if (kv.second == "GT") gt_key = kv.first;
}

// One BCF2 record (l_shared, l_indiv, shared, indiv) at p.  GT is kept raw for
// the samples in sel (all samples if sel is null): 2 ints each, vector_end and
// absent values as INT32_MIN + 1.
// Carriers of a bi-allelic record from its int8 diploid GT bytes g (2 per sample of
// the file): byte j of sample k's pair carries id 2 k + side when it is Unphased(1)
// (4) in slot 0 or Phased(1) (5) in slot 1 (haplotype.rs:27-36); a vector_end byte
// (-127) in either slot is a ploidy error (haplotype.rs:24-26).  Without a sample
// selection the bytes are swept 8 at a time (SWAR: most are 0|0 and skipped whole).
static void gt8_carriers(const int8_t *g, size_t ns, const std::vector<size_t> *sel, std::vector<uint32_t> &car,
                         int &status) {
    car.clear();
    auto one = [&](size_t k, int8_t a, int8_t b) {
        if (a == -127 || b == -127) status = TFBS_E_PLOIDY;
        if (a == 4) car.push_back((uint32_t)(2 * k));
        if (b == 5) car.push_back((uint32_t)(2 * k + 1));
    };
    if (sel) {
        for (size_t k = 0; k < sel->size(); k++) one(k, g[2 * (*sel)[k]], g[2 * (*sel)[k] + 1]);
        return;
    }
    const uint64_t P = 0x0504050405040504ull, V = 0x8181818181818181ull, L = 0x0101010101010101ull,
                   H = 0x8080808080808080ull;
    size_t j = 0;
    for (; j + 8 <= 2 * ns; j += 8) {
        uint64_t x;
        memcpy(&x, g + j, 8);
        const uint64_t a = x ^ P, b = x ^ V;  // zero bytes: a carrier allele / a vector_end
        if ((((a - L) & ~a) | ((b - L) & ~b)) & H)
            for (size_t q = j; q < j + 8; q += 2) one(q / 2, g[q], g[q + 1]);
    }
    for (; j < 2 * ns; j += 2) one(j / 2, g[j], g[j + 1]);
}

// The shared part of a record (CHROM .. ALT; INFO is not read): position, rlen, REF,
// ALT; n_allele and n_fmt for the per-sample part.
static int decode_shared(Cur sh, BcfRecord &r, int32_t &chrom, uint32_t &n_allele, uint32_t &n_fmt) {
    int32_t pos, rlen;
    uint32_t nai, nfs;
    if (!sh.need(24)) return fail(TFBS_E_PARSE, "short BCF record");
    memcpy(&chrom, sh.p, 4);
    memcpy(&pos, sh.p + 4, 4);
    memcpy(&rlen, sh.p + 8, 4);
    memcpy(&nai, sh.p + 16, 4);
    memcpy(&nfs, sh.p + 20, 4);
    sh.p += 24;
    r.pos = (uint64_t)(int64_t)pos;
    r.rlen = (uint32_t)std::max(rlen, 0);
    n_allele = nai >> 16;
    n_fmt = nfs >> 24;
    r.n_alleles = n_allele;
    r.ref.clear();
    r.alt.clear();
    int t;
    uint32_t n;
    if (!typed(sh, t, n) || !sh.need(n * type_size(t))) return fail(TFBS_E_PARSE, "bad BCF ID");
    sh.p += n * type_size(t);
    for (uint32_t a = 0; a < n_allele; a++) {
        if (!typed(sh, t, n) || !sh.need(n)) return fail(TFBS_E_PARSE, "bad BCF allele");
        std::string al((const char *)sh.p, n);
        sh.p += n;
        while (!al.empty() && al.back() == '\0') al.pop_back();
        if (a == 0) r.ref = al;
        else if (a == 1) r.alt = al;
    }
    return TFBS_OK;
}

// Carriers mode: the carriers of a bi-allelic record's GT payload g (vt, vn as typed,
// ns samples of the file), after r.gt_status was set from vn.
static void gt_carriers(const unsigned char *g, int vt, uint32_t vn, size_t ns, const std::vector<size_t> *sel,
                        BcfRecord &r) {
    if (vt == 1 && vn == 2) {
        gt8_carriers((const int8_t *)g, ns, sel, r.carriers, r.gt_status);
        return;
    }
    if (vn < 2) return;
    const size_t sz = type_size(vt), nk = sel ? sel->size() : ns;  // wider ints: the first two values of every sample
    const int64_t ve = vt == 1 ? -127 : vt == 2 ? -32767 : (int64_t)INT32_MIN + 1;
    for (size_t k = 0; k < nk; k++) {
        const size_t s = sel ? (*sel)[k] : k;
        Cur c{g + sz * vn * s, g + sz * vn * (s + 1)};
        int64_t a = 0, b = 0;
        read_int(c, vt, a);
        read_int(c, vt, b);
        if (a == ve || b == ve) r.gt_status = TFBS_E_PLOIDY;
        if (a == 4) r.carriers.push_back((uint32_t)(2 * k));
        if (b == 5) r.carriers.push_back((uint32_t)(2 * k + 1));
    }
}

static int decode_bcf_record(const unsigned char *&p, const unsigned char *end, size_t ns, int gt_key,
                             const std::vector<size_t> *sel, bool carriers, BcfRecord &r, int32_t &chrom) {
    uint32_t l_shared, l_indiv;
    memcpy(&l_shared, p, 4);
    memcpy(&l_indiv, p + 4, 4);
    p += 8;
    if ((size_t)(end - p) < (size_t)l_shared + l_indiv) return fail(TFBS_E_PARSE, "truncated BCF record");
    Cur sh{p, p + l_shared};
    Cur in{p + l_shared, p + l_shared + l_indiv};
    p += l_shared + l_indiv;
    uint32_t n_allele, n_fmt;
    if (int rc = decode_shared(sh, r, chrom, n_allele, n_fmt)) return rc;
    const size_t nk = sel ? sel->size() : ns;
    r.carriers.clear();
    r.gt_status = TFBS_OK;
    if (carriers) {  // load_diffs' view of the record only (bi-allelic: carriers, ploidy)
        r.gt.clear();
        if (n_allele == 2 && nk) r.gt_status = TFBS_E_PLOIDY;  // (no GT field: every GT is empty)
    } else {
        r.gt.assign(2 * nk, INT32_MIN + 1);
    }
    for (uint32_t f = 0; f < n_fmt; f++) {
        int kt;
        uint32_t kn;
        int64_t key;
        if (!typed(in, kt, kn) || kn != 1 || !read_int(in, kt, key)) return fail(TFBS_E_PARSE, "bad FORMAT key");
        int vt;
        uint32_t vn;
        if (!typed(in, vt, vn)) return fail(TFBS_E_PARSE, "bad FORMAT type");
        const size_t sz = type_size(vt);
        if (!in.need(sz * vn * ns)) return fail(TFBS_E_PARSE, "truncated FORMAT data");
        if (carriers) {
            if (key == gt_key && n_allele == 2 && nk && vt >= 1 && vt <= 3) {
                r.gt_status = vn >= 2 ? TFBS_OK : TFBS_E_PLOIDY;  // one value per sample: glen 1
                gt_carriers(in.p, vt, vn, ns, sel, r);
            }
        } else if (key == gt_key && vt == 1 && vn == 2) {  // the common diploid int8 layout
            const int8_t *g = (const int8_t *)in.p;
            int32_t *o = r.gt.data();
            for (size_t k = 0; k < nk; k++) {
                const size_t s = sel ? (*sel)[k] : k;
                const int8_t a = g[2 * s], b = g[2 * s + 1];
                o[2 * k] = a == -127 ? INT32_MIN + 1 : a;
                o[2 * k + 1] = b == -127 ? INT32_MIN + 1 : b;
            }
        } else if (key == gt_key && vt >= 1 && vt <= 3) {
            const int64_t ve = vt == 1 ? -127 : vt == 2 ? -32767 : (int64_t)INT32_MIN + 1;
            const unsigned char *base = in.p;
            for (size_t k = 0; k < nk; k++) {
                const size_t s = sel ? (*sel)[k] : k;
                Cur c{base + sz * vn * s, base + sz * vn * (s + 1)};
                for (uint32_t q = 0; q < vn && q < 2; q++) {
                    int64_t v;
                    read_int(c, vt, v);
                    r.gt[2 * k + q] = v == ve ? INT32_MIN + 1 : (int32_t)v;
                }
            }
        }
        in.p += sz * vn * ns;
    }
    return TFBS_OK;
}

Bcf::~Bcf() {
    discard_ahead();
    if (f) fclose(f);
    if (getenv("TFBS_BCF_TIMING"))
        fprintf(stderr, "tfbs_bcf_timing {\"read_s\": %.4f, \"inflate_s\": %.4f, \"erase_s\": %.4f, \"scan_s\": %.4f, "
                        "\"decode_s\": %.4f, \"ahead_wait_s\": %.4f, \"inflated_bytes\": %llu}\n",
                t_read, t_inflate, t_erase, t_scan, t_decode, t_ahead_wait, (unsigned long long)n_inflated);
}

int Bcf::open(const std::string &p, uint32_t nthreads) {
    path = p;
    use_fast_inflate = !(getenv("TFBS_BCF_ZLIB") && atoi(getenv("TFBS_BCF_ZLIB")));
    threads = nthreads ? nthreads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char *e = getenv("TFBS_BCF_THREADS")) threads = std::max(1, atoi(e));
    if (const char *e = getenv("TFBS_BCF_CHUNK_KB")) chunk = std::max<size_t>(1, (size_t)atoll(e)) << 10;
    condense = !(getenv("TFBS_BCF_CONDENSED") && atoi(getenv("TFBS_BCF_CONDENSED")) == 0);
    read_ahead = !(getenv("TFBS_BCF_READAHEAD") && atoi(getenv("TFBS_BCF_READAHEAD")) == 0);
    int rc = rewind();
    if (rc) return rc;
    if ((rc = load_csi())) return rc;
    sel.resize(samples.size());
    for (size_t i = 0; i < sel.size(); i++) sel[i] = i;
    all_samples = true;
    return TFBS_OK;
}

int Bcf::set_carriers_mode(bool on) {
    carriers_mode = on;
    cur = -1;  // the decoded records change: drop the window
    return rewind();
}

int Bcf::select(const std::vector<size_t> &s) {
    for (size_t i : s)
        if (i >= samples.size()) return fail(TFBS_E_ARG, "sample index out of range");
    sel = s;
    all_samples = sel.size() == samples.size();
    for (size_t i = 0; all_samples && i < sel.size(); i++) all_samples = sel[i] == i;
    cur = -1;  // decoded GT columns change: drop the window
    return rewind();
}

// (Re)start at the first record: header parsed again, window emptied.
int Bcf::rewind() {
    discard_ahead();
    if (f) fclose(f);
    f = fopen(path.c_str(), "rb");
    if (!f) return fail(TFBS_E_IO, "Could not open file " + path);
    cbuf.clear();
    dbuf.clear();
    doff = 0;
    in_eof = done = seen = false;
    cmode = false;
    cblk.clear();
    win.clear();
    last_beg = last_pos = 0;
    unsigned char m[4] = {0, 0, 0, 0};
    const size_t got = fread(m, 1, 4, f);
    fseek(f, 0, SEEK_SET);
    bgzf = got == 4 && m[0] == 0x1f && m[1] == 0x8b && m[2] == 8 && (m[3] & 4);
    if (!bgzf) {  // plain gzip members: inflate the whole file at once
        std::string raw;
        int rc = read_file(path, raw);
        if (rc) return rc;
        std::string all;
        if ((rc = bgzf_inflate(raw, all))) return rc;
        dbuf.assign(all);
        in_eof = true;
    }
    // the header in small reads (a full chunk inflates hundreds of MB of records
    // that a fetch's seek would then inflate again)
    const size_t big = chunk;
    chunk = std::min<size_t>(big, 256u << 10);
    struct Restore {
        size_t &c, v;
        ~Restore() { c = v; }
    } restore{chunk, big};
    while (dbuf.size() < 9 && !in_eof)
        if (int rc = inflate_more()) return rc;
    if (dbuf.size() < 9 || memcmp(dbuf.data(), "BCF\2", 4) != 0) return fail(TFBS_E_PARSE, "not a BCF2 file: " + path);
    uint32_t l_text;
    memcpy(&l_text, dbuf.data() + 5, 4);
    while (dbuf.size() < 9ull + l_text && !in_eof)
        if (int rc = inflate_more()) return rc;
    if (9ull + l_text > dbuf.size()) return fail(TFBS_E_PARSE, "truncated BCF header");
    std::vector<std::string> s, c;
    parse_bcf_header(std::string(dbuf.data() + 9, l_text), s, c, gt_key);
    if (samples.empty() && contigs.empty()) {
        samples = std::move(s);
        contigs = std::move(c);
    }
    doff = 9 + l_text;
    return TFBS_OK;
}

// CSI (htslib's coordinate-sorted index, SAM/VCF index spec): BGZF-compressed
// "CSI\1", min_shift, depth, aux, then per reference its bins (bin, loffset,
// chunks of [begin, end) virtual offsets).  Only the chunk starts are kept, as
// (bin end, start) per bin, suffix-minimised over bins sorted by end: every
// record with pos + rlen > beg sits in a chunk of a bin that ends after beg.
int Bcf::load_csi() {
    csi.clear();
    std::string raw, txt;
    {
        std::ifstream in(path + ".csi", std::ios::binary);
        if (!in || !bgzf) return TFBS_OK;  // no index: sweep from the start
        std::stringstream ss;
        ss << in.rdbuf();
        raw = ss.str();
    }
    if (int rc = bgzf_inflate(raw, txt)) return rc;
    const unsigned char *p = (const unsigned char *)txt.data(), *e = p + txt.size();
    auto rd = [&](void *dst, size_t n) {
        if ((size_t)(e - p) < n) return false;
        memcpy(dst, p, n);
        p += n;
        return true;
    };
    char magic[4];
    int32_t min_shift, depth, l_aux, n_ref;
    if (!rd(magic, 4) || memcmp(magic, "CSI\1", 4) != 0 || !rd(&min_shift, 4) || !rd(&depth, 4) || !rd(&l_aux, 4) ||
        min_shift < 0 || depth < 0 || min_shift + 3 * depth > 62 || l_aux < 0 || (size_t)(e - p) < (size_t)l_aux)
        return fail(TFBS_E_PARSE, "bad CSI index " + path + ".csi");
    p += l_aux;
    if (!rd(&n_ref, 4) || n_ref < 0) return fail(TFBS_E_PARSE, "bad CSI index " + path + ".csi");
    const uint64_t n_bins_valid = ((1ull << (3 * (depth + 1))) - 1) / 7;  // bins above are pseudo-bins
    csi.resize((size_t)n_ref);
    for (int32_t r = 0; r < n_ref; r++) {
        int32_t n_bin;
        if (!rd(&n_bin, 4) || n_bin < 0) return fail(TFBS_E_PARSE, "bad CSI index " + path + ".csi");
        auto &bins = csi[r];
        for (int32_t i = 0; i < n_bin; i++) {
            uint32_t bin;
            uint64_t loff;
            int32_t n_chunk;
            if (!rd(&bin, 4) || !rd(&loff, 8) || !rd(&n_chunk, 4) || n_chunk < 0)
                return fail(TFBS_E_PARSE, "bad CSI index " + path + ".csi");
            uint64_t lo = UINT64_MAX;
            for (int32_t c = 0; c < n_chunk; c++) {
                uint64_t cb, ce;
                if (!rd(&cb, 8) || !rd(&ce, 8)) return fail(TFBS_E_PARSE, "bad CSI index " + path + ".csi");
                lo = std::min(lo, cb);
            }
            if (bin >= n_bins_valid || lo == UINT64_MAX) continue;
            int level = 0;
            while (level < depth && bin >= ((1ull << (3 * (level + 1))) - 1) / 7) level++;
            const uint64_t first = ((1ull << (3 * level)) - 1) / 7;
            const int shift = min_shift + 3 * (depth - level);
            bins.push_back({(bin - first + 1) << shift, lo});
        }
        std::sort(bins.begin(), bins.end());
        for (size_t i = bins.size(); i-- > 1;) bins[i - 1].second = std::min(bins[i - 1].second, bins[i].second);
    }
    if (csi.size() < contigs.size()) csi.resize(contigs.size());
    return TFBS_OK;
}

uint64_t Bcf::csi_start(int contig, uint64_t beg) const {
    if (csi.empty()) return 0;
    const auto &bins = csi[(size_t)contig];
    auto it = std::upper_bound(bins.begin(), bins.end(), std::make_pair(beg, UINT64_MAX));
    return it == bins.end() ? UINT64_MAX : it->second;
}

// Restart the stream at virtual offset voff (block at voff >> 16, byte voff & 0xFFFF of it).
int Bcf::seek(int contig, uint64_t voff) {
    discard_ahead();
    if (fseeko(f, (off_t)(voff >> 16), SEEK_SET) != 0) return fail(TFBS_E_IO, "seek failed in " + path);
    cbuf.clear();
    dbuf.clear();
    doff = 0;
    in_eof = done = seen = false;
    cmode = false;
    cblk.clear();
    win.clear();
    last_pos = 0;
    cur = contig;
    const size_t u = (size_t)(voff & 0xFFFF);
    // the condensed stream takes over after the block at voff: read it in a small round
    const size_t big = chunk;
    if (condensed()) chunk = std::min<size_t>(big, 256u << 10);
    struct Restore {
        size_t &c, v;
        ~Restore() { c = v; }
    } restore{chunk, big};
    while (dbuf.size() < u && !in_eof)
        if (int rc = inflate_more()) return rc;
    if (dbuf.size() < u) return fail(TFBS_E_PARSE, "CSI offset past the end of " + path);
    doff = u;
    return TFBS_OK;
}

// Read up to `chunk` compressed bytes, inflate every complete BGZF block in
// parallel and append the output to dbuf.
static double bcf_now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// The complete BGZF blocks at the start of c: their deflate data and inflated sizes
// (out: offset of a block's bytes after the blocks before it); used = bytes they take.
struct BgzfSpan {
    size_t off, len, out, isize;
};
static int bgzf_spans(const std::string &cb, const std::string &path, std::vector<BgzfSpan> &blks, size_t &used) {
    size_t o = 0, out = 0;
    const unsigned char *c = (const unsigned char *)cb.data();
    while (o + 18 <= cb.size()) {
        if (c[o] != 0x1f || c[o + 1] != 0x8b || c[o + 2] != 8 || !(c[o + 3] & 4))
            return fail(TFBS_E_PARSE, "corrupt BGZF block header in " + path);
        const size_t xlen = c[o + 10] | (c[o + 11] << 8);
        size_t bsize = 0;
        for (size_t x = o + 12; x + 4 <= o + 12 + xlen && x + 4 <= cb.size();) {
            const size_t slen = c[x + 2] | (c[x + 3] << 8);
            if (c[x] == 'B' && c[x + 1] == 'C' && slen == 2 && x + 6 <= cb.size()) bsize = (c[x + 4] | (c[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        if (!bsize) {
            if (o + 12 + xlen <= cb.size()) return fail(TFBS_E_PARSE, "BGZF block without BSIZE in " + path);
            break;
        }
        if (o + bsize > cb.size()) break;
        if (bsize < 12 + xlen + 8) return fail(TFBS_E_PARSE, "corrupt BGZF block size in " + path);
        uint32_t isize;
        memcpy(&isize, c + o + bsize - 4, 4);
        blks.push_back({o + 12 + xlen, bsize - 12 - xlen - 8, out, isize});
        out += isize;
        o += bsize;
    }
    used = o;
    return TFBS_OK;
}

// zlib's raw inflate of exactly isize bytes (where inflate_raw_fast declines)
static bool inflate_zlib(const unsigned char *in, size_t len, uint8_t *out, size_t isize) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return false;
    zs.next_in = (Bytef *)in;
    zs.avail_in = (uInt)len;
    zs.next_out = (Bytef *)out;
    zs.avail_out = (uInt)isize;
    const int rc = inflate(&zs, Z_FINISH);
    const bool ok = rc == Z_STREAM_END && zs.total_out == isize;
    inflateEnd(&zs);
    return ok;
}

int Bcf::inflate_more() {
    if (in_eof) return TFBS_OK;
    double t0 = bcf_now();
    if (doff) {
        dbuf.erase_front(doff);
        doff = 0;
    }
    double t1 = bcf_now();
    t_erase += t1 - t0;
    const size_t have = cbuf.size();
    cbuf.resize(have + chunk);
    const size_t got = fread(&cbuf[have], 1, chunk, f);
    cbuf.resize(have + got);
    t0 = bcf_now();
    t_read += t0 - t1;
    const bool file_end = got < chunk;
    std::vector<BgzfSpan> blks;
    size_t o = 0;
    if (int rc = bgzf_spans(cbuf, path, blks, o)) return rc;
    if (file_end && o < cbuf.size() && blks.empty()) return fail(TFBS_E_PARSE, "truncated BGZF file " + path);
    const size_t out0 = dbuf.size();
    dbuf.resize_uninit(out0 + (blks.empty() ? 0 : blks.back().out + blks.back().isize));
    const unsigned char *c = (const unsigned char *)cbuf.data();
    std::vector<int> bad(blks.size(), 0);
    par_for(blks.size(), blks.size() >= 4 ? threads : 1, [&](size_t i) {
        const BgzfSpan &b = blks[i];
        if (!b.isize) return;
        uint8_t *dst = (uint8_t *)&dbuf[out0 + b.out];
        if (use_fast_inflate && inflate_raw_fast(c + b.off, b.len, dst, b.isize) == 0) return;
        bad[i] = !inflate_zlib(c + b.off, b.len, dst, b.isize);
    });
    t_inflate += bcf_now() - t0;
    for (const BgzfSpan &b : blks) n_inflated += b.isize;
    for (int x : bad)
        if (x) return fail(TFBS_E_IO, "corrupt BGZF data in " + path);
    cbuf.erase(0, o);
    if (file_end && cbuf.empty()) in_eof = true;
    return TFBS_OK;
}

// Decode the next run of complete records of contig `cur` into the window.
// Records of other contigs are skipped unread; once the contig's records are
// over (a later contig follows them) the stream is done.
int Bcf::fill() {
    std::vector<size_t> offs;
    const double ts = bcf_now();
    for (;;) {
        size_t o = doff;
        const unsigned char *d = (const unsigned char *)dbuf.data();
        while (o + 8 <= dbuf.size()) {
            uint32_t ls, li;
            memcpy(&ls, d + o, 4);
            memcpy(&li, d + o + 4, 4);
            const size_t n = 8 + (size_t)ls + li;
            if (o + n > dbuf.size()) break;
            if (ls < 24) return fail(TFBS_E_PARSE, "short BCF record");
            int32_t chrom, pos;
            memcpy(&chrom, d + o + 8, 4);
            memcpy(&pos, d + o + 12, 4);
            if (chrom < 0 || (size_t)chrom >= contigs.size()) return fail(TFBS_E_PARSE, "BCF record with unknown contig");
            if (chrom == cur) {
                const uint64_t p = (uint64_t)(int64_t)pos;
                if (seen && p < last_pos)
                    return fail(TFBS_E_PARSE, "BCF records are not sorted by position (an indexed BCF is): " + path);
                seen = true;
                last_pos = p;
                offs.push_back(o);
            } else if (seen) {
                done = true;
                break;
            }
            o += n;
        }
        doff = o;
        if (done || !offs.empty()) break;
        if (in_eof) {
            if (doff + 8 <= dbuf.size()) return fail(TFBS_E_PARSE, "truncated BCF record");
            done = true;
            break;
        }
        if (int rc = inflate_more()) return rc;
    }
    const double td = bcf_now();
    t_scan += td - ts;
    const size_t base = win.size();
    win.resize(base + offs.size());
    std::vector<int> rcs(offs.size(), TFBS_OK);
    const unsigned char *end = (const unsigned char *)dbuf.data() + dbuf.size();
    const std::vector<size_t> *s = all_samples ? nullptr : &sel;
    par_for(offs.size(), offs.size() >= 64 ? threads : 1, [&](size_t i) {
        const unsigned char *p = (const unsigned char *)dbuf.data() + offs[i];
        int32_t chrom;
        rcs[i] = decode_bcf_record(p, end, samples.size(), gt_key, s, carriers_mode, win[base + i], chrom);
    });
    t_decode += bcf_now() - td;
    for (size_t i = 0; i < rcs.size(); i++)
        if (rcs[i]) {  // decode again on this thread for the (thread-local) error message
            const unsigned char *p = (const unsigned char *)dbuf.data() + offs[i];
            int32_t chrom;
            BcfRecord r;
            return decode_bcf_record(p, end, samples.size(), gt_key, s, carriers_mode, r, chrom);
        }
    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// The condensed stream (carriers mode): CBlock per inflated BGZF block.
uint8_t CBlock::at(uint32_t off) const {
    if (!raw.empty()) return raw[off];
    auto it = std::lower_bound(ex.begin(), ex.end(), off << 8);
    if (it != ex.end() && (*it >> 8) == off) return (uint8_t)*it;
    const uint8_t c = bg[off >> 6];
    return c < 2 ? (uint8_t)(2 + ((off ^ c) & 1)) : c;
}

void CBlock::read(uint32_t off, uint32_t m, uint8_t *dst) const {
    if (!raw.empty()) {
        memcpy(dst, raw.data() + off, m);
        return;
    }
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t q = off + i;
        const uint8_t c = bg[q >> 6];
        dst[i] = c < 2 ? (uint8_t)(2 + ((q ^ c) & 1)) : c;
    }
    for (auto it = std::lower_bound(ex.begin(), ex.end(), off << 8); it != ex.end() && (*it >> 8) < off + m; ++it)
        dst[(*it >> 8) - off] = (uint8_t)*it;
}

// Per 64-byte line of d (full lines only): the bytes that match the alternating
// backgrounds -- code 0: 2 at even offsets, 3 at odd ones; code 1: the other way
// round -- as bit masks m[2 l], m[2 l + 1].
__attribute__((target("avx2"))) static inline void line_masks_avx2(const uint8_t *d, uint32_t nl, uint64_t *m) {
    const __m256i p0 = _mm256_set1_epi16(0x0302), p1 = _mm256_set1_epi16(0x0203);
    for (uint32_t l = 0; l < nl; l++) {
        const __m256i a = _mm256_loadu_si256((const __m256i *)(d + 64ull * l)),
                      b = _mm256_loadu_si256((const __m256i *)(d + 64ull * l + 32));
        m[2 * l] = (uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, p0)) |
                   ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, p0)) << 32);
        m[2 * l + 1] = (uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, p1)) |
                       ((uint64_t)(uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, p1)) << 32);
    }
}
static inline void line_masks_sse2(const uint8_t *d, uint32_t nl, uint64_t *m) {
    const __m128i p0 = _mm_set1_epi16(0x0302), p1 = _mm_set1_epi16(0x0203);
    for (uint32_t l = 0; l < nl; l++) {
        uint64_t r0 = 0, r1 = 0;
        for (int k = 0; k < 4; k++) {
            const __m128i x = _mm_loadu_si128((const __m128i *)(d + 64ull * l + 16 * k));
            r0 |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, p0)) << (16 * k);
            r1 |= (uint64_t)(uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(x, p1)) << (16 * k);
        }
        m[2 * l] = r0;
        m[2 * l + 1] = r1;
    }
}

// Condense n inflated bytes d into b: per line the background code with the most
// matching bytes (a line that matches an alternating one whole is decided by the
// masks alone), then the other bytes as exceptions; ex, mk: the thread's scratch.
// (Compiled twice: with AVX2 + POPCNT where the CPU has them, and plain x86-64.)
template <bool kAvx2>
static inline __attribute__((always_inline)) void condense_body(const uint8_t *d, uint32_t n, CBlock &b,
                                                                std::vector<uint32_t> &ex, std::vector<uint64_t> &mk) {
    b.n = n;
    b.raw.clear();
    const uint32_t nl = (n + 63) / 64, nfull = n / 64, lim = n / 16;
    b.bg.resize(nl);
    if (mk.size() < 2ull * nl) mk.resize(2ull * nl);
    if (ex.size() < (size_t)lim + 64) ex.resize((size_t)lim + 64);
    if (kAvx2) line_masks_avx2(d, nfull, mk.data());
    else line_masks_sse2(d, nfull, mk.data());
    uint8_t *bg = b.bg.data();
    uint32_t *e = ex.data(), *const e_lim = ex.data() + lim;
    for (uint32_t l = 0; l < nl; l++) {
        const uint8_t *p = d + 64ull * l;
        const uint32_t m = std::min<uint32_t>(64, n - 64 * l);
        const uint64_t valid = m == 64 ? ~0ull : (1ull << m) - 1;
        uint64_t ok[4];
        if (l < nfull) {
            ok[0] = mk[2 * l];
            ok[1] = mk[2 * l + 1];
            if (ok[0] == ~0ull || ok[1] == ~0ull) {
                bg[l] = ok[0] == ~0ull ? 0 : 1;
                continue;
            }
        } else {
            ok[0] = ok[1] = 0;
            for (uint32_t i = 0; i < m; i++) {
                ok[0] |= (uint64_t)(p[i] == 2 + (i & 1)) << i;
                ok[1] |= (uint64_t)(p[i] == 3 - (i & 1)) << i;
            }
        }
        // the constant backgrounds from the alternating masks: a byte equal to 2 at an
        // even offset matches code 0 there, at an odd offset code 1
        const uint64_t even = 0x5555555555555555ull;
        ok[2] = (ok[0] & even) | (ok[1] & ~even);
        ok[3] = (ok[1] & even) | (ok[0] & ~even);
        int best = 0, bc = __builtin_popcountll(ok[0] & valid);
        for (int c = 1; c < 4; c++) {
            const int k = __builtin_popcountll(ok[c] & valid);
            if (k > bc) bc = k, best = c;
        }
        bg[l] = (uint8_t)best;
        for (uint64_t miss = valid & ~ok[best]; miss; miss &= miss - 1) {
            const uint32_t i = (uint32_t)__builtin_ctzll(miss);
            *e++ = ((64 * l + i) << 8) | p[i];
        }
        if (e > e_lim) {  // not GT-like: keep the bytes
            b.raw.assign(d, d + n);
            b.bg.clear();
            b.bg.shrink_to_fit();
            b.ex.clear();
            return;
        }
    }
    b.ex.assign(ex.data(), e);
}
__attribute__((target("avx2,popcnt,bmi"))) static void condense_avx2(const uint8_t *d, uint32_t n, CBlock &b,
                                                                     std::vector<uint32_t> &ex,
                                                                     std::vector<uint64_t> &mk) {
    condense_body<true>(d, n, b, ex, mk);
}
static void condense_block(const uint8_t *d, uint32_t n, CBlock &b, std::vector<uint32_t> &ex,
                           std::vector<uint64_t> &mk) {
    static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("popcnt");
    if (avx2) condense_avx2(d, n, b, ex, mk);
    else condense_body<false>(d, n, b, ex, mk);
}

size_t Bcf::sblock(uint64_t o) const {
    size_t lo = 0, hi = cblk.size();  // the last block with a0 <= o
    while (hi - lo > 1) {
        const size_t mid = (lo + hi) / 2;
        if (cblk[mid].a0 <= o) lo = mid;
        else hi = mid;
    }
    return lo;
}

void Bcf::sread(uint64_t o, size_t n, uint8_t *dst) const {
    size_t hint = sblock(o);
    sread_from(hint, o, n, dst);
}

void Bcf::sread_from(size_t &hint, uint64_t o, size_t n, uint8_t *dst) const {
    size_t bi = hint < cblk.size() && cblk[hint].a0 <= o ? hint : sblock(o);
    while (bi + 1 < cblk.size() && cblk[bi].a0 + cblk[bi].n <= o) bi++;
    hint = bi;
    for (; n; bi++) {
        const CBlock &b = cblk[bi];
        const uint32_t off = (uint32_t)(o - b.a0), m = (uint32_t)std::min<uint64_t>(n, b.n - off);
        b.read(off, m, dst);
        dst += m;
        o += m;
        n -= m;
    }
}

// Read a chunk of compressed bytes and inflate its complete BGZF blocks on the reader's
// threads, each into a thread-local buffer that is condensed at once.
int Bcf::condense_chunk(std::vector<CBlock> &out, bool &eof, double &tr, double &ti) {
    out.clear();
    double t0 = bcf_now();
    const size_t have = cbuf.size();
    cbuf.resize(have + chunk);
    const size_t got = fread(&cbuf[have], 1, chunk, f);
    cbuf.resize(have + got);
    double t1 = bcf_now();
    tr += t1 - t0;
    const bool file_end = got < chunk;
    std::vector<BgzfSpan> blks;
    size_t used = 0;
    if (int rc = bgzf_spans(cbuf, path, blks, used)) return rc;
    if (file_end && used < cbuf.size() && blks.empty()) return fail(TFBS_E_PARSE, "truncated BGZF file " + path);
    std::vector<size_t> nz;  // (empty blocks -- the EOF marker -- add nothing)
    for (size_t i = 0; i < blks.size(); i++)
        if (blks[i].isize) nz.push_back(i);
    out.resize(nz.size());
    std::vector<int> bad(nz.size(), 0);
    const unsigned char *c = (const unsigned char *)cbuf.data();
    par_for(nz.size(), nz.size() >= 4 ? threads : 1, [&](size_t j) {
        thread_local std::vector<uint8_t> buf;
        thread_local std::vector<uint32_t> ex;
        thread_local std::vector<uint64_t> mk;
        const BgzfSpan &s = blks[nz[j]];
        if (buf.size() < s.isize) buf.resize(s.isize);
        if (!(use_fast_inflate && inflate_raw_fast(c + s.off, s.len, buf.data(), s.isize) == 0) &&
            !inflate_zlib(c + s.off, s.len, buf.data(), s.isize)) {
            bad[j] = 1;
            return;
        }
        condense_block(buf.data(), (uint32_t)s.isize, out[j], ex, mk);
    });
    ti += bcf_now() - t1;
    for (int x : bad)
        if (x) return fail(TFBS_E_IO, "corrupt BGZF data in " + path);
    cbuf.erase(0, used);
    eof = file_end && cbuf.empty();
    return TFBS_OK;
}

void Bcf::discard_ahead() {
    if (ahead.th.joinable()) ahead.th.join();
    ahead.blk.clear();
    ahead.rc = TFBS_OK;
}

// The next chunk's condensed blocks onto the stream: the read-ahead's (waited for), or
// read here; then the read-ahead of the one after starts.
int Bcf::inflate_condensed() {
    if (in_eof) return TFBS_OK;
    size_t k = 0;  // the blocks wholly before the next record are done with
    while (k < cblk.size() && cblk[k].a0 + cblk[k].n <= spos) k++;
    if (k) cblk.erase(cblk.begin(), cblk.begin() + (long)k);
    std::vector<CBlock> got;
    bool eof = false;
    if (ahead.th.joinable()) {
        const double t0 = bcf_now();
        ahead.th.join();
        t_ahead_wait += bcf_now() - t0;
        t_read += ahead.tr;
        t_inflate += ahead.ti;
        ahead.tr = ahead.ti = 0;
        if (ahead.rc) {
            const int rc = ahead.rc;
            ahead.rc = TFBS_OK;
            return fail(rc, ahead.err);
        }
        got.swap(ahead.blk);
        eof = ahead.eof;
    } else if (int rc = condense_chunk(got, eof, t_read, t_inflate)) {
        return rc;
    }
    const size_t base = cblk.size();
    cblk.reserve(base + got.size());
    for (CBlock &b : got) {
        b.a0 = send;
        send += b.n;
        n_inflated += b.n;
        cblk.push_back(std::move(b));
    }
    if (eof) {
        in_eof = true;
    } else if (read_ahead) {
        ahead.th = std::thread([this] {
            ahead.rc = condense_chunk(ahead.blk, ahead.eof, ahead.tr, ahead.ti);
            if (ahead.rc) ahead.err = tfbs_last_error();
        });
    }
    return TFBS_OK;
}

// fill() over the condensed stream.  The bytes already inflated (the header round,
// a seek) start it as one kept block.
int Bcf::fill_condensed() {
    if (!cmode) {
        cblk.clear();
        spos = send = 0;
        if (dbuf.size() > doff) {
            CBlock b;
            b.n = (uint32_t)(dbuf.size() - doff);
            b.raw.assign(dbuf.data() + doff, dbuf.data() + dbuf.size());
            send = b.n;
            cblk.push_back(std::move(b));
        }
        dbuf.clear();
        doff = 0;
        cmode = true;
    }
    std::vector<uint64_t> offs;
    const double ts = bcf_now();
    size_t hint = 0;
    for (;;) {
        uint64_t o = spos;
        while (o + 8 <= send) {
            uint8_t h[16];  // the lengths, CHROM and POS in one read
            sread_from(hint, o, (size_t)std::min<uint64_t>(16, send - o), h);
            uint32_t ls, li;
            memcpy(&ls, h, 4);
            memcpy(&li, h + 4, 4);
            const uint64_t n = 8 + (uint64_t)ls + li;
            if (o + n > send) break;
            if (ls < 24) return fail(TFBS_E_PARSE, "short BCF record");
            int32_t chrom, pos;
            memcpy(&chrom, h + 8, 4);
            memcpy(&pos, h + 12, 4);
            if (chrom < 0 || (size_t)chrom >= contigs.size()) return fail(TFBS_E_PARSE, "BCF record with unknown contig");
            if (chrom == cur) {
                const uint64_t p = (uint64_t)(int64_t)pos;
                if (seen && p < last_pos)
                    return fail(TFBS_E_PARSE, "BCF records are not sorted by position (an indexed BCF is): " + path);
                seen = true;
                last_pos = p;
                offs.push_back(o);
            } else if (seen) {
                done = true;
                break;
            }
            o += n;
        }
        spos = o;
        if (done || !offs.empty()) break;
        if (in_eof) {
            if (spos + 8 <= send) return fail(TFBS_E_PARSE, "truncated BCF record");
            done = true;
            break;
        }
        if (int rc = inflate_condensed()) return rc;
    }
    const double td = bcf_now();
    t_scan += td - ts;
    const size_t base = win.size();
    win.resize(base + offs.size());
    std::vector<int> rcs(offs.size(), TFBS_OK);
    par_for(offs.size(), offs.size() >= 64 ? threads : 1,
            [&](size_t i) { rcs[i] = decode_condensed(offs[i], win[base + i]); });
    t_decode += bcf_now() - td;
    for (size_t i = 0; i < rcs.size(); i++)
        if (rcs[i]) {
            BcfRecord r;  // again on this thread for the (thread-local) error message
            return decode_condensed(offs[i], r);
        }
    return TFBS_OK;
}

// decode_bcf_record in carriers mode over the condensed stream: the shared part and
// the FORMAT descriptors are read back; an int8 diploid GT payload of all samples is
// not: its carriers are the differing bytes of its blocks (a background byte, 2 or
// 3, is allele 0 in either slot), or a kept block's bytes.
int Bcf::decode_condensed(uint64_t o, BcfRecord &r) const {
    uint8_t h[8];
    sread(o, 8, h);
    uint32_t ls, li;
    memcpy(&ls, h, 4);
    memcpy(&li, h + 4, 4);
    thread_local std::vector<uint8_t> sh, gbuf;
    sh.resize(ls);
    sread(o + 8, ls, sh.data());
    int32_t chrom;
    uint32_t n_allele, n_fmt;
    if (int rc = decode_shared(Cur{sh.data(), sh.data() + ls}, r, chrom, n_allele, n_fmt)) return rc;
    const std::vector<size_t> *sel_p = all_samples ? nullptr : &sel;
    const size_t ns = samples.size(), nk = sel_p ? sel_p->size() : ns;
    r.carriers.clear();
    r.gt.clear();
    r.gt_status = (n_allele == 2 && nk) ? TFBS_E_PLOIDY : TFBS_OK;  // (no GT field: every GT is empty)
    uint64_t ip = o + 8 + ls;
    const uint64_t ie = ip + li;
    for (uint32_t f = 0; f < n_fmt; f++) {
        uint8_t tb[24];
        const size_t m = (size_t)std::min<uint64_t>(sizeof tb, ie - ip);
        sread(ip, m, tb);
        Cur in{tb, tb + m};
        int kt, vt;
        uint32_t kn, vn;
        int64_t key;
        if (!typed(in, kt, kn) || kn != 1 || !read_int(in, kt, key)) return fail(TFBS_E_PARSE, "bad FORMAT key");
        if (!typed(in, vt, vn)) return fail(TFBS_E_PARSE, "bad FORMAT type");
        ip += (uint64_t)(in.p - tb);
        const uint64_t payload = (uint64_t)type_size(vt) * vn * ns;
        if (ie - ip < payload) return fail(TFBS_E_PARSE, "truncated FORMAT data");
        if (key == gt_key && n_allele == 2 && nk && vt >= 1 && vt <= 3) {
            r.gt_status = vn >= 2 ? TFBS_OK : TFBS_E_PLOIDY;  // one value per sample: glen 1
            if (vt == 1 && vn == 2 && !sel_p) {
                const uint64_t g0 = ip, g1 = ip + payload;
                size_t most = 0;  // (at most one carrier per differing byte: one allocation)
                for (size_t bi = sblock(g0); bi < cblk.size() && cblk[bi].a0 < g1; bi++) {
                    const CBlock &b = cblk[bi];
                    if (!b.raw.empty()) {
                        most += b.n;
                        continue;
                    }
                    const uint32_t lo = (uint32_t)(std::max(g0, b.a0) - b.a0),
                                   hi = (uint32_t)(std::min<uint64_t>(g1, b.a0 + b.n) - b.a0);
                    most += (size_t)(std::lower_bound(b.ex.begin(), b.ex.end(), hi << 8) -
                                     std::lower_bound(b.ex.begin(), b.ex.end(), lo << 8));
                }
                r.carriers.reserve(std::min<size_t>(most, 2 * ns));
                for (size_t bi = sblock(g0); bi < cblk.size() && cblk[bi].a0 < g1; bi++) {
                    const CBlock &b = cblk[bi];
                    const uint32_t lo = (uint32_t)(std::max(g0, b.a0) - b.a0),
                                   hi = (uint32_t)(std::min<uint64_t>(g1, b.a0 + b.n) - b.a0);
                    auto one = [&](uint32_t off, int8_t v) {
                        const uint64_t q = b.a0 + off - g0;
                        if (v == -127) r.gt_status = TFBS_E_PLOIDY;
                        if (v == (q & 1 ? 5 : 4)) r.carriers.push_back((uint32_t)q);  // 2 k + slot
                    };
                    if (!b.raw.empty()) {
                        for (uint32_t off = lo; off < hi; off++)
                            if ((b.raw[off] & 0xFE) != 2) one(off, (int8_t)b.raw[off]);
                    } else {
                        for (auto it = std::lower_bound(b.ex.begin(), b.ex.end(), lo << 8);
                             it != b.ex.end() && (*it >> 8) < hi; ++it)
                            one(*it >> 8, (int8_t)(uint8_t)*it);
                    }
                }
            } else if (vn >= 2) {
                gbuf.resize(payload);
                sread(ip, payload, gbuf.data());
                gt_carriers(gbuf.data(), vt, vn, ns, sel_p, r);
            }
        }
        ip += payload;
    }
    return TFBS_OK;
}

int Bcf::contig_index(const std::string &name) const {
    for (size_t i = 0; i < contigs.size(); i++)
        if (contigs[i] == name) return (int)i;
    return -1;
}

int Bcf::fetch(int contig, uint64_t beg, uint64_t end, std::vector<const BcfRecord *> &out) {
    out.clear();
    if (contig < 0 || (size_t)contig >= contigs.size()) return TFBS_OK;
    const bool back = contig != cur || beg < last_beg;
    if (indexed()) {
        // seek when the sweep would rewind, or when the query's first record lies
        // past everything read so far (a sparse BED over a large file)
        const uint64_t v = csi_start(contig, beg);
        if (v == UINT64_MAX) {  // nothing on this contig ends after beg
            win.clear();
            cur = contig;
            done = true;
            last_beg = beg;
            return TFBS_OK;
        }
        const off_t fpos = ftello(f);
        if (back || (fpos >= 0 && (v >> 16) > (uint64_t)fpos)) {
            if (int rc = seek(contig, v)) return rc;
        }
    } else if (back) {
        if (int rc = rewind()) return rc;
        cur = contig;
    }
    last_beg = beg;
    // drop what no later query (beg' >= beg) can overlap
    size_t k = 0;
    while (k < win.size() && win[k].pos + win[k].rlen <= beg) k++;
    if (k) win.erase(win.begin(), win.begin() + k);
    if (win.size() > 4096)
        win.erase(std::remove_if(win.begin(), win.end(), [&](const BcfRecord &r) { return r.pos + r.rlen <= beg; }),
                  win.end());
    while (!done && (win.empty() || win.back().pos < end))
        if (int rc = condensed() ? fill_condensed() : fill()) return rc;
    for (const BcfRecord &r : win) {
        if (r.pos >= end) break;
        if (r.pos + r.rlen > beg) out.push_back(&r);
    }
    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// FASTA (.fai)
// ---------------------------------------------------------------------------
int Fasta::open(const std::string &path) {
    this->path = path;
    std::ifstream fi(path + ".fai");
    if (!fi) return fail(TFBS_E_IO, "Error while opening the reference genome '" + path + "' (.fai missing)");
    std::string line;
    while (std::getline(fi, line)) {
        std::istringstream ls(line);
        std::string name;
        FaiEntry e;
        if (std::getline(ls, name, '\t') && (ls >> e.len >> e.off >> e.lbases >> e.lwidth)) idx[name] = e;
    }
    f = fopen(path.c_str(), "rb");
    if (!f) return fail(TFBS_E_IO, "Error while opening the reference genome '" + path + "'");
    return TFBS_OK;
}
Fasta::~Fasta() {
    if (f) fclose(f);
}
int Fasta::fetch(const std::string &chrom, uint64_t start, uint64_t stop, std::string &out) {
    out.clear();
    auto it = idx.find(chrom);
    if (it == idx.end()) return fail(TFBS_E_RANGE, "Error while seeking in reference genome file: unknown " + chrom);
    const FaiEntry &e = it->second;
    if (start > e.len) return fail(TFBS_E_RANGE, "Error while seeking in reference genome file");
    stop = std::min(stop, e.len);
    uint64_t pos = start;
    while (pos < stop) {
        const uint64_t line = pos / e.lbases, col = pos % e.lbases;
        const uint64_t take = std::min<uint64_t>(e.lbases - col, stop - pos);
        if (fseeko(f, (off_t)(e.off + line * e.lwidth + col), SEEK_SET)) return fail(TFBS_E_IO, "seek failed");
        const size_t old = out.size();
        out.resize(old + take);
        if (fread(&out[old], 1, take, f) != take) return fail(TFBS_E_IO, "short FASTA read");
        pos += take;
    }
    return TFBS_OK;
}

// ---------------------------------------------------------------------------
// BED (bed.rs:9-19): tab separated chrom, start, end[, ...]; raw start/end kept
// as an inclusive Range.  Empty lines and '#'/track/browser lines are skipped.
// ---------------------------------------------------------------------------
int load_bed(const std::string &path, const std::string &chrom, std::vector<std::pair<uint64_t, uint64_t>> &out) {
    std::ifstream in(path);
    if (!in) return fail(TFBS_E_IO, "Bed file " + path + " does not exist");
    std::string line;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty() || line[0] == '#' || line.rfind("track", 0) == 0 || line.rfind("browser", 0) == 0) continue;
        std::vector<std::string> f;
        std::string x;
        std::istringstream ls(line);
        while (std::getline(ls, x, '\t')) f.push_back(x);
        if (f.size() < 3) return fail(TFBS_E_PARSE, "bad BED line in " + path);
        if (f[0] != chrom) continue;
        char *e1 = nullptr, *e2 = nullptr;
        unsigned long long s = strtoull(f[1].c_str(), &e1, 10), e = strtoull(f[2].c_str(), &e2, 10);
        if (*e1 || *e2 || f[1].empty() || f[2].empty()) return fail(TFBS_E_PARSE, "bad BED coordinates in " + path);
        out.push_back({s, e});
    }
    return TFBS_OK;
}

// range.rs:43-87 RangeStack: stable sort by start, merge while last.overlaps(next).
std::vector<std::pair<uint64_t, uint64_t>> merge_ranges(std::vector<std::pair<uint64_t, uint64_t>> r) {
    std::stable_sort(r.begin(), r.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::vector<std::pair<uint64_t, uint64_t>> out;
    for (auto &x : r) {
        if (!out.empty()) {
            auto &l = out.back();
            const bool ov = (x.first >= l.first && x.first <= l.second) || (x.second >= l.first && x.second <= l.second);
            if (ov) {
                l.first = std::min(l.first, x.first);
                l.second = std::max(l.second, x.second);
                continue;
            }
        }
        out.push_back(x);
    }
    return out;
}

}  // namespace tfbs
