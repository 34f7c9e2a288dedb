// File formats around the scoring path.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace tfbs {

int bgzf_inflate(const std::string &in, std::string &out);
int bgzf_block(const char *data, size_t n, std::string &out);

// BGZF writer with the block boundaries of BGzWriter (main.rs:267-276): a
// block every kBlock input bytes and at each flush().  Full blocks are queued
// and deflated in parallel (`threads`), then written in order, so the bytes
// are those of a one-block-at-a-time writer.
class BgzfWriter {
  public:
    static constexpr size_t kBlock = 65280;  // htslib/bgzip's BGZF_BLOCK_SIZE of input per block
    int open(const std::string &path, uint32_t threads = 1);
    int write(const char *p, size_t n);
    // For whole BGZF blocks made elsewhere (tfbs_batch_rows_bgzf): the open block,
    // if it holds anything, is ended and written, the stream flushed; returns the
    // file descriptor to append the blocks to (or < 0 with the error set).
    int raw_fd();
    // after blocks were written to raw_fd() at explicit offsets: the stream goes on at `at`
    int seek_to(uint64_t at);
    int flush();
    int close();
    ~BgzfWriter();

  private:
    int drain();
    FILE *f = nullptr;
    uint32_t threads = 1;
    std::string raw;                   // queued input: blocks back to back, then the open block
    std::vector<size_t> ends;          // end offset in raw of each queued (closed) block
};

struct BcfRecord {
    uint64_t pos = 0;       // 0-based
    uint32_t rlen = 0;
    uint32_t n_alleles = 0;
    std::string ref, alt;   // alleles[0], alleles[1] (alt empty if a single allele)
    std::vector<int32_t> gt;  // 2 raw GT ints per selected sample, INT32_MIN+1 = vector_end / absent
    // carriers mode (Bcf::set_carriers_mode; raw gt left empty): load_diffs' carriers of
    // a bi-allelic record (haplotype.rs:16-41: 2 k + 0 iff GT[0] = Unphased(1), 2 k + 1
    // iff GT[1] = Phased(1), k the selected sample), found while the record is decoded
    // on the reader's threads; gt_status TFBS_E_PLOIDY if some selected sample's GT
    // does not have 2 alleles (raised when a region uses the record)
    std::vector<uint32_t> carriers;
    int gt_status = 0;
};

// Streaming BCF2 reader (f2; replaces rust_htslib's IndexedReader::fetch +
// records(), haplotype.rs:78-82).  BGZF blocks are inflated chunk by chunk in
// parallel threads, record boundaries are found serially and records are
// decoded in parallel, for one contig at a time, keeping GT only for the
// selected samples.  fetch() keeps a window of the records that can still
// overlap a later query, so a sweep with nondecreasing `beg` (the run flow's
// sorted merged regions) reads the file once; a query that goes backwards or
// to another contig rewinds to the start of the file.  Input must be sorted
// by position within a contig (an indexed BCF is); unsorted input fails.
// With a CSI index (<path>.csi, as bcftools index writes it) a query that
// would rewind, or whose first record lies beyond what has been read, seeks
// to the index's chunk start instead (IndexedReader::fetch's seek); the
// sweep itself is unchanged.
// Raw DEFLATE (RFC 1951) of in[0, in_len) into exactly out_len bytes (inflate.cpp);
// 0 on success, nonzero when it cannot decode the stream exactly (the caller then
// inflates with zlib).
int inflate_raw_fast(const uint8_t *in, size_t in_len, uint8_t *out, size_t out_len);

// A byte buffer that grows without zero-filling and drops consumed bytes from the
// front by moving only what is left (the reader's inflated stream: hundreds of MB
// per round, of which std::string's resize zero-filled and erase moved everything).
class RawBuf {
  public:
    const char *data() const { return p.get(); }
    char *data() { return p.get(); }
    size_t size() const { return n; }
    void clear() { n = 0; }
    char &operator[](size_t i) { return p[i]; }
    void resize_uninit(size_t m) {
        if (m > cap) {
            const size_t c = std::max(m, cap + cap / 2);
            std::unique_ptr<char[]> q(new char[c]);
            if (n) memcpy(q.get(), p.get(), n);
            p = std::move(q);
            cap = c;
        }
        n = m;
    }
    void erase_front(size_t k) {
        k = std::min(k, n);
        if (k < n) memmove(p.get(), p.get() + k, n - k);
        n -= k;
    }
    void assign(const std::string &s) {
        resize_uninit(s.size());
        if (!s.empty()) memcpy(p.get(), s.data(), s.size());
    }

  private:
    std::unique_ptr<char[]> p;
    size_t n = 0, cap = 0;
};

// One inflated BGZF block of a carriers-mode stream, condensed (Bcf::fill_condensed):
// GT columns are nearly all 0|0 -- bytes 2 and 3 -- so a block is kept as a background
// code per 64-byte line (0: 2 at even offsets and 3 at odd ones, 1: the other way
// round, 2: all 2, 3: all 3) and the bytes that differ from it, (offset << 8 | byte)
// ascending; a block with more than 1/16 of its bytes differing keeps its bytes
// (`raw`).  Exact: every byte can be read back.
struct CBlock {
    uint64_t a0 = 0;              // offset of its first byte in the condensed stream
    uint32_t n = 0;               // its bytes (> 0)
    std::vector<uint8_t> raw;     // dense block; empty when condensed
    std::vector<uint8_t> bg;      // per 64-byte line: its background code
    std::vector<uint32_t> ex;     // the bytes that differ from the background
    uint8_t at(uint32_t off) const;
    void read(uint32_t off, uint32_t n, uint8_t *dst) const;
};

class Bcf {
  public:
    int open(const std::string &path, uint32_t threads = 0);
    // GT columns kept, in this order (default: all samples); rewinds the stream.
    int select(const std::vector<size_t> &sel);
    // records keep their carriers instead of raw GT (the run flow; rewinds the stream)
    int set_carriers_mode(bool on);
    int contig_index(const std::string &name) const;
    // records with pos < end && pos + rlen > beg, in file order; pointers stay
    // valid until the next fetch
    int fetch(int contig, uint64_t beg, uint64_t end, std::vector<const BcfRecord *> &out);
    // The records of the last fetch that no later fetch from beg_next on can return
    // (pos + rlen <= beg_next): their carriers may be moved out (the run flow's fetch
    // stage, which knows its next region), the others are copied.
    bool dropped_before(const BcfRecord *r, uint64_t beg_next) const { return r->pos + r->rlen <= beg_next; }
    std::vector<uint32_t> take_carriers(const BcfRecord *r) {
        return std::move(const_cast<BcfRecord *>(r)->carriers);  // (r is one of this reader's window)
    }
    ~Bcf();
    std::vector<std::string> samples, contigs;

    bool indexed() const { return !csi.empty(); }
    // seconds so far in file reads, inflate + condense, record boundary scans (with the
    // inflate rounds they wait for: of them, waits for the read-ahead), decodes
    void phase_seconds(double &read, double &inflate, double &scan, double &ahead_wait, double &decode) const {
        read = t_read, inflate = t_inflate, scan = t_scan, ahead_wait = t_ahead_wait, decode = t_decode;
    }

  private:
    int rewind();
    int inflate_more();
    int fill();
    // carriers mode over the condensed stream: BGZF blocks inflated and condensed on
    // the reader's threads (CBlock: the inflated bytes never reach memory in full),
    // record boundaries found serially, records decoded in parallel
    int fill_condensed();
    bool condensed() const { return carriers_mode && condense && bgzf; }
    int inflate_condensed();
    // the next `chunk` compressed bytes' complete BGZF blocks, inflated and condensed
    // on the reader's threads (a0 unset); reads f and cbuf only
    int condense_chunk(std::vector<CBlock> &out, bool &eof, double &tr, double &ti);
    // read-ahead (TFBS_BCF_READAHEAD=0: off): once a chunk is in, the next one is read
    // and condensed on a background thread while the caller scans, decodes and does
    // its own work; inflate_condensed takes it over, seek/rewind discard it
    struct Ahead {
        std::thread th;
        std::vector<CBlock> blk;
        bool eof = false;
        int rc = 0;
        std::string err;
        double tr = 0, ti = 0;
    } ahead;
    bool read_ahead = true;
    double t_ahead_wait = 0;  // (of t_scan) waiting for the read-ahead to finish
    void discard_ahead();
    void sread(uint64_t o, size_t n, uint8_t *dst) const;  // bytes [o, o + n) of the condensed stream
    // sread with the block search from *hint on (a walk in stream order)
    void sread_from(size_t &hint, uint64_t o, size_t n, uint8_t *dst) const;
    size_t sblock(uint64_t o) const;                       // the block holding byte o
    int decode_condensed(uint64_t o, BcfRecord &r) const;
    int load_csi();
    // virtual offset to start reading for records with pos + rlen > beg on
    // `contig` (the smallest chunk start of the CSI bins ending after beg);
    // UINT64_MAX: no such record; 0 with no index.
    uint64_t csi_start(int contig, uint64_t beg) const;
    int seek(int contig, uint64_t voff);
    // per contig: (bin end, smallest chunk start over this and every later entry)
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> csi;
    std::string path;
    FILE *f = nullptr;
    uint32_t threads = 1;
    size_t chunk = 8u << 20;            // compressed bytes read per inflate round
    bool use_fast_inflate = true;       // inflate_raw_fast, zlib where it fails (TFBS_BCF_ZLIB=1: zlib only)
    // TFBS_BCF_TIMING: seconds per phase (printed when the reader closes); scan_s
    // includes the inflate rounds a fill needs
    double t_read = 0, t_inflate = 0, t_erase = 0, t_scan = 0, t_decode = 0;
    uint64_t n_inflated = 0;
    bool bgzf = true, in_eof = false, done = false, seen = false;
    std::string cbuf;                   // compressed tail not yet inflated
    RawBuf dbuf;                        // inflated bytes from doff on
    size_t doff = 0;
    int gt_key = -1;
    std::vector<size_t> sel;
    bool all_samples = true;
    bool carriers_mode = false;
    bool condense = true;               // carriers mode reads the condensed stream (TFBS_BCF_CONDENSED=0: off)
    bool cmode = false;                 // the stream is condensed from spos on (reset by rewind / seek)
    std::vector<CBlock> cblk;           // condensed blocks, in stream order (consumed ones dropped)
    uint64_t spos = 0, send = 0;        // next record / end of the condensed stream
    int cur = -1;                       // contig of the window
    uint64_t last_beg = 0, last_pos = 0;
    std::vector<BcfRecord> win;         // window of decoded records of contig `cur`, file order
};

class Fasta {
  public:
    int open(const std::string &path);
    // bio::io::fasta::IndexedReader::fetch(chrom, start, stop) + read: [start, stop), truncated at the end
    int fetch(const std::string &chrom, uint64_t start, uint64_t stop, std::string &out);
    ~Fasta();

  private:
    struct FaiEntry {
        uint64_t len = 0, off = 0, lbases = 0, lwidth = 0;
    };
    std::string path;
    std::map<std::string, FaiEntry> idx;
    FILE *f = nullptr;
};

int load_bed(const std::string &path, const std::string &chrom, std::vector<std::pair<uint64_t, uint64_t>> &out);
std::vector<std::pair<uint64_t, uint64_t>> merge_ranges(std::vector<std::pair<uint64_t, uint64_t>> r);

}  // namespace tfbs
