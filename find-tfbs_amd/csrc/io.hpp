// File formats around the scoring path.
#pragma once

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace tfbs {

int bgzf_inflate(const std::string &in, std::string &out);
int bgzf_block(const char *data, size_t n, std::string &out);

class BgzfWriter {
  public:
    static constexpr size_t kBlock = 65280;  // htslib/bgzip's BGZF_BLOCK_SIZE of input per block
    int open(const std::string &path);
    int write(const char *p, size_t n);
    int flush();
    int close();
    ~BgzfWriter();

  private:
    int emit();
    FILE *f = nullptr;
    std::string buf;
};

struct BcfRecord {
    uint64_t pos = 0;       // 0-based
    uint32_t rlen = 0;
    uint32_t n_alleles = 0;
    std::string ref, alt;   // alleles[0], alleles[1] (alt empty if a single allele)
    std::vector<int32_t> gt;  // 2 raw GT ints per sample (all samples), INT32_MIN+1 = vector_end
};

class Bcf {
  public:
    int open(const std::string &path);
    int contig_index(const std::string &name) const;
    void fetch(int contig, uint64_t beg, uint64_t end, std::vector<const BcfRecord *> &out) const;
    std::vector<std::string> samples, contigs;

  private:
    std::vector<std::vector<BcfRecord>> per_contig;
    std::vector<std::vector<uint64_t>> max_end;
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
