#!/usr/bin/env python3
"""Synthetic find-tfbs input set: FASTA (+.fai), BED, BCF (BGZF, BCF2 GT), samples
file and HOCOMOCO-format PWMs + thresholds, from the SURVEY.md 8(d) generator
(the same regions bench.py scans).  Used by the run-flow parity test
(tests/test_gpu_parity.py) and by tools/bench_run.py.

Layout of the synthetic chromosome "chr1": merged region j is [1000 + 400 j,
1200 + 400 j]; the bases of every region's extended window come from the
generator; the rest of the chromosome is A.  Variants: the generator's records,
each sample's GT written as phased pairs (left alt = 1 -> GT[0] = 4 (Unphased(1)),
right alt -> GT[1] = 5 (Phased(1)), references 2 / 3), which load_diffs
(haplotype.rs:34-41) reads back as the same carrier sets.

Usage: python tools/synth_dataset.py OUTDIR [--samples N] [--regions R] [--pwms P]
       [--length-config C] [--seed S] [--indel-pct I]
"""
import argparse
import os
import struct
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


BGZF_BLOCK = 65280


def bgzf_blocks(data, block_offsets=None):
    """BGZF framing (SAM spec 4.1): <= 64 KiB-input deflate blocks + the EOF block.
    block_offsets (a list) receives each block's compressed file offset."""
    out = bytearray()
    for i in range(0, len(data), BGZF_BLOCK):
        if block_offsets is not None:
            block_offsets.append(len(out))
        chunk = bytes(data[i:i + BGZF_BLOCK])
        co = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = co.compress(chunk) + co.flush()
        bsize = len(comp) + 25
        out += struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
        out += comp
        out += struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def reg2bin(beg, end, min_shift, depth):
    """htslib hts_reg2bin: the smallest bin holding [beg, end)."""
    end -= 1
    s, t = min_shift, ((1 << (3 * depth)) - 1) // 7
    for lev in range(depth, 0, -1):
        if beg >> s == end >> s:
            return t + (beg >> s)
        s += 3
        t -= 1 << (3 * (lev - 1))
    return 0


def csi_index(spans, block_offsets, contig_len, min_shift=14):
    """A CSI index (htslib's format, as `bcftools index` writes it, without the
    optional pseudo-bin) for one contig.  spans: per record in file order
    (pos0, rlen, uncompressed start, uncompressed end) in the BGZF stream."""
    max_len = contig_len + 256
    depth, sz = 0, 1 << min_shift
    while max_len > sz:
        depth += 1
        sz <<= 3

    def voff(u):
        k = u // BGZF_BLOCK
        if k >= len(block_offsets):  # end of the last block
            k = len(block_offsets) - 1
            return (block_offsets[k] << 16) | (u - k * BGZF_BLOCK)
        return (block_offsets[k] << 16) | (u % BGZF_BLOCK)

    bins = {}
    for pos0, rlen, u0, u1 in spans:
        b = reg2bin(pos0, pos0 + max(rlen, 1), min_shift, depth)
        ch = bins.setdefault(b, [])
        v0, v1 = voff(u0), voff(u1)
        if ch and ch[-1][1] == v0:
            ch[-1][1] = v1
        else:
            ch.append([v0, v1])
    body = b"CSI\1" + struct.pack("<iii", min_shift, depth, 0) + struct.pack("<i", 1)
    body += struct.pack("<i", len(bins))
    for b in sorted(bins):
        ch = bins[b]
        body += struct.pack("<IQi", b, ch[0][0], len(ch))
        for v0, v1 in ch:
            body += struct.pack("<QQ", v0, v1)
    body += struct.pack("<Q", 0)
    return bgzf_blocks(body)


def typed_str(s):
    b = s.encode()
    if len(b) < 15:
        return bytes([(len(b) << 4) | 7]) + b
    return bytes([0xF7, 0x11, len(b)]) + b  # length as a typed int8


def bcf_record(chrom, pos0, ref, alt, gt_pairs):
    """One BCF2 record: no QUAL/ID/FILTER/INFO, FORMAT GT as int8 pairs."""
    n_sample = gt_pairs.shape[0]
    shared = struct.pack("<iiif", chrom, pos0, len(ref), struct.unpack("<f", struct.pack("<I", 0x7F800001))[0])
    shared += struct.pack("<II", (2 << 16) | 0, (1 << 24) | n_sample)
    shared += typed_str("") + typed_str(ref) + typed_str(alt) + bytes([0x00])  # ID '.', alleles, FILTER none
    indiv = bytes([0x11, 1, 0x21]) + gt_pairs.astype(np.int8).tobytes()  # key GT (dict index 1), 2 x int8
    return struct.pack("<II", len(shared), len(indiv)) + shared + indiv


class BgzfStream:
    """BGZF framing written as the data comes (fixed BGZF_BLOCK-byte blocks, so a
    record's uncompressed offset u lies in block u // BGZF_BLOCK, as csi_index assumes),
    the blocks deflated on a thread pool (zlib drops the GIL); block_offsets receives
    each block's compressed file offset."""

    def __init__(self, f, level=6, threads=16):
        import concurrent.futures as cf
        self.f, self.level, self.pending, self.size = f, level, bytearray(), 0
        self.block_offsets, self.pos = [], 0
        self.ex = cf.ThreadPoolExecutor(threads)
        self.threads = threads

    def _blocks(self, chunks):
        def one(chunk):
            co = zlib.compressobj(self.level, zlib.DEFLATED, -15)
            comp = co.compress(chunk) + co.flush()
            return (struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, len(comp) + 25) + comp +
                    struct.pack("<II", zlib.crc32(chunk) & 0xFFFFFFFF, len(chunk)))
        for b in self.ex.map(one, chunks):
            self.block_offsets.append(self.pos)
            self.f.write(b)
            self.pos += len(b)

    def write(self, data):
        self.pending += data
        self.size += len(data)
        n = len(self.pending) // BGZF_BLOCK
        if n >= 4 * self.threads:
            self._blocks([bytes(self.pending[i * BGZF_BLOCK:(i + 1) * BGZF_BLOCK]) for i in range(n)])
            del self.pending[:n * BGZF_BLOCK]

    def close(self):
        n = (len(self.pending) + BGZF_BLOCK - 1) // BGZF_BLOCK
        self._blocks([bytes(self.pending[i * BGZF_BLOCK:(i + 1) * BGZF_BLOCK]) for i in range(n)])
        self.f.write(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
        self.ex.shutdown()


def make_dataset(out, n_samples=200, n_regions=20, n_pwms=8, length_config=2, seed=3, indel_pct=0, index=True,
                 keep_gt=True, level=6, edges=False):
    """keep_gt=False: the returned records carry no GT arrays (large runs: the BCF is
    streamed out region by region, records of a region sorted; regions are 400 bp
    apart and their extended windows do not overlap, so the file is sorted).
    edges=True: per region three more records at the fetch window's edges (SURVEY.md
    8(c), the cases no reference fixture pins): an SNV at the window's last base
    (pos0 = ext.end), one just past it (pos0 = ext.end + 1: outside the half-open
    fetch(ext.start, ext.end + 1)), and a 3-base deletion starting two bases left of
    ext.start that reaches into the window (fetched, left out of the patch)."""
    import tfbs_pkg
    T = tfbs_pkg.load()
    os.makedirs(out, exist_ok=True)
    names = T.synth_write_pwms(out, n_pwms, length_config, seed)
    ps = T.parse_pwm_files(os.path.join(out, "pwms.txt"), os.path.join(out, "thr"), 1e-4, names)
    lmax = ps.max_length
    samples = ["S%05d" % i for i in range(n_samples)]
    H = 2 * n_samples
    regions, records = [], []
    chrom_len = 1000 + 400 * n_regions + 1000
    seq = bytearray(b"A" * chrom_len)
    header = ("##fileformat=VCFv4.2\n##FILTER=<ID=PASS,Description=\"All filters passed\">\n"
              "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
              "##contig=<ID=chr1,length=%d>\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t%s\n"
              % (chrom_len, "\t".join(samples))).encode() + b"\0"
    bcf = os.path.join(out, "genotypes.bcf")
    spans = []
    last_pos = -1
    with open(bcf, "wb") as f:
        z = BgzfStream(f, level)
        z.write(b"BCF\2\2" + struct.pack("<I", len(header)) + header)
        for j in range(n_regions):
            if j and j % 1000 == 0:  # progress for long runs (stderr)
                print("synth_dataset: %d / %d regions" % (j, n_regions), file=sys.stderr, flush=True)
            r = T.SynthRegion(seed, j, n_samples, lmax, indel_pct)
            s, e = r.merged
            regions.append((s, e))
            es = r.ext_start
            seq[es:es + len(r.ref)] = r.ref.encode()
            recs = []
            extra = []
            if edges:
                ee = es + len(r.ref) - 1  # ext.end (inclusive)
                erng = np.random.default_rng(seed * 7919 + j)
                for p0, rl in ((ee, 1), (ee + 1, 1), (es - 2, 4)):
                    if p0 < 0:
                        continue
                    ref_b = bytes(seq[p0:p0 + rl]).decode()
                    alt_b = ref_b[0] if rl > 1 else "ACGT"[("ACGT".index(ref_b) + 1 + int(erng.integers(3))) % 4]
                    car = np.sort(erng.choice(H, size=max(1, H // 5), replace=False))
                    extra.append((p0, ref_b, alt_b, car.tolist()))
            for pos, ref, alt, car in list(r.records) + extra:
                gt = np.empty((n_samples, 2), dtype=np.int8)
                gt[:, 0] = 2
                gt[:, 1] = 3
                car = np.asarray(car, dtype=np.int64)
                car = car[car < H]
                gt[car[car % 2 == 0] // 2, 0] = 4
                gt[car[car % 2 == 1] // 2, 1] = 5
                recs.append({"chrom": "chr1", "pos0": pos, "rlen": len(ref), "alleles": [ref, alt], "gt": gt})
            recs.sort(key=lambda x: x["pos0"])
            for rec in recs:
                assert rec["pos0"] >= last_pos, "records out of order across regions"
                last_pos = rec["pos0"]
                u0 = z.size
                z.write(bcf_record(0, rec["pos0"], rec["alleles"][0], rec["alleles"][1], rec["gt"]))
                spans.append((rec["pos0"], rec["rlen"], u0, z.size))
                if not keep_gt:
                    rec = {k: v for k, v in rec.items() if k != "gt"}
                records.append(rec)
        z.close()
    if index:
        with open(bcf + ".csi", "wb") as f:
            f.write(csi_index(spans, z.block_offsets, chrom_len))
    # FASTA + .fai
    fa = os.path.join(out, "genome.fa")
    with open(fa, "w") as f:
        f.write(">chr1\n")
        for i in range(0, chrom_len, 60):
            f.write(seq[i:i + 60].decode() + "\n")
    with open(fa + ".fai", "w") as f:
        f.write("chr1\t%d\t6\t60\t61\n" % chrom_len)
    # BED (half-open in the file; find-tfbs reads [start, end] inclusive, bed.rs:15)
    bed = os.path.join(out, "regions.bed")
    with open(bed, "w") as f:
        for s, e in regions:
            f.write("chr1\t%d\t%d\n" % (s, e))
    with open(os.path.join(out, "samples"), "w") as f:
        f.write("\n".join(samples) + "\n")
    return {"dir": out, "fasta": fa, "bed": bed, "bcf": bcf, "samples": samples, "names": names,
            "pwm_file": os.path.join(out, "pwms.txt"), "thr_dir": os.path.join(out, "thr"),
            "records": records, "regions": regions}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--samples", type=int, default=200)
    ap.add_argument("--regions", type=int, default=20)
    ap.add_argument("--pwms", type=int, default=8)
    ap.add_argument("--length-config", type=int, default=2)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--indel-pct", type=int, default=0)
    ap.add_argument("--no-index", action="store_true", help="no <bcf>.csi")
    a = ap.parse_args()
    d = make_dataset(a.out, a.samples, a.regions, a.pwms, a.length_config, a.seed, a.indel_pct, not a.no_index)
    print("wrote %s: %d records, %d regions, %d samples" % (d["bcf"], len(d["records"]), len(d["regions"]),
                                                           len(d["samples"])))


if __name__ == "__main__":
    main()
