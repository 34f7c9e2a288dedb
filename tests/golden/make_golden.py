#!/usr/bin/env python3
"""Regenerate the golden fixtures under tests/golden/ from the reference's test_data.

The inputs in tests/golden/test_data/ are byte copies of find-tfbs v1.0.1
test_data/ (data files only).  This script derives two small fixtures from them:

* ``expected_output_{1,2}.vcf`` -- the decompressed text of the reference's
  BGZF outputs (main.rs:548-568 compares gz bytes; those bytes come from
  miniz-sys 0.1.12 and are not reproducible with zlib, so parity is on text).
* ``genotypes{,2}.records.json`` -- the BCF records decoded by a tiny,
  independent BCF2 reader (below), so the oracle can be fed the same variants
  without sharing the product's BCF reader (find-tfbs_amd/csrc/bcf.cpp).

Run: python tests/golden/make_golden.py
"""
import gzip
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "test_data")

INT8_VE, INT16_VE, INT32_VE = -127, -32767, -2147483647  # BCF2 vector_end sentinels


def _typed(buf, off):
    """Decode a BCF2 typed-value descriptor; returns (type, count, new offset)."""
    d = buf[off]
    off += 1
    t, n = d & 0x0F, d >> 4
    if n == 15:
        vt, vn, off = _typed(buf, off)
        assert vn == 1
        n, off = _ints(buf, off, vt, 1)
        n = n[0]
    return t, n, off


def _ints(buf, off, t, n):
    fmt = {1: "b", 2: "h", 3: "i"}[t]
    size = {1: 1, 2: 2, 3: 4}[t]
    vals = list(struct.unpack_from("<%d%s" % (n, fmt), buf, off))
    ve = {1: INT8_VE, 2: INT16_VE, 3: INT32_VE}[t]
    vals = [INT32_VE if v == ve else v for v in vals]
    return vals, off + n * size


def read_bcf(path):
    raw = gzip.decompress(open(path, "rb").read())  # BGZF = concatenated gzip members
    assert raw[:5] == b"BCF\x02\x02", raw[:5]
    (l_text,) = struct.unpack_from("<I", raw, 5)
    text = raw[9 : 9 + l_text].rstrip(b"\x00").decode()
    off = 9 + l_text
    # string dictionary: PASS first, then FILTER/INFO/FORMAT IDs in order (IDX= when present)
    sdict = {0: "PASS"}
    contigs = []
    samples = []
    nxt = 1
    for line in text.split("\n"):
        if line.startswith("##contig=<"):
            cid = line.split("ID=")[1].split(",")[0].rstrip(">")
            contigs.append(cid)
        elif line.startswith(("##FILTER=<", "##INFO=<", "##FORMAT=<")):
            fid = line.split("ID=")[1].split(",")[0].rstrip(">")
            if fid == "PASS":
                continue
            if "IDX=" in line:
                idx = int(line.split("IDX=")[1].split(",")[0].rstrip(">"))
            else:
                idx = nxt
            sdict[idx] = fid
            nxt = max(nxt, idx + 1)
        elif line.startswith("#CHROM"):
            samples = line.split("\t")[9:]
    records = []
    while off < len(raw):
        l_shared, l_indiv = struct.unpack_from("<II", raw, off)
        off += 8
        sh = raw[off : off + l_shared]
        ind = raw[off + l_shared : off + l_shared + l_indiv]
        off += l_shared + l_indiv
        chrom, pos, rlen = struct.unpack_from("<iii", sh, 0)
        n_allele_info, n_fmt_sample = struct.unpack_from("<II", sh, 16)
        n_allele, n_info = n_allele_info >> 16, n_allele_info & 0xFFFF
        n_fmt, n_sample = n_fmt_sample >> 24, n_fmt_sample & 0xFFFFFF
        p = 24
        t, n, p = _typed(sh, p)  # ID
        p += n
        alleles = []
        for _ in range(n_allele):
            t, n, p = _typed(sh, p)
            alleles.append(sh[p : p + n].decode())
            p += n
        q = 0
        gts = None
        for _ in range(n_fmt):
            kt, kn, q = _typed(ind, q)
            key, q = _ints(ind, q, kt, 1)
            vt, vn, q = _typed(ind, q)
            size = {1: 1, 2: 2, 3: 4, 5: 4, 7: 1}[vt]
            if sdict.get(key[0]) == "GT":
                vals, _ = _ints(ind, q, vt, vn * n_sample)
                gts = [vals[i * vn : (i + 1) * vn] for i in range(n_sample)]
            q += vn * n_sample * size
        records.append(
            {"chrom": contigs[chrom], "pos0": pos, "rlen": rlen, "alleles": alleles, "gt": gts}
        )
    return {"samples": samples, "contigs": contigs, "records": records}


def main():
    for i in (1, 2):
        src = os.path.join(DATA, "expected_output_%d.vcf.gz" % i)
        with open(os.path.join(HERE, "expected_output_%d.vcf" % i), "wb") as f:
            f.write(gzip.decompress(open(src, "rb").read()))
    for name in ("genotypes", "genotypes2"):
        rec = read_bcf(os.path.join(DATA, name + ".bcf"))
        with open(os.path.join(HERE, name + ".records.json"), "w") as f:
            json.dump(rec, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
