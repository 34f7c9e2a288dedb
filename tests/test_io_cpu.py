"""f2-f4 file formats on the CPU: BCF decode vs the independent fixture decoder,
FASTA fetch vs the oracle driver, BGZF write/read, BED merge vs the oracle."""
import gzip
import json
import os
import random
import sys

import pytest

import oracle_py as O
from helpers import GOLD, TD, T


def test_bcf_reader_matches_fixture_decoder():
    for name in ("genotypes", "genotypes2"):
        want = json.load(open(os.path.join(GOLD, name + ".records.json")))
        r = T.BcfReader(os.path.join(TD, name + ".bcf"))
        assert r.samples == want["samples"]
        got = r.fetch("chr1", 0, 250)
        assert len(got) == len(want["records"])
        for g, w in zip(got, want["records"]):
            assert (g["pos0"], g["rlen"], g["ref"], g["alt"]) == (w["pos0"], w["rlen"], w["alleles"][0],
                                                                  w["alleles"][1])
            assert g["gt"] == w["gt"]


def test_bcf_fetch_overlap_semantics():
    r = T.BcfReader(os.path.join(TD, "genotypes2.bcf"))  # one record, POS0 = 100, rlen 1
    assert len(r.fetch("chr1", 100, 101)) == 1
    assert len(r.fetch("chr1", 97, 114)) == 1
    assert r.fetch("chr1", 101, 200) == []   # pos + rlen > beg fails
    assert r.fetch("chr1", 0, 100) == []     # pos < end fails (half-open end)


def test_fasta_fetch_matches_oracle_driver():
    fa = os.path.join(TD, "reference_genome.fa")
    fai = O.read_fai(fa + ".fai")
    for (s, e) in [(0, 10), (97, 114), (95, 120), (240, 260), (249, 250), (0, 250)]:
        assert T.fasta_fetch(fa, "chr1", s, e) == O.fasta_fetch(fa, fai, "chr1", s, e)


def test_bgzf_roundtrip_and_framing(tmp_path):
    text = open(os.path.join(GOLD, "expected_output_2.vcf")).read() * 3000  # > one 64 KiB block
    p = tmp_path / "x.vcf.gz"
    T.bgzf_write(str(p), text, flushes=2)
    assert T.bgzf_read(str(p)) == text
    assert gzip.decompress(p.read_bytes()).decode() == text
    raw = p.read_bytes()
    assert raw[-28:] == bytes([0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43, 2, 0, 0x1b, 0, 3, 0,
                               0, 0, 0, 0, 0, 0, 0, 0])
    # the reference fixtures decode with the same reader
    for i in (1, 2):
        assert T.bgzf_read(os.path.join(TD, "expected_output_%d.vcf.gz" % i)) == \
            open(os.path.join(GOLD, "expected_output_%d.vcf" % i)).read()


def test_merge_ranges_matches_oracle():
    rnd = random.Random(2)
    for _ in range(200):
        rs = [(s, s + rnd.randint(0, 30)) for s in (rnd.randint(0, 300) for _ in range(rnd.randint(0, 20)))]
        assert T.merge_ranges(rs) == O.merge_ranges(rs)


def test_synthetic_bcf_roundtrip(tmp_path):
    """tools/synth_dataset.py writes a BGZF BCF2 file; the native reader (f2) returns
    the same records, alleles and raw GT pairs (unphased/phased 0/1 encodings)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path), n_samples=40, n_regions=6, indel_pct=20)
    r = T.BcfReader(d["bcf"])
    assert r.samples == d["samples"]
    got = r.fetch("chr1", 0, 10 ** 9)
    assert len(got) == len(d["records"]) > 0
    for g, w in zip(got, d["records"]):
        assert (g["pos0"], g["rlen"], g["ref"], g["alt"], g["n_alleles"]) == \
            (w["pos0"], w["rlen"], w["alleles"][0], w["alleles"][1], 2)
        assert g["gt"] == w["gt"].astype(int).tolist()


def _want(records, beg, end, sel):
    return [(w["pos0"], w["rlen"], w["alleles"][0], w["alleles"][1], w["gt"][sel].astype(int).tolist())
            for w in records if w["pos0"] < end and w["pos0"] + w["rlen"] > beg]


def test_bcf_stream_sweep_select_and_rewind(tmp_path, monkeypatch):
    """Streaming reader: 1 KiB read chunks (records and BGZF blocks span chunks),
    a sample subset in permuted order, a sweep of overlapping windows with
    nondecreasing beg (the run flow's access pattern), then queries that go
    backwards (rewind); every answer equals a brute-force filter of the records."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import numpy as np
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path), n_samples=70, n_regions=25, indel_pct=25, seed=9)
    monkeypatch.setenv("TFBS_BCF_CHUNK_KB", "1")
    r = T.BcfReader(d["bcf"])
    sel = [5, 3, 69, 0, 41, 41, 12]
    r.select(sel)
    sel = np.asarray(sel)
    got = lambda b, e: [(g["pos0"], g["rlen"], g["ref"], g["alt"], g["gt"]) for g in r.fetch("chr1", b, e)]
    n_hit = 0
    for (s, e) in d["regions"]:
        for b, z in ((s - 40, e + 40), (s - 5, s + 30), (e - 10, e + 200)):
            w = _want(d["records"], b, z, sel)
            n_hit += len(w)
            assert got(b, z) == w
    assert n_hit > 0
    for (s, e) in reversed(d["regions"][:6]):
        assert got(s - 30, e + 30) == _want(d["records"], s - 30, e + 30, sel)
    assert got(0, 10 ** 9) == _want(d["records"], 0, 10 ** 9, sel)


def test_bcf_csi_seek_matches_brute_force(tmp_path, monkeypatch):
    """CSI-indexed fetch (IndexedReader::fetch, haplotype.rs:78-79): the same BCF with
    and without its index answers a query sequence with forward jumps over many
    regions (seek past unread blocks), backward jumps (seek instead of rewind),
    repeated and empty windows identically to a brute-force filter of the records.
    Small read chunks make the forward seeks real."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import shutil

    import numpy as np
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "a"), n_samples=90, n_regions=60, indel_pct=30, seed=4)
    plain = str(tmp_path / "plain.bcf")
    shutil.copy(d["bcf"], plain)
    monkeypatch.setenv("TFBS_BCF_CHUNK_KB", "2")
    ri, rp = T.BcfReader(d["bcf"]), T.BcfReader(plain)
    assert ri.indexed and not rp.indexed
    sel = [7, 1, 88, 40]
    ri.select(sel)
    rp.select(sel)
    sel = np.asarray(sel)
    rnd = random.Random(3)
    regs = d["regions"]
    queries = [(s - 30, e + 30) for (s, e) in regs[::7]]                       # sparse forward sweep
    queries += [(s - 30, e + 30) for (s, e) in reversed(regs[10:20])]          # backwards
    queries += [(0, 500), (10 ** 8, 10 ** 8 + 5), (regs[-1][1] + 100, 10 ** 9)]  # before / after everything
    for _ in range(40):
        a = rnd.randint(0, regs[-1][1] + 500)
        queries.append((a, a + rnd.randint(0, 2000)))
    n_hit = 0
    for b, e in queries:
        want = _want(d["records"], b, e, sel)
        n_hit += len(want)
        for r in (ri, rp):
            got = [(g["pos0"], g["rlen"], g["ref"], g["alt"], g["gt"]) for g in r.fetch("chr1", b, e)]
            assert got == want, (r.indexed, b, e)
    assert n_hit > 50


def test_csi_fixture_index_loads():
    """The reference's own test_data/*.bcf.csi (htslib-written, depth 0) parse and
    give the same records as the sweep (test_bcf_reader_matches_fixture_decoder)."""
    for name in ("genotypes", "genotypes2"):
        r = T.BcfReader(os.path.join(TD, name + ".bcf"))
        assert r.indexed
        want = json.load(open(os.path.join(GOLD, name + ".records.json")))
        for b, e in [(97, 118), (0, 250), (100, 101), (101, 200), (0, 100)]:
            got = [(g["pos0"], g["rlen"]) for g in r.fetch("chr1", b, e)]
            assert got == [(w["pos0"], w["rlen"]) for w in want["records"]
                           if w["pos0"] < e and w["pos0"] + w["rlen"] > b]


def test_bcf_stream_rejects_unsorted(tmp_path):
    """An indexed BCF is position-sorted; the streaming reader fails loudly on
    records that go backwards instead of silently missing them."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import numpy as np
    import struct
    import synth_dataset
    header = ("##fileformat=VCFv4.2\n##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
              "##contig=<ID=chr1,length=1000>\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\n").encode() + b"\0"
    body = bytearray(b"BCF\2\2" + struct.pack("<I", len(header)) + header)
    gt = np.array([[4, 3]], dtype=np.int8)
    for pos in (100, 50):
        body += synth_dataset.bcf_record(0, pos, "A", "C", gt)
    p = str(tmp_path / "unsorted.bcf")
    open(p, "wb").write(synth_dataset.bgzf_blocks(body))
    r = T.BcfReader(p)
    with pytest.raises(Exception, match="not sorted"):
        r.fetch("chr1", 0, 1000)


def _carriers_from_gt(gt):
    """load_diffs (haplotype.rs:16-41) on raw GT pairs: 2 k iff GT[0] = Unphased(1) (4),
    2 k + 1 iff GT[1] = Phased(1) (5); a vector_end (INT32_MIN + 1) in either slot
    makes glen != 2: the ploidy error."""
    ve = -2 ** 31 + 1
    ids, bad = [], False
    for k, (a, b) in enumerate(gt):
        bad |= a == ve or b == ve
        if a == 4:
            ids.append(2 * k)
        if b == 5:
            ids.append(2 * k + 1)
    return ids, bad


@pytest.mark.parametrize("sel", [None, [5, 3, 69, 0, 41, 41, 12]])
def test_bcf_carriers_mode_matches_raw_gt(tmp_path, sel):
    """The run flow's reader mode: carrier ids found while decoding (8 GT bytes at a
    time without a selection) equal load_diffs on the raw GT of the same records --
    carriers at every byte of a word, in the tail, both phasings, haploid / missing
    samples (ploidy status) -- with and without a sample selection."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import struct

    import numpy as np
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "s"), n_samples=70, n_regions=12, indel_pct=25, seed=6)
    # hand-made records: 70 samples (140 GT bytes: 17 words + a 4-byte tail)
    ns = 70
    header = ("##fileformat=VCFv4.2\n##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
              "##contig=<ID=chr1,length=100000>\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" +
              "\t".join("S%d" % i for i in range(ns)) + "\n").encode() + b"\0"
    body = bytearray(b"BCF\2\2" + struct.pack("<I", len(header)) + header)
    rnd = np.random.default_rng(1)
    gts = []
    for pos in range(100, 1300, 100):
        g = np.full((ns, 2), [2, 3], dtype=np.int8)           # 0|0
        k = rnd.choice(ns, size=rnd.integers(0, 12), replace=False)
        g[k, 0] = rnd.choice([4, 5, 2, 3], size=len(k))       # 1/., 1|., 0/., 0|.
        g[k, 1] = rnd.choice([4, 5, 2, 3], size=len(k))
        if pos == 300:
            g[ns - 1, 1] = 5                                  # the last byte of the tail
        if pos == 500:
            g[:4] = [[4, 5]] * 4                              # a whole word of carriers
        if pos == 700:
            g[33, 1] = -127                                   # haploid sample: ploidy error
        if pos == 900:
            g[0, 0] = -127                                    # empty GT
        gts.append(g)
        body += synth_dataset.bcf_record(0, pos, "A", "C", g)
    hand = str(tmp_path / "hand.bcf")
    open(hand, "wb").write(synth_dataset.bgzf_blocks(body))
    n_bad = n_car = 0
    for path in (d["bcf"], hand):
        raw, car = T.BcfReader(path), T.BcfReader(path)
        if sel is not None:
            raw.select(sel)
            car.select(sel)
        car.set_carriers_mode(True)
        for b, e in ((0, 500), (400, 900), (850, 10 ** 9)):
            rr, cc = raw.fetch("chr1", b, e), car.fetch("chr1", b, e)
            assert [(r["pos0"], r["ref"], r["alt"]) for r in rr] == [(c["pos0"], c["ref"], c["alt"]) for c in cc]
            for r, c in zip(rr, cc):
                ids, bad = _carriers_from_gt(r["gt"])
                assert c["carriers"] == ids, (path, r["pos0"])
                assert (c["gt_status"] != 0) == bad, (path, r["pos0"])
                n_bad += bad
                n_car += len(ids)
    assert n_car > 50 and (n_bad > 0 or sel is not None)


@pytest.mark.parametrize("readahead", [0, 1])
@pytest.mark.parametrize("chunk_kb", [None, 1, 7])
def test_bcf_condensed_stream_matches_dense(tmp_path, monkeypatch, chunk_kb, readahead):
    """Carriers mode reads the condensed stream (io.hpp CBlock: per 64-byte line a
    background code -- alternating 2/3 either way round, all 2, all 3 -- plus the
    differing bytes; blocks that are not GT-like kept whole).  Against the dense
    stream (TFBS_BCF_CONDENSED=0) on a file built to hit every case: phased 0|0,
    unphased 0/0 (constant background), both mixed within a line, common variants
    (blocks kept whole), random bytes, vector_end (ploidy), GT payloads spanning
    several BGZF blocks and read chunks, odd-length shared parts (the alternation's
    parity flips between records), multi-allelic records, a sample selection (the
    payload read back) and a CSI seek (the condensed stream restarting mid-file); with
    and without the read-ahead (the next chunk condensed on a background thread, dropped
    by a seek)."""
    monkeypatch.setenv("TFBS_BCF_READAHEAD", str(readahead))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import struct

    import numpy as np
    import synth_dataset
    if chunk_kb:
        monkeypatch.setenv("TFBS_BCF_CHUNK_KB", str(chunk_kb))
    ns = 23000  # 46 000 GT bytes: payloads cross BGZF blocks
    header = ("##fileformat=VCFv4.2\n##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
              "##contig=<ID=chr1,length=1000000>\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" +
              "\t".join("S%d" % i for i in range(ns)) + "\n").encode() + b"\0"
    body = bytearray(b"BCF\2\2" + struct.pack("<I", len(header)) + header)
    rnd = np.random.default_rng(11)
    spans = []
    for j, pos in enumerate(range(100, 100 + 40 * 3001, 3001)):
        kind = j % 8
        g = np.full((ns, 2), [2, 3], dtype=np.int8)                       # 0|0
        if kind == 1:
            g[:] = 2                                                      # 0/0 0/0: constant 2
        elif kind == 2:
            g[: ns // 2] = 2                                              # both backgrounds in one record
            g[ns // 3: ns // 3 + 5] = [[3, 3]]                            # and all-3 runs
        elif kind == 3:
            k = rnd.random(ns) < 0.3                                      # a common variant: kept blocks
            g[k, 0] = 4
        elif kind == 4:
            g[:] = rnd.integers(-128, 128, size=(ns, 2))                  # noise
        f = rnd.random(ns) < 0.01
        g[f, 0] = rnd.choice([4, 5, 2, 3], size=f.sum())
        g[f, 1] = rnd.choice([4, 5, 2, 3], size=f.sum())
        if kind == 5:
            g[rnd.integers(ns), rnd.integers(2)] = -127                   # vector_end
        ref, alt = ("A", "C") if kind != 6 else ("ACG", "A")
        if kind == 7:
            ref, alt = "AT", "A"                                          # odd-length alleles: parity flips
        u0 = len(body)
        body += synth_dataset.bcf_record(0, pos, ref, alt + "T" * (j % 3), g)
        spans.append((pos, len(ref), u0, len(body)))
    path = str(tmp_path / "mix.bcf")
    offs = []
    open(path, "wb").write(synth_dataset.bgzf_blocks(bytes(body), offs))
    open(path + ".csi", "wb").write(synth_dataset.csi_index(spans, offs, 1000000))

    def read(condensed, sel=None, queries=((0, 10 ** 9),)):
        monkeypatch.setenv("TFBS_BCF_CONDENSED", "1" if condensed else "0")
        r = T.BcfReader(path)
        if sel is not None:
            r.select(sel)
        r.set_carriers_mode(True)
        return [[(c["pos0"], c["ref"], c["alt"], c["carriers"], c["gt_status"]) for c in r.fetch("chr1", b, e)]
                for b, e in queries]

    qs = ((0, 500), (450, 9000), (50000, 60000), (90000, 91000), (20000, 33000), (100000, 10 ** 9))
    for sel in (None, [5, 3, 22999, 0, 41, 41, 12000]):
        want, got = read(False, sel, qs), read(True, sel, qs)
        assert got == want
        assert sum(len(q) for q in want) > 12
        assert sum(len(c[3]) for q in want for c in q) > (1000 if sel is None else 0)
        assert any(c[4] != 0 for q in want for c in q) or sel is not None


def test_inflate_raw_matches_zlib():
    """tfbs_inflate_raw (the BCF reader's DEFLATE decoder, inflate.cpp) == zlib on raw
    streams of every block type (stored, fixed, dynamic), every zlib level and strategy,
    sizes around its copy steps, short periods (the GT columns' 2-byte runs) and random
    bytes; truncated or corrupted streams fail or decode, never overrun."""
    import ctypes as C
    import random
    import zlib

    L = T.lib()

    def fast(comp, n):
        out = C.create_string_buffer(max(n, 1) + 16)
        return L.tfbs_inflate_raw(comp, len(comp), out, n), out.raw[:n]

    rnd = random.Random(7)
    checked = 0
    for trial in range(600):
        kind = trial % 6
        n = rnd.choice([0, 1, 2, 7, 8, 9, 15, 16, 17, 63, 64, 65, 1000, 4096, 20000, 65280])
        if kind == 0:
            data = bytes(rnd.randrange(256) for _ in range(n))
        elif kind == 1:
            data = bytes(rnd.choice(b"ACGT") for _ in range(n))
        elif kind == 2:
            data = (b"\x02\x03" * (n // 2 + 1))[:n]
        elif kind == 3:
            d = bytearray((b"\x02\x03" * (n // 2 + 1))[:n])
            for _ in range(n // 50 + 1):
                if n:
                    d[rnd.randrange(n)] = rnd.choice([4, 5])
            data = bytes(d)
        elif kind == 4:
            data = bytes(rnd.randrange(3) for _ in range(n))
        else:
            per = rnd.randint(1, 40)
            pat = bytes(rnd.randrange(256) for _ in range(per))
            data = (pat * (n // per + 1))[:n]
        for level in (0, 1, 6, 9):
            for strat in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE):
                co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strat)
                comp = co.compress(data) + co.flush()
                rc, out = fast(comp, len(data))
                assert rc == 0 and out == data, (trial, kind, n, level, strat)
                checked += 1
                if trial % 20 == 0 and len(comp) > 4:
                    rc, out = fast(comp[:len(comp) // 2], len(data))
                    assert rc != 0 or out == data
                    bad = bytearray(comp)
                    bad[len(bad) // 2] ^= 0x55
                    fast(bytes(bad), len(data))
    assert checked == 600 * 16


def _dynamic_block(lit_lens, dist_lens, symbols):
    """A raw DEFLATE stream of one final dynamic block with the given literal/length and
    distance code lengths (written one by one through a complete code-length code:
    lengths 0 -> '0', 1 -> '10', 2 -> '11') and the literal symbols (< 256) then EOB."""
    bits = []

    def put(v, n):  # LSB first
        bits.extend((v >> i) & 1 for i in range(n))

    def code(c, n):  # Huffman codes MSB first
        bits.extend((c >> (n - 1 - i)) & 1 for i in range(n))

    def canon(lens):  # RFC 1951 3.2.2
        count = [sum(1 for x in lens if x == ln) if ln else 0 for ln in range(16)]
        codes, nxt, c = {}, {}, 0
        for ln in range(1, 16):
            c = (c + count[ln - 1]) << 1
            nxt[ln] = c
        for s, ln in enumerate(lens):
            if ln:
                codes[s] = (nxt[ln], ln)
                nxt[ln] += 1
        return codes

    put(1, 1)
    put(2, 2)
    put(len(lit_lens) - 257, 5)
    put(len(dist_lens) - 1, 5)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl = [0] * 19
    cl[0], cl[1], cl[2] = 1, 2, 2
    put(18 - 4, 4)
    for k in range(18):
        put(cl[order[k]], 3)
    cc = canon(cl)
    for ln in list(lit_lens) + list(dist_lens):
        code(*cc[ln])
    lc = canon(lit_lens)
    for s in list(symbols) + [256]:
        code(*lc[s])
    while len(bits) % 8:
        bits.append(0)
    return bytes(sum(bits[i + j] << j for j in range(8)) for i in range(0, len(bits), 8))


def test_inflate_raw_rejects_incomplete_codes():
    """A dynamic block whose literal/length code is incomplete (two codes of length 2)
    is refused, as zlib refuses it ('invalid literal/lengths set'), even though every
    symbol the stream uses has a code and the output length matches; a single distance
    code of length 1 (zlib's allowed incomplete case) and complete codes still decode."""
    import ctypes as C
    import zlib

    L = T.lib()

    def fast(comp, n):
        out = C.create_string_buffer(max(n, 1) + 16)
        return L.tfbs_inflate_raw(comp, len(comp), out, n), out.raw[:n]

    lit = [0] * 257
    lit[65], lit[256] = 2, 2  # incomplete: 2 of 4 codes of length 2
    bad = _dynamic_block(lit, [1], [65] * 4)
    with pytest.raises(zlib.error):
        zlib.decompressobj(-15).decompress(bad)
    rc, _ = fast(bad, 4)
    assert rc != 0
    lit[66], lit[67] = 2, 2  # complete; the one distance code of length 1 stays allowed
    good = _dynamic_block(lit, [1], [65, 66, 67, 65])
    assert zlib.decompressobj(-15).decompress(good) == b"ABCA"
    rc, out = fast(good, 4)
    assert rc == 0 and out == b"ABCA"
