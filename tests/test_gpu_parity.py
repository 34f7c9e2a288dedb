"""GPU parity: the HIP scan through the C ABI against the CPU oracle.

Integer work, so every comparison is bit-exact: match lists, per-sample L/R
count vectors per (bed, inner range, pattern_id) key, and the VCF row text.
"""
import json
import os
import random

import pytest

import oracle_py as O
from helpers import GOLD, TD, T, build_batch, make_regions_synth, run_oracle, run_product, synth_patterns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if T.device_count() == 0:
        pytest.fail("gpu test without a visible HIP device")


def _hap(s, start=0):
    return [(c, start + i) for i, c in enumerate(s)]


# ------------------------------------------------------------ pattern.rs:268-301 on the GPU
def test_matches_reference_vectors():
    c, g = T.Weight(0, 1000, 0, 0), T.Weight(0, 0, 1000, 0)
    pwm = T.Pattern.PWM([c, g], "pwm", 5, 1500)
    m = T.matches(pwm, [("A", 10), ("C", 11), ("G", 12), ("T", 13)], ())
    assert m == [T.Match(T.Range(11, 12), 5, ())]

    w = [T.Weight(0, 0, 100, 0), T.Weight(100, 0, 0, 0), T.Weight(0, 0, 0, 100), T.Weight(100, 0, 0, 0),
         T.Weight(100, 0, 0, 0)]
    pad = [("N", 0), ("G", 1), ("A", 2), ("T", 3), ("A", 4), ("A", 5), ("N", 6)]
    nopad = pad[1:-1]
    p499 = T.Pattern.PWM(w, "Example", 123, 499)
    p500 = T.Pattern.PWM(w, "Example", 123, 500)
    assert len(T.matches(p499, pad)) == 1 and len(T.matches(p499, nopad)) == 1
    assert len(T.matches(p500, pad)) == 0 and len(T.matches(p500, nopad)) == 0
    assert T.matches(T.Pattern.OtherPattern("x", 1), pad) == []


def _rand_pwm(rnd, L, scale=1000):
    return [[rnd.randint(-3 * scale, scale) for _ in range(4)] + [0] for _ in range(L)]


@pytest.mark.parametrize("mfma", ["0", "1"])
def test_matches_fuzz_vs_oracle(monkeypatch, mfma):
    """Random PWMs of length 1..40 (fast LUT path and the >32 generic path, or the
    matrix-core path), haplotypes up to 700 bases (several 256-window passes), N bases,
    non-affine positions."""
    monkeypatch.setenv("TFBS_MFMA", mfma)
    rnd = random.Random(1)
    pats = []
    for i in range(48):
        L = rnd.choice([1, 2, 3, 4, 5, 7, 8, 11, 15, 16, 17, 24, 29, 30, 31, 32, 33, 36, 40])
        w = _rand_pwm(rnd, L)
        best = sum(max(r[:4]) for r in w)
        worst = sum(min(r[:4]) for r in w)
        ms = rnd.randint(worst, best) if rnd.random() < 0.8 else best - rnd.randint(0, 3000)
        pats.append(T.Pattern.PWM([T.Weight(*r[:4]) for r in w], "P%d" % i, i // 2, ms, i % 2))
    pats.append(T.Pattern.OtherPattern("other", 99))
    sc = T.Scanner(pats)
    try:
        for trial in range(12):
            n = rnd.choice([0, 1, 5, 31, 64, 65, 200, 257, 513, 700])
            seq = "".join(rnd.choice("ACGTACGTACGTN" if trial % 3 == 0 else "ACGT") for _ in range(n))
            pos = []
            p = 1000
            for i in range(n):  # non-decreasing positions with repeats and skips
                pos.append(p)
                p += rnd.choice([0, 1, 1, 1, 3]) if trial % 2 else 1
            hap = list(zip(seq, pos))
            got = sc.matches_all(hap)
            for i, p_ in enumerate(pats):
                w5 = [wt.acgtn for wt in p_.weights]
                want = O.matches(w5, p_.min_score, hap, kind=p_.kind)
                assert got[i] == want, (trial, i, len(w5))
    finally:
        sc.close()


def _scores(w4, seq):
    """Window scores of pattern.rs:125-135 (N = 0), i32 wrapping."""
    L = len(w4)
    out = []
    for i in range(len(seq) - L + 1):
        s = 0
        for j in range(L):
            c = "ACGTN".index(seq[i + j])
            s += w4[j][c] if c < 4 else 0
        out.append(((s + 2**31) % 2**32) - 2**31)
    return out


def octet_boundary_patterns(rnd, seq):
    """PWMs placed on the edges of the 16-bit octet path (plan.cpp): thresholds tied
    with / one below a real window score, biased thresholds of exactly -32768 and
    -32769, block ranges of 32767 and 32768, i32-wrapping weights, thresholds above
    the best score."""
    pats = []

    def add(w4, ms):
        pats.append(T.Pattern.PWM([T.Weight(*r) for r in w4], "B%d" % len(pats), len(pats) // 2, ms,
                                  len(pats) % 2))

    for L in (1, 4, 9, 16, 23, 32):
        w4 = [[rnd.randint(-2100, 0) for _ in range(4)] for _ in range(L)]
        best = sum(max(r) for r in w4)
        sc = sorted(_scores(w4, seq.replace("N", "A")))
        top = sc[-1 - rnd.randint(0, 5)]
        add(w4, top)          # tie: never a hit for that window
        add(w4, top - 1)      # one below: a hit
        add(w4, best - 32768)  # biased threshold exactly -32768 (octet)
        add(w4, best - 32769)  # -32769: quad
        add(w4, best)          # nothing can exceed the best score
        add(w4, best + 5)
    # a block whose range is exactly 32767 (octet) / 32768 (quad)
    for span in (32767, 32768):
        w4 = [[0, -span, 0, 0]] + [[0, 0, 0, 0]] * 3 + [[rnd.randint(-50, 50) for _ in range(4)] for _ in range(4)]
        add(w4, -span + 10)
        add(w4, 20)
    # i32 wrap (pattern.rs sums in i32): quad path must wrap like the reference
    w4 = [[2**30, 2**30 - 7, -2**31, 5] for _ in range(6)]
    add(w4, 0)
    add(w4, -2**31)
    return pats


@pytest.mark.parametrize("mfma", ["0", "1"])
def test_octet_boundaries_vs_oracle(monkeypatch, mfma):
    """With TFBS_MFMA=1 the same patterns split between the matrix-core path (weights
    within the two int8 digits) and the LUT path (the rest)."""
    monkeypatch.setenv("TFBS_MFMA", mfma)
    rnd = random.Random(5)
    base = "".join(rnd.choice("ACGT") for _ in range(700))
    pats = octet_boundary_patterns(rnd, base)
    st = T.PatternSet.from_patterns(pats).plan_stats(mfma=mfma == "1")
    if mfma == "1":
        assert st["n_mfma_strands"] > 0 and st["n_quad_strands"] > 0, st
    else:
        assert st["n_octet_strands"] > 0 and st["n_quad_strands"] > 0, st
    sc = T.Scanner(pats)
    try:
        for trial, seq in enumerate([base, base[:300] + "N" + base[301:520] + "NN" + base[522:], base[:33], ""]):
            hap = _hap(seq, 5000)
            got = sc.matches_all(hap)
            for i, p_ in enumerate(pats):
                w5 = [wt.acgtn for wt in p_.weights]
                assert got[i] == O.matches(w5, p_.min_score, hap, kind=p_.kind), (trial, i)
    finally:
        sc.close()


def test_mfma_split_edges_vs_oracle(monkeypatch):
    """The matrix-core path's FP6 upper bound (mfma.cpp): weight spans from 1 to 2^20
    (scales 1 .. ~10^5, every FP6 grid range), all-negative and all-positive columns,
    thresholds tied with / one below real window scores (the bound must never drop an
    exact hit), thresholds below every score (every tile fires), N bases (one-hot zero,
    bound term c_j >= 0), and a strand whose sum could wrap i32 (LUT path)."""
    monkeypatch.setenv("TFBS_MFMA", "1")
    rnd = random.Random(11)
    base = "".join(rnd.choice("ACGT") for _ in range(600))
    seqs = [base, base[:100] + "N" * 3 + base[103:400] + "N" + base[401:], base[:40], ""]
    pats = []

    def add(w4, ms):
        pats.append(T.Pattern.PWM([T.Weight(*r) for r in w4], "S%d" % len(pats), len(pats) // 2, ms,
                                  len(pats) % 2))

    for L in (1, 3, 8, 15, 16, 17, 24, 31, 32):
        for mx in (1, 2, 7, 8, 15, 16, 127, 1000, 4400, 32385, 1 << 20):
            kind = rnd.randrange(3)  # mixed signs, all negative, all positive
            lo, hi = (-mx, mx) if kind == 0 else ((-mx, -1) if kind == 1 else (1, mx))
            if lo > hi:
                lo, hi = hi, lo
            w4 = [[rnd.randint(lo, hi) for _ in range(4)] for _ in range(L)]
            sc = sorted(_scores(w4, base))
            top = sc[-1 - rnd.randint(0, 3)] if sc else 0
            add(w4, top)
            add(w4, top - 1)
            if mx in (4400, 1 << 20):
                add(w4, sc[0] - 1 if sc else -1)  # every window hits
    w4 = [[2**30, 0, -5, 7]] * 2 + [[rnd.randint(-100, 100) for _ in range(4)] for _ in range(6)]
    pats.append(T.Pattern.PWM([T.Weight(*r) for r in w4], "LUT", 9999, sorted(_scores(w4, base))[-2], 0))
    st = T.PatternSet.from_patterns(pats).plan_stats(mfma=True)
    assert st["n_mfma_strands"] == len(pats) - 1, st
    sc = T.Scanner(pats)
    try:
        for trial, seq in enumerate(seqs):
            hap = _hap(seq, 7000)
            got = sc.matches_all(hap)
            for i, p_ in enumerate(pats):
                w5 = [wt.acgtn for wt in p_.weights]
                assert got[i] == O.matches(w5, p_.min_score, hap, kind=p_.kind), (trial, i)
    finally:
        sc.close()


# ------------------------------------------------------------ main.rs:548-568 through the product
def _c1(bcf_json, beds_files, samples_file=True):
    rec = json.load(open(os.path.join(GOLD, bcf_json)))
    ps = T.parse_pwm_files(os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["ACGT"])
    merged, beds = O.load_peak_files([os.path.join(TD, b) for b in beds_files], "chr1", 0)
    names = rec["samples"]
    want = [l.strip() for l in open(os.path.join(TD, "samples")) if len(l.rstrip("\n")) > 1]
    sel = [i for i, s in enumerate(names) if s in set(want)] if samples_file else list(range(len(names)))
    fai = O.read_fai(os.path.join(TD, "reference_genome.fa.fai"))
    b = T.RegionBatch(ps, len(sel))
    for name, _ in beds:
        b.add_bed(name)
    for (s, e) in merged:
        es, ee = b.ext(s, e)
        ref = O.fasta_fetch(os.path.join(TD, "reference_genome.fa"), fai, "chr1", es, ee + 1)
        b.begin(s, e, ref)
        for bi, a, z in T.select_inner_peaks((s, e), beds):
            b.add_inner(bi, a, z)
        for r in rec["records"]:
            if r["chrom"] == "chr1" and r["pos0"] < ee + 1 and r["pos0"] + r["rlen"] > es:
                b.add_record_gt(r["pos0"], len(r["alleles"]), r["alleles"][0], r["alleles"][1],
                                [r["gt"][i] for i in sel])
        b.end()
    sc = T.Scanner(ps)
    b.scan(sc)
    rows, _ = b.rows("chr1")
    sc.close()
    header = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT" + "".join("\t" + names[i] for i in sel) + "\n"
    return header + rows


def test_integration_no_polymorphism():
    assert _c1("genotypes.records.json", ["regions1.bed", "regions2.bed"]) == \
        open(os.path.join(GOLD, "expected_output_1.vcf")).read()


def test_integration_one_polymorphism():
    assert _c1("genotypes2.records.json", ["regions1.bed", "regions2.bed"]) == \
        open(os.path.join(GOLD, "expected_output_2.vcf")).read()


@pytest.mark.parametrize("bcf,expected", [("genotypes.bcf", 1), ("genotypes2.bcf", 2)])
def test_run_end_to_end_matches_reference_outputs(tmp_path, bcf, expected):
    """main.rs:548-568 through the native flow (BCF reader, FASTA, BED merge, GPU scan,
    BGZF writer): decompressed text identical to the reference's expected_output_N."""
    out = tmp_path / "out.vcf.gz"
    T.run("chr1", os.path.join(TD, bcf), [os.path.join(TD, "regions1.bed"), os.path.join(TD, "regions2.bed")],
          os.path.join(TD, "reference_genome.fa"), os.path.join(TD, "samples"),
          os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["ACGT"], str(out), False, False, 0, 1, 0, False)
    want = open(os.path.join(GOLD, "expected_output_%d.vcf" % expected)).read()
    assert T.bgzf_read(str(out)) == want
    assert not os.path.exists(str(out) + ".part")


def test_cli_binary(tmp_path):
    import subprocess
    exe = os.path.join(os.path.dirname(T.__file__), "bin", "find-tfbs-amd")
    out = tmp_path / "cli.vcf.gz"
    r = subprocess.run([exe, "--chromosome", "chr1", "--input", os.path.join(TD, "genotypes2.bcf"),
                        "--bed", os.path.join(TD, "regions1.bed") + "," + os.path.join(TD, "regions2.bed"),
                        "--reference", os.path.join(TD, "reference_genome.fa"), "--samples",
                        os.path.join(TD, "samples"), "--pwm_file", os.path.join(TD, "pwm_definitions.txt"),
                        "--pwm_threshold_directory", TD, "--pwm_threshold", "0.0001", "--pwm_names", "ACGT",
                        "--output", str(out), "--threads", "2"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert T.bgzf_read(str(out)) == open(os.path.join(GOLD, "expected_output_2.vcf")).read()
    # a missing bed file fails like bed.rs:34's panic (non-zero exit)
    r2 = subprocess.run([exe, "--chromosome", "chr1", "--input", os.path.join(TD, "genotypes2.bcf"), "--bed",
                         "/nonexistent.bed", "--reference", os.path.join(TD, "reference_genome.fa"), "--pwm_file",
                         os.path.join(TD, "pwm_definitions.txt"), "--pwm_threshold_directory", TD,
                         "--pwm_threshold", "0.0001", "--pwm_names", "ACGT", "--output", str(tmp_path / "y.gz")],
                        capture_output=True, text=True, timeout=120)
    assert r2.returncode != 0


def test_config1_regions1_only():
    # BASELINE.json configs[0]: genotypes2.bcf + regions1.bed + ACGT -> the same single row
    got = _c1("genotypes2.records.json", ["regions1.bed"])
    assert got.splitlines()[1:] == open(os.path.join(GOLD, "expected_output_2.vcf")).read().splitlines()[1:]


# ------------------------------------------------------------ synthetic regions vs the oracle
def _compare(ps, n_samples, beds, regions, min_maf=0):
    okeys, orows, _ = run_oracle(ps, n_samples, beds, regions, min_maf=min_maf)
    sc = T.Scanner(ps)
    try:
        # dense download, the device key reduction and the device per-sample encoding
        # (f1) the run flow uses
        for reduce, encode in ((False, False), (True, False), (True, True)):
            pkeys, prows, b = run_product(sc, ps, n_samples, beds, regions, min_maf=min_maf, reduce=reduce,
                                          encode=encode)
            assert len(okeys) == len(pkeys)
            for i, (a, z) in enumerate(zip(okeys, pkeys)):
                assert a.keys() == z.keys(), (reduce, i)
                for k in a:
                    assert a[k] == z[k], (reduce, i, k)
            assert prows == orows, (reduce, encode)
    finally:
        sc.close()
    return b


@pytest.mark.parametrize("mfma", ["0", "1"])
@pytest.mark.parametrize("config,indel,n_samples,n_regions", [(2, 0, 150, 16), (3, 0, 60, 6), (5, 30, 80, 10)])
def test_synthetic_regions_vs_oracle(tmp_path, monkeypatch, config, indel, n_samples, n_regions, mfma):
    """Both scan paths: the LUT kernels and (TFBS_MFMA=1) the int8 matrix-core kernel."""
    monkeypatch.setenv("TFBS_MFMA", mfma)
    ps, _ = synth_patterns(tmp_path, 12 if config != 3 else 40, config, 100 + config, thr=1e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(7 + config, 0, n_regions, n_samples, ps.max_length, indel)
    b = _compare(ps, n_samples, beds, regions)
    assert b.num_haplotypes > n_regions


@pytest.mark.parametrize("thr", [0.5, 0.05])
def test_dense_hits_vs_oracle(tmp_path, monkeypatch, thr):
    """Loose thresholds (p 0.5 / 0.05: most / many windows hit) through the count path:
    the matrix-core kernel's candidate queues fill and drain mid-haplotype many times, and
    the workgroup's pooled final drain carries hundreds of entries per wave."""
    monkeypatch.setenv("TFBS_MFMA", "1")
    ps, _ = synth_patterns(tmp_path, 6, 3, 61, thr=thr)
    n_regions = 4
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(17, 0, n_regions, 40, ps.max_length, 10)
    b = _compare(ps, 40, beds, regions)
    assert b.num_haplotypes > n_regions


@pytest.mark.parametrize("thr", [1e-3, 0.05])
def test_reuse_indel_haplotypes_without_own_runs_vs_oracle(tmp_path, monkeypatch, thr):
    """Reference-window reuse across indels when a haplotype's own columns hold no diff
    run but the reference's do: a deletion running to the window's last base (the
    haplotype is a prefix of the reference: one segment, no run in its columns, the
    reference's columns past it a run to the end), alone or with SNVs carried by other
    haplotypes, one region per case and several in one batch (so a missing run list
    cannot borrow a neighbour's).  Found by the C5 full-size golden digests: the
    haplotype's reference-column runs were not stored when its own list was empty."""
    monkeypatch.setenv("TFBS_MFMA", "1")
    ps, _ = synth_patterns(tmp_path, 12, 5, 83, thr=thr)
    n_samples = 40
    H = 2 * n_samples
    rnd = random.Random(9)
    regions, ranges = [], []
    for j in range(8):
        r = T.SynthRegion(41, j, n_samples, ps.max_length, 0)
        s, e = r.merged
        es = s - ps.max_length + 1
        ref = r.ref
        recs = []
        q = len(ref) - 2 - j  # the deletion's first base; it runs to the last base
        dele = list(range(0, H, 3))
        recs.append(("car", es + q, ref[q:], ref[q], dele))
        if j % 2:  # SNVs carried by other haplotypes (their own runs come first in the run array)
            for t in (5, 40, 77):
                alt = "ACGT"[("ACGT".index(ref[t]) + 1) % 4]
                recs.append(("car", es + t, ref[t], alt, sorted(rnd.sample([h for h in range(H) if h % 3], 9))))
        if j == 4:  # an insertion at the end too
            recs.append(("car", es + len(ref) - 1, ref[-1], ref[-1] + "AC", list(range(1, H, 7))))
        recs.sort(key=lambda x: x[1])
        regions.append({"merged": (s, e), "ref": ref, "records": recs})
        ranges.append((s, e))
    beds = [("synthetic.bed", ranges)]
    b = _compare(ps, n_samples, beds, regions)
    assert b.num_scan_windows < b.num_windows
    for k in range(len(regions)):  # one region per batch
        _compare(ps, n_samples, [("synthetic.bed", [ranges[k]])], [regions[k]])


@pytest.mark.parametrize("thr,fast_max_u,cor", [(1e-3, None, None), (0.05, None, None), (1e-3, "0", None),
                                                (0.05, "40", None), (0.05, None, ("0", None)),
                                                (1e-3, None, ("16", "200"))])
def test_reference_window_reuse_vs_oracle(tmp_path, monkeypatch, thr, fast_max_u, cor):
    """Reference-window reuse (HAP_DEDUP, ref_fixup_kernel) on its edge cases, against
    the oracle: an SNV every haplotype carries (no reference group: the helper copy of
    the reference supplies the hits), N runs in the reference, haplotypes with indels
    (reused before the first indel, scanned after it), 40 nested inner ranges (the fix-up's path past 32 ranges) and
    p = 0.05 thresholds (over 64 reference hits per region: the overflow list; with
    small candidate lists, the candidate overflow list and its regrowth).  fast_max_u:
    regions of more distinct haplotypes than that leave key_fast_kernel for the list
    pass of key_asm_kernel (0: every region; 40: some -- both kernels in one reduction);
    the region with 40 inner ranges always takes that pass.  cor: key_fast_kernel's
    corrections in its global arena instead of LDS (every region -- its counter
    chunks too --, or past 16 entries with an arena of 200 that fills: those regions
    go to key_asm_kernel)."""
    monkeypatch.setenv("TFBS_MFMA", "1")
    if fast_max_u is not None:
        monkeypatch.setenv("TFBS_KEY_FAST_MAXU", fast_max_u)
    if cor is not None:
        monkeypatch.setenv("TFBS_KEY_COR_LDS", cor[0])
        if cor[1] is not None:
            monkeypatch.setenv("TFBS_KEY_COR_CAP", cor[1])
    ps, _ = synth_patterns(tmp_path, 10, 3, 71, thr=thr)
    n_samples, n_regions = 60, 6
    H = 2 * n_samples
    rnd = random.Random(5)
    regions, ranges = [], []
    for j in range(n_regions):
        r = T.SynthRegion(31, j, n_samples, ps.max_length, 20 if j == 3 else 0)
        s, e = r.merged
        es = s - ps.max_length + 1
        ref = list(r.ref)
        if j == 2:  # N runs away from the variant sites
            for q in range(10, 18):
                ref[q] = "N"
        ref = "".join(ref)
        recs = [("car", pos, rf, alt, car) for pos, rf, alt, car in r.records
                if j != 2 or not any(10 <= pos - es + t < 18 for t in range(len(rf)))]
        if j in (0, 4):  # every haplotype carries one SNV: no reference group
            q = len(ref) // 2
            while ref[q] == "N" or any(rec[1] == es + q for rec in recs):
                q += 1
            recs.append(("car", es + q, ref[q], "ACGT"[("ACGT".index(ref[q]) + 1) % 4], list(range(H))))
        regions.append({"merged": (s, e), "ref": ref, "records": recs})
        ranges.append((s, e))
        if j == 5:  # 40 nested inner ranges sharing the merged start
            ranges.extend((s, s + 1 + k) for k in range(39))
    beds = [("synthetic.bed", ranges)]
    b = _compare(ps, n_samples, beds, regions)
    assert b.num_scan_windows < b.num_windows
    monkeypatch.setenv("TFBS_DEDUP", "0")  # the same job scanning every window
    b0 = _compare(ps, n_samples, beds, regions)
    assert b0.num_scan_windows > b.num_scan_windows
    if thr > 0.01:
        # 8 list entries per wave: candidates spill to the overflow list, which
        # itself overflows (16 entries): the scan grows it and runs again
        monkeypatch.setenv("TFBS_DEDUP", "1")
        monkeypatch.setenv("TFBS_CAND_CAP", "64")
        monkeypatch.setenv("TFBS_CAND_OVER_CAP", "16")
        # and varying-key lists of 8 keys / 32 counts: the key reduction grows them and reruns
        monkeypatch.setenv("TFBS_VAR_CAP", "8")
        _compare(ps, n_samples, beds, regions)


def test_long_region_vs_oracle(tmp_path, monkeypatch):
    """A 33 kb merged region next to a short one, 40 samples, 60 SNVs each with
    random carriers, against the oracle: a count of the long region could pass 2^16,
    so the key assembly keeps its LDS counters u32 there (packed u16 in the other)."""
    monkeypatch.setenv("TFBS_MFMA", "1")
    ps, _ = synth_patterns(tmp_path, 6, 3, 91, thr=1e-3)
    lmax = ps.max_length
    rnd = random.Random(7)
    n_samples = 40
    H = 2 * n_samples
    regions, ranges = [], []
    for (s, e) in ((5000, 5000 + 33000), (60000, 60200)):
        es = s - lmax + 1
        n = e - s + 2 * lmax - 1
        ref = "".join(rnd.choice("ACGT") for _ in range(n))
        recs = []
        for q in sorted(rnd.sample(range(n), 60)):
            alt = rnd.choice([c for c in "ACGT" if c != ref[q]])
            recs.append(("car", es + q, ref[q], alt, sorted(rnd.sample(range(H), rnd.randint(1, 12)))))
        regions.append({"merged": (s, e), "ref": ref, "records": recs})
        ranges.append((s, e))
    b = _compare(ps, n_samples, [("synthetic.bed", ranges)], regions)
    assert b.num_haplotypes > 20


def test_multi_bed_duplicate_and_nested_inner_peaks(tmp_path):
    """Several bed sources, duplicate ranges (double count), a range that is never selected
    (strictly inside a 3-way merge, bed.rs:77/89), empty ranges, Ns in the reference."""
    ps, _ = synth_patterns(tmp_path, 8, 2, 55, thr=2e-3)
    n = 40
    base = T.SynthRegion(3, 1, n, ps.max_length)
    ref = list(base.ref)
    for i in range(30, 36):
        ref[i] = "N"
    ref = "".join(ref)
    s0 = base.merged[0]
    beds = [("a.bed", [(s0, s0 + 80), (s0 + 80, s0 + 120), (s0, s0 + 80)]),
            ("b.bed", [(s0 + 120, s0 + 200), (s0 + 90, s0 + 100), (s0 + 130, s0 + 129)]),
            ("c.bed", [(s0 + 60, s0 + 70)])]
    merged = O.merge_ranges([r for _, rs in beds for r in rs])
    assert merged[0] == (s0, s0 + 200)
    recs = [("car", p, r, a, c) for p, r, a, c in base.records if not (base.ext_start + 30 <= p < base.ext_start + 36)]
    regions = [{"merged": merged[0], "ref": ref, "records": recs}]
    _compare(ps, n, beds, regions)


def test_gt_decoding_and_reference_collisions(tmp_path):
    """Raw GT ints (unphased/phased/missing), multi-allelic records, a REF allele
    longer than the window, and two groups that patch to the same sequence."""
    ps, _ = synth_patterns(tmp_path, 6, 2, 77, thr=5e-3)
    rnd = random.Random(4)
    n = 30
    base = T.SynthRegion(5, 2, n, ps.max_length)
    es = base.ext_start
    ref = base.ref
    recs = []
    VE = -2147483647
    gt_choices = [(4, 3), (2, 5), (4, 5), (4, 4), (5, 5), (2, 3), (0, 1), (2, 2)]
    for k, (off, alt) in enumerate([(20, None), (40, None), (41, None), (60, None)]):
        p = es + off
        r0 = ref[off]
        a = rnd.choice([c for c in "ACGT" if c != r0])
        gts = [list(rnd.choice(gt_choices)) for _ in range(n)]
        recs.append(("gt", p, 2, r0, a, gts))
    # multi-allelic: counted as a variant, no diffs
    recs.append(("gt", es + 50, 3, ref[50], "A", [[VE, VE]] * n))
    # a deletion starting before the window (filtered by patch_haplotype, haplotype.rs:95)
    recs.append(("gt", es - 2, 2, "AC", "A", [[4, 3]] * 5 + [[2, 3]] * (n - 5)))
    # the same SNV twice at one position: groups {d} and {d, d} differ but ...
    r0 = ref[80]
    a = "A" if r0 != "A" else "C"
    recs.append(("gt", es + 80, 2, r0, a, [[4, 3]] * 10 + [[2, 3]] * (n - 10)))
    recs.append(("gt", es + 80, 2, r0, a, [[4, 3]] * 3 + [[2, 3]] * (n - 3)))
    regions = [{"merged": base.merged, "ref": ref, "records": recs}]
    beds = [("x.bed", [base.merged])]
    _compare(ps, n, beds, regions)


def test_min_maf_filter(tmp_path):
    ps, _ = synth_patterns(tmp_path, 10, 2, 8, thr=1e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(6)])]
    regions = make_regions_synth(21, 0, 6, 100, ps.max_length)
    _compare(ps, 100, beds, regions, min_maf=3)


def test_large_scan_counts_are_invariant_to_tiling(tmp_path, monkeypatch):
    """Size-independent property at a larger size: counts do not depend on the LDS
    tile size or on haplotypes-per-workgroup (the kernels' only tunables)."""
    ps, _ = synth_patterns(tmp_path, 60, 3, 9)
    b = T.RegionBatch(ps, 2000)
    b.synth_fill(13, 0, 200)
    res = []
    for mfma, tb, hpb in [("0", "32", "64"), ("0", "8", "4"), ("0", "64", "16"), ("1", "12", "5"),
                          ("1", "64", "64"), ("1", "28", "32")]:
        monkeypatch.setenv("TFBS_MFMA", mfma)
        monkeypatch.setenv("TFBS_TILE_BLOCKS", tb)
        monkeypatch.setenv("TFBS_HAPS_PER_BLOCK", hpb)
        monkeypatch.setenv("TFBS_MFMA_LDS_KB", tb)
        monkeypatch.setenv("TFBS_MFMA_HAPS_PER_BLOCK", hpb)
        sc = T.Scanner(ps)
        b.scan(sc)
        res.append([b.keys(r) for r in (0, 57, 199)])
        rows_dense, _ = b.rows("chr1")
        b.scan(sc, upload=False, reduce=True)  # device key reduction gives the same keys and rows
        assert [b.keys(r) for r in (0, 57, 199)] == res[-1]
        assert b.rows("chr1")[0] == rows_dense
        sc.close()
    assert all(r == res[0] for r in res)
    assert rows_dense.count("\n") > 0


@pytest.mark.parametrize("n", [120, 300])
def test_many_variant_regions_vs_oracle(tmp_path, n):
    """Regions with 64 and ~90 distinct diffs: both haplotype-grouping paths of the
    host (64-bit diff masks / sorted diff lists) through the GPU scan vs the oracle;
    at 300 samples the regions have > 255 distinct haplotypes, beyond the device
    encoding's u8 membership (those keys take the host path)."""
    from helpers import many_variant_regions
    ps, _ = synth_patterns(tmp_path, 10, 2, 31, thr=2e-3)
    regions = many_variant_regions(n, ps.max_length)
    beds = [("synthetic.bed", [tuple(r["merged"]) for r in regions])]
    _compare(ps, n, beds, regions)


@pytest.mark.parametrize("indel,per_batch,subset,index", [(0, 5, False, True), (25, 0, False, False),
                                                          (10, 3, True, True)])
def test_run_flow_on_synthetic_bcf_vs_oracle(tmp_path, indel, per_batch, subset, index):
    """f2-f4 + the scan at a larger size than test_data: a synthetic BCF/FASTA/BED set
    (tools/synth_dataset.py) through tfbs_run (streaming BCF reader, batches of
    merged regions, device key reduction, BGZF writer) vs the oracle's run() on the
    same records; decompressed VCF text identical.  subset: a samples file naming
    a shuffled subset plus an unknown name (main.rs:293-314 keeps BCF order)."""
    import gzip
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "data"), n_samples=80, n_regions=14, n_pwms=10,
                                   length_config=2, seed=7, indel_pct=indel, index=index)
    out = tmp_path / "out.vcf.gz"
    samples_file = os.path.join(d["dir"], "samples")
    wanted = d["samples"]
    if subset:
        import random as _random
        wanted = _random.Random(5).sample(d["samples"], 23)
        samples_file = str(tmp_path / "wanted.txt")
        open(samples_file, "w").write("\n".join(wanted + ["NOT_IN_BCF"]) + "\n")
    T.run("chr1", d["bcf"], [d["bed"]], d["fasta"], samples_file, d["pwm_file"], d["thr_dir"], 2e-3, d["names"],
          str(out), threads=4, regions_per_batch=per_batch)
    got = gzip.open(str(out), "rt").read()
    recs = [dict(r, gt=r["gt"].astype(int).tolist()) for r in d["records"]]
    want = O.run("chr1", recs, [d["bed"]], d["fasta"], d["samples"], wanted + (["NOT_IN_BCF"] if subset else []),
                 d["pwm_file"], d["thr_dir"], 2e-3, d["names"])
    assert got == want
    assert got.count("\n") > 1  # some rows


@pytest.mark.parametrize("index", [True, False])
def test_run_flow_fetch_edges_vs_oracle(tmp_path, index):
    """The fetch window's edges (parity unpinned by the reference's
    fixtures): per region an SNV at ext.end (fetched and patched), one at ext.end + 1
    (outside the half-open fetch(ext.start, ext.end + 1), haplotype.rs:78-79) and a
    deletion starting left of ext.start that reaches into the window (fetched: its
    carriers form their own groups; not patched: patch_haplotype keeps diffs with
    ext.start <= pos, haplotype.rs:95-96).  The product's rows equal the oracle's,
    which restates htslib's overlap rule (pos < end and pos + rlen > beg); with and
    without the CSI index."""
    import gzip
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "data"), n_samples=60, n_regions=12, n_pwms=10,
                                   length_config=2, seed=13, indel_pct=10, index=index, edges=True)
    out = tmp_path / "edges.vcf.gz"
    T.run("chr1", d["bcf"], [d["bed"]], d["fasta"], None, d["pwm_file"], d["thr_dir"], 2e-3, d["names"], str(out),
          threads=4, regions_per_batch=5)
    got = gzip.open(str(out), "rt").read()
    recs = [dict(r, gt=r["gt"].astype(int).tolist()) for r in d["records"]]
    want = O.run("chr1", recs, [d["bed"]], d["fasta"], d["samples"], d["samples"], d["pwm_file"], d["thr_dir"], 2e-3,
                 d["names"])
    assert got == want
    assert got.count("\n") > 10


@pytest.mark.parametrize("index", [True, False])
def test_run_devices_shards_same_text(tmp_path, index):
    """Multi-device run flow: the merged regions cut into one block per
    listed device, each with its own BCF reader (CSI seek to its block, or a sweep from
    the file start), FASTA reader, prep thread and ctx; rows concatenated in merged-peak
    order with POS renumbered.  2, 3 and 8 contexts on this one GPU give the text of a
    single device, which equals the oracle's run()."""
    import gzip
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "data"), n_samples=60, n_regions=37, n_pwms=12,
                                   length_config=2, seed=8, indel_pct=15, index=index)
    args = ("chr1", d["bcf"], [d["bed"]], d["fasta"], os.path.join(d["dir"], "samples"), d["pwm_file"],
            d["thr_dir"], 2e-3, d["names"])
    texts = []
    for devs, per_batch in [(None, 4), ([0, 0], 4), ([0, 0, 0], 3), ([0] * 8, 2), ([0] * 16, 1)]:
        out = tmp_path / ("out%d.vcf.gz" % len(texts))
        T.run(*args, str(out), threads=4, regions_per_batch=per_batch, devices=devs)
        texts.append(gzip.open(str(out), "rt").read())
        assert not [f for f in os.listdir(str(tmp_path)) if ".part" in f]  # spills removed
    assert all(t == texts[0] for t in texts[1:])
    recs = [dict(r, gt=r["gt"].astype(int).tolist()) for r in d["records"]]
    want = O.run("chr1", recs, [d["bed"]], d["fasta"], d["samples"], d["samples"], d["pwm_file"], d["thr_dir"],
                 2e-3, d["names"])
    assert texts[0] == want
    assert want.count("\n") > 10


def test_run_async_rows_writer_same_text(tmp_path, monkeypatch):
    """The one-device run flow hands each drained slot of BGZF blocks to the ctx's writer
    thread (copy back + write, in order) and goes on with the next batch.  With the
    writer held back (TFBS_ROWS_WRITER_DELAY_US) and two blocks per launch (every call
    cycles the three slots, so the next call's launches meet slots whose copies have
    not run yet, and a slot that held a one-block remainder grows under them) the output
    equals the synchronous writes' (TFBS_RUN_ASYNC_WRITE=0)."""
    import gzip
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "data"), n_samples=2000, n_regions=30, n_pwms=10,
                                   length_config=2, seed=21, indel_pct=10)
    args = ("chr1", d["bcf"], [d["bed"]], d["fasta"], None, d["pwm_file"], d["thr_dir"], 2e-3, d["names"])
    monkeypatch.setenv("TFBS_BGZF_BATCH_BLOCKS", "2")
    texts = []
    for asyn, delay in ((0, 0), (1, 0), (1, 3000)):
        monkeypatch.setenv("TFBS_RUN_ASYNC_WRITE", str(asyn))
        monkeypatch.setenv("TFBS_ROWS_WRITER_DELAY_US", str(delay))
        out = tmp_path / ("async%d.vcf.gz" % len(texts))
        T.run(*args, str(out), threads=4, regions_per_batch=3)
        texts.append(gzip.open(str(out), "rt").read())
    assert texts[1] == texts[0] and texts[2] == texts[0]
    assert texts[0].count("\n") > 20


def test_cli_gpus_and_devices(tmp_path):
    """--gpus N / --devices LIST on the command line: same text as one device."""
    import gzip
    import subprocess
    import sys as _sys
    _sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import synth_dataset
    d = synth_dataset.make_dataset(str(tmp_path / "data"), n_samples=30, n_regions=12, n_pwms=6,
                                   length_config=2, seed=5, indel_pct=10)
    exe = os.path.join(os.path.dirname(T.__file__), "bin", "find-tfbs-amd")
    texts = []
    for extra in ([], ["--gpus", "1"], ["--devices", "0,0,0"]):
        out = tmp_path / ("cli%d.vcf.gz" % len(texts))
        r = subprocess.run([exe, "--chromosome", "chr1", "--input", d["bcf"], "--bed", d["bed"], "--reference",
                            d["fasta"], "--pwm_file", d["pwm_file"], "--pwm_threshold_directory", d["thr_dir"],
                            "--pwm_threshold", "0.002", "--pwm_names", ",".join(d["names"]), "--output", str(out),
                            "--threads", "3", "--regions_per_batch", "2"] + extra,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        texts.append(gzip.open(str(out), "rt").read())
    assert texts[0] == texts[1] == texts[2]
    assert texts[0].count("\n") > 1


def test_reduce_zero_samples_after_keys(tmp_path):
    """A batch with no samples has no haplotype and no key (main.rs:500-534 counts
    nothing), also when its ctx just reduced a batch with keys (reused device buffers)."""
    ps, _ = synth_patterns(tmp_path, 8, 2, 41, thr=5e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(3)])]
    sc = T.Scanner(ps)
    try:
        full = build_batch(ps, 30, beds, make_regions_synth(3, 0, 3, 30, ps.max_length))
        full.scan(sc, reduce=True)
        assert sum(len(full.keys(r)) for r in range(3)) > 0
        empty = build_batch(ps, 0, beds, make_regions_synth(3, 0, 3, 0, ps.max_length))
        empty.scan(sc, reduce=True)
        for r in range(3):
            assert empty.keys(r) == {}
            assert empty.region_rows(r, "chr1")[0] == ""
    finally:
        sc.close()


@pytest.mark.parametrize("mfma", ["0", "1"])
def test_ds_ties_at_the_fifth_decimal_vs_oracle(monkeypatch, mfma):
    """counts_as_genotypes' DS = {:.4} of the f32 2 (x - lo) / (hi - lo) (main.rs:439-498):
    with hi - lo = 64 (a multiple of 32) a sample at x - lo odd lands exactly on a 5th
    decimal 5 (1/32 = 0.03125 -> '0.0312', 63/32 = 1.96875 -> '1.9688': ties to even, as
    Rust >= 1.67 and printf('%.4f') print them).  A one-column 'A' PWM hits
    every A of the inner range; per-sample counts are set by A->C SNVs on either
    haplotype: 2 a0 (both reference), 2 (a0 - 32) (32 SNVs on both), 2 a0 - 1 and
    2 (a0 - 32) + 1 (one SNV / 31 SNVs on one side) and a spread of others.  Device keys,
    rows (dense, device reduction, device encoding) == the oracle's, and the tie texts
    are in the rows."""
    monkeypatch.setenv("TFBS_MFMA", mfma)
    ps = T.PatternSet.from_patterns([T.Pattern.PWM([T.Weight(1000, 0, 0, 0)], "A1", 0, 999, 0)])
    n = 12
    s0, e0 = 2000, 2199  # inner = merged: 200 bases, ext = the same (L_max 1)
    rnd = random.Random(5)
    ref = "".join(rnd.choice("AACGT") for _ in range(e0 - s0 + 1))
    a_pos = [s0 + i for i, c in enumerate(ref) if c == "A"]
    assert len(a_pos) > 64
    # haplotype h carries the SNVs at a_pos[:k_h]
    k = {0: 0, 1: 0, 2: 32, 3: 32, 4: 1, 5: 0, 6: 31, 7: 32}
    for s in range(4, n):
        k[2 * s], k[2 * s + 1] = rnd.randint(0, 32), rnd.randint(0, 32)
    recs = []
    for j, p in enumerate(a_pos[:32]):
        car = sorted(h for h in range(2 * n) if k.get(h, 0) > j)
        if car:
            recs.append(("car", p, "A", "C", car))
    regions = [{"merged": (s0, e0), "ref": ref, "records": recs}]
    beds = [("ties.bed", [(s0, e0)])]
    _compare(ps, n, beds, regions)
    okeys, orows, _ = run_oracle(ps, n, beds, regions)
    row = [r for r in orows.split("\n") if r][0].split("\t")
    assert "1|1:1.9688" in row and "0|0:0.0312" in row, row[9:]
