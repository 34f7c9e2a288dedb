"""Pin the CPU oracle (oracle/tfbs_oracle.c) against every offline-runnable test
vector of the reference.  CPU only."""
import os

import oracle_py as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TD = os.path.join(GOLD, "test_data")

REF = [("A", 0), ("C", 1), ("G", 2), ("T", 3)]  # haplotype.rs:162-169


# ---------------------------------------------------------------- range.rs:93-107
def test_range_contains_overlaps():
    L = O.lib()
    # Range::contains is overlaps with a point range
    for p, want in [(100, 1), (105, 1), (110, 1), (99, 0), (111, 0)]:
        assert L.orc_range_overlaps(100, 110, p, p) == want
    # asymmetric overlaps (range.rs:18-21): a range that strictly contains self is not "overlapping"
    assert L.orc_range_overlaps(5, 20, 3, 30) == 0
    assert L.orc_range_overlaps(3, 30, 5, 20) == 1


# ---------------------------------------------------------------- haplotype.rs:172-254
def test_patch_haplotype_with_no_diff():
    assert O.patch_haplotype((1, 2), [], REF) == [("C", 1), ("G", 2)]
    assert O.patch_haplotype((0, 2), [], REF) == [("A", 0), ("C", 1), ("G", 2)]
    assert O.patch_haplotype((0, 5), [], REF) == [("A", 0), ("C", 1), ("G", 2), ("T", 3)]


def test_patch_haplotype_one_snp():
    assert O.patch_haplotype((1, 2), [(100, "A", "C")], REF) == [("C", 1), ("G", 2)]
    assert O.patch_haplotype((1, 2), [(1, "C", "N")], REF) == [("N", 1), ("G", 2)]
    assert O.patch_haplotype((1, 2), [(2, "G", "A")], REF) == [("C", 1), ("A", 2)]


def test_patch_haplotype_two_snp():
    assert O.patch_haplotype((1, 2), [(1, "C", "N"), (2, "G", "A")], REF) == [("N", 1), ("A", 2)]
    assert O.patch_haplotype((1, 2), [(1, "C", "N"), (4, "G", "A")], REF) == [("N", 1), ("G", 2)]


def test_patch_haplotype_one_insert():
    assert O.patch_haplotype((1, 2), [(1, "C", "NN")], REF) == [("N", 1), ("N", 1), ("G", 2)]
    assert O.patch_haplotype((1, 2), [(2, "G", "NN")], REF) == [("C", 1), ("N", 2), ("N", 2)]
    assert O.patch_haplotype((1, 2), [(3, "T", "NN")], REF) == [("C", 1), ("G", 2)]


def test_patch_haplotype_one_deletion():
    assert O.patch_haplotype((1, 2), [(1, "CG", "C")], REF) == [("C", 1)]
    assert O.patch_haplotype((1, 2), [(2, "GT", "G")], REF) == [("C", 1), ("G", 2)]
    assert O.patch_haplotype((1, 2), [(0, "AC", "A")], REF) == [("C", 1), ("G", 2)]


def test_patch_haplotype_quirks():
    # REF mismatch panics (haplotype.rs:126-128) -> error code
    assert O.patch_haplotype((1, 2), [(1, "G", "A")], REF) == -2
    # MNP panics (haplotype.rs:141-142)
    assert O.patch_haplotype((1, 2), [(1, "CG", "TA")], REF) == -3
    # overlapping diffs on one haplotype truncate it (haplotype.rs:147-149)
    assert O.patch_haplotype((0, 3), [(0, "AC", "A"), (1, "C", "T")], REF) == [("A", 0)]
    # ... unless the walk is already at/after the window end: one ref base at ref_position is
    # emitted, even past range.end (haplotype.rs:144-146)
    assert O.patch_haplotype((0, 3), [(1, "CG", "C"), (2, "G", "T")], REF) == [("A", 0), ("C", 1), ("T", 3)]
    assert O.patch_haplotype((0, 2), [(1, "CG", "C"), (2, "G", "T")], REF) == [("A", 0), ("C", 1), ("T", 3)]
    assert O.patch_haplotype((0, 3), [(1, "CGT", "C"), (2, "G", "T")], REF) == [("A", 0), ("C", 1)]


# ---------------------------------------------------------------- pattern.rs:268-301
def test_matches():
    w = [[0, 1000, 0, 0, 0], [0, 0, 1000, 0, 0]]
    hap = [("A", 10), ("C", 11), ("G", 12), ("T", 13)]
    assert O.matches(w, 1500, hap) == [(11, 12)]


def test_match_gataa():
    w = [[0, 0, 100, 0, 0], [100, 0, 0, 0, 0], [0, 0, 0, 100, 0], [100, 0, 0, 0, 0], [100, 0, 0, 0, 0]]
    pad = [("N", 0), ("G", 1), ("A", 2), ("T", 3), ("A", 4), ("A", 5), ("N", 6)]
    nopad = [("G", 1), ("A", 2), ("T", 3), ("A", 4), ("A", 5)]
    assert len(O.matches(w, 499, pad)) == 1
    assert len(O.matches(w, 499, nopad)) == 1
    assert len(O.matches(w, 500, pad)) == 0
    assert len(O.matches(w, 500, nopad)) == 0


def test_matches_other_pattern_and_short_haplotype():
    w = [[0, 1000, 0, 0, 0], [0, 0, 1000, 0, 0]]
    assert O.matches(w, 1500, [("C", 1)]) == []  # haplotype shorter than the PWM
    assert O.matches(w, -10**9, [("C", 1), ("G", 2)], kind=1) == []  # OtherPattern never matches


def test_matches_indel_positions():
    # Match end is pos-based, not index-based (pattern.rs:156): an inserted base repeats the pos.
    w = [[0, 1000, 0, 0, 0], [0, 0, 1000, 0, 0], [0, 0, 0, 1000, 0]]
    hap = [("C", 5), ("G", 5), ("T", 6)]
    assert O.matches(w, 2500, hap) == [(5, 7)]


# ---------------------------------------------------------------- pattern.rs:192-260 (RC vectors)
GATA1_P = [[322, -754, 193, -65], [-490, 565, 200, -898], [1022, -2694, -3126, 105], [-4400, -4400, 1375, -3903],
           [1377, -4400, -4400, -4400], [-3325, -3126, -4400, 1363], [1347, -3126, -3325, -2584],
           [1296, -3573, -1421, -2584], [-570, -357, 969, -2311], [393, -220, 304, -1022], [304, -144, 250, -705]]
GATA1_N = [[-705, 250, -144, 304], [-1022, 304, -220, 393], [-2311, 969, -357, -570], [-2584, -1421, -3573, 1296],
           [-2584, -3325, -3126, 1347], [1363, -4400, -3126, -3325], [-4400, -4400, -4400, 1377],
           [-3903, 1375, -4400, -4400], [105, -3126, -2694, 1022], [-898, 200, 565, -490], [-65, 193, -754, 322]]
GATA2_P = [[333, -754, 281, -210], [-415, 551, 327, -1525], [1093, -2961, -3325, -74], [-4400, -3903, 1371, -3573],
           [1355, -2694, -3325, -3903], [-2584, -1770, -1600, 1268], [1229, -1561, -2034, -1421],
           [1117, -2311, -291, -2311], [-516, -40, 814, -1681], [509, -357, 388, -1818], [509, -543, 91, -415]]
GATA2_N = [[-415, 91, -543, 509], [-1818, 388, -357, 509], [-1681, 814, -40, -516], [-2311, -291, -2311, 1117],
           [-1421, -2034, -1561, 1229], [1268, -1600, -1770, -2584], [-3903, -3325, -2694, 1355],
           [-3573, 1371, -3903, -4400], [-74, -3325, -2961, 1093], [-1525, 327, 551, -415], [-210, 281, -754, 333]]


def _rc(w4):
    L = O.lib()
    flat = O.arr(O.C.c_int32, [x for r in w4 for x in (r + [0])])
    out = (O.C.c_int32 * (5 * len(w4)))()
    L.orc_reverse_complement(flat, len(w4), out)
    return [[out[5 * j + c] for c in range(4)] for j in range(len(w4))]


def test_reverse_complement_vectors():
    assert _rc(GATA1_P) == GATA1_N
    assert _rc(GATA2_P) == GATA2_N


def test_parse_pwm_files_synthetic_gata(tmp_path):
    """pattern.rs:192-260 with the float text reconstructed from the pinned integers
    (the HOCOMOCO source file is absent)."""
    pwm = tmp_path / "pwms.txt"
    lines = []
    for name, w in [("OTHER_NOT_WANTED", GATA2_P[:3]), ("GATA1_HUMAN.H11MO.1.A", GATA1_P),
                    ("GATA2_HUMAN.H11MO.1.A", GATA2_P)]:
        lines.append(">" + name)
        lines += ["\t".join("%.3f" % (x / 1000.0) for x in row) for row in w]
    pwm.write_text("\n".join(lines) + "\n")
    thr = tmp_path / "thr"
    thr.mkdir()
    (thr / "GATA1_HUMAN.H11MO.1.A.thr").write_text("1.000\t0.5\n4.683\t0.0011\n5.000\t0.0009\n")
    (thr / "GATA2_HUMAN.H11MO.1.A.thr").write_text("5.314\t0.002\n6.0\t0.001\n")
    pats = O.Patterns.from_files(str(pwm), str(thr), 0.001, ["GATA1_HUMAN.H11MO.1.A", "GATA2_HUMAN.H11MO.1.A"])
    got = pats.as_list()
    assert len(got) == 4
    want = [(GATA1_P, 0, 4683, 0), (GATA1_N, 0, 4683, 1), (GATA2_P, 1, 5314, 0), (GATA2_N, 1, 5314, 1)]
    for g, (w, pid, ms, d) in zip(got, want):
        assert [r[:4] for r in g["weights"]] == w
        assert all(r[4] == 0 for r in g["weights"])
        assert (g["pattern_id"], g["min_score"], g["direction"]) == (pid, ms, d)


def test_parse_threshold_acgt():
    v = O.C.c_int32()
    r = O.lib().orc_parse_threshold_file(os.path.join(TD, "ACGT.thr").encode(), 0.0001, O.C.byref(v))
    assert r == 1 and v.value == 3999  # min_score 3999 at 1e-4
    r = O.lib().orc_parse_threshold_file(os.path.join(TD, "ACGT.thr").encode(), 1.0, O.C.byref(v))
    assert r == 0  # no p-value > 1.0 -> None


def test_parse_weight_rounding():
    v = O.C.c_int32()
    for s, want in [("1.0", 1000), ("-28.912716067144597", -28913), ("2.999", 2999), ("0.0005", 1),
                    ("-0.0005", -1), ("1e-3", 1)]:
        assert O.lib().orc_parse_weight(s.encode(), O.C.byref(v)) == 0
        assert v.value == want, s
    assert O.lib().orc_parse_weight(b"abc", O.C.byref(v)) < 0
    assert O.lib().orc_parse_weight(b"0x10", O.C.byref(v)) < 0


# ---------------------------------------------------------------- main.rs:570-671
def test_count_matches():
    m1 = ((10, 11), 0, [(0, 0)])
    ml1 = [m1]
    ml2 = [((20, 21), 0, [(0, 0)])]
    ml3 = [((4, 5), 0, [(0, 0)])]
    ml4 = [((3, 4), 0, [(0, 0)])]
    ml5 = [((21, 22), 0, [(0, 0)])]
    ml6 = [((4, 5), 9, [(1, 1)])]
    ml7 = [((17, 18), 11, [(1, 1)])]
    MEP, ERY = 0, 1
    r1, r2 = (5, 20), (15, 25)
    ip = [(MEP, 5, 20)]
    ip2 = [(MEP, 5, 20), (ERY, 15, 25)]
    c = O.count_matches_by_sample
    assert c(2, ml1, ip) == {(MEP, r1, 0): ([1, 0], [0, 0])}
    assert c(2, ml1, ip) == c(2, ml2, ip)
    assert c(2, ml1, ip) == c(2, ml3, ip)
    assert c(2, ml4, ip) == c(2, ml5, ip)
    assert c(2, ml4, ip) == {}
    assert c(2, ml6, ip) == {(MEP, r1, 9): ([0, 0], [0, 1])}
    assert c(2, ml1, ip2) == {(MEP, r1, 0): ([1, 0], [0, 0])}
    assert c(2, ml2, ip2) == {(MEP, r1, 0): ([1, 0], [0, 0]), (ERY, r2, 0): ([1, 0], [0, 0])}
    assert c(2, ml1, ip2) == c(2, ml3, ip2)
    assert c(2, ml4, ip2) == {}
    assert c(2, ml5, ip2) == {(ERY, r2, 0): ([1, 0], [0, 0])}
    assert c(2, ml6, ip2) == {(MEP, r1, 9): ([0, 0], [0, 1])}
    assert c(2, ml7, ip2) == {(MEP, r1, 11): ([0, 0], [0, 1]), (ERY, r2, 11): ([0, 0], [0, 1])}


def test_count_matches_duplicate_inner_double_counts():
    # the same Range twice in one bed list is one HashMap key hit twice (main.rs:503-505)
    got = O.count_matches_by_sample(1, [((10, 11), 3, [(0, 0)])], [(0, 5, 20), (0, 5, 20)])
    assert got == {(0, (5, 20), 3): ([2], [0])}


# ---------------------------------------------------------------- main.rs:439-498
def test_counts_as_genotypes():
    assert O.counts_as_genotypes([1, 1], [0, 0]) is None
    maf, info, gts = O.counts_as_genotypes([0, 1, 1, 1], [2, 3, 3, 3])
    assert info == "COUNTS=2,4;freqs=1/0/3" and gts == "\t0|0:0.0\t1|1:2.0\t1|1:2.0\t1|1:2.0" and maf == 1
    maf, info, gts = O.counts_as_genotypes([0, 1, 2, 3, 4], [0, 0, 0, 0, 0])
    # thr1 = (0+4000)/4 = 1000, thr3 = 3000: 1 -> 0|1 (1000 !< 1000), 2 -> 0|1, 3 -> 1|1
    assert info == "COUNTS=0,1,2,3,4;freqs=1/2/2"
    assert gts == "\t0|0:0.0\t0|1:0.5000\t0|1:1.0000\t1|1:1.5000\t1|1:2.0"
    assert maf == 3  # zero=1, one=2, two=2: two wins the tie over one -> zero + one


# ---------------------------------------------------------------- bed.rs:67-96
def test_merge_bed():
    merged, beds = O.load_peak_files([os.path.join(TD, "regions1.bed"), os.path.join(TD, "regions2.bed")], "chr1", 0)
    assert merged == [(100, 115), (118, 130), (150, 160), (161, 165), (180, 210)]
    assert dict(beds) == {
        "regions1.bed": [(100, 110), (120, 130), (150, 160), (180, 190), (200, 210)],
        "regions2.bed": [(110, 115), (118, 125), (161, 165), (190, 200)],
    }
    assert sum(e - s for s, e in merged) == 71


# ---------------------------------------------------------------- main.rs:548-568 (text of the gz fixtures)
def _run(bcf_json):
    import json
    rec = json.load(open(os.path.join(GOLD, bcf_json)))
    samples = [l.strip() for l in open(os.path.join(TD, "samples")) if len(l.rstrip("\n")) > 1]
    return O.run("chr1", rec["records"], [os.path.join(TD, "regions1.bed"), os.path.join(TD, "regions2.bed")],
                 os.path.join(TD, "reference_genome.fa"), rec["samples"], samples,
                 os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["ACGT"])


def test_integration_no_polymorphism():
    assert _run("genotypes.records.json") == open(os.path.join(GOLD, "expected_output_1.vcf")).read()


def test_integration_one_polymorphism():
    assert _run("genotypes2.records.json") == open(os.path.join(GOLD, "expected_output_2.vcf")).read()
