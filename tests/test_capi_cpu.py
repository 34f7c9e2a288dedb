"""CPU-side checks of the product library (no GPU calls): symbol exports, the
host parsers / patcher / genotype encoder against the oracle, and batch
construction (grouping, dedup) against the oracle's haplotype counts."""
import os
import random
import re

import pytest

import oracle_py as O
from helpers import GOLD, TD, T, make_regions_synth, pattern_dicts, run_oracle, synth_patterns

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "tfbs_amd.h")).read()
    decls = set(re.findall(r"^\s*(?:const\s+)?[\w ]+?\**\s*\*?(tfbs_\w+)\(", hdr, re.M))
    assert len(decls) > 40
    lib = T.lib()
    for name in sorted(decls):
        assert hasattr(lib, name), name
    declared = {s[0] for s in T._capi.SIGNATURES}
    assert decls == declared, decls ^ declared


def test_no_device_means_loud_failure():
    if T.device_count() > 0:
        pytest.skip("a GPU is visible")
    ps = T.parse_pwm_files(os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["ACGT"])
    with pytest.raises(T.TfbsError) as ei:
        T.Scanner(ps)
    assert ei.value.code == T.TFBS_E_NODEVICE


def test_parse_pwm_files_matches_oracle(tmp_path):
    ps, names = synth_patterns(tmp_path, 40, 3, 11)
    orc = O.Patterns.from_files(str(tmp_path / "pwms.txt"), str(tmp_path / "thr"), 1e-4, names)
    assert pattern_dicts(ps) == orc.as_list()
    ps2, _ = synth_patterns(tmp_path, 40, 3, 11, thr=1e-3, forward_only=True)
    orc2 = O.Patterns.from_files(str(tmp_path / "pwms.txt"), str(tmp_path / "thr"), 1e-3, names, add_reverse=False)
    assert pattern_dicts(ps2) == orc2.as_list()


def test_parse_acgt_fixture():
    ps = T.parse_pwm_files(os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["ACGT"])
    pl = ps.to_list()
    assert [p.min_score for p in pl] == [3999, 3999]
    assert [w.acgtn for w in pl[0].weights] == [[1000, 0, 0, 0, 0], [0, 1000, 0, 0, 0], [0, 0, 1000, 0, 0],
                                                [0, 0, 0, 1000, 0]]
    assert pl[1].weights == pl[0].weights  # ACGT is its own reverse complement
    assert T.parse_threshold_file(os.path.join(TD, "ACGT.thr"), 0.0001) == 3999
    assert T.parse_threshold_file(os.path.join(TD, "ACGT.thr"), 1.0) is None
    with pytest.raises(T.TfbsError):
        T.parse_threshold_file(os.path.join(TD, "missing.thr"), 0.1)
    with pytest.raises(T.TfbsError):  # main.rs:238: no pattern loaded
        T.parse_pwm_files(os.path.join(TD, "pwm_definitions.txt"), TD, 0.0001, ["NOPE"])


def test_parse_weight_matches_oracle():
    rnd = random.Random(5)
    vals = ["1.0", "-0.0005", "0.0005", "2.5e-3", "-28.912716067144597", "1e10", "inf", "-inf", "nan", "5.", ".5"]
    vals += ["%.*f" % (rnd.randint(0, 7), rnd.uniform(-20, 20)) for _ in range(300)]
    for s in vals:
        v = O.C.c_int32()
        assert O.lib().orc_parse_weight(s.encode(), O.C.byref(v)) == 0, s
        assert T.parse_weight(s) == v.value, s


REF = [("A", 0), ("C", 1), ("G", 2), ("T", 3)]


@pytest.mark.parametrize("rng,diffs", [
    ((1, 2), []), ((0, 2), []), ((0, 5), []),
    ((1, 2), [(100, "A", "C")]), ((1, 2), [(1, "C", "N")]), ((1, 2), [(2, "G", "A")]),
    ((1, 2), [(1, "C", "N"), (2, "G", "A")]), ((1, 2), [(1, "C", "N"), (4, "G", "A")]),
    ((1, 2), [(1, "C", "NN")]), ((1, 2), [(2, "G", "NN")]), ((1, 2), [(3, "T", "NN")]),
    ((1, 2), [(1, "CG", "C")]), ((1, 2), [(2, "GT", "G")]), ((1, 2), [(0, "AC", "A")]),
    ((0, 3), [(0, "AC", "A"), (1, "C", "T")]), ((0, 3), [(1, "CG", "C"), (2, "G", "T")]),
    ((0, 2), [(1, "CG", "C"), (2, "G", "T")]), ((0, 3), [(1, "CGT", "C"), (2, "G", "T")]),
])
def test_patch_haplotype_matches_reference_vectors(rng, diffs):
    want = O.patch_haplotype(rng, diffs, REF)
    got = T.patch_haplotype(rng, [T.Diff(*d) for d in diffs], REF)
    assert [(n.nuc, n.pos) for n in got] == want


def test_patch_haplotype_errors():
    with pytest.raises(T.TfbsError) as e1:
        T.patch_haplotype((1, 2), [T.Diff(1, "G", "A")], REF)
    assert e1.value.code == -3
    with pytest.raises(T.TfbsError) as e2:
        T.patch_haplotype((1, 2), [T.Diff(1, "CG", "TA")], REF)
    assert e2.value.code == -4


def test_patch_haplotype_fuzz_vs_oracle():
    rnd = random.Random(7)
    for _ in range(400):
        n = rnd.randint(1, 30)
        ref = [("ACGTN"[rnd.randrange(5)], 10 + i) for i in range(n)]
        diffs = []
        for _ in range(rnd.randint(0, 5)):
            p = rnd.randint(5, 10 + n + 3)
            r0 = ref[p - 10][0] if 10 <= p < 10 + n else "A"
            kind = rnd.randrange(3)
            if kind == 0:
                d = (p, r0, rnd.choice("ACGTN"))
            elif kind == 1:
                d = (p, r0, r0 + "".join(rnd.choice("ACGT") for _ in range(rnd.randint(1, 3))))
            else:
                d = (p, r0 + "".join(rnd.choice("ACGT") for _ in range(rnd.randint(1, 3))), r0)
            diffs.append(d)
        rng = (rnd.randint(8, 14), rnd.randint(14, 10 + n + 3))
        want = O.patch_haplotype(rng, diffs, ref)
        if isinstance(want, int):
            with pytest.raises(T.TfbsError):
                T.patch_haplotype(rng, [T.Diff(*d) for d in diffs], ref)
        else:
            got = T.patch_haplotype(rng, [T.Diff(*d) for d in diffs], ref)
            assert [(x.nuc, x.pos) for x in got] == want, (rng, diffs)


def test_counts_as_genotypes_fuzz_vs_oracle():
    rnd = random.Random(3)
    for _ in range(300):
        n = rnd.randint(1, 40)
        top = rnd.choice([1, 3, 10, 33, 64, 1000])
        v1 = [rnd.randint(0, top) for _ in range(n)]
        v2 = [rnd.randint(0, top) for _ in range(n)]
        want = O.counts_as_genotypes(v1, v2)
        got = T.counts_as_genotypes(v1, v2)
        if want is None:
            assert got is None
        else:
            maf, info, gts = want
            counts, gmaf, f0, f1, f2, ggts = got
            assert gmaf == maf and ggts == gts
            assert info == "COUNTS=%s;freqs=%d/%d/%d" % (",".join(map(str, counts)), f0, f1, f2)


@pytest.mark.parametrize("indel", [0, 30])
def test_batch_grouping_matches_oracle(tmp_path, indel):
    """Distinct-haplotype construction (groups, patch, dedup, reference group) on the
    host matches the oracle's number_of_haplotypes / variant_count per region."""
    ps, _ = synth_patterns(tmp_path, 6, 2 if not indel else 5, 4)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(12)])]
    regions = make_regions_synth(9, 0, 12, 200, ps.max_length, indel)
    _, _, stats = run_oracle(ps, 200, beds, regions)
    from helpers import build_batch
    b = build_batch(ps, 200, beds, regions)
    for i, (nh, nv, _) in enumerate(stats):
        assert b.region_stats(i) == (nh, nv)
    assert b.num_haplotypes == sum(s[0] for s in stats)
    assert b.num_windows > 0 and b.num_effective_windows >= b.num_windows


def _plan(w4, ms):
    p = T.Pattern.PWM([T.Weight(*r) for r in w4], "x", 0, ms, 0)
    return T.PatternSet.from_patterns([p]).plan_stats()


def test_plan_octet_eligibility():
    """plan.cpp: a strand takes the 16-bit octet path iff every 4-column block spans
    <= 32767, no i32 wrap is possible and min_score - sum(block maxima) >= -32768."""
    w = [[0, -1000, -500, -2000]] * 8          # best 0, worst -16000
    assert _plan(w, -32768)["n_octet_strands"] == 1
    assert _plan(w, -32769)["n_quad_strands"] == 1
    assert _plan(w, 10**6)["n_octet_strands"] == 1  # threshold above the best: thr clamps to 0
    span = [[0, -32767, 0, 0]] + [[0, 0, 0, 0]] * 3
    assert _plan(span, -100)["n_octet_strands"] == 1
    span = [[0, -32768, 0, 0]] + [[0, 0, 0, 0]] * 3
    assert _plan(span, -100)["n_quad_strands"] == 1
    assert _plan([[2**30, 0, 0, 0]] * 2, 0)["n_quad_strands"] == 1
    long = [[0, 1, 2, 3]] * 33
    st = _plan(long, 5)
    assert st["n_generic_strands"] == 1 and st["n_fast_tiles"] == 0


def test_plan_tiles_cover_every_strand(tmp_path):
    ps, _ = synth_patterns(tmp_path, 120, 3, 4)
    for tb in (8, 16, 32):
        st = ps.plan_stats(tb)
        assert st["n_octet_strands"] + st["n_quad_strands"] + st["n_generic_strands"] == len(ps)
        assert st["max_tile_blocks"] <= max(tb, 8)


def test_batch_grouping_beyond_64_distinct_diffs(tmp_path):
    """The 64-bit diff-mask grouping and the sorted-list fallback (> 64 distinct
    diffs in a region) agree with the oracle's distinct-haplotype counts."""
    from helpers import build_batch, many_variant_regions
    ps, _ = synth_patterns(tmp_path, 4, 2, 6)
    n = 120
    regions = many_variant_regions(n, ps.max_length)
    beds = [("synthetic.bed", [tuple(r["merged"]) for r in regions])]
    _, _, stats = run_oracle(ps, n, beds, regions)
    b = build_batch(ps, n, beds, regions)
    for i, (nh, nv, _) in enumerate(stats):
        assert b.region_stats(i) == (nh, nv)
    assert max(s[1] for s in stats) > 64


def _window_score(w4, window):
    """apply_pwm (pattern.rs:125-135): i32 sum, N = 0."""
    return sum(w4[j]["ACGT".index(ch)] for j, ch in enumerate(window) if ch != "N")


def test_mfma_bound_is_sound():
    """The FP6 bound the matrix-core scan filters with (mfma.cpp): for random patterns
    (weight spans 1 .. 2^20, mixed / all-negative / all-positive columns, thresholds at,
    below and above real scores) and random windows with N, 8 * score <= 8 c + scale * q8,
    every window with score > min_score (pattern.rs:151) is a candidate (q8 > t8), and the
    window's 11-bit field q8 + 1023 - t8 neither borrows nor carries."""
    rnd = random.Random(21)
    checked = hits = 0
    for trial in range(160):
        L = rnd.choice([1, 2, 5, 8, 9, 15, 16, 17, 24, 31, 32])
        mx = rnd.choice([1, 3, 8, 100, 1000, 4400, 32385, 1 << 20])
        kind = trial % 3
        lo, hi = (-mx, mx) if kind == 0 else ((-mx, -1) if kind == 1 else (1, mx))
        if lo > hi:
            lo, hi = hi, lo
        w4 = [[rnd.randint(lo, hi) for _ in range(4)] for _ in range(L)]
        windows = ["".join(rnd.choice("ACGT" if t % 4 else "ACGTN") for _ in range(L)) for t in range(60)]
        best = "".join("ACGT"[max(range(4), key=lambda b: w4[j][b])] for j in range(L))
        windows.append(best)
        scores = sorted(_window_score(w4, x) for x in windows)
        ms = rnd.choice([scores[-1], scores[-1] - 1, scores[len(scores) // 2], scores[0] - 1, scores[-1] + 5])
        ps = T.PatternSet.from_patterns([T.Pattern.PWM([T.Weight(*r) for r in w4], "B", 1, ms)])
        for x in windows:
            b = ps.mfma_bound(0, x)
            assert b["eligible"] == 1
            sc = _window_score(w4, x)
            assert 8 * sc <= 8 * b["c"] + b["scale"] * b["q8"], (trial, x, sc, b)
            # the packed two-strand fields (scan_mfma.hip): V = q8 + 1023 - t8 in [0, 2048)
            assert -1024 < b["t8"] <= 0 and 0 <= b["q8"] + 1023 - b["t8"] < 2048, (trial, x, b)
            if sc > ms:
                hits += 1
                assert b["q8"] > b["t8"], (trial, x, sc, ms, b)
            checked += 1
    assert checked > 9000 and hits > 100


def test_mfma_bound_eligibility():
    """Strands whose window sums could wrap i32 (the reference wraps, pattern.rs:125-135)
    and strands longer than 32 stay off the matrix-core path."""
    wrap = [T.Weight(2**30, 0, 0, 0)] * 2
    ok = [T.Weight(2**29, 0, 0, 0)] * 3
    long_ = [T.Weight(1, 0, 0, 0)] * 33
    ps = T.PatternSet.from_patterns([T.Pattern.PWM(wrap, "w", 1, 0), T.Pattern.PWM(ok, "o", 2, 0),
                                     T.Pattern.PWM(long_, "l", 3, 0)])
    assert ps.mfma_bound(0, "AA")["eligible"] == 0
    assert ps.mfma_bound(1, "AAA")["eligible"] == 1
    assert ps.mfma_bound(2, "A" * 33)["eligible"] == 0


@pytest.mark.parametrize("indel", [0, 30])
def test_prep_overlap_same_batch(tmp_path, indel, monkeypatch):
    """tfbs_synth_fill_batch commits chunk k while it builds chunk k + 1 (build_regions and
    commit_regions on two threads, disjoint Batch fields: batch.hpp).  The packed batch must
    not depend on it: every region's input digest and stats with the overlap on equal the
    serial order's (TFBS_PREP_OVERLAP=0).  Two host threads make 128-region chunks, so 300
    regions take three chunks and two overlapped commits."""
    ps, _ = synth_patterns(str(tmp_path), 12, 3, 5)
    monkeypatch.setenv("TFBS_HOST_THREADS", "2")
    got = {}
    for ov in ("0", "1"):
        monkeypatch.setenv("TFBS_PREP_OVERLAP", ov)
        b = T.RegionBatch(ps, 400, keep_membership=True)
        b.synth_fill(7, 0, 300, indel)
        got[ov] = (b.num_regions, b.num_windows, b.num_effective_windows,
                   [(b.region_stats(r), b.input_digest(r)) for r in range(b.num_regions)])
    assert got["0"][0] == 300
    assert got["0"] == got["1"]
