"""Device haplotype grouping (tfbs_batch_set_build_device; haplotype.rs:16-88 on the
GPU, build_gpu.hip): SNV-only regions are grouped and patched from the device's
masks; regions with indels, N in the window, diffs outside it or two records at
one position are grouped on the device and only their distinct groups patched on
the host (batch.cpp mask_finish, with HashMap::insert's collision rule).  A batch
built so must be the batch the host builds -- per region the same distinct
haplotypes in the same order, packed bases, carrier counts, reference group,
keys and membership (tfbs_batch_region_input_digest), the same scan statistics
(reference-window reuse masks included) -- and scan to the same keys and rows.
Regions the device does not take (unsorted carriers, a repeated diff, more than 64
applied records or 2047 distinct diff masks) are built on the host in the same
batch."""
import os
import random

import pytest

from helpers import T, build_batch, make_regions_synth, synth_patterns

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if T.device_count() == 0:
        pytest.fail("gpu test without a visible HIP device")


def _same_batches(host, dev):
    assert dev.num_regions == host.num_regions
    for r in range(host.num_regions):
        assert dev.input_digest(r) == host.input_digest(r), r
    assert dev.num_haplotypes == host.num_haplotypes
    assert dev.num_windows == host.num_windows
    assert dev.num_effective_windows == host.num_effective_windows
    assert dev.num_scan_windows == host.num_scan_windows


def _c3_patterns(tmp_path):
    names = T.synth_write_pwms(str(tmp_path), 600, 3, 3)
    return T.parse_pwm_files(os.path.join(str(tmp_path), "pwms.txt"), os.path.join(str(tmp_path), "thr"), 1e-4, names)


def test_device_grouping_c3_batch(tmp_path):
    """The C3 generator (50 000 samples, SNVs only): 300 regions grouped on the device ==
    the host build, scanned to the same keys and rows."""
    ps = _c3_patterns(tmp_path)
    host = T.RegionBatch(ps, 50000)
    host.synth_fill(3, 0, 300, 0)
    dev = T.RegionBatch(ps, 50000, build_device=0)
    dev.synth_fill(3, 0, 300, 0)
    nd, nh = dev.build_stats()
    assert (nd, nh) == (300, 0), (nd, nh)
    _same_batches(host, dev)
    sc = T.Scanner(ps)
    try:
        host.scan(sc, reduce=True)
        want = [host.key_digest_sum(r) for r in range(300)]
        dev.scan(sc, reduce=True)
        assert [dev.key_digest_sum(r) for r in range(300)] == want
        del host, dev
        # rows (~14 MB of text per region) of a dozen regions
        host = T.RegionBatch(ps, 50000)
        host.synth_fill(3, 1000, 12, 0)
        dev = T.RegionBatch(ps, 50000, build_device=0)
        dev.synth_fill(3, 1000, 12, 0)
        host.scan(sc, reduce=True)
        want_rows, _ = host.rows("chr1")
        dev.scan(sc, reduce=True)
        got_rows, _ = dev.rows("chr1")  # membership fetched from the device
        assert got_rows == want_rows
        dev.scan(sc, reduce=True, encode=True)  # pair tables from the device membership
        got_rows, _ = dev.rows("chr1")
        assert got_rows == want_rows
    finally:
        sc.close()


@pytest.mark.parametrize("dev_patch", ["1", "0"])
def test_device_grouping_indels_mixed(tmp_path, monkeypatch, dev_patch):
    """C5-like regions (3 % indels: about half the regions have one): every region grouped
    on the device, the indel ones patched on the host; with TFBS_DEV_PATCH=0 the SNV-only
    ones on the device and the rest built on the host."""
    monkeypatch.setenv("TFBS_DEV_PATCH", dev_patch)
    ps, _ = synth_patterns(tmp_path, 12, 5, 105, thr=1e-3)
    host = T.RegionBatch(ps, 2000)
    host.synth_fill(5, 0, 120, 3)
    dev = T.RegionBatch(ps, 2000, build_device=0)
    dev.synth_fill(5, 0, 120, 3)
    nd, nh = dev.build_stats()
    if dev_patch == "1":
        assert (nd, nh) == (120, 0), (nd, nh)
    else:
        assert nd > 0 and nh > 0, (nd, nh)
    _same_batches(host, dev)
    sc = T.Scanner(ps)
    try:
        host.scan(sc, reduce=True, encode=True)
        want, _ = host.rows("chr1")
        dev.scan(sc, reduce=True, encode=True)
        got, _ = dev.rows("chr1")
    finally:
        sc.close()
    assert got == want


def _edge_regions(n_samples, lmax):
    """One region per case; each built through the region API."""
    rnd = random.Random(7)
    H = 2 * n_samples
    regs = []

    def base(j):
        r = T.SynthRegion(91, j, n_samples, lmax)
        s, e = r.merged
        return r.ref, (s, e), s - lmax + 1

    def snv(ref, es, p, car):
        rb = ref[p]
        return ("car", es + p, rb, rnd.choice([c for c in "ACGT" if c != rb]), car)

    # 0: plain SNVs, random carriers (device)
    ref, m, es = base(0)
    regs.append({"merged": m, "ref": ref,
                 "records": [snv(ref, es, p, sorted(rnd.sample(range(H), rnd.randint(1, H // 3))))
                             for p in sorted(rnd.sample(range(len(ref)), 12))]})
    # 1: no records at all (device: one group, the reference)
    ref, m, es = base(1)
    regs.append({"merged": m, "ref": ref, "records": []})
    # 2: every haplotype carries a variant (no reference group: a helper copy)
    ref, m, es = base(2)
    ps_ = sorted(rnd.sample(range(len(ref)), 2))
    regs.append({"merged": m, "ref": ref, "records": [snv(ref, es, ps_[0], list(range(0, H, 2))),
                                                      snv(ref, es, ps_[1], list(range(1, H, 2)))]})
    # 3: two records at one position (host)
    ref, m, es = base(3)
    p = len(ref) // 2
    alts = [c for c in "ACGT" if c != ref[p]]
    regs.append({"merged": m, "ref": ref, "records": [("car", es + p, ref[p], alts[0], [0, 5, 9]),
                                                      ("car", es + p, ref[p], alts[1], [1, 6])]})
    # 4: carriers out of order (host)
    ref, m, es = base(4)
    regs.append({"merged": m, "ref": ref, "records": [snv(ref, es, 10, [7, 3, 11]), snv(ref, es, 20, [2, 4])]})
    # 5: an N in the window (host)
    ref, m, es = base(5)
    ref = ref[:30] + "N" + ref[31:]
    regs.append({"merged": m, "ref": ref, "records": [snv(ref, es, 10, [1, 2, 3])]})
    # 6: more than 2047 distinct diff masks (host): 14 SNVs, each on half the haplotypes
    ref, m, es = base(6)
    regs.append({"merged": m, "ref": ref,
                 "records": [snv(ref, es, p, sorted(rnd.sample(range(H), H // 2)))
                             for p in sorted(rnd.sample(range(len(ref)), 14))]})
    # 7: an insertion among SNVs (host), 8: a multi-allelic record among SNVs (device: not applied)
    ref, m, es = base(7)
    regs.append({"merged": m, "ref": ref, "records": [snv(ref, es, 5, [0, 1]),
                                                      ("car", es + 9, ref[9], ref[9] + "AC", [2, 3])]})
    ref, m, es = base(8)
    regs.append({"merged": m, "ref": ref, "records": [snv(ref, es, 5, [0, 3, 8]),
                                                      ("gt", es + 12, 3, ref[12], "A", [[4, 5]] * n_samples)]})
    # 9: 64 SNVs (the widest mask) on the device, 10: 65 (host)
    for j, ns in ((9, 64), (10, 65)):
        ref, m, es = base(j)
        regs.append({"merged": m, "ref": ref,
                     "records": [snv(ref, es, p, sorted(rnd.sample(range(H), 2)))
                                 for p in sorted(rnd.sample(range(len(ref)), ns))]})
    # 11: a collision (device grouping, host patch): a deletion starting before the
    # window (patch_haplotype drops it, haplotype.rs:95) on haplotypes {0, 1}, an SNV on
    # {0, 2}: the groups [del, snv] and [snv] patch to one sequence, [snv] (later in
    # Vec<Diff> order) wins and haplotype 0 joins the reference group
    ref, m, es = base(11)
    regs.append({"merged": m, "ref": ref, "records": [("car", es - 2, "AC", "A", [0, 1]),
                                                      snv(ref, es, 40, [0, 2])]})
    # 12: an insertion and a deletion on one haplotype, a deletion over the window's end
    ref, m, es = base(12)
    n = len(ref)
    regs.append({"merged": m, "ref": ref, "records": [("car", es + 9, ref[9], ref[9] + "GT", [3, 4, 5]),
                                                      ("car", es + 30, ref[30:33], ref[30], [4, 6]),
                                                      ("car", es + n - 2, ref[n - 2:], ref[n - 2], [7])]})
    return regs


def test_device_grouping_edge_cases(tmp_path):
    ps, _ = synth_patterns(tmp_path, 8, 2, 106, thr=1e-3)
    n_samples = 1500
    regions = _edge_regions(n_samples, ps.max_length)
    beds = [("synthetic.bed", [reg["merged"] for reg in regions])]
    host = build_batch(ps, n_samples, beds, regions)
    dev = T.RegionBatch(ps, n_samples, build_device=0)
    for name, _ in beds:
        dev.add_bed(name)
    for reg in regions:
        s, e = reg["merged"]
        dev.begin(s, e, reg["ref"])
        for (bi, a, z) in T.select_inner_peaks((s, e), beds):
            dev.add_inner(bi, a, z)
        for rec in reg["records"]:
            if rec[0] == "car":
                dev.add_record_carriers(rec[1], rec[2], rec[3], rec[4])
            else:
                dev.add_record_gt(rec[1], rec[2], rec[3], rec[4], rec[5])
        dev.end()
    nd, nh = dev.build_stats()
    assert (nd, nh) == (10, 3), (nd, nh)  # on the host: 4 (unsorted carriers), 6 (masks), 10 (65 records)
    _same_batches(host, dev)
    sc = T.Scanner(ps)
    try:
        host.scan(sc, reduce=True, encode=True)
        want, _ = host.rows("chr1")
        want_keys = [host.keys(i) for i in range(host.num_regions)]
        dev.scan(sc, reduce=True, encode=True)
        got, _ = dev.rows("chr1")
        got_keys = [dev.keys(i) for i in range(dev.num_regions)]
    finally:
        sc.close()
    assert got_keys == want_keys
    assert got == want


def test_device_grouping_ref_mismatch_fails_like_host(tmp_path):
    """A REF base that is not the window's: the host build's error (haplotype.rs:108-111)."""
    ps, _ = synth_patterns(tmp_path, 4, 2, 107, thr=1e-3)
    r = T.SynthRegion(5, 0, 10, ps.max_length)
    s, e = r.merged
    es = s - ps.max_length + 1
    wrong = [c for c in "ACGT" if c != r.ref[7]][0]
    for dev in (None, 0):
        b = T.RegionBatch(ps, 10, build_device=dev)
        b.add_bed("x.bed")
        b.begin(s, e, r.ref)
        b.add_inner(0, s, e)
        b.add_record_carriers(es + 7, wrong, "A" if wrong != "A" else "C", [1, 2])
        with pytest.raises(T.TfbsError, match="doesn't match"):
            b.end()
