"""GPU parity at the BASELINE.json sizes.

The batch the bench times is scanned here exactly as bench.py builds it (same
generator, seeds, PWM sets and thresholds), and checked three ways:

* against the oracle (oracle/tfbs_oracle.c, the C restatement of main.rs:94-154,
  500-534 and 439-498): every region of C3 and C5 (10 000 each) and a spread of
  10 000+ C4 regions (1 250+ per shard) through the oracle's committed per-region digests
  (tests/golden/fullsize_<W>.npz, tests/golden/make_fullsize_digests.py: a linear
  sketch of count_matches_by_sample's per-sample L/R vectors and XXH64 of the row
  text without POS); every region of C2, and ~125 C3/C5 regions (a spread, the
  10 with the most distinct haplotypes, the 10 with the most variant records --
  C5's indel-dense ones --, every region with N runs) against the live oracle key
  by key and row by row (POS aside: the oracle numbers rows over its own subset);
* the device per-sample encoding (tfbs_batch_encode: the rows formatted from
  per-sample codes) against the oracle on the same regions;
* device key reduction (the run flow's tfbs_batch_reduce) against the dense
  count download over the WHOLE batch, region by region, through
  tfbs_batch_region_digest (keys + every distinct haplotype's count);
* C4: 100 000 regions scanned as one batch (a 28 GB count matrix: u64 count
  offsets) and as 8 static region shards of 12 500 (the multi-GPU partition,
  SURVEY.md 8(e)), run one after the other on this GPU: identical digests for
  every region, the golden oracle digests on the spread and the live oracle on
  a few regions of every shard.

C2/C3 carry no N in the reference (the generator draws ACGT only); the C3
batch gets extra regions whose reference holds N runs (appended after the
generator's regions, so they sit in the last haplotype groups).
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest
import xxhash

import oracle_py as O
from helpers import GOLD, T, pattern_dicts

pytestmark = pytest.mark.gpu

# workload: (samples, regions, pwms, length_config, indel_pct, seed) -- SURVEY.md 8(d)
C2 = (1000, 1000, 10, 2, 0, 2)
C3 = (50000, 10000, 600, 3, 0, 3)
C4 = (50000, 100000, 600, 3, 0, 4)
C5 = (50000, 10000, 600, 5, 30, 5)
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if T.device_count() == 0:
        pytest.fail("gpu test without a visible HIP device")


def _patterns(tmp, cfg):
    n_samples, n_regions, n_pwms, lc, indel, seed = cfg
    names = T.synth_write_pwms(str(tmp), n_pwms, lc, seed)
    return T.parse_pwm_files(os.path.join(str(tmp), "pwms.txt"), os.path.join(str(tmp), "thr"), 1e-4, names)


def _n_regions(seed, first, count, n_samples, lmax, indel):
    """Regions after the generator's: its region + N runs in the reference (none over
    a variant's REF bases, which patch_haplotype checks, haplotype.rs:119-128)."""
    out = []
    for j in range(first, first + count):
        r = T.SynthRegion(seed, j, n_samples, lmax, indel)
        ref = list(r.ref)
        busy = set()
        for pos, rf, _, _ in r.records:
            busy.update(range(pos - r.ext_start, pos - r.ext_start + len(rf)))
        k = j - first
        for a, z in [(3 + 7 * k, 6 + 7 * k), (100 + k, 101 + k), (len(ref) - 9, len(ref) - 5)]:
            for i in range(a, min(z, len(ref))):
                if i not in busy:
                    ref[i] = "N"
        out.append({"merged": r.merged, "ref": "".join(ref), "records": r.records})
    return out


def _append_regions(b, regions):
    bed = b.beds.index("synthetic.bed")
    for reg in regions:
        s, e = reg["merged"]
        b.begin(s, e, reg["ref"])
        b.add_inner(bed, s, e)
        for pos, ref, alt, car in reg["records"]:
            b.add_record_carriers(pos, ref, alt, car)
        b.end()


def _strip_pos(rows):
    out = []
    for line in rows.splitlines():
        f = line.split("\t", 2)
        out.append(f[0] + "\t" + f[2])
    return out


def _keys_digest(keys):
    """xxh3 over a region's count_matches_by_sample map: key identity + both vectors."""
    h = xxhash.xxh3_64()
    for k in sorted(keys):
        h.update(repr(k).encode())
        h.update(np.ascontiguousarray(keys[k][0], dtype=np.uint32).tobytes())
        h.update(np.ascontiguousarray(keys[k][1], dtype=np.uint32).tobytes())
    return h.hexdigest()


def _rows_digest(rows):
    h = xxhash.xxh3_64()
    for r in rows:
        h.update(r.encode())
        h.update(b"\n")
    return h.hexdigest()


def _oracle_regions(ps, n_samples, seed, indel, jobs, digest=False):
    """jobs: [(product region index, merged, ref, records)] -> {index: (keys, rows)} on
    host threads (ctypes drops the GIL), one oracle Job per thread; digest=True keeps
    only sha1 digests of both (wide spreads at 50 000 samples)."""
    pats = pattern_dicts(ps)
    ranges = sorted({tuple(j[1]) for j in jobs})

    def work(chunk):
        job = O.Job(n_samples, "chr1", pats, [("synthetic.bed", ranges)])
        res = {}
        try:
            for idx, merged, ref, recs in chunk:
                assert job.begin(merged[0], merged[1], ref) == 0
                for pos, rf, alt, car in recs:
                    assert job.add_record_carriers(pos, rf, alt, car) == 0
                assert job.end() == 0
                keys, rows = job.keys_np(), _strip_pos(job.rows())
                res[idx] = (_keys_digest(keys), _rows_digest(rows)) if digest else (keys, rows)
                job.clear_rows()
        finally:
            job.close()
        return res

    n = max(1, min(THREADS, len(jobs)))
    chunks = [jobs[i::n] for i in range(n)]
    out = {}
    with cf.ThreadPoolExecutor(n) as ex:
        for r in ex.map(work, chunks):
            out.update(r)
    return out


def _synth_jobs(seed, indices, n_samples, lmax, indel):
    jobs = []
    for j in indices:
        r = T.SynthRegion(seed, j, n_samples, lmax, indel)
        jobs.append((j, r.merged, r.ref, r.records))
    return jobs


def _check_vs_oracle(b, ref, label, digest=False, keys=True, rows=True):
    """b: scanned batch (counts present); ref: {region: (oracle keys, oracle rows)}, or
    their _keys_digest / _rows_digest (digest=True); keys / rows: which to compare."""
    n_rows = 0
    for idx in sorted(ref):
        okeys, orows = ref[idx]
        if keys:
            pkeys = b.keys_np(idx)
            if digest:
                assert _keys_digest(pkeys) == okeys, (label, idx)
            else:
                assert pkeys.keys() == okeys.keys(), (label, idx)
                for k in okeys:
                    assert np.array_equal(pkeys[k][0], okeys[k][0]) and np.array_equal(pkeys[k][1], okeys[k][1]), \
                        (label, idx, k)
        if rows:
            prows = _strip_pos(b.region_rows(idx, "chr1")[0])
            assert (_rows_digest(prows) if digest else prows) == orows, (label, idx)
            n_rows += len(prows)
    return n_rows


def _spread(n, count):
    """~count region indices over [0, n): both ends, the last haplotype groups, even spacing."""
    idx = set(range(0, 8)) | set(range(max(0, n - 12), n))
    step = max(1, n // max(1, count - len(idx)))
    idx |= set(range(0, n, step))
    return sorted(i for i in idx if i < n)


def _digests(b):
    return [b.digest(r) for r in range(b.num_regions)]


def _golden(name, cfg):
    """The oracle's per-region digests of workload `name` (tests/golden/make_fullsize_digests.py)."""
    g = np.load(os.path.join(GOLD, "fullsize_%s.npz" % name))
    assert tuple(int(x) for x in g["config"]) == cfg, ("golden file for another configuration", name)
    return g


def _check_golden(label, want_idx, want, got):
    bad = [int(i) for i, a, b in zip(want_idx, want, got) if a != b]
    assert not bad, (label, len(bad), bad[:10])


def _fullsize(tmp_path, cfg, n_full, golden=None, n_extra_n=0, n_top=0, build_device=None):
    """Every region of the batch against the oracle's golden digests (golden: the workload
    name; tests/golden/fullsize_<W>.npz, made by the oracle over the same generator): the
    canonical sketch of count_matches_by_sample's per-sample vectors after the device key
    reduction, and XXH64 of the row text after the device encoding (tfbs_batch_region_digests
    vs orc_job_digests).  Besides, against the live oracle key by key and row by row: ~n_full
    regions spread over the batch, the n_top regions with the most distinct haplotypes and
    the n_top with the most variant records (C5's indel-dense ones), and the n_extra_n regions
    with N runs appended after the generator's.  build_device: the batch is grouped there as
    bench.py builds it; those regions' rows are then also made as BGZF blocks on the device
    (tfbs_batch_rows_bgzf), inflated and compared with the oracle's.  Without golden digests
    (C2) every region is checked live."""
    n_samples, n_regions, _, _, indel, seed = cfg
    ps = _patterns(tmp_path, cfg)
    lmax = ps.max_length
    b = T.RegionBatch(ps, n_samples, build_device=build_device)
    b.synth_fill(seed, 0, n_regions, indel)
    if build_device is not None:
        dev_regions, _ = b.build_stats()
        assert dev_regions > n_regions // 2, dev_regions
    extra = _n_regions(seed, n_regions, n_extra_n, n_samples, lmax, indel) if n_extra_n else []
    _append_regions(b, extra)
    assert b.num_regions == n_regions + n_extra_n
    g = _golden(golden, cfg) if golden else None
    if g is not None:
        assert list(g["regions"]) == list(range(n_regions))
    sc = T.Scanner(ps)
    try:
        # the run flow's path: device key reduction
        b.scan(sc, reduce=True)
        reduced = _digests(b)
        n_golden = 0
        if g is not None:  # every region's keys vs the oracle
            keys, _, _ = b.region_digests(0, n_regions, threads=THREADS, rows=False)
            _check_golden("keys", range(n_regions), g["keys"], keys)
            n_golden = n_regions
        full = set(_spread(n_regions, n_full) if n_full < n_regions else range(n_regions))
        if n_top:
            st = [b.region_stats(i) for i in range(n_regions)]
            full |= set(sorted(range(n_regions), key=lambda i: -st[i][0])[:n_top])
            full |= set(sorted(range(n_regions), key=lambda i: -st[i][1])[:n_top])
        jobs = _synth_jobs(seed, sorted(full), n_samples, lmax, indel)
        jobs += [(n_regions + k, r["merged"], r["ref"], r["records"]) for k, r in enumerate(extra)]
        ref = _oracle_regions(ps, n_samples, seed, indel, jobs)
        # the device key reduction: every checked region's keys and rows in full
        n_full_rows = _check_vs_oracle(b, ref, "reduce")
        # the device per-sample encoding (f1) the run flow formats rows from, 2 000
        # regions at a time: every region's row digest, the live regions' text
        n_enc = n_rows = n_bgzf = 0
        for r0 in range(0, b.num_regions, 2000):
            r1 = min(b.num_regions, r0 + 2000)
            b.encode(sc, r0, r1)
            n_enc += _check_vs_oracle(b, {i: ref[i] for i in ref if r0 <= i < r1}, "encode", keys=False)
            if g is not None and r0 < n_regions:
                e1 = min(r1, n_regions)
                _, rows, nr = b.region_digests(r0, e1, threads=THREADS, keys=False)
                _check_golden("rows", range(r0, e1), g["rows"][r0:e1], rows)
                _check_golden("n_rows", range(r0, e1), g["n_rows"][r0:e1], nr)
                n_rows += int(nr.sum())
            if build_device is not None:  # the device BGZF writer's rows of the live regions vs the oracle's
                import gzip
                for i in sorted(x for x in ref if r0 <= x < r1):
                    data, _, nr, _ = b.rows_bgzf(sc, "chr1", 0, 1, i, i + 1)
                    got = _strip_pos(gzip.decompress(data).decode()) if data else []
                    assert got == ref[i][1], ("bgzf", i)
                    n_bgzf += nr
        assert n_enc == n_full_rows
        if build_device is not None:
            assert n_bgzf == n_full_rows
        # dense download over the same batch, rescanned
        b.scan(sc, upload=False, download=True)
        assert _digests(b) == reduced
        _check_vs_oracle(b, {i: ref[i] for i in list(ref)[:24]}, "dense")
    finally:
        sc.close()
    return b, n_rows + n_full_rows, n_golden, len(ref)


def test_c2_full_vs_oracle(tmp_path):
    """C2 in full: 1 000 samples x 1 000 regions x 10 PWMs, every region vs the live oracle."""
    b, n_rows, _, n_live = _fullsize(tmp_path, C2, C2[1])
    assert n_live == C2[1] and n_rows > 100


def test_c3_full_batch_vs_oracle(tmp_path):
    """C3 as bench.py times it (50 000 samples, 10 000 regions, 600 PWMs = 1 200 strands,
    ~1.18 M distinct haplotypes, one batch, SNV-only regions grouped on the GPU), plus
    6 regions with N runs at its end (built on the host); the device BGZF rows of the
    100-region subset against the oracle's."""
    b, n_rows, n_golden, n_live = _fullsize(tmp_path, C3, 100, "C3", n_extra_n=6, n_top=10, build_device=0)
    assert n_golden == C3[1] and n_live >= 100 and n_rows > 300_000
    assert b.num_haplotypes > 1_000_000


def test_c5_full_batch_vs_oracle(tmp_path):
    """C5: C3 with 30 % indels (non-affine positions, variable-length haplotypes) and
    PWMs of length 25-30 (K depth 2 of the matrix-core kernel)."""
    b, n_rows, n_golden, n_live = _fullsize(tmp_path, C5, 100, "C5", n_extra_n=4, n_top=10, build_device=0)
    assert n_golden == C5[1] and n_live >= 100 and n_rows > 0


def test_c4_shards_equal_unsharded(tmp_path):
    """C4: 100 000 regions as one batch vs 8 static shards of 12 500 (the multi-GPU
    partition, one after the other on this GPU): identical digests region by region;
    the oracle on a spread of every shard's regions."""
    n_samples, n_regions, _, _, indel, seed = C4
    ps = _patterns(tmp_path, C4)
    lmax = ps.max_length
    sc = T.Scanner(ps)
    try:
        whole = T.RegionBatch(ps, n_samples, keep_membership=False)
        whole.synth_fill(seed, 0, n_regions, indel)
        whole.scan(sc, reduce=True)
        want = _digests(whole)
        del whole
        n_shards = 8
        g = _golden("C4", C4)
        gidx = [int(i) for i in g["regions"]]
        got, checked, n_golden = [], 0, 0
        for k in range(n_shards):
            r0, r1 = k * n_regions // n_shards, (k + 1) * n_regions // n_shards
            b = T.RegionBatch(ps, n_samples)
            b.synth_fill(seed, r0, r1 - r0, indel)
            b.scan(sc, reduce=True)
            got += _digests(b)
            sel = [q for q, i in enumerate(gidx) if r0 <= i < r1]
            with cf.ThreadPoolExecutor(THREADS) as ex:  # one region per call (ctypes drops the GIL)
                dg = list(ex.map(lambda q: b.region_digests(gidx[q] - r0, gidx[q] - r0 + 1, threads=1), sel))
            for name, f in (("keys", 0), ("rows", 1), ("n_rows", 2)):
                _check_golden("C4 " + name, [gidx[q] for q in sel], g[name][sel], [d[f][0] for d in dg])
            n_golden += len(sel)
            local = [0, (r1 - r0) // 2, r1 - r0 - 1] + list(range(3, r1 - r0, (r1 - r0) // 5))
            jobs = [(i, m, rf, rc) for (i, m, rf, rc) in _synth_jobs(seed, [r0 + i for i in local], n_samples, lmax,
                                                                      indel)]
            jobs = [(i - r0, m, rf, rc) for (i, m, rf, rc) in jobs]
            ref = _oracle_regions(ps, n_samples, seed, indel, jobs)
            _check_vs_oracle(b, ref, "shard%d" % k)
            checked += len(ref)
            del b
        assert len(got) == len(want)
        bad = [i for i in range(n_regions) if got[i] != want[i]]
        assert not bad, bad[:10]
        assert checked >= 40 and n_golden == len(gidx) >= 1000
    finally:
        sc.close()


def test_c4_region_x_pwm_shards_sum_to_unsharded(tmp_path):
    """C4's 2-D split (bench.py --shard regions_x_pwms): one region block of the C4
    generator scanned with all 600 PWMs and as 2 pattern_id shards (both strands of a
    PWM together, the whole set's window L_max): per region the shards' order-free key
    digests add up to the unsharded digest, and their rows together are its rows."""
    import bench

    n_samples, _, _, _, indel, seed = C4
    n_regions = 3000
    rows_at = _spread(n_regions, 60)  # rows of 50 000 samples are 0.4 MB each: text on a spread
    ps = _patterns(tmp_path, C4)
    whole = T.RegionBatch(ps, n_samples)
    whole.synth_fill(seed, 0, n_regions, indel)
    sc = T.Scanner(ps)
    try:
        whole.scan(sc, reduce=True)
        want = [whole.key_digest_sum(r) for r in range(n_regions)]
        want_rows = [sorted(_strip_pos(whole.region_rows(r, "chr1")[0])) for r in rows_at]
    finally:
        sc.close()
    del whole
    got = [0] * n_regions
    got_rows = [[] for _ in rows_at]
    pids = []
    for part in range(2):
        sub = bench.shard_patterns(T, ps, part, 2)
        pids.append({p.pattern_id for p in sub.to_list()})
        b = T.RegionBatch(sub, n_samples, window_lmax=ps.max_length)
        b.synth_fill(seed, 0, n_regions, indel)
        sc = T.Scanner(sub)
        try:
            b.scan(sc, reduce=True)
            for r in range(n_regions):
                got[r] = (got[r] + b.key_digest_sum(r)) % (1 << 64)
            for q, r in enumerate(rows_at):
                got_rows[q] += _strip_pos(b.region_rows(r, "chr1")[0])
        finally:
            sc.close()
        del b
    assert not pids[0] & pids[1] and len(pids[0] | pids[1]) == 600
    bad = [r for r in range(n_regions) if got[r] != want[r]]
    assert not bad, bad[:10]
    assert [sorted(x) for x in got_rows] == want_rows
    assert sum(len(x) for x in want_rows) > 200


@pytest.mark.parametrize("cfg", [C2, (2000, 300, 40, 3, 30, 7)], ids=["C2", "indels"])
def test_step_graph_replays_equal_plain_steps(tmp_path, cfg):
    """tfbs_step (bench.py's step: scan + assembly + wait; from the third step alike on
    one hipGraph replay of the scan's and the assembly's launches) gives exactly the
    keys of plain tfbs_scan + tfbs_batch_reduce, after several replays, on C2 and on a
    batch with indels; a new upload of another batch does not replay the old graph."""
    n_samples, n_regions, _, _, indel, seed = cfg
    ps = _patterns(tmp_path, cfg)
    sc = T.Scanner(ps)
    L = T.lib()
    try:
        b = T.RegionBatch(ps, n_samples, keep_membership=False)
        b.synth_fill(seed, 0, n_regions, indel)
        b.scan(sc, reduce=True)
        want = _digests(b)
        for _ in range(6):
            T.check(L.tfbs_step(sc.h, b.h))
        T.check(L.tfbs_batch_reduce(sc.h, b.h))
        assert _digests(b) == want
        b2 = T.RegionBatch(ps, n_samples, keep_membership=False)
        b2.synth_fill(seed + 1, 0, n_regions // 2, indel)
        b2.scan(sc, reduce=True)
        want2 = _digests(b2)
        for _ in range(5):
            T.check(L.tfbs_step(sc.h, b2.h))
        T.check(L.tfbs_batch_reduce(sc.h, b2.h))
        assert _digests(b2) == want2
        T.check(L.tfbs_batch_upload(sc.h, b.h))  # back to the first batch: a new image, a new graph
        for _ in range(4):
            T.check(L.tfbs_step(sc.h, b.h))
        T.check(L.tfbs_batch_reduce(sc.h, b.h))
        assert _digests(b) == want
    finally:
        del sc
