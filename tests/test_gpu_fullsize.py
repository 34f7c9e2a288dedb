"""GPU parity at the BASELINE.json sizes.

The batch the bench times is scanned here exactly as bench.py builds it (same
generator, seeds, PWM sets and thresholds), and checked three ways:

* against the oracle (oracle/tfbs_oracle.c, the C restatement of main.rs:94-154,
  500-534 and 439-498): every region of C2, and for C3/C5 >= 1 000 regions (a
  deterministic spread: first, last, the last haplotype group, evenly spaced
  ones; the 50 with the most distinct haplotypes and the 50 with the most
  variant records -- C5's indel-dense ones --; every region with N runs) key
  by key -- the per-sample L/R vectors of count_matches_by_sample -- and row by
  row (POS aside: the oracle numbers rows over its own region subset), in full
  on 100 of them and through xxh3 digests of the same on the rest;
* the device per-sample encoding (tfbs_batch_encode: the rows formatted from
  per-sample codes) against the oracle on the same regions;
* device key reduction (the run flow's tfbs_batch_reduce) against the dense
  count download over the WHOLE batch, region by region, through
  tfbs_batch_region_digest (keys + every distinct haplotype's count);
* C4: 100 000 regions scanned as one batch (a 28 GB count matrix: u64 count
  offsets) and as 8 static region shards of 12 500 (the multi-GPU partition,
  SURVEY.md 8(e)), run one after the other on this GPU: identical digests for
  every region, and the oracle on a spread of regions of every shard.

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
from helpers import T, pattern_dicts

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


def _fullsize(tmp_path, cfg, n_check, n_extra_n=0, n_top=0, build_device=None):
    """n_check regions spread over the batch (all of them if n_check >= its size), the
    n_top regions with the most distinct haplotypes and the n_top with the most
    variant records, and the n_extra_n regions with N runs, against the oracle:
    key by key and row by row on a 100-region subset, by xxh3 digests of the same
    (count_matches_by_sample vectors of every key after the key reduction, row
    text after the device encoding) on all of them.  build_device: the batch is
    grouped there as bench.py builds it (SNV-only regions' haplotypes grouped on
    the GPU); the 100-region subset's rows are then also made as BGZF blocks on
    the device (tfbs_batch_rows_bgzf), inflated and compared with the oracle's."""
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
    sc = T.Scanner(ps)
    try:
        # the run flow's path: device key reduction
        b.scan(sc, reduce=True)
        reduced = _digests(b)
        check = set(_spread(n_regions, n_check) if n_check < n_regions else range(n_regions))
        if n_top:
            st = [b.region_stats(i) for i in range(n_regions)]
            check |= set(sorted(range(n_regions), key=lambda i: -st[i][0])[:n_top])
            check |= set(sorted(range(n_regions), key=lambda i: -st[i][1])[:n_top])
        check = sorted(check)
        full = set(check) if len(check) <= 100 else {check[i] for i in _spread(len(check), 100)}
        jobs = _synth_jobs(seed, check, n_samples, lmax, indel)
        jobs += [(n_regions + k, r["merged"], r["ref"], r["records"]) for k, r in enumerate(extra)]
        full |= {n_regions + k for k in range(len(extra))}
        ref = _oracle_regions(ps, n_samples, seed, indel, [j for j in jobs if j[0] in full])
        dig = _oracle_regions(ps, n_samples, seed, indel, [j for j in jobs if j[0] not in full], digest=True)
        # the device key reduction: every checked region's keys (rows in full on the subset)
        n_full = _check_vs_oracle(b, ref, "reduce")
        _check_vs_oracle(b, dig, "reduce", digest=True, rows=False)
        # the device per-sample encoding (f1) the run flow formats rows from, 2 000
        # regions at a time: every checked region's rows
        n_enc = n_rows = n_bgzf = 0
        for r0 in range(0, b.num_regions, 2000):
            r1 = min(b.num_regions, r0 + 2000)
            b.encode(sc, r0, r1)
            n_enc += _check_vs_oracle(b, {i: ref[i] for i in ref if r0 <= i < r1}, "encode", keys=False)
            n_rows += _check_vs_oracle(b, {i: dig[i] for i in dig if r0 <= i < r1}, "encode", digest=True, keys=False)
            if build_device is not None:  # the device BGZF writer's rows of the subset vs the oracle's
                import gzip
                for i in sorted(x for x in ref if r0 <= x < r1):
                    data, _, nr, _ = b.rows_bgzf(sc, "chr1", 0, 1, i, i + 1)
                    got = _strip_pos(gzip.decompress(data).decode()) if data else []
                    assert got == ref[i][1], ("bgzf", i)
                    n_bgzf += nr
        assert n_enc == n_full
        if build_device is not None:
            assert n_bgzf == n_full
        n_rows += n_enc
        # dense download over the same batch, rescanned
        b.scan(sc, upload=False, download=True)
        assert _digests(b) == reduced
        _check_vs_oracle(b, {i: ref[i] for i in list(ref)[:24]}, "dense")
    finally:
        sc.close()
    return b, n_rows, len(ref) + len(dig)


def test_c2_full_vs_oracle(tmp_path):
    """C2 in full: 1 000 samples x 1 000 regions x 10 PWMs, every region vs the oracle."""
    b, n_rows, n_checked = _fullsize(tmp_path, C2, C2[1])
    assert n_checked == C2[1] and n_rows > 100


def test_c3_full_batch_vs_oracle(tmp_path):
    """C3 as bench.py times it (50 000 samples, 10 000 regions, 600 PWMs = 1 200 strands,
    ~1.18 M distinct haplotypes, one batch, SNV-only regions grouped on the GPU), plus
    6 regions with N runs at its end (built on the host); the device BGZF rows of the
    100-region subset against the oracle's."""
    b, n_rows, n_checked = _fullsize(tmp_path, C3, 1000, n_extra_n=6, n_top=50, build_device=0)
    assert n_checked >= 1000 and n_rows > 0
    assert b.num_haplotypes > 1_000_000


def test_c5_full_batch_vs_oracle(tmp_path):
    """C5: C3 with 30 % indels (non-affine positions, variable-length haplotypes) and
    PWMs of length 25-30 (K depth 2 of the matrix-core kernel)."""
    b, n_rows, n_checked = _fullsize(tmp_path, C5, 1000, n_extra_n=4, n_top=50, build_device=0)
    assert n_checked >= 1000 and n_rows > 0


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
        got, checked = [], 0
        for k in range(n_shards):
            r0, r1 = k * n_regions // n_shards, (k + 1) * n_regions // n_shards
            b = T.RegionBatch(ps, n_samples)
            b.synth_fill(seed, r0, r1 - r0, indel)
            b.scan(sc, reduce=True)
            got += _digests(b)
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
        assert checked >= 40
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
