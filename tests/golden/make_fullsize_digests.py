"""Oracle digests of every region of the full-size workloads, for tests/test_gpu_fullsize.py.

TEST INFRASTRUCTURE: runs the CPU oracle (oracle/tfbs_oracle.c, the C restatement of
main.rs:94-154, 395-534 and haplotype.rs:13-156) over the same synthetic regions bench.py
times (the product's deterministic generator, SURVEY.md 8(d): C3 and C5 in full, 10 000
regions each; C4 a spread of 10 000+ of its 100 000, 1 250+ per shard of 12 500) and writes per region

  keys[i]   the oracle's orc_job_digests key sketch (count_matches_by_sample vectors),
  rows[i]   XXH64 of the region's rows without POS,
  n_rows[i] their number,

to tests/golden/fullsize_<W>.npz (plain uint64 arrays: numpy.load needs no pickle).
The GPU test computes the same digests from the product (tfbs_batch_region_digests)
and compares every region.  Run in the build container (no GPU needed):

    python3 tests/golden/make_fullsize_digests.py C3 C5 C4 [--threads 8]
"""
import argparse
import concurrent.futures as cf
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_py as O  # noqa: E402
from helpers import T, pattern_dicts  # noqa: E402

# workload: (samples, regions, pwms, length_config, indel_pct, seed) -- as tests/test_gpu_fullsize.py
WORKLOADS = {
    "C3": (50000, 10000, 600, 3, 0, 3),
    "C4": (50000, 100000, 600, 3, 0, 4),
    "C5": (50000, 10000, 600, 5, 30, 5),
}


def spread(n, count):
    """~count region indices over [0, n): both ends and even spacing (C4's checked set)."""
    idx = set(range(0, 8)) | set(range(max(0, n - 12), n))
    step = max(1, n // max(1, count - len(idx)))
    idx |= set(range(0, n, step))
    return sorted(i for i in idx if i < n)


def region_indices(name):
    n = WORKLOADS[name][1]
    return spread(n, 10000) if name == "C4" else list(range(n))


def golden_path(name):
    return os.path.join(HERE, "fullsize_%s.npz" % name)


def make(name, threads):
    n_samples, n_regions, n_pwms, lc, indel, seed = WORKLOADS[name]
    with tempfile.TemporaryDirectory() as tmp:
        names = T.synth_write_pwms(tmp, n_pwms, lc, seed)
        ps = T.parse_pwm_files(os.path.join(tmp, "pwms.txt"), os.path.join(tmp, "thr"), 1e-4, names)
    pats = pattern_dicts(ps)
    lmax = ps.max_length
    idx = region_indices(name)
    keys = np.zeros(len(idx), dtype=np.uint64)
    rows = np.zeros(len(idx), dtype=np.uint64)
    nrows = np.zeros(len(idx), dtype=np.uint64)
    # every thread's job covers all merged ranges of the synthetic BED (inner peaks select
    # by overlap, main.rs:62-72), as the product's synthetic batch registers them
    ranges = sorted({tuple(T.SynthRegion(seed, j, n_samples, lmax, indel).merged) for j in idx})

    def work(part):
        job = O.Job(n_samples, "chr1", pats, [("synthetic.bed", ranges)])
        try:
            for q in part:
                r = T.SynthRegion(seed, idx[q], n_samples, lmax, indel)
                assert job.begin(r.merged[0], r.merged[1], r.ref) == 0
                for pos, rf, alt, car in r.records:
                    assert job.add_record_carriers(pos, rf, alt, car) == 0
                assert job.end() == 0
                keys[q], rows[q], nrows[q] = job.digests()
                job.clear_rows()
        finally:
            job.close()

    t0 = time.time()
    parts = [list(range(k, len(idx), threads)) for k in range(threads)]
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, parts))
    np.savez(golden_path(name), regions=np.asarray(idx, dtype=np.uint64), keys=keys, rows=rows, n_rows=nrows,
             config=np.asarray(WORKLOADS[name], dtype=np.uint64))
    print("%s: %d regions, %d rows, %.0f s" % (name, len(idx), int(nrows.sum()), time.time() - t0), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="+", choices=sorted(WORKLOADS))
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    for w in a.workloads:
        make(w, a.threads)


if __name__ == "__main__":
    main()
