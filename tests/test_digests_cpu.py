"""The full-size golden digests (tests/golden/fullsize_<W>.npz) and the function that
makes them (the oracle's orc_job_digests), on the CPU.

* orc_xxh64 is XXH64: python's xxhash on random inputs of every length class.
* orc_job_digests is what its header says: recomputed here from the oracle's own
  per-sample vectors (keys_np: a linear sketch with splitmix64 weights) and from its
  row text (XXH64 of the rows with the POS field removed), on C2-shaped regions.
* The golden files cover what tests/test_gpu_fullsize.py checks: every C3 / C5
  region, 1 000+ C4 regions, the workload configuration recorded beside them, and
  they load without pickle.
"""
import os
import tempfile

import numpy as np
import pytest
import xxhash

import oracle_py as O
from helpers import GOLD, T, pattern_dicts

M64 = (1 << 64) - 1


def _splitmix(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _mix(h, x):
    h ^= (x + 0x9E3779B97F4A7C15 + ((h << 6) & M64) + (h >> 2)) & M64
    h = (h * 0xFF51AFD7ED558CCD) & M64
    return h ^ (h >> 33)


def test_oracle_xxh64_is_xxh64():
    L = O.lib()
    rnd = np.random.default_rng(5)
    for n in list(range(0, 70)) + [100, 1000, 4097]:
        b = rnd.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 12345):
            assert L.orc_xxh64(b, n, seed) == xxhash.xxh64(b, seed=seed).intdigest(), (n, seed)


def test_oracle_region_digests_recomputed():
    n_samples, seed = 1000, 2
    with tempfile.TemporaryDirectory() as tmp:
        names = T.synth_write_pwms(tmp, 10, 2, seed)
        ps = T.parse_pwm_files(os.path.join(tmp, "pwms.txt"), os.path.join(tmp, "thr"), 1e-4, names)
    regs = [T.SynthRegion(seed, j, n_samples, ps.max_length, 0) for j in range(30)]
    job = O.Job(n_samples, "chr1", pattern_dicts(ps), [("synthetic.bed", sorted({tuple(r.merged) for r in regs}))])
    w = np.array([_splitmix(h) for h in range(2 * n_samples)], dtype=np.uint64)
    total_rows = 0
    try:
        for r in regs:
            assert job.begin(r.merged[0], r.merged[1], r.ref) == 0
            for pos, rf, alt, car in r.records:
                assert job.add_record_carriers(pos, rf, alt, car) == 0
            assert job.end() == 0
            k, rw, nr = job.digests()
            s = 0
            for (_, (a, b), pid), (lv, rv) in job.keys_np().items():
                with np.errstate(over="ignore"):
                    S = int((lv.astype(np.uint64) * w[0::2]).sum() + (rv.astype(np.uint64) * w[1::2]).sum())
                h = 0x2545F4914F6CDD1D
                for x in (0, a, b, pid, S & M64):
                    h = _mix(h, x)
                s = (s + h) & M64
            x = xxhash.xxh64()
            rows = job.rows().splitlines(True)
            for line in rows:
                x.update(line.split("\t", 2)[2].encode())
            assert (k, rw, nr) == (s, x.intdigest(), len(rows))
            total_rows += nr
            job.clear_rows()
    finally:
        job.close()
    assert total_rows > 5


@pytest.mark.parametrize("name,config,n_min", [
    ("C3", (50000, 10000, 600, 3, 0, 3), 10000),
    ("C5", (50000, 10000, 600, 5, 30, 5), 10000),
    ("C4", (50000, 100000, 600, 3, 0, 4), 1000),
])
def test_golden_fullsize_files(name, config, n_min):
    g = np.load(os.path.join(GOLD, "fullsize_%s.npz" % name))  # allow_pickle=False (the default)
    assert tuple(int(x) for x in g["config"]) == config
    n = len(g["regions"])
    assert n >= n_min and all(len(g[k]) == n for k in ("keys", "rows", "n_rows"))
    if name != "C4":
        assert list(g["regions"]) == list(range(config[1]))
    assert int(g["n_rows"].sum()) > 10 * n  # tens of varying keys per region at 50 000 samples
    assert len(set(g["keys"].tolist())) == n  # no two regions share a key sketch
