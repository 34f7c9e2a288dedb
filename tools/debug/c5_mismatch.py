"""Which C5 regions' keys differ from the oracle's golden digests, under which build
switches (GPU).  Usage: python tools/debug/c5_mismatch.py [n_regions] -- prints per
variant the mismatching regions among the first n, and for the first one the keys
whose vectors differ (against the live oracle)."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(n, variant):
    import oracle_py as O
    from helpers import T, pattern_dicts
    g = np.load(os.path.join(ROOT, "tests/golden/fullsize_C5.npz"))
    n_samples, _, n_pwms, lc, indel, seed = (50000, 10000, 600, 5, 30, 5)
    tmp = tempfile.mkdtemp()
    names = T.synth_write_pwms(tmp, n_pwms, lc, seed)
    ps = T.parse_pwm_files(os.path.join(tmp, "pwms.txt"), os.path.join(tmp, "thr"), 1e-4, names)
    b = T.RegionBatch(ps, n_samples, build_device=None if variant == "host" else 0)
    b.synth_fill(seed, 0, n, indel)
    sc = T.Scanner(ps)
    b.scan(sc, reduce=True)
    keys, _, _ = b.region_digests(0, n, threads=16, rows=False)
    bad = [i for i in range(n) if int(keys[i]) != int(g["keys"][i])]
    print(variant, "mismatches", len(bad), bad[:40], flush=True)
    if bad and variant == "default":
        j = bad[0]
        pats = pattern_dicts(ps)
        r = T.SynthRegion(seed, j, n_samples, ps.max_length, indel)
        job = O.Job(n_samples, "chr1", pats, [("synthetic.bed", [tuple(r.merged)])])
        job.begin(r.merged[0], r.merged[1], r.ref)
        for pos, rf, alt, car in r.records:
            job.add_record_carriers(pos, rf, alt, car)
        job.end()
        ok = job.keys_np()
        pk = b.keys_np(j)
        print("region", j, "ext_start", r.ext_start, "len", len(r.ref), "records",
              [(p - r.ext_start, a, c, len(car)) for p, a, c, car in r.records])
        print("keys oracle", len(ok), "product", len(pk), "only oracle", len(set(ok) - set(pk)),
              "only product", len(set(pk) - set(ok)))
        nd = 0
        for k in sorted(set(ok) & set(pk)):
            dl = np.nonzero(ok[k][0] != pk[k][0])[0]
            dr = np.nonzero(ok[k][1] != pk[k][1])[0]
            if len(dl) or len(dr):
                nd += 1
                if nd <= 8:
                    s = dl[0] if len(dl) else dr[0]
                    side = 0 if len(dl) else 1
                    car_of = [i for i, (p, a, c, car) in enumerate(r.records) if (2 * s + side) in set(car)]
                    print(" key", k, "L diff", len(dl), "R diff", len(dr), "first sample", s, "side", side,
                          "oracle", int(ok[k][side][s]), "product", int(pk[k][side][s]), "records carried", car_of)
        print("keys differing", nd)
        job.close()
    sc.close()


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    if len(sys.argv) > 2:
        run(n, sys.argv[2])
    else:
        for v, env in (("default", {}), ("nodedup", {"TFBS_DEDUP": "0"}), ("nodevpatch", {"TFBS_DEV_PATCH": "0"}),
                       ("host", {})):
            e = dict(os.environ, **env)
            r = subprocess.run([sys.executable, __file__, str(n), v], env=e, timeout=600)
            if r.returncode:
                sys.exit(r.returncode)
