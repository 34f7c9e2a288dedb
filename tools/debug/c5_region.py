"""One C5 region (24) against the live oracle on the GPU, with subsets of its records
(the deletion reaching the window's end alone, with the others, ...), with and without
reference-window reuse."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402
from helpers import T, pattern_dicts  # noqa: E402

n_samples, seed, indel = int(sys.argv[1]) if len(sys.argv) > 1 else 50000, 5, 30
tmp = tempfile.mkdtemp()
names = T.synth_write_pwms(tmp, 600, 5, seed)
ps = T.parse_pwm_files(os.path.join(tmp, "pwms.txt"), os.path.join(tmp, "thr"), 1e-4, names)
pats = pattern_dicts(ps)
r = T.SynthRegion(seed, 24, n_samples, ps.max_length, indel)
es = r.ext_start
recs = r.records
subsets = {"all": list(range(len(recs))), "del_end": [25], "del_end+snv0": [0, 25],
           "no_del_end": [i for i in range(len(recs)) if i != 25], "last3": [23, 24, 25]}
sc = T.Scanner(ps)
for name, sub in subsets.items():
    b = T.RegionBatch(ps, n_samples)
    bed = b.add_bed("synthetic.bed")
    b.begin(r.merged[0], r.merged[1], r.ref)
    b.add_inner(bed, r.merged[0], r.merged[1])
    for i in sub:
        pos, rf, alt, car = recs[i]
        b.add_record_carriers(pos, rf, alt, car)
    b.end()
    b.scan(sc, reduce=True)
    pk = b.keys_np(0)
    job = O.Job(n_samples, "chr1", pats, [("synthetic.bed", [tuple(r.merged)])])
    job.begin(r.merged[0], r.merged[1], r.ref)
    for i in sub:
        pos, rf, alt, car = recs[i]
        job.add_record_carriers(pos, rf, alt, car)
    job.end()
    ok = job.keys_np()
    job.close()
    nd = sum(1 for k in set(ok) | set(pk) if k not in ok or k not in pk or not (
        np.array_equal(ok[k][0], pk[k][0]) and np.array_equal(ok[k][1], pk[k][1])))
    print(name, "records", len(sub), "haplotypes", b.region_stats(0), "keys", len(ok), len(pk), "differing", nd, flush=True)
