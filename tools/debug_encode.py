"""Debug: rows through the device encoding vs the host path (tfbs_batch_reduce only)
for test_reference_window_reuse_vs_oracle's job; prints the first differing rows."""
import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
os.environ["TFBS_MFMA"] = "1"
from helpers import T, build_batch, synth_patterns  # noqa: E402

tmp = tempfile.mkdtemp()
ps, _ = synth_patterns(tmp, 10, 3, 71, thr=float(sys.argv[1]) if len(sys.argv) > 1 else 1e-3)
n_samples, n_regions = 60, 6
H = 2 * n_samples
regions, ranges = [], []
for j in range(n_regions):
    r = T.SynthRegion(31, j, n_samples, ps.max_length, 20 if j == 3 else 0)
    s, e = r.merged
    es = s - ps.max_length + 1
    ref = list(r.ref)
    if j == 2:
        for q in range(10, 18):
            ref[q] = "N"
    ref = "".join(ref)
    recs = [("car", pos, rf, alt, car) for pos, rf, alt, car in r.records
            if j != 2 or not any(10 <= pos - es + t < 18 for t in range(len(rf)))]
    if j in (0, 4):
        q = len(ref) // 2
        while ref[q] == "N" or any(rec[1] == es + q for rec in recs):
            q += 1
        recs.append(("car", es + q, ref[q], "ACGT"[("ACGT".index(ref[q]) + 1) % 4], list(range(H))))
    regions.append({"merged": (s, e), "ref": ref, "records": recs})
    ranges.append((s, e))
    if j == 5:
        ranges.extend((s, s + 1 + k) for k in range(39))
beds = [("synthetic.bed", ranges)]
sc = T.Scanner(ps)
b = build_batch(ps, n_samples, beds, regions)
b.scan(sc, reduce=True)
want = [b.region_rows(i, "chr1")[0].splitlines() for i in range(b.num_regions)]
b.encode(sc)
got = [b.region_rows(i, "chr1")[0].splitlines() for i in range(b.num_regions)]
for i in range(b.num_regions):
    st = b.region_stats(i)
    print("region", i, "stats", st, "rows", len(want[i]), len(got[i]))
    for a, z in zip(want[i], got[i]):
        if a != z:
            print("HOST:", a[:400])
            print("ENC: ", z[:400])
            break
sc.close()
