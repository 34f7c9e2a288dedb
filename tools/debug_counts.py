#!/usr/bin/env python3
"""Debug helper: the synthetic-regions parity case under several MFMA tunables;
prints, per variant, the mismatching keys against the oracle (diff histogram)."""
import collections
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import T, make_regions_synth, run_oracle, run_product, synth_patterns  # noqa: E402


def main():
    config, indel, n_samples, n_regions = [int(x) for x in (sys.argv[1:5] or [2, 0, 150, 16])]
    d = tempfile.mkdtemp()
    ps, _ = synth_patterns(d, 12 if config != 3 else 40, config, 100 + config, thr=1e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(7 + config, 0, n_regions, n_samples, ps.max_length, indel)
    okeys, _, _ = run_oracle(ps, n_samples, beds, regions)
    import oracle_py as O
    os.environ["TFBS_MFMA"] = "1"
    sc = T.Scanner(ps)
    pats = ps.to_list()
    for ri in range(len(regions)):
        ref = regions[ri]["ref"]
        hap = [(c, 5000 + i) for i, c in enumerate(ref)]
        got = sc.matches_all(hap)
        for pi, p_ in enumerate(pats):
            want = O.matches([wt.acgtn for wt in p_.weights], p_.min_score, hap, kind=p_.kind)
            if got[pi] != want:
                print("matches region", ri, "pattern", pi, "id", p_.pattern_id, "len", len(p_), "min", p_.min_score,
                      "hap len", len(hap), "got", got[pi], "want", want)
    sc.close()
    for var in [dict(), dict(TFBS_MFMA_HAPS_PER_BLOCK="4"), dict(TFBS_MFMA_LDS_KB="8"), dict(TFBS_MFMA="0")]:
        os.environ["TFBS_MFMA"] = "1"
        os.environ.pop("TFBS_MFMA_HAPS_PER_BLOCK", None)
        os.environ.pop("TFBS_MFMA_LDS_KB", None)
        os.environ.update(var)
        sc = T.Scanner(ps)
        pkeys, _, b = run_product(sc, ps, n_samples, beds, regions)
        bad = 0
        for i, (a, z) in enumerate(zip(okeys, pkeys)):
            for k in sorted(set(a) | set(z)):
                if a.get(k) != z.get(k):
                    bad += 1
                    if bad <= 6:
                        av, zv = a.get(k), z.get(k)
                        if av and zv:
                            h = collections.Counter(
                                (x - y) for ax, zx in zip(av, zv) for x, y in zip(zx, ax))
                        else:
                            h = None
                        print(var, "region", i, "key", k, "oracle" if av else "-", "product" if zv else "-",
                              "diff hist", h, "region_stats", b.region_stats(i))
        print(var, "mismatching keys", bad, flush=True)
        sc.close()


if __name__ == "__main__":
    main()
