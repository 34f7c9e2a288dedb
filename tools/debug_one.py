#!/usr/bin/env python3
"""Debug helper: matches_all of one synthetic region's reference (config 2 patterns)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import T, make_regions_synth, synth_patterns  # noqa: E402
import oracle_py as O  # noqa: E402

d = tempfile.mkdtemp()
ps, _ = synth_patterns(d, 12, 2, 102, thr=1e-3)
regions = make_regions_synth(9, 0, 16, 150, ps.max_length, 0)
ref = regions[int(sys.argv[1]) if len(sys.argv) > 1 else 2]["ref"]
hap = [(c, 5000 + i) for i, c in enumerate(ref)]
sc = T.Scanner(ps)
got = sc.matches_all(hap)
for pi, p_ in enumerate(ps.to_list()):
    want = O.matches([wt.acgtn for wt in p_.weights], p_.min_score, hap, kind=p_.kind)
    print("pattern", pi, "len", len(p_), "got", got[pi], "want", want, "OK" if got[pi] == want else "MISMATCH")
