#!/usr/bin/env python3
"""Row formatting A/B on one box: a C3 batch (--regions) scanned, reduced and
device-encoded once, then tfbs_batch_format_rows timed --rounds times (TFBS_LIB
selects the library build).  Prints the median seconds and the rows / bytes."""
import argparse
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tfbs_pkg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--regions", type=int, default=2000)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--threads", type=int, default=16)
a = ap.parse_args()
T = tfbs_pkg.load()
L = T.lib()
d = tempfile.mkdtemp()
names = T.synth_write_pwms(d, 600, 3, 3)
ps = T.parse_pwm_files(os.path.join(d, "pwms.txt"), os.path.join(d, "thr"), 1e-4, names)
b = T.RegionBatch(ps, 50000, keep_membership=True)
b.synth_fill(3, 0, a.regions, 0)
sc = T.Scanner(ps, device=0)
T.check(L.tfbs_batch_upload(sc.h, b.h))
T.check(L.tfbs_scan(sc.h, b.h))
T.check(L.tfbs_ctx_sync(sc.h))
T.check(L.tfbs_batch_reduce(sc.h, b.h))
te = []
for _ in range(a.rounds):  # the bench's device encoding: 512 regions per call
    t = time.perf_counter()
    for r0 in range(0, b.num_regions, 512):
        b.encode(sc, r0, min(b.num_regions, r0 + 512))
    te.append(time.perf_counter() - t)
print("encode (512 regions per call) median %.4f s min %.4f s" % (statistics.median(te), min(te)))
b.encode(sc, 0, b.num_regions)
ts = []
for _ in range(a.rounds):
    t = time.perf_counter()
    nr, nb = b.format_rows("chr1", 0, a.threads, 0, b.num_regions)
    ts.append(time.perf_counter() - t)
print("lib %s rows %d bytes %d median %.4f s min %.4f s" % (os.environ.get("TFBS_LIB", "in-tree"), nr, nb,
                                                            statistics.median(ts), min(ts)))
