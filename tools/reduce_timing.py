"""First and repeated tfbs_batch_reduce / encode on one C3 batch: how much of the key
reduction is one-time allocation (pinned staging, first-touch pages) rather than work.
Usage: reduce_timing.py [regions]"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfbs_pkg  # noqa: E402

T = tfbs_pkg.load()
L = T.lib()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
d = tempfile.mkdtemp()
names = T.synth_write_pwms(d, 600, 3, 3)
ps = T.parse_pwm_files(os.path.join(d, "pwms.txt"), os.path.join(d, "thr"), 1e-4, names)
sc = T.Scanner(ps)
b = T.RegionBatch(ps, 50000, build_device=0)
b.synth_fill(3, 0, n, 0)
T.check(L.tfbs_batch_upload(sc.h, b.h))
T.check(L.tfbs_scan(sc.h, b.h))
T.check(L.tfbs_ctx_sync(sc.h))
for k in range(3):
    t = time.perf_counter()
    T.check(L.tfbs_batch_reduce(sc.h, b.h))
    t1 = time.perf_counter()
    b.encode(sc, 0, 512, device_codes=True)
    t2 = time.perf_counter()
    print("pass %d: reduce %.4f s, encode(512 regions) %.4f s" % (k, t1 - t, t2 - t1), flush=True)
sc.close()
