"""The device BGZF row writer alone, for profiling: a C3-shaped batch (device
grouping), scan, key reduction, per-sample encoding with the codes left on the
device, then tfbs_batch_rows_bgzf to /dev/null.  Usage: bgzf_only.py [regions]"""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tfbs_pkg  # noqa: E402

T = tfbs_pkg.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
d = tempfile.mkdtemp()
names = T.synth_write_pwms(d, 600, 3, 3)
ps = T.parse_pwm_files(os.path.join(d, "pwms.txt"), os.path.join(d, "thr"), 1e-4, names)
b = T.RegionBatch(ps, 50000, build_device=0)
b.synth_fill(3, 0, n, 0)
sc = T.Scanner(ps)
b.scan(sc, reduce=True)
b.encode(sc, 0, n, device_codes=True)
fd = os.open(os.devnull, os.O_WRONLY)
t = time.perf_counter()
nw, _, nr, nb = b.rows_bgzf(sc, "chr1", 0, 1, 0, n, fd=fd)
print("rows %d text %.3g bgzf %.3g seconds %.3f" % (nr, nb, nw, time.perf_counter() - t))
sc.close()
