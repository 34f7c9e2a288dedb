"""The first BGZF block whose inflated bytes differ from the host rows (the C3 BGZF
test's case), with the bytes around the first difference: debug aid for the device
BGZF writer.  Usage: bgzf_diff.py [regions] [chunk]"""
import os
import struct
import sys
import tempfile
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import tfbs_pkg  # noqa: E402

T = tfbs_pkg.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 150
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 64
d = tempfile.mkdtemp()
names = T.synth_write_pwms(d, 600, 3, 3)
ps = T.parse_pwm_files(os.path.join(d, "pwms.txt"), os.path.join(d, "thr"), 1e-4, names)
b = T.RegionBatch(ps, 50000)
b.synth_fill(3, 0, n, 0)
sc = T.Scanner(ps)
b.scan(sc, reduce=True)
want, _ = b.rows("chr1")
want = want.encode()
data, fake = b"", 1
for r0 in range(0, n, chunk):
    r1 = min(n, r0 + chunk)
    b.encode(sc, r0, r1, device_codes=True)
    part, fake, _, _ = b.rows_bgzf(sc, "chr1", 0, fake, r0, r1)
    data += part
i, at, k, bad = 0, 0, 0, 0
while i < len(data):
    bsize = struct.unpack_from("<H", data, i + 16)[0] + 1
    crc, isize = struct.unpack_from("<II", data, i + bsize - 8)
    raw = zlib.decompress(data[i + 18:i + bsize - 8], -15)
    exp = want[at:at + isize]
    if raw != exp or zlib.crc32(raw) != crc:
        j = next((q for q in range(min(len(raw), len(exp))) if raw[q] != exp[q]), min(len(raw), len(exp)))
        print("block %d at %d isize %d: inflated %s expected (len %d vs %d), crc stored %08x of inflated %08x; "
              "first diff at %d: got %r want %r" % (k, at, isize, "==" if raw == exp else "!=", len(raw), len(exp),
                                                   crc, zlib.crc32(raw), j, raw[max(0, j - 20):j + 20],
                                                   exp[max(0, j - 20):j + 20]))
        bad += 1
        if bad >= 5:
            break
    i += bsize
    at += isize
    k += 1
print("blocks %d bad %d" % (k, bad))
sc.close()
