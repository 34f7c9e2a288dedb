#!/usr/bin/env python3
"""A/B the scan kernel's tunables in ONE process on one batch (interleaved rounds).

Usage: python tools/tune.py [--regions N] [--rounds R] VAR=a,b,c [VAR2=x,y ...]
Each variant is a full assignment of the listed environment variables; the
ctx reads them at creation.  Prints median/min kernel ms per variant and
checks that every variant produces identical counts.
"""
import argparse
import itertools
import os
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tfbs_pkg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--regions", type=int, default=2000)
    ap.add_argument("--samples", type=int, default=50000)
    ap.add_argument("--pwms", type=int, default=600)
    ap.add_argument("--length-config", type=int, default=3)
    ap.add_argument("--indel-pct", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("vars", nargs="*")
    a = ap.parse_args()
    T = tfbs_pkg.load()
    d = tempfile.mkdtemp()
    names = T.synth_write_pwms(d, a.pwms, a.length_config, 3)
    ps = T.parse_pwm_files(os.path.join(d, "pwms.txt"), os.path.join(d, "thr"), 1e-4, names)
    b = T.RegionBatch(ps, a.samples, keep_membership=True)
    b.synth_fill(3, 0, a.regions, a.indel_pct)
    keys, vals = [], []
    for v in a.vars:
        k, x = v.split("=")
        keys.append(k)
        vals.append(x.split(","))
    variants = list(itertools.product(*vals)) or [()]
    L = T.lib()
    times = {v: [] for v in variants}
    ref_counts = None
    scanners = {}
    for v in variants:
        for k, x in zip(keys, v):
            os.environ[k] = x
        scanners[v] = T.Scanner(ps)
    for r in range(a.rounds):
        for v in variants:
            sc = scanners[v]
            b.scan(sc, upload=True, download=(r == 0))
            T.check(L.tfbs_scan(sc.h, b.h))
            times[v].append(L.tfbs_ctx_last_scan_ms(sc.h))
            if r == 0:
                T.check(L.tfbs_batch_download(sc.h, b.h))
                key = [b.keys(i) for i in (0, b.num_regions // 2, b.num_regions - 1)]
                if ref_counts is None:
                    ref_counts = key
                elif key != ref_counts:
                    print("MISMATCH in variant", dict(zip(keys, v)))
    print("regions=%d haps=%d windows=%.3g cells=%.3g" % (a.regions, b.num_haplotypes, b.num_windows, b.num_cell_ops))
    for v in variants:
        t = times[v]
        print("%-60s median %8.2f ms  min %8.2f ms  -> %.3g windows/s" % (
            " ".join("%s=%s" % kv for kv in zip(keys, v)), statistics.median(t), min(t),
            b.num_windows / (statistics.median(t) / 1e3)))


if __name__ == "__main__":
    main()
