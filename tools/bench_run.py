#!/usr/bin/env python3
"""End-to-end run flow (main.rs:234-393 through tfbs_run: BCF decode, FASTA/BED,
distinct haplotypes, GPU scan, device key reduction, rows, BGZF VCF) on a
synthetic dataset (tools/synth_dataset.py).  Prints one JSON line.

Usage: python tools/bench_run.py [--samples 1000] [--regions 1000] [--pwms 10]
       [--length-config 2] [--threads 16] [--regions-per-batch 512]
"""
import argparse
import ctypes
import gzip
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1000)
    ap.add_argument("--regions", type=int, default=1000)
    ap.add_argument("--pwms", type=int, default=10)
    ap.add_argument("--length-config", type=int, default=2)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--regions-per-batch", type=int, default=512)
    ap.add_argument("--threshold", type=float, default=1e-4)
    a = ap.parse_args()
    import synth_dataset
    import tfbs_pkg
    T = tfbs_pkg.load()
    work = tempfile.mkdtemp(prefix="tfbs_run_")
    t = time.perf_counter()
    d = synth_dataset.make_dataset(work, a.samples, a.regions, a.pwms, a.length_config, a.seed)
    t_gen = time.perf_counter() - t
    out = os.path.join(work, "out.vcf.gz")
    t = time.perf_counter()
    r = T.BcfReader(d["bcf"])  # streaming reader (f2): parallel BGZF inflate + BCF2 decode of the whole contig
    n = ctypes.c_size_t()
    T.check(T.lib().tfbs_bcf_fetch(r.h, b"chr1", 0, 1 << 40, ctypes.byref(n)))
    t_bcf = time.perf_counter() - t
    assert n.value == len(d["records"])
    n_rec = len(d["records"])
    del r
    t = time.perf_counter()
    T.run("chr1", d["bcf"], [d["bed"]], d["fasta"], None, d["pwm_file"], d["thr_dir"], a.threshold, d["names"], out,
          threads=a.threads, regions_per_batch=a.regions_per_batch)
    t_run = time.perf_counter() - t
    with gzip.open(out, "rt") as f:
        rows = sum(1 for _ in f) - 1
    print(json.dumps({
        "workload": "run flow, %d samples x %d regions x %d PWMs (both strands)" % (a.samples, a.regions, a.pwms),
        "records": n_rec, "rows": rows, "bcf_bytes": os.path.getsize(d["bcf"]), "vcf_gz_bytes": os.path.getsize(out),
        "run_s": t_run, "regions_per_s": a.regions / t_run, "bcf_decode_s": t_bcf, "dataset_gen_s": t_gen,
        "threads": a.threads}))


if __name__ == "__main__":
    main()
