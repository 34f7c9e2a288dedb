#!/usr/bin/env python3
"""End-to-end run flow (main.rs:234-393 through tfbs_run: BCF decode, FASTA/BED,
distinct haplotypes, GPU scan, device key reduction, rows, BGZF VCF) on a
synthetic dataset (tools/synth_dataset.py).  Prints one JSON line.

Usage: python tools/bench_run.py [--samples 50000] [--regions 1000] [--pwms 600]
       [--length-config 3] [--threads 16] [--regions-per-batch 512] [--devices 0,0]
       [--oracle-seconds 6]

The line carries the oracle's end-to-end leg on the same generator and regions
(bench.cpu_baseline: load_diffs + patch + find_all_matches + count + rows on the
box's share of host threads, inputs generated before its clock), next to the run.
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
    ap.add_argument("--samples", type=int, default=50000)
    ap.add_argument("--regions", type=int, default=1000)
    ap.add_argument("--pwms", type=int, default=600)
    ap.add_argument("--length-config", type=int, default=3)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--regions-per-batch", type=int, default=512)
    ap.add_argument("--threshold", type=float, default=1e-4)
    ap.add_argument("--devices", default=None, help="comma list of HIP devices (tfbs_run --devices)")
    ap.add_argument("--oracle-seconds", type=float, default=6.0, help="budget of the oracle's e2e leg (0: skip)")
    a = ap.parse_args()
    import synth_dataset
    import tfbs_pkg
    T = tfbs_pkg.load()
    work = tempfile.mkdtemp(prefix="tfbs_run_")
    t = time.perf_counter()
    d = synth_dataset.make_dataset(work, a.samples, a.regions, a.pwms, a.length_config, a.seed, keep_gt=False)
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
    devices = [int(x) for x in a.devices.split(",")] if a.devices else None
    os.environ["TFBS_RUN_TIMING"] = "1"  # per-shard phase seconds on stderr
    # the process's first device use (HIP runtime, the device's context and code objects:
    # 0.1-0.6 s, the most on a fresh box) timed apart: a context made and released on
    # each device before the run's clock -- tfbs_run warms the runtime itself too, so the
    # run alone does not depend on it; both rates are in the line
    t = time.perf_counter()
    warm_ps = T.parse_pwm_files(d["pwm_file"], d["thr_dir"], a.threshold, d["names"])
    for dev in sorted(set(devices or [0])):
        T.Scanner(warm_ps, device=dev).close()
    t_warm = time.perf_counter() - t
    t = time.perf_counter()
    T.run("chr1", d["bcf"], [d["bed"]], d["fasta"], None, d["pwm_file"], d["thr_dir"], a.threshold, d["names"], out,
          threads=a.threads, regions_per_batch=a.regions_per_batch, devices=devices)
    t_run = time.perf_counter() - t
    rows = 0
    with gzip.open(out, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            rows += chunk.count(b"\n")
    rows -= 1  # the header
    line = {
        "workload": "run flow (tfbs_run: BCF decode + FASTA/BED + distinct haplotypes + scan + key assembly + "
                    "device encode + device BGZF rows), %d samples x %d regions x %d PWMs (both strands), "
                    "threshold %g" % (a.samples, a.regions, a.pwms, a.threshold),
        "devices": a.devices or "0", "records": n_rec, "rows": rows, "bcf_bytes": os.path.getsize(d["bcf"]),
        "vcf_gz_bytes": os.path.getsize(out), "run_s": t_run, "regions_per_s": a.regions / t_run,
        "device_warmup_s": t_warm, "regions_per_s_with_device_warmup": a.regions / (t_run + t_warm),
        "bcf_decode_alone_s": t_bcf, "dataset_gen_s": t_gen, "threads": a.threads,
        "regions_per_batch": a.regions_per_batch}
    if a.oracle_seconds > 0:  # the oracle's end-to-end leg on the same generator (bench.py's CPU baseline)
        import bench
        args = argparse.Namespace(seed=a.seed, samples=a.samples, regions=a.regions, indel_pct=0)
        ps = T.parse_pwm_files(d["pwm_file"], d["thr_dir"], a.threshold, d["names"])
        cb = bench.cpu_baseline(T, ps, args, a.oracle_seconds)
        e2e = cb["matrix"]["e2e_t%d" % cb["cores"]]
        line["oracle_e2e"] = {"regions_per_s": e2e["regions_per_s"], "threads": cb["cores"],
                              "regions": e2e["regions"], "kind": "port",
                              "note": "oracle/tfbs_oracle.c: load_diffs + patch + find_all_matches + "
                                      "count_matches_by_sample + counts_as_genotypes + rows, per-region inputs "
                                      "generated before its clock (no BCF decode)"}
        line["vs_oracle_e2e"] = line["regions_per_s"] / e2e["regions_per_s"]
    print(json.dumps(line))


if __name__ == "__main__":
    main()
