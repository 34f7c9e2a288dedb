#!/usr/bin/env python3
"""Benchmark: haplotype-windows scored/sec of the MI355X PWM scan (BASELINE.json).

Workload (default, BASELINE.json configs[2] = SURVEY.md section 8d "C3"): per
GPU, 10 000 merged regions x 201 bp of a synthetic chromosome, 50 000 phased
samples (100 000 haplotypes), Poisson(20) variant sites per region with
carrier counts ~ 1/k, 600 synthetic HOCOMOCO-format PWMs (L 8..30) on both
strands (1 200 patterns), threshold 1e-4.  Regions are reduced to distinct
haplotypes on the host (untimed, as the reference does before scanning) and
packed into HBM; one timed step = one tfbs_scan over every distinct haplotype
x pattern window of the rank's batch.

Multi-GPU (torchrun, one rank per GPU): rank r scans regions
[r*R, (r+1)*R) of the same synthetic chromosome -- weak scaling, no collective
on the data path; a barrier + max-over-ranks bracket the timed region.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X spec (MI355X_MICROARCH.md, chip table)
VALU_PEAK_TOPS = 78.64      # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz int32 lane-ops/s
# dense FP4/FP6 MFMA: 4x the ~2.5 PF dense BF16 rate (MI355X_MICROARCH.md, MFMA table:
# v_mfma_scale_f32_32x32x64_f8f6f4 with FP4/FP6 operands)
MFMA_F6_PEAK_TOPS = 10000.0
# ops of the one-hot formulation per (window, strand, column): 4 bases x 1 FP6
# digit = 4 multiply-adds (scan_mfma.hip); padding (K, windows, strands) and the
# exact rescoring of the rare candidate windows excluded
MFMA_OPS_PER_CELL = 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--regions", type=int, default=10000, help="regions per GPU")
    ap.add_argument("--samples", type=int, default=50000)
    ap.add_argument("--pwms", type=int, default=600)
    ap.add_argument("--length-config", type=int, default=3)
    ap.add_argument("--indel-pct", type=int, default=0)
    ap.add_argument("--threshold", type=float, default=1e-4)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for the timing reductions (gloo: rehearse several ranks on one GPU)")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def workload_name(args):
    """BASELINE.json configs: C2 = 1 k samples x 10 PWMs (lengths 8-15), C3 = 50 k x 600
    PWMs per GPU (C4 is C3 sharded over 8 GPUs), C5 = C3 with 30 % indels and PWMs of length 25-30."""
    key = (args.samples, args.pwms, args.length_config, args.indel_pct)
    return {(1000, 10, 2, 0): "C2", (50000, 600, 3, 0): "C3", (50000, 600, 5, 30): "C5"}.get(key, "custom")


def cpu_baseline(T, ps, args, budget_s):
    """The oracle (C restatement of the reference algorithm) on host threads over a
    bounded sample of the same workload's regions, 50-region chunks per worker as
    main.rs:375-381.  Returns the cpu_baseline object."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import concurrent.futures as cf

    import oracle_py as O
    from helpers import pattern_dicts

    pats = pattern_dicts(ps)
    threads = max(1, min(16, os.cpu_count() or 1))
    lmax = ps.max_length

    def run_regions(idx):
        job = O.Job(args.samples, "chr1", pats, [("synthetic.bed", [])])
        wall = 0.0
        for j in idx:
            r = T.SynthRegion(args.seed, j, args.samples, lmax, args.indel_pct)
            t0 = time.perf_counter()
            rc = job.begin(r.merged[0], r.merged[1], r.ref)
            for pos, ref, alt, car in r.records:
                rc |= job.add_record_carriers(pos, ref, alt, car)
            rc |= job.end()
            wall += time.perf_counter() - t0
            assert rc == 0
        job.close()
        return wall

    # calibrate on one region, then size the sample to ~budget_s of wall time
    t1 = run_regions([0])
    per_thread = max(1, int(budget_s / max(t1, 1e-3)))
    n = min(args.regions, threads * per_thread)
    idx = list(range(n))
    csize = max(1, min(50, n // threads))  # the reference's 50-peak chunks, split further for small samples
    chunks = [idx[i:i + csize] for i in range(0, n, csize)]
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(run_regions, chunks))
    wall = time.perf_counter() - t0
    b = T.RegionBatch(ps, args.samples, keep_membership=False)
    b.synth_fill(args.seed, 0, n, args.indel_pct)
    return {"value": b.num_windows / wall, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": "%d of the %d regions (%d distinct haplotypes, %.3g windows), %d samples, %d patterns; "
                      "oracle/tfbs_oracle.c restating the reference scan + count + genotype path, %d threads, "
                      "%.1f s wall" % (n, args.regions, b.num_haplotypes, b.num_windows, args.samples, len(ps),
                                       threads, wall)}


def shard_batch(T, ps, args, rank):
    """Rank r's share: merged regions [r R, (r+1) R) of the synthetic
    chromosome, reduced to distinct haplotypes and packed on the host."""
    batch = T.RegionBatch(ps, args.samples, keep_membership=False)
    batch.synth_fill(args.seed, rank * args.regions, args.regions, args.indel_pct)
    return batch


def job_totals(dist, elapsed, windows, regions, eff, device):
    """Max-over-ranks wall time and whole-job sums.  Regions shard with no exchange, so
    the only collectives are these scalar reductions around the timed region."""
    if dist is None:
        return elapsed, float(windows), float(regions), float(eff)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    w = torch.tensor([windows, regions, eff], dtype=torch.float64, device=device)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    tot = [float(x) for x in w.tolist()]
    return float(t.item()), tot[0], tot[1], tot[2]


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        if args.dist_backend == "gloo":  # rehearsal: ranks may share a GPU
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)

    import tfbs_pkg

    T = tfbs_pkg.load()
    work = tempfile.mkdtemp(prefix="tfbs_bench_%d_" % rank)
    names = T.synth_write_pwms(work, args.pwms, args.length_config, args.seed)
    ps = T.parse_pwm_files(os.path.join(work, "pwms.txt"), os.path.join(work, "thr"), args.threshold, names)
    sc = T.Scanner(ps, device=local)
    t_prep = time.perf_counter()
    batch = shard_batch(T, ps, args, rank)
    t_prep = time.perf_counter() - t_prep
    t_up = time.perf_counter()
    batch.scan(sc, upload=True, download=False)
    T.check(T.lib().tfbs_ctx_sync(sc.h))
    t_up = time.perf_counter() - t_up

    L = T.lib()
    for _ in range(args.warmup):
        T.check(L.tfbs_scan(sc.h, batch.h))
    T.check(L.tfbs_ctx_sync(sc.h))

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    kernel_ms, mfma_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        T.check(L.tfbs_scan(sc.h, batch.h))
        kernel_ms.append(L.tfbs_ctx_last_scan_ms(sc.h))  # waits for this step's end event
        mfma_ms.append(L.tfbs_ctx_last_mfma_ms(sc.h))   # the matrix-core kernel alone (-1: none ran)
    T.check(L.tfbs_ctx_sync(sc.h))
    if dist is not None:
        import torch
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()

    # after the timed region: the two ways the counts leave the GPU
    t_red = time.perf_counter()
    T.check(L.tfbs_batch_reduce(sc.h, batch.h))
    t_red = time.perf_counter() - t_red
    t_dense = time.perf_counter()
    T.check(L.tfbs_batch_download(sc.h, batch.h))
    t_dense = time.perf_counter() - t_dense

    windows = batch.num_windows
    regions = batch.num_regions
    elapsed, tot_windows, tot_regions, tot_eff = job_totals(dist, elapsed, windows, regions,
                                                             batch.num_effective_windows,
                                                             "cuda" if args.dist_backend == "nccl" else "cpu")

    if rank == 0:
        steps = args.steps
        value = tot_windows * steps / elapsed
        kms = sum(kernel_ms) / len(kernel_ms)
        pattern_bytes = 0
        for p in ps.to_list():
            pattern_bytes += ((len(p) + 15) // 16) * 1536 + 16 * len(p) + 24
        alg_bytes = batch.input_bytes + batch.output_bytes + pattern_bytes
        achieved = alg_bytes / (kms / 1e3) / 1e9
        traffic = None
        if os.path.exists(args.pmc_summary):
            try:
                pm = json.load(open(args.pmc_summary))
                if (pm.get("workload") == "C3" and pm.get("regions") == args.regions
                        and pm.get("scan_path") == ("mfma" if min(mfma_ms) > 0 else "lut")):
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cell_tops = batch.num_cell_ops / (kms / 1e3) / 1e12
        mms = sum(mfma_ms) / len(mfma_ms)
        hbm = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
               "note": "algorithmic bytes/launch = packed haplotypes + metadata + pattern tables + u32 counts; "
                       "the scan is compute bound"}
        if mms > 0:  # the matrix-core kernel scored every strand of this workload
            mops = MFMA_OPS_PER_CELL * batch.num_cell_ops / (mms / 1e3) / 1e12
            roof = {"bound": "mfma", "achieved": mops, "peak": MFMA_F6_PEAK_TOPS, "unit": "TOPS",
                    "frac": mops / MFMA_F6_PEAK_TOPS, "traffic": traffic,
                    "kernel": "scan_mfma_kernel<staged, K depth> (one launch per depth, 4 streams)",
                    "kernel_ms": mms,
                    "note": "achieved = 8 ops per (window, strand, column) of the FP4 one-hot x FP6 bound-digit "
                            "GEMM / the MFMA phase's HIP-event time (first launch to last, joined on the ctx "
                            "stream; tools/trace_phase.py gives the same phase from the rocprofv3 trace); "
                            "traffic = HBM bytes of the phase's dispatches from PMC"}
        else:
            roof = hbm
        path = "mfma" if mms > 0 else "lut"
        out = {
            "metric": "haplotype-windows scored/sec",
            "value": value,
            "unit": "windows/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp4xfp6->f32 bound + int32 exact" if path == "mfma" else "int32",
            "data": "synthetic (SURVEY.md 8d generator; no HOCOMOCO/BCF download possible)",
            "config": {
                "workload": workload_name(args),
                "samples": args.samples, "haplotypes": 2 * args.samples, "regions_per_gpu": args.regions,
                "region_bp": 201, "pwms": args.pwms, "patterns": len(ps), "threshold": args.threshold,
                "indel_pct": args.indel_pct, "distinct_haplotypes_per_gpu": batch.num_haplotypes,
                "windows_per_step": int(tot_windows), "parallelism": "region shard x%d" % world,
                "scan_path": path,
            },
            "regions_per_s": tot_regions * steps / elapsed,
            "effective_windows_per_s": tot_eff * steps / elapsed,
            "kernel_ms_avg": kms,
            "host_prep_s": t_prep,
            "upload_s": t_up,
            "key_reduce_s": t_red,
            "dense_download_s": t_dense,
            "roofline": roof,
            "hbm_roofline": hbm,
            "valu_roofline": {"bound": "valu", "achieved": cell_tops, "peak": VALU_PEAK_TOPS,
                              "unit": "T column-lookups/s vs T int32 lane-ops/s",
                              "frac": cell_tops / VALU_PEAK_TOPS},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(T, ps, args, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    sc.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
