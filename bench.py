#!/usr/bin/env python3
"""Benchmark: haplotype-windows scored/sec of the MI355X PWM scan (BASELINE.json).

Workloads (--workload, default C3 = BASELINE.json configs[2]):
  C2  1 000 samples x 1 000 regions x 10 PWMs (L 8-15), seed 2
  C3  50 000 samples x 10 000 regions x 600 PWMs (L 8-30), seed 3     (per GPU)
  C4  C3's generator with seed 4, 12 500 regions per GPU (100 000 over 8 GPUs)
  C5  C3 with 30 % indels and PWMs of length 25-30, seed 5
Regions are 201 bp merged BED rows of a synthetic chromosome with Poisson(20)
variant sites and carrier counts ~ 1/k; PWMs are synthetic HOCOMOCO-format
matrices with exact 1e-4 thresholds, both strands.  The host reduces every
region to its distinct haplotypes and packs them into HBM (untimed, as the
reference builds them before scanning); one timed step = tfbs_scan (every
distinct haplotype x pattern window of the rank's batch) + tfbs_batch_assemble +
tfbs_batch_assemble_wait (every region's keyed counts: reference-window reuse
resolved, classified, varying counts compacted; the host checks every list).

Multi-GPU (one rank per GPU; `--gpus N` without WORLD_SIZE starts torchrun with
N ranks itself, before anything touches a GPU): weak scaling, no collective on
the data path; a barrier + max-over-ranks bracket the timed region.
  --shard regions         rank r scans regions [r R, (r+1) R) -- the static
                          contiguous region shard tfbs_run --devices uses
                          (SURVEY.md 8(e)); R = regions per GPU
  --shard regions_x_pwms  the 2-D region x PWM split (BASELINE config C4): P
                          pattern shards (--pwm-shards, pattern_id % P, both
                          strands of a PWM on one rank) x N / P region blocks
                          of P R regions; rank r = block r // P, pattern shard
                          r % P; every rank keeps the whole set's windows
                          (tfbs_batch_set_window_lmax), so the per-key counts
                          of the P shards of a block are the unsharded run's
                          (the host merges disjoint pattern_id keys)

Besides `value` the line carries an end-to-end leg over the same batch (host
prep + upload + scan + device key reduction + device per-sample encoding + the
VCF rows as BGZF blocks made on the GPU), the roofline of the dominant kernel
(HIP events around its launches on the ctx stream; traffic, the rocprofv3 MFMA
phase and the SQ instruction mix from the PMC passes and kernel trace of the
same bench command, tools/profile_round.sh, used only when they profiled this
same library build) and the CPU baseline (the oracle, scan-only and end-to-end,
1 thread and the box's share of threads).
"""
import argparse
import ctypes
import json
import math
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
CPU_THREADS_MAX = 16        # the GPU box's CPU share for one GPU (os.cpu_count() shows the whole host)

WORKLOADS = {  # samples, regions per GPU, pwms, length config, indel %, seed
    "C2": (1000, 1000, 10, 2, 0, 2),
    "C3": (50000, 10000, 600, 3, 0, 3),
    "C4": (50000, 12500, 600, 3, 0, 4),
    "C5": (50000, 10000, 600, 5, 30, 5),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: as many as fill --min-seconds, at least 5, from the warmup's pace)")
    ap.add_argument("--min-seconds", type=float, default=5.0,
                    help="without --steps: the timed loop's length to aim for (long enough for a GPU-busy sampler)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="C3", choices=sorted(WORKLOADS))
    ap.add_argument("--regions", type=int, default=None, help="regions per GPU (workload default)")
    ap.add_argument("--samples", type=int, default=None)
    ap.add_argument("--pwms", type=int, default=None)
    ap.add_argument("--length-config", type=int, default=None)
    ap.add_argument("--indel-pct", type=int, default=None)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--threshold", type=float, default=1e-4)
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="budget of each CPU baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end leg (profiling passes)")
    ap.add_argument("--host-build", action="store_true",
                    help="reduce haplotypes to distinct ones on the host only (no device grouping)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for the timing reductions (gloo: rehearse several ranks on one GPU)")
    ap.add_argument("--shard", default="regions", choices=["regions", "regions_x_pwms"])
    ap.add_argument("--pwm-shards", type=int, default=None,
                    help="pattern shards of --shard regions_x_pwms (default 2 on an even rank count, else 1)")
    a = ap.parse_args()
    w = WORKLOADS[a.workload]
    for name, v in zip(("samples", "regions", "pwms", "length_config", "indel_pct", "seed"), w):
        if getattr(a, name) is None:
            setattr(a, name, v)
    a.custom = tuple(getattr(a, n) for n in ("samples", "regions", "pwms", "length_config", "indel_pct",
                                              "seed")) != w
    return a


def workload_key(args):
    """What a PMC summary must match to be this run's traffic (profiles/pmc_traffic_<workload>.json)."""
    return {"workload": args.workload, "samples": args.samples, "regions": args.regions, "pwms": args.pwms,
            "length_config": args.length_config, "indel_pct": args.indel_pct, "seed": args.seed,
            "threshold": args.threshold}


def library_sha256():
    """SHA-256 of the product library this process loads (find-tfbs_amd/_capi.LIB_PATH)."""
    import hashlib
    import tfbs_pkg

    path = tfbs_pkg.load()._capi.LIB_PATH
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def pmc_profile(args, path):
    """The PMC passes and kernel trace of this same bench configuration AND library build
    (profiles/pmc_traffic_<workload>.json, tools/pmc_traffic.py: stamped with the profiled
    library's SHA-256), or (None, reason): a profile of another build is refused."""
    f = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % args.workload)
    if not os.path.exists(f):
        return None, "no %s" % os.path.relpath(f, ROOT)
    try:
        pm = json.load(open(f))
    except ValueError:
        return None, "unreadable %s" % os.path.relpath(f, ROOT)
    if pm.get("config") != workload_key(args) or pm.get("scan_path") != path:
        return None, "%s is for another configuration" % os.path.relpath(f, ROOT)
    if pm.get("library_sha256") != library_sha256():
        return None, "%s profiled another library build (sha256 %s)" % (os.path.relpath(f, ROOT),
                                                                       str(pm.get("library_sha256"))[:12])
    return pm, "%s (%s)" % (os.path.relpath(f, ROOT), pm.get("source", ""))


def cpu_baseline(T, ps, args, budget_s):
    """The oracle (oracle/tfbs_oracle.c, the C restatement of the reference algorithm,
    gcc -O3 -march=x86-64-v3) on host threads over a bounded sample of the workload's
    regions, 50-region chunks per worker as main.rs:375-381: scan-only (load_diffs +
    patch + find_all_matches, no count/rows) and end-to-end (+ count_matches_by_sample,
    counts_as_genotypes, rows), each on 1 thread and on the box's share of threads.
    Region inputs are generated before the clock starts."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import concurrent.futures as cf

    import numpy as np
    import oracle_py as O
    from helpers import pattern_dicts

    pats = pattern_dicts(ps)
    lmax = ps.max_length
    tmax = max(1, min(CPU_THREADS_MAX, os.cpu_count() or 1))

    def gen(j):
        r = T.SynthRegion(args.seed, j, args.samples, lmax, args.indel_pct)
        return (r.merged, r.ref, [(p, rf, a, np.asarray(c, dtype=np.uint32)) for p, rf, a, c in r.records])

    regs = [gen(0)]

    def run_regions(idx, scan_only):
        job = O.Job(args.samples, "chr1", pats, [("synthetic.bed", [regs[j][0] for j in idx])])
        job.set_scan_only(scan_only)
        for j in idx:
            merged, ref, recs = regs[j]
            rc = job.begin(merged[0], merged[1], ref)
            for pos, rf, alt, car in recs:
                rc |= job.add_record_carriers_np(pos, rf, alt, car)
            rc |= job.end()
            assert rc == 0
            job.clear_rows()
        ph = job.phase_seconds()
        job.close()
        return ph

    t1 = {}
    for scan_only in (True, False):
        t0 = time.perf_counter()
        run_regions([0], scan_only)
        t1[scan_only] = max(time.perf_counter() - t0, 1e-3)
    sizes = {(so, th): max(th, min(args.regions, int(th * budget_s / t1[so])))
             for so in (True, False) for th in (1, tmax)}
    ncpu = os.cpu_count() or 1
    if ncpu > tmax:  # every host CPU the box shows (its share is tmax): the scan-only leg's sample, ncpu threads
        sizes[(True, ncpu)] = max(ncpu, sizes[(True, tmax)])
    n_max = max(sizes.values())
    regs += [gen(j) for j in range(1, n_max)]
    matrix = {}
    for (scan_only, threads), n in sizes.items():
        csize = max(1, min(50, n // threads))  # the reference's 50-peak chunks, split for small samples
        chunks = [list(range(i, min(n, i + csize))) for i in range(0, n, csize)]
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(lambda c: run_regions(c, scan_only), chunks))
        wall = time.perf_counter() - t0
        b = T.RegionBatch(ps, args.samples, keep_membership=False)
        b.synth_fill(args.seed, 0, n, args.indel_pct)
        phases = [sum(p[k] for p in res) for k in range(3)]
        matrix["%s_t%d" % ("scan" if scan_only else "e2e", threads)] = {
            "windows_per_s": b.num_windows / wall, "regions_per_s": n / wall, "regions": n, "threads": threads,
            "wall_s": wall, "windows": b.num_windows,
            "phase_thread_s": {"load_diffs_patch": phases[0], "find_all_matches": phases[1],
                               "count_rows": phases[2]}}
    best = matrix["scan_t%d" % tmax]
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = ncpu
    return {"value": best["windows_per_s"], "unit": "windows/s", "cores": tmax, "kind": "port",
            "host_cpus": {"os_cpu_count": ncpu, "sched_affinity": affinity, "share_used": tmax,
                          "note": "the GPU box shows every host CPU but grants one GPU's job a share of %d; "
                                  "scan_t%d runs the scan-only sample on all %d" % (tmax, ncpu, ncpu)
                          if ncpu > tmax else "all host CPUs used"},
            "sample": "scan-only leg on %d threads: %d of the %d regions of this workload (%d samples, %d "
                      "patterns, %.3g windows); oracle/tfbs_oracle.c (C restatement of the reference scan; gcc "
                      "-O3 -march=x86-64-v3), inputs generated before the clock; matrix: scan-only and "
                      "end-to-end on 1 and %d threads" % (
                          tmax, best["regions"], args.regions, args.samples, len(ps), best["windows"], tmax),
            "matrix": matrix}


def host_bgzf_sample(T, batch, sc, threads, n_regions=8):
    """The host writer (zlib level 6 deflate, the run flow's TFBS_GPU_BGZF=0 and
    multi-device path) on the rows of the first regions: its single-thread rate and
    the time the batch's text would take on `threads` threads at that rate."""
    L = T.lib()
    import ctypes as C
    batch.encode(sc, 0, min(n_regions, batch.num_regions))
    text = b"".join(batch.region_rows(i, "chr1")[0].encode() for i in range(min(n_regions, batch.num_regions)))
    if not text:
        return None
    t = time.perf_counter()
    T.check(L.tfbs_bgzf_write_file(os.devnull.encode(), C.c_char_p(text), len(text), 0))
    dt = time.perf_counter() - t
    return {"sample_bytes": len(text), "seconds_1_thread": dt, "mb_per_s_1_thread": len(text) / dt / 1e6}


def shard_plan(args, rank, world):
    """(first region, regions, pattern shard index, pattern shards) of rank r (SURVEY.md
    8(e)): the 1-D region shard, or the 2-D region x PWM split (module docstring)."""
    if getattr(args, "shard", "regions") == "regions_x_pwms":
        p = args.pwm_shards or (2 if world % 2 == 0 else 1)
        if p < 1 or world % p:
            raise SystemExit("--shard regions_x_pwms: %d ranks are not a multiple of --pwm-shards %d" % (world, p))
        block = rank // p
        return block * p * args.regions, p * args.regions, rank % p, p
    return rank * args.regions, args.regions, 0, 1


def shard_patterns(T, ps, part, parts):
    """The rank's pattern shard: pattern_id % parts == part (both strands of a PWM
    share their id, pattern.rs:73-77)."""
    return ps if parts == 1 else ps.subset(lambda pid: pid % parts == part)


def shard_batch(T, ps, args, rank, world=1, window_lmax=None, build_device=None):
    """Rank r's share: its merged regions of the synthetic chromosome
    (shard_plan), reduced to distinct haplotypes (grouped on build_device where the
    region is SNV-only, else on the host) and packed (with the haplotype -> distinct
    membership the rows need); ps is the rank's pattern shard, window_lmax the whole
    pattern set's L_max when it is a shard."""
    first, count, _, _ = shard_plan(args, rank, world)
    batch = T.RegionBatch(ps, args.samples, keep_membership=True, window_lmax=window_lmax,
                          build_device=build_device)
    batch.synth_fill(args.seed, first, count, args.indel_pct)
    return batch


def job_totals(dist, device, elapsed, sums):
    """Max-over-ranks wall time and whole-job sums.  Regions shard with no exchange, so
    the only collectives are these scalar reductions around the timed region."""
    if dist is None:
        return elapsed, [float(x) for x in sums]
    import torch
    t = torch.tensor(elapsed if isinstance(elapsed, list) else [elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    w = torch.tensor(sums, dtype=torch.float64, device=device)
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    tl = [float(x) for x in t.tolist()]
    return (tl if isinstance(elapsed, list) else tl[0]), [float(x) for x in w.tolist()]


def launch_ranks(args):
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start the same command under
    torch.distributed.run with N ranks on this node as a child process -- nothing here
    has touched a GPU -- and exit with its status."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one JSON line on stdout, from rank 0: every rank's other output (library chatter
    # such as gloo's connection messages included) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w") if rank == 0 else None
    os.dup2(2, 1)
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        if args.dist_backend == "gloo":  # rehearsal: ranks may share a GPU
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)
    rdev = "cuda" if args.dist_backend == "nccl" else "cpu"

    import tfbs_pkg

    T = tfbs_pkg.load()
    threads = max(1, min(CPU_THREADS_MAX, os.cpu_count() or 1))
    work = tempfile.mkdtemp(prefix="tfbs_bench_%d_" % rank)
    names = T.synth_write_pwms(work, args.pwms, args.length_config, args.seed)
    ps_all = T.parse_pwm_files(os.path.join(work, "pwms.txt"), os.path.join(work, "thr"), args.threshold, names)
    first, count, part, parts = shard_plan(args, rank, world)
    ps = shard_patterns(T, ps_all, part, parts)
    sc = T.Scanner(ps, device=local)
    L = T.lib()

    # ---- end-to-end leg, once: host prep, upload, scan, device key reduction, rows
    t_prep = time.perf_counter()
    batch = shard_batch(T, ps, args, rank, world, window_lmax=ps_all.max_length if parts > 1 else None,
                        build_device=None if args.host_build else local)
    dev_regions, host_regions = batch.build_stats()
    patched_regions = batch.patch_stats()
    t_prep = time.perf_counter() - t_prep
    gen_s, build_s, prep_wall, fill_s = batch.prep_seconds()  # prep_wall: build_region + commit, no generation
    t_up = time.perf_counter()
    T.check(L.tfbs_batch_upload(sc.h, batch.h))
    t_up = time.perf_counter() - t_up
    wl_entries, wl_s = (ctypes.c_uint64 * 2)(), ctypes.c_double()
    T.check(L.tfbs_ctx_window_lists(sc.h, wl_entries, ctypes.byref(wl_s)))
    t_scan1 = time.perf_counter()
    T.check(L.tfbs_scan(sc.h, batch.h))
    T.check(L.tfbs_ctx_sync(sc.h))
    t_scan1 = time.perf_counter() - t_scan1
    t_red = time.perf_counter()
    T.check(L.tfbs_batch_reduce(sc.h, batch.h))
    t_red = time.perf_counter() - t_red
    n_rows = n_row_bytes = n_bgzf = 0
    t_rows = t_enc = 0.0
    host_bgzf = None
    if not args.no_e2e:
        # device per-sample encoding, then the rows as BGZF blocks made on the device
        # (tfbs_batch_rows_bgzf: heads on the host, genotype text + deflate + CRC32 on the
        # GPU), 512 regions at a time (the run flow's batch); the blocks reach host memory
        # (the file write is not timed)
        fake = 1
        devnull = os.open(os.devnull, os.O_WRONLY)
        for r0 in range(0, batch.num_regions, 512):
            r1 = min(batch.num_regions, r0 + 512)
            t = time.perf_counter()
            batch.encode(sc, r0, r1, device_codes=True)
            t_enc += time.perf_counter() - t
            t = time.perf_counter()
            nw, fake, nr, nb = batch.rows_bgzf(sc, "chr1", 0, fake, r0, r1, fd=devnull)
            t_rows += time.perf_counter() - t
            n_rows += nr
            n_row_bytes += nb
            n_bgzf += nw
        os.close(devnull)
        rows_split = (ctypes.c_double * 2)()
        T.check(L.tfbs_ctx_rows_bgzf_seconds(sc.h, rows_split))
        host_bgzf = host_bgzf_sample(T, batch, sc, threads)

    # ---- timed loop: one step = the scan and the key assembly of the rank's batch
    # (tfbs_scan: the matrix-core / LUT kernels' hit lists and the reference hits;
    # tfbs_batch_assemble: overflow candidates rescored, spill records bucketed, every
    # region's keys assembled -- reference-window reuse resolved per haplotype --,
    # classified and the varying keys' counts compacted; tfbs_batch_assemble_wait:
    # the host waits and checks every list, rescanning if one overflowed)
    # (tfbs_step: the same three calls in one; from the third step alike on, the scan's
    # and the assembly's launches replay as one hipGraph)
    def step():
        T.check(L.tfbs_step(sc.h, batch.h))

    def step_plain():
        T.check(L.tfbs_scan(sc.h, batch.h))
        T.check(L.tfbs_batch_assemble(sc.h, batch.h))
        T.check(L.tfbs_batch_assemble_wait(sc.h, batch.h))

    for _ in range(args.warmup):
        step()
    T.check(L.tfbs_ctx_sync(sc.h))
    if args.steps is None:  # K from the pace of a few more untimed steps (every rank the same K: the max)
        t = time.perf_counter()
        for _ in range(3):
            step()
        T.check(L.tfbs_ctx_sync(sc.h))
        pace = (time.perf_counter() - t) / 3
        k = max(5, min(100000, int(math.ceil(args.min_seconds / max(pace, 1e-6)))))
        if dist is not None:
            import torch
            kt = torch.tensor([k], dtype=torch.int64, device=rdev)
            dist.all_reduce(kt, op=dist.ReduceOp.MAX)
            k = int(kt.item())
        args.steps = k

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    T.check(L.tfbs_ctx_sync(sc.h))
    if dist is not None:
        import torch
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    # the steps' device times (HIP events), read after further steps outside the timed
    # loop: reading them syncs on each step's events, which is not part of a step
    kernel_ms, mfma_ms, asm_ms = [], [], []
    for _ in range(min(args.steps, 10)):
        step_plain()  # (graph steps carry no timing events)
        kernel_ms.append(L.tfbs_ctx_last_scan_ms(sc.h))  # the scan's launches (HIP events)
        mfma_ms.append(L.tfbs_ctx_last_mfma_ms(sc.h))   # the matrix-core kernel alone (-1: none ran)
        asm_ms.append(L.tfbs_ctx_last_assemble_ms(sc.h))  # the assembly's launches
    T.check(L.tfbs_ctx_sync(sc.h))
    # the last step's list counters (device atomics, one per wave): candidates, the part
    # of them in the waves' global lists, hit-list pairs, spill records, overflow
    lc = (ctypes.c_uint64 * 5)()
    T.check(L.tfbs_ctx_scan_counters(sc.h, lc))
    list_counters = {"candidates": lc[2], "candidates_global": lc[3], "hit_pairs": lc[4], "spill_records": lc[0],
                     "candidates_overflow": lc[1],
                     # bytes the scan writes to its lists: 8 per global candidate and per hit pair,
                     # 12 per spill / overflow record, 4 per wave's hit count
                     "list_bytes": 8 * (lc[3] + lc[4]) + 12 * (lc[0] + lc[1])}

    # the dense download, for reference (the run flow uses the key reduction)
    t_dense = time.perf_counter()
    T.check(L.tfbs_batch_download(sc.h, batch.h))
    t_dense = time.perf_counter() - t_dense

    e2e_s = prep_wall + t_up + t_scan1 + t_red + t_enc + t_rows
    if host_bgzf:
        host_bgzf["estimate_s_%d_threads" % threads] = n_row_bytes / (host_bgzf["mb_per_s_1_thread"] * 1e6 * threads)
    per_rank_ms = [elapsed * 1e3 / args.steps]
    if dist is not None:  # every rank's ms per step, as the collective saw them
        import torch
        g = [torch.zeros(1, dtype=torch.float64, device=rdev) for _ in range(world)]
        dist.all_gather(g, torch.tensor(per_rank_ms, dtype=torch.float64, device=rdev))
        per_rank_ms = [float(x.item()) for x in g]
    (elapsed, e2e_max), tot = job_totals(dist, rdev, [elapsed, e2e_s],
                                         [batch.num_windows, batch.num_regions, batch.num_effective_windows,
                                          n_rows, n_row_bytes, batch.num_scan_windows, n_bgzf])
    tot_windows, tot_regions, tot_eff, tot_rows, tot_row_bytes, tot_scan, tot_bgzf = tot

    if rank == 0:
        steps = args.steps
        value = tot_windows * steps / elapsed
        kms = sum(kernel_ms) / len(kernel_ms)
        mms = sum(mfma_ms) / len(mfma_ms)
        ams = sum(asm_ms) / len(asm_ms)
        path = "mfma" if mms > 0 else "lut"
        prof, traffic_src = pmc_profile(args, path)
        traffic = prof["hbm_bytes_per_step"] if prof else None
        pattern_bytes = 0
        for p in ps.to_list():
            pattern_bytes += ((len(p) + 15) // 16) * 1536 + 16 * len(p) + 24
        # the scan's outputs are sparse (haplotype, key) hit lists (8 bytes per hit, a few MB
        # per step): no dense count matrix is written for the matrix-core path
        alg_bytes = batch.input_bytes + pattern_bytes + (batch.output_bytes if mms <= 0 else 0)
        # executed work: the cells of the windows the scan reads (reference-window
        # reuse leaves the others to the reference's result)
        scan_cells = batch.num_scan_cell_ops
        cell_tops = scan_cells / (kms / 1e3) / 1e12
        if mms > 0:  # the matrix-core kernel scored every strand of this workload
            mops = MFMA_OPS_PER_CELL * scan_cells / (mms / 1e3) / 1e12
            rp = prof.get("rocprof_phase_ms") if prof else None
            roof = {"bound": "mfma", "achieved": mops, "peak": MFMA_F6_PEAK_TOPS, "unit": "TFLOP/s",
                    "frac": mops / MFMA_F6_PEAK_TOPS, "traffic": traffic,
                    "kernel": "scan_mfma_all_kernel<staged> (one launch: a workgroup per group of 64 haplotypes over every super tile; TFBS_SCAN_MERGED=0: scan_mfma_kernel<staged, K depth>, one launch per depth class)",
                    "kernel_ms": mms,
                    # the same figure on the rocprofv3 kernel trace's MFMA phase (same library build)
                    "rocprof_phase_ms": rp,
                    "frac_rocprof": (MFMA_OPS_PER_CELL * scan_cells / (rp / 1e3) / 1e12 / MFMA_F6_PEAK_TOPS
                                     if rp else None),
                    "traffic_per_algorithmic_byte": traffic / alg_bytes if traffic else None,
                    "frac_source": "frac: HIP events on the ctx stream around the MFMA phase (this run); "
                                   "frac_rocprof: the same phase on the rocprofv3 kernel trace of this build "
                                   "(profiles/pmc_traffic_<W>.json)",
                    "list_counters": list_counters,
                    "write_per_list_byte": (prof["write_bytes"] / list_counters["list_bytes"]
                                            if prof and prof.get("write_bytes") and list_counters["list_bytes"]
                                            else None),
                    "sq": prof.get("sq") if prof else None,
                    "note": "achieved = 8 ops per (window, strand, column) cell of the FP4 one-hot x FP6 "
                            "bound-digit GEMM x %.4g cells the scan reads (of %.4g: reference-window reuse) / "
                            "the MFMA phase's HIP-event time (first launch to last, joined on the ctx stream; "
                            "tools/trace_phase.py reads the same phase from the rocprofv3 trace); traffic = HBM "
                            "bytes of the phase's dispatches per step, FETCH_SIZE x2 (gfx950) + WRITE_SIZE, "
                            "from %s" % (scan_cells, batch.num_cell_ops, traffic_src)}
            hbm_ms = mms
        else:
            roof = None
            hbm_ms = kms
        achieved = alg_bytes / (hbm_ms / 1e3) / 1e9
        hbm = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
               "note": "algorithmic bytes/step = packed haplotypes + metadata (%d B) + pattern tables (%d B)%s; "
                       "the scan is compute bound" % (
                           batch.input_bytes, pattern_bytes,
                           " + u32 counts (%d B)" % batch.output_bytes if mms <= 0 else
                           " (the sparse hit lists, 8 B per hit, are not counted)")}
        if roof is None:
            roof = hbm
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
                "workload": args.workload + ("-custom" if args.custom else ""),
                "samples": args.samples, "haplotypes": 2 * args.samples, "regions_per_gpu": args.regions,
                "regions_per_rank_batch": count,
                "region_bp": 201, "pwms": args.pwms, "patterns": len(ps), "threshold": args.threshold,
                "indel_pct": args.indel_pct, "seed": args.seed,
                "distinct_haplotypes_per_gpu": batch.num_haplotypes,
                "windows_per_step": int(tot_windows),
                "parallelism": ("region shard x%d" % world if parts == 1 else
                                "region x PWM shard: %d region blocks x %d pattern shards" % (world // parts, parts)),
                "scan_path": path,
                "scanned_windows_per_step": int(tot_scan),
                "window_list_entries": [int(wl_entries[0]), int(wl_entries[1])],
            },
            "value_note": "windows of every distinct haplotype resolved per second, scan AND key assembly in "
                          "the timed step (the reference scores each window and counts its hits per key, "
                          "main.rs:94-154, 500-534); a haplotype's windows whose bases and positions equal the "
                          "region's reference window take the reference window's hits in the assembly (reference-"
                          "window reuse, exact; TFBS_DEDUP=0 scans them all); scanned_windows_per_s counts the "
                          "windows the kernels read",
            "step": "tfbs_step = tfbs_scan + tfbs_batch_assemble + tfbs_batch_assemble_wait (host sync and "
                    "list check every step; from the third step alike the launches replay as one hipGraph): "
                    "scan kernels, overflow rescoring, spill bucketing, key assembly + classification + "
                    "varying-count compaction of every region of the batch",
            "step_device_ms": {"scan": kms, "mfma_phase": mms, "assemble": ams},
            "ranks": {"world_size": world, "backend": args.dist_backend if dist is not None else None,
                      "ms_per_step": per_rank_ms},
            "scanned_windows_per_s": tot_scan * steps / elapsed,
            "scan_regions_per_s": tot_regions * steps / elapsed,
            "effective_windows_per_s": tot_eff * steps / elapsed,
            "end_to_end": {
                # definition v3 (round 3 on): host prep wall (build_region + commit; the synthetic
                # generation excluded) + upload + scan + key reduction + device encode + device BGZF
                # rows written to /dev/null.  v2 (round 2) summed the whole synthetic fill and host rows.
                "definition": "v3",
                "regions_per_s": tot_regions / e2e_max,
                "windows_per_s": tot_windows / e2e_max,
                "seconds": e2e_max,
                "note": "one pass over the rank's batch: haplotype reconstruction (load_diffs/group on the GPU "
                        "for SNV-only regions, else on the host; patch/dedup/pack on %d host threads, a chunk's "
                        "layout commit overlapping the next chunk's build; the synthetic records are generated "
                        "before each chunk, outside the clock, as for the CPU baseline) + upload "
                        "+ scan + device key reduction + device "
                        "per-sample encoding + the VCF rows as BGZF blocks made on the GPU and written out (%d rows, "
                        "%.3g bytes of text deflated to %.3g bytes, to /dev/null)" % (
                            threads, tot_rows, tot_row_bytes, tot_bgzf),
                "bgzf_bytes": int(tot_bgzf),
                "host_bgzf_writer": host_bgzf,
                "rank0_phases_s": {"host_prep_wall": prep_wall, "synthetic_generation_wall": fill_s - prep_wall,
                                   "synthetic_generation_thread_s": gen_s, "build_region_thread_s": build_s,
                                   "upload": t_up, "upload_window_lists": wl_s.value, "scan": t_scan1,
                                   "key_reduce": t_red,
                                   "device_encode": t_enc, "rows_bgzf": t_rows,
                                   "rows_bgzf_host_plan": rows_split[0] if not args.no_e2e else 0.0,
                                   "rows_bgzf_device_and_write": rows_split[1] if not args.no_e2e else 0.0},
                "rows": int(tot_rows),
                "regions_grouped_on_device": int(dev_regions),
                "regions_built_on_host": int(host_regions),
                "regions_grouped_on_device_patched_on_host": int(patched_regions),
            },
            "kernel_ms_avg": kms,
            "dense_download_s": t_dense,
            "roofline": roof,
            "hbm_roofline": hbm,
            "vs_valu_peak": {"achieved": cell_tops, "peak": VALU_PEAK_TOPS,
                             "unit": "T column-lookups/s vs T int32 lane-ops/s",
                             "ratio": cell_tops / VALU_PEAK_TOPS,
                             "note": "not a roofline: the executed (window, strand, column) lookups per second "
                                     "against the chip's int32 VALU peak (one lane-op per lookup); > 1 means "
                                     "no VALU formulation of the scan could reach this rate"},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(T, ps, args, args.cpu_seconds)
        print(json.dumps(out), file=json_out, flush=True)
    sc.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
