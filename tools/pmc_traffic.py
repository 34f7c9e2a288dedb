#!/usr/bin/env python3
"""profiles/pmc_traffic_<workload>.json: HBM bytes per scan step of the MFMA
phase (bench.py's roofline.traffic) from the FETCH_SIZE and WRITE_SIZE passes
tools/profile_round.sh ran over the same bench.py arguments, with the MFMA phase
of the same run's kernel trace (tools/trace_phase.py: mfma_phase.json) and the SQ
pass, all stamped with the SHA-256 of the library they profiled: bench.py uses
the file only when that hash is the running library's.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (rocprofv3), summed over the last
step's scan_mfma_kernel dispatches (tools/pmc_summary.py).  On gfx950
FETCH_SIZE reports half the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section): it is doubled; WRITE_SIZE is taken as is.

Usage: python tools/pmc_traffic.py OUT_DIR [bench.py args...]
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    root = sys.argv[1]
    sys.argv = ["bench.py"] + sys.argv[2:]
    import bench
    args = bench.parse()
    f = json.load(open(os.path.join(root, "pmc_fetch", "pmc_summary.json")))
    w = json.load(open(os.path.join(root, "pmc_write", "pmc_summary.json")))
    fetch, write = f["FETCH_SIZE"] * 1024, w["WRITE_SIZE"] * 1024
    out = {"config": bench.workload_key(args), "scan_path": "mfma", "library_sha256": bench.library_sha256(),
           "kernels": f.get("_kernels"), "dispatches": f.get("_dispatches"),
           "fetch_size_bytes": fetch, "fetch_bytes_x2": 2 * fetch, "write_bytes": write,
           "hbm_bytes_per_step": 2 * fetch + write,
           "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes over `bench.py %s "
                     "--steps 2 --warmup 0 --no-cpu --no-e2e`, the last step's scan_mfma_kernel dispatches "
                     "summed, FETCH_SIZE x2" % " ".join(sys.argv[1:])}
    ph = os.path.join(root, "mfma_phase.json")
    if os.path.exists(ph):  # the kernel trace of the same command (--kernel-trace --stats pass)
        p = json.load(open(ph))
        out["rocprof_phase_ms"] = p["phase_ms_mean_after_first"]
        out["rocprof_per_kernel_ms"] = p["per_kernel_ms_mean"]
    sq = os.path.join(root, "pmc_sq", "pmc_summary.json")
    if os.path.exists(sq):  # the SQ pass: instruction mix of the same dispatches
        q = json.load(open(sq))
        out["sq"] = {k: v for k, v in q.items() if not k.startswith("_")}
    dst = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % args.workload)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
