#!/usr/bin/env python3
"""MFMA scan phase from a rocprofv3 kernel trace.

One scan step launches one scan_mfma_kernel per K depth, spread over four
streams, so the step's MFMA phase is the union of those dispatches: from the
first start to the last end of each run of consecutive scan_mfma dispatches
(the counts memset that opens every step ends a run).  This is the figure
bench.py's roofline divides by (HIP events around the launches on the ctx
stream); per-kernel averages are listed beside it.

Usage: python tools/trace_phase.py TRACE_CSV [OUT_JSON]
"""
import csv
import json
import re
import statistics
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
    steps, cur = [], []
    for r in rows:
        if re.search(r"scan_mfma(_all)?_kernel", r["Kernel_Name"]):
            cur.append(r)
        elif cur:
            steps.append(cur)
            cur = []
    if cur:
        steps.append(cur)
    per_kernel = {}
    out_steps = []
    for st in steps:
        t0 = min(int(r["Start_Timestamp"]) for r in st)
        t1 = max(int(r["End_Timestamp"]) for r in st)
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st)
        out_steps.append({"dispatches": len(st), "phase_ms": (t1 - t0) / 1e6, "sum_of_kernel_ms": busy / 1e6})
        for r in st:
            m = re.search(r"scan_mfma(_all)?_kernel<[^>]*>", r["Kernel_Name"])
            key = m.group(0) if m else r["Kernel_Name"][:60]
            per_kernel.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    timed = out_steps[1:] if len(out_steps) > 1 else out_steps  # the first step is the warmup
    out = {"source": sys.argv[1], "steps": out_steps,
           "phase_ms_mean_after_first": statistics.mean(s["phase_ms"] for s in timed) if timed else None,
           "per_kernel_ms_mean": {k: statistics.mean(v) for k, v in sorted(per_kernel.items())}}
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
