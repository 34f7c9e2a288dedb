#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc pass over bench.py: counters summed over the
dispatches of the last scan step's MFMA phase (every scan_mfma_kernel dispatch
after the last non-MFMA dispatch that precedes them -- one per K depth and hap
group chunk), plus the dispatches' kernel names.

Usage: python tools/pmc_summary.py PMC_DIR [KERNEL]  -> PMC_DIR/pmc_summary.json
       KERNEL (a substring of the kernel name): that kernel's last dispatch instead
       (e.g. key_fast_kernel), -> PMC_DIR/pmc_summary_KERNEL.json
"""
import csv
import glob
import json
import os
import re
import sys


def last_phase(rows):
    """Dispatch ids of the last run of consecutive scan_mfma_kernel dispatches."""
    names = {}
    for r in rows:
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    run, best = [], []
    for d in sorted(names):
        if re.search(r"scan_mfma(_all)?_kernel", names[d]):
            run.append(d)
        else:
            if run:
                best = run
            run = []
    return set(run or best), names


def last_of(rows, sub):
    """The last dispatch of a kernel whose name contains sub."""
    names = {}
    for r in rows:
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    ds = [d for d in sorted(names) if sub in names[d]]
    return ({ds[-1]} if ds else set()), names


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else None
    files = glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)
    out = {"_files": files}
    for f in files:
        rows = list(csv.DictReader(open(f)))
        take, names = last_of(rows, sub) if sub else last_phase(rows)
        if not take:
            continue
        kern = {}
        for r in rows:
            d = int(r["Dispatch_Id"])
            if d in take:
                out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for d in sorted(take):
            m = re.search(r"scan_mfma(_all)?_kernel<[^>]*>", names[d])
            k = m.group(0) if m else names[d].split("(")[0][-60:]
            kern[k] = kern.get(k, 0) + 1
        out["_dispatches"] = len(take)
        out["_kernels"] = kern
    name = "pmc_summary.json" if not sub else "pmc_summary_%s.json" % sub
    json.dump(out, open(os.path.join(root, name), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
