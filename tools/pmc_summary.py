#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for the scan kernels: per-dispatch counter sums."""
import csv
import glob
import json
import os
import sys

out = {}
root = sys.argv[1]
for f in glob.glob(os.path.join(root, "pmc_counter_collection.csv")) + glob.glob(
        os.path.join(root, "*", "pmc_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    # the last scan step: the last run of consecutive scan dispatches (one per
    # K depth for the MFMA path), counters summed over its dispatches
    kinds = {}
    for r in rows:
        kinds[int(r["Dispatch_Id"])] = "scan_" in r["Kernel_Name"]
    ids = sorted(kinds)
    last = []
    for d in ids:
        if kinds[d]:
            last = last + [d] if last and last[-1] == ids[ids.index(d) - 1] else [d]
    if not last:
        continue
    take = set(last)
    seen = set()
    for r in rows:
        d = int(r["Dispatch_Id"])
        if d in take:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out["_kernel"] = r["Kernel_Name"][:60]
            out["_dispatches"] = len(take)
            out["_grid"] = r["Grid_Size"]
            out["_vgpr"] = r["VGPR_Count"]
            out["_lds"] = r["LDS_Block_Size"]
json.dump(out, open(os.path.join(root, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
