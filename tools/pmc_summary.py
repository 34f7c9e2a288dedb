#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for the scan kernels: per-dispatch counter sums."""
import csv
import glob
import json
import os
import sys

out = {}
root = sys.argv[1]
for f in glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    disp = sorted({int(r["Dispatch_Id"]) for r in rows if "scan_" in r["Kernel_Name"]})
    if not disp:
        continue
    d = disp[-1]  # last scan dispatch of the run (warm)
    for r in rows:
        if int(r["Dispatch_Id"]) == d and "scan_" in r["Kernel_Name"]:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out["_kernel"] = r["Kernel_Name"][:60]
            out["_grid"] = r["Grid_Size"]
            out["_vgpr"] = r["VGPR_Count"]
            out["_lds"] = r["LDS_Block_Size"]
json.dump(out, open(os.path.join(root, "pmc_summary.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
