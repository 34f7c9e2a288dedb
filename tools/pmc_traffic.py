#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json (roofline.traffic for bench.py) from the
FETCH_SIZE / WRITE_SIZE passes of tools/gpu_round.sh.

Usage: python tools/pmc_traffic.py gpurun_out/TAG [regions] [scan_path]
FETCH_SIZE and WRITE_SIZE are KiB per dispatch (rocprofv3); the dominant scan
kernel's last dispatch is used.  The gfx950 x2 correction of FETCH_SIZE applies
to 16-B-per-lane streaming reads only (MI355X_MICROARCH.md, HBM); the scan's
memory-side reads are the staging copies of the tables and the haplotype words
(16-B and 4-B per lane), so both the raw and the corrected figures are kept and
the raw one is reported."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    root = sys.argv[1]
    regions = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    path = sys.argv[3] if len(sys.argv) > 3 else "mfma"
    s = json.load(open(os.path.join(root, "sum_pmc_fetch.json")))
    s.update(json.load(open(os.path.join(root, "sum_pmc_write.json"))))
    fetch, write = s["FETCH_SIZE"] * 1024, s["WRITE_SIZE"] * 1024
    out = {"workload": "C3", "regions": regions, "scan_path": path, "kernel": s.get("_kernel"),
           "fetch_bytes": fetch, "write_bytes": write, "hbm_bytes_per_launch": fetch + write,
           "fetch_bytes_x2_corrected": 2 * fetch,
           "source": os.path.join(root, "sum_pmc_{fetch,write}.json") + " (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, "
                     "separate passes, last scan dispatch)"}
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
