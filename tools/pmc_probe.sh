#!/bin/bash
# SQ instruction counters and the MFMA-phase time of one library build (the
# product, or a tools/probe_build.sh probe) on the C3 bench workload.
# Usage: tools/pmc_probe.sh OUTDIR [LIB]   (LIB: path of a libtfbs_amd.so)
set -o pipefail
OUT=${1:?outdir}; LIB=${2:-}
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export TFBS_LIB=$LIB
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu --no-e2e > $OUT/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py $OUT/pmc_sq > $OUT/pmc_sq.json || exit 1
python3 - $OUT <<'PY'
import json, sys
o = sys.argv[1]
b = json.load(open(o + "/bench.json")); p = json.load(open(o + "/pmc_sq.json"))
print(o, "mfma_phase_ms %.2f" % b["roofline"]["kernel_ms"], "VALU %.3g MFMA %.3g SALU %.3g LDS %.3g conflicts %.3g" % (
    p["SQ_INSTS_VALU"], p["SQ_INSTS_MFMA"], p["SQ_INSTS_SALU"], p["SQ_INSTS_LDS"], p["SQ_LDS_BANK_CONFLICT"]))
PY
