#!/bin/bash
# PMC passes over the scan (separate rocprofv3 runs; counters per MI355X_MICROARCH.md).
# Usage: tools/pmc.sh OUTDIR [bench args...]
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu "${BARGS[@]}" > $OUT/$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $OUT/$name.log; return 1; }
}
BARGS=("$@")
run fetch FETCH_SIZE && run write WRITE_SIZE && run sq1 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES && run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && python3 tools/pmc_summary.py $OUT
