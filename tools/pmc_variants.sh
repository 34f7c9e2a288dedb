#!/bin/bash
# One PMC pass (instruction mix + cycles) of the tune.py workload per library
# build: the in-tree one and find-tfbs_amd/lib/probe<NAME> for each NAME.
# Usage: bash tools/pmc_variants.sh OUTDIR NAME...
OUT=gpurun_out/${1:-pmcv}; shift
mkdir -p $OUT
export TMPDIR=/tmp TFBS_MFMA=1
set="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
for v in default "$@"; do
  lib=""
  [ $v != default ] && lib=find-tfbs_amd/lib/probe$v/libtfbs_amd.so
  TFBS_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$v/x -o pmc -- python3 tools/tune.py --regions 2000 --rounds 1 > $OUT/$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/$v.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/$v > $OUT/$v.json 2>&1
  echo "== $v: $(python3 -c "import json;d=json.load(open('$OUT/$v.json'));print({k:d.get(k) for k in ['SQ_INSTS_VALU','SQ_INSTS_MFMA','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_WAVE_CYCLES','SQ_WAIT_INST_ANY','GRBM_GUI_ACTIVE','SQ_VALU_MFMA_BUSY_CYCLES']})")"
done
