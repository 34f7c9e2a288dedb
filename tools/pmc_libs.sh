#!/bin/bash
# One PMC pass (instruction mix + cycles) of the tune.py workload per library
# build: "base" (in-tree) and find-tfbs_amd/lib/probe<NAME>; prints a table.
# Usage: bash tools/pmc_libs.sh TAG LENGTH_CONFIG NAME...
OUT=gpurun_out/${1:?tag}; shift
LC=${1:-3}; shift
mkdir -p $OUT
export TMPDIR=/tmp
set="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
for v in base "$@"; do
  if [ $v = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$v/libtfbs_amd.so; fi
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/lc${LC}_$v -o pmc -- python3 tools/tune.py --regions 2000 --rounds 1 --length-config $LC > $OUT/lc${LC}_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/lc${LC}_$v.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/lc${LC}_$v > /dev/null 2>&1
  python3 -c "
import json;d=json.load(open('$OUT/lc${LC}_$v/pmc_summary.json'))
m=d.get('SQ_INSTS_MFMA',1)
print('lc$LC %-8s VALU %.3g (%.1f/MFMA) MFMA %.3g SALU %.3g LDS %.3g waveCyc %.3g waitInst %.3g gui %.3g mfmaBusy %.3g' % ('$v', d.get('SQ_INSTS_VALU',0), d.get('SQ_INSTS_VALU',0)/m, m, d.get('SQ_INSTS_SALU',0), d.get('SQ_INSTS_LDS',0), d.get('SQ_WAVE_CYCLES',0), d.get('SQ_WAIT_INST_ANY',0), d.get('GRBM_GUI_ACTIVE',0), d.get('SQ_VALU_MFMA_BUSY_CYCLES',0)))"
done
unset TFBS_LIB
