#!/bin/bash
# One GPU session of kernel experiments: tune.py over env variants and over
# probe builds (tools/probe_build.sh), then the PMC passes of tools/pmc_mfma.sh.
# Usage: bash tools/exp.sh OUTDIR "ENV=a,b ..." LIB_NAME...
OUT=gpurun_out/${1:-exp}; shift
VARS=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/tune.py --regions 2000 --rounds 5 $VARS > $OUT/tune_default.log 2>&1 || { tail -5 $OUT/tune_default.log; exit 1; }
for lib in "$@"; do
  TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so timeout -k 10 300 python tools/tune.py --regions 2000 --rounds 5 > $OUT/tune_$lib.log 2>&1 || { tail -5 $OUT/tune_$lib.log; exit 1; }
done
for f in $OUT/tune_*.log; do echo "== $f"; grep -h "median\|probe4\|MISMATCH" $f | sort | uniq -c | sort -rn | head -8; done
