#!/bin/bash
# A/B the scan kernel of two library builds on the same box: alternating tune.py
# runs (the in-tree build vs find-tfbs_amd/lib/old/libtfbs_amd.so).
# Usage: bash tools/ab.sh OUTDIR [length-configs...]
OUT=gpurun_out/${1:-ab}; shift
mkdir -p $OUT
for lc in ${@:-3}; do
  for rep in 1 2; do
    TFBS_LIB=find-tfbs_amd/lib/old/libtfbs_amd.so timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 3 --length-config $lc > $OUT/old_lc${lc}_$rep.log 2>&1 || exit 1
    timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 3 --length-config $lc > $OUT/new_lc${lc}_$rep.log 2>&1 || exit 1
  done
done
for f in $OUT/*.log; do echo "$(basename $f): $(grep -h median $f | sed "s/  */ /g")"; done
