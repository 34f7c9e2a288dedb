#!/bin/bash
# Same-box A/B of library builds: the in-tree build ("base") and each
# find-tfbs_amd/lib/probe<NAME>/libtfbs_amd.so, on tools/tune.py batches of
# the given length configs (2: L 8-15 = K depth 1 only, 3: C3's mix, 5: L 25-30
# = depth 2 only), then a GPU parity subset per build.  Every step has its own
# time limit; the first failure ends the script.
# Usage: bash tools/exp_libs.sh TAG "LENGTH_CONFIGS" NAME...
OUT=gpurun_out/${1:?tag}; shift
LCS=${1:-3}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for lc in $LCS; do
  for rep in 1 2; do
    for lib in base "$@"; do
      if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
      timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 4 --length-config $lc > $OUT/${lib}_lc${lc}_$rep.log 2>&1 || { echo "tune $lib failed"; tail -5 $OUT/${lib}_lc${lc}_$rep.log; exit 1; }
    done
  done
done
unset TFBS_LIB
for lib in "$@"; do
  TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fuzz or split_edges or synthetic_regions or dense_hits or invariant" > $OUT/parity_$lib.log 2>&1 || { echo "parity $lib FAILED"; tail -20 $OUT/parity_$lib.log; exit 1; }
  echo "parity $lib: $(tail -1 $OUT/parity_$lib.log)"
done
for f in $OUT/*_lc*.log; do echo "$(basename $f .log): $(grep -h median $f | sed 's/  */ /g')"; done
