#!/bin/bash
# Same-box kernel times of the in-tree build and probe/variant builds
# (find-tfbs_amd/lib/probe<NAME>) on one command: rocprofv3 --kernel-trace --stats
# per build, then the kernels matching PATTERN (average ns, calls) side by side.
# Usage: bash tools/ab_kernels.sh TAG PATTERN "COMMAND" NAME...
OUT=gpurun_out/${1:?tag}; PAT=$2; CMD=$3; shift 3
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
    timeout -k 10 ${ABT:-200} rocprofv3 --kernel-trace --stats -d $OUT/${lib}_$rep -o t --output-format csv -- $CMD > $OUT/${lib}_$rep.log 2>&1 || { echo "$lib failed"; tail -5 $OUT/${lib}_$rep.log; exit 1; }
    f=$(find $OUT/${lib}_$rep -name '*kernel_stats.csv' | head -1)
    echo "$lib rep$rep: $(grep -h -E "$PAT" $f | awk -F, '{gsub(/"/,"",$1); printf "%s calls=%s avg_us=%.1f total_ms=%.2f | ", substr($1,1,40), $2, $4/1000, $3/1e6}')"
  done
done
