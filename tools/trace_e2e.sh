#!/bin/bash
# Kernel trace of one bench run's end-to-end leg (device grouping, scan, assembly,
# encode, BGZF rows): rocprofv3 --kernel-trace --stats over bench.py with one timed
# step and no CPU baseline.  Usage: tools/trace_e2e.sh TAG [bench.py args]
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- python3 bench.py "$@" --steps 1 --warmup 0 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "trace failed"; tail -5 $OUT/bench.err; exit 1; }
cp "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv | cut -d, -f1-4 | sed 's/(tfbs::[^)]*)//; s/tfbs::(anonymous namespace):://'
