#!/bin/bash
# One measured configuration on the GPU box: the bench line, a rocprofv3 kernel
# trace (--kernel-trace --stats) of the same command, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ counters; separate runs as MI355X_MICROARCH.md's
# HBM section prescribes), each step under its own time limit, stopping at the
# first failure.  Summaries land in gpurun_out/TAG/ (and
# profiles/pmc_traffic_<workload>.json, which bench.py reads back when its
# arguments match).
# Usage: tools/profile_round.sh TAG [bench.py args, e.g. --workload C5]
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step bench
timeout -k 10 400 python3 bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- python3 bench.py "$@" --steps 3 --warmup 1 --no-cpu --no-e2e > $OUT/prof.log 2>&1 || { echo "rocprof trace failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_phase.py "$(find $OUT/prof -name '*kernel_trace.csv' | head -1)" $OUT/mfma_phase.json > /dev/null || exit 1
cp "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" $OUT/kernel_stats.csv
for pass in fetch:FETCH_SIZE write:WRITE_SIZE "sq:SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
  name=${pass%%:*}; counters=${pass#*:}
  step "pmc $name"
  timeout -s KILL 300 rocprofv3 --pmc $counters --output-format csv -d $OUT/pmc_$name -o pmc -- python3 bench.py "$@" --steps 2 --warmup 0 --no-cpu --no-e2e > $OUT/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -20 $OUT/pmc_$name.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/pmc_$name > /dev/null || exit 1
done
python3 tools/pmc_traffic.py $OUT "$@" > $OUT/pmc_traffic.json || exit 1
cp profiles/pmc_traffic_*.json $OUT/ 2>/dev/null
step done
