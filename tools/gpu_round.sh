#!/bin/bash
# One GPU session: parity tests, the default bench, a rocprofv3 kernel trace and
# PMC passes (separate, as MI355X_MICROARCH.md's HBM section prescribes).
# Usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1
echo "gpu tests rc=$?"; tail -3 $OUT/gpu_tests.log
timeout -k 10 500 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/prof.log 2>&1 || { echo "rocprof trace failed"; tail -20 $OUT/prof.log; exit 1; }
python3 tools/trace_phase.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) $OUT/mfma_phase.json > /dev/null
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu "$@" > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu "$@" > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -20 $OUT/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o pmc -- python3 bench.py --steps 2 --warmup 0 --no-cpu "$@" > $OUT/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 $OUT/pmc_sq.log; }
for p in pmc_fetch pmc_write pmc_sq; do python3 tools/pmc_summary.py $OUT/$p > $OUT/sum_$p.json 2>&1; done
find $OUT -name "*.csv" | head -20
