#!/bin/bash
# Round-4 iteration check on the GPU box: selected GPU tests (pytest -k EXPR, or
# none when EXPR is "-"), the key assembly's phase clocks (TFBS_KF_PROF) for the
# in-tree build and the probe builds named after it, and optionally the 50k-sample
# run flow (RUNFLOW=1).  Usage: tools/gpu_iter_r4.sh TAG EXPR [PROBE...]
set -o pipefail
T=${1:?tag}; K=${2:--}; shift 2
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
if [ "$K" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in base "$@"; do
  if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
  TFBS_KF_PROF=1 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $O/kf_$lib.json 2> $O/kf_$lib.err || { echo "$lib failed"; tail -5 $O/kf_$lib.err; exit 1; }
  echo "$lib: $(grep -o '"ms_per_step": [0-9.]*' $O/kf_$lib.json) $(grep -o '"assemble": [0-9.]*' $O/kf_$lib.json)"
  grep "kf prof" $O/kf_$lib.err | tail -1
done
unset TFBS_LIB
if [ "${RUNFLOW:-0}" = 1 ]; then
  timeout -k 10 600 python3 tools/bench_run.py --samples 50000 --regions 1000 > $O/run_50k.json 2> $O/run_50k.err || { echo "run flow failed"; tail -5 $O/run_50k.err; exit 1; }
  grep -h tfbs_run_timing $O/run_50k.err; tail -c 700 $O/run_50k.json
fi
