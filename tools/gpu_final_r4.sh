# Round-4 measurement set, part A (the GPU suite and the C3 profile) or B (the
# other workloads' bench lines and the run flow).  Usage: tools/gpu_final_r4.sh TAG A|B
set -o pipefail
T=${1:?tag}; PART=${2:-A}
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" = A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1
  rc=$?; tail -5 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  bash tools/profile_round.sh ${T}_c3 || exit 1
  bash tools/pmc_scan_stalls.sh ${T}_stall || exit 1
else
  for w in C2 C4 C5; do
    timeout -k 10 400 python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
    echo "$w: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$w.json) $(grep -o '"regions_per_s": [0-9.]*' $O/bench_$w.json | head -1)"
  done
  timeout -k 10 600 python3 tools/bench_run.py --samples 50000 --regions 1000 > $O/run_50k.json 2> $O/run_50k.err || { echo "run flow failed"; tail -5 $O/run_50k.err; exit 1; }
  tail -c 600 $O/run_50k.json
  timeout -k 10 600 python3 tools/bench_run.py --samples 50000 --regions 1000 --devices 0,0 --oracle-seconds 0 > $O/run_50k_2dev.json 2> $O/run_50k_2dev.err || { echo "run flow (2 shards) failed"; tail -5 $O/run_50k_2dev.err; exit 1; }
  tail -c 400 $O/run_50k_2dev.json
fi
