# End-of-round check of HEAD: the GPU suite, the C3 profile set (bench line, kernel trace, PMC
# passes) and the C4 / C5 bench lines.
set -o pipefail
T=${1:-r3f}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1
rc=$?
tail -20 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh ${T}_c3 --cpu-seconds 4 || exit 1
for w in C4 C5; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 4 > $O/bench_$(echo $w | tr C c).json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
done
