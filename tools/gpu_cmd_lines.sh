# The GPU suite, then the bench line of every BASELINE config (C3 first) at HEAD.
set -o pipefail
T=${1:-lines}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for w in C3 C2 C4 C5; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 4 > $O/bench_$(echo $w | tr C c).json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
done
