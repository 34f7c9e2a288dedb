# The GPU suite, then the C3 bench line without the CPU leg and a kernel trace of the bench.
set -o pipefail
O=gpurun_out/${1:-q1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=10 > $O/gpu_tests.log 2>&1
rc=$?
tail -16 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $O/prof.log 2>&1
