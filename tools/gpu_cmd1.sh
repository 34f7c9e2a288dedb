# GPU suite, the C3 bench line, a kernel trace of the bench and the multi-rank rehearsals.
set -o pipefail
O=gpurun_out/${1:-sp1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1
rc=$?
tail -30 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 4 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/prof.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --gpus 2 --dist-backend gloo --workload C2 --steps 5 --warmup 2 --no-cpu > $O/b2.json 2> $O/b2.err || exit 1
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --shard regions_x_pwms --regions 2000 --steps 5 --warmup 2 --no-cpu > $O/b2x.json 2> $O/b2x.err
