# The BGZF and device-build tests, then the C3 bench line (no CPU leg) and its kernel trace.
set -o pipefail
O=gpurun_out/${1:-z1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py tests/test_gpu_build.py -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1
rc=$?
tail -15 $O/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/prof.log 2>&1
