# The device-grouping tests, then the whole GPU suite, the C3 bench line and a kernel trace.
set -o pipefail
O=gpurun_out/${1:-b1}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -x -v --timeout 240 --timeout-method thread > $O/build_tests.log 2>&1
rc=$?
tail -30 $O/build_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_cmd1.sh ${1:-b1}
