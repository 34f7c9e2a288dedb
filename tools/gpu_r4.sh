# Round-4 GPU check: the GPU suite (or the tests named in TESTS), then the C3 profile
# set (bench line, kernel trace, PMC passes).  Usage: tools/gpu_r4.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-r4}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 "${K[@]}" > $O/gpu_tests.log 2>&1
rc=$?
tail -25 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh ${T}_c3 --no-cpu || exit 1
bash tools/pmc_scan_stalls.sh ${T}_stall || exit 1
