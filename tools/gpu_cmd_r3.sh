# Round-3 check of HEAD: the GPU suite, then the C3 profile set (bench line, kernel trace, PMC passes).
set -o pipefail
T=${1:-r3a}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=25 > $O/gpu_tests.log 2>&1
rc=$?
tail -30 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh ${T}_c3 --cpu-seconds 4 || exit 1
bash tools/pmc_bgzf.sh ${T}_bgzf || exit 1
