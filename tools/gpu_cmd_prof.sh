# Parity of the reuse paths, then the round's profile set (bench line, kernel trace, PMC traffic and SQ
# passes: tools/profile_round.sh) and the SQ stall passes (tools/pmc_stalls.sh).
set -o pipefail
T=${1:-p1}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_c3_full_batch_vs_oracle -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh $T --cpu-seconds 4 || exit 1
bash tools/pmc_stalls.sh ${T}_stalls
