# Parity of the in-tree build (parity suite + C3/C5 full batches), then same-box timing against
# find-tfbs_amd/lib/probe<NAME> builds (tools/ab_probes.sh).
set -o pipefail
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_c3_full_batch_vs_oracle tests/test_gpu_fullsize.py::test_c5_full_batch_vs_oracle -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_probes.sh $T "$@"
