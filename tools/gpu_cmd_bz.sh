# BGZF kernel work: the device-BGZF parity tests on the in-tree build, then same-box kernel times
# of the in-tree build against variant builds (tools/ab_kernels.sh).
set -o pipefail
T=${1:-bz}; shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernels.sh ${T}_ab "bgzf_wave|row_cum|bgzf_block" "python3 tools/bgzf_only.py 1000" "$@"
