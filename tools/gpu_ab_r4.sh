# Round-4 A/B: the BGZF tests, key assembly diagnostics, then the in-tree scan (B
# prefetch) against the probe builds named on the command line (tools/exp_libs.sh,
# C3 mix), and the device BGZF writer (look-back placement) against probechain.
set -o pipefail
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/bgzf_tests.log 2>&1 || { tail -20 gpurun_out/$T/bgzf_tests.log; exit 1; }
tail -1 gpurun_out/$T/bgzf_tests.log
TFBS_DEBUG_OVER=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > gpurun_out/$T/diag.json 2> gpurun_out/$T/diag.err || { tail -5 gpurun_out/$T/diag.err; exit 1; }
grep "regions left\|assembly: spill" gpurun_out/$T/diag.err | tail -3
for rep in 1 2; do
  for lib in base chain; do
    if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
    echo "bgzf $lib: $(timeout -k 10 200 python3 tools/bgzf_only.py 1000 2>&1 | tail -1)"
  done
done
unset TFBS_LIB
bash tools/exp_libs.sh ${T}_x 3 "$@"
