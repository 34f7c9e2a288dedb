# Round-4 A/B: key assembly diagnostics, then the in-tree scan (B prefetch) against
# the probe builds named on the command line (tools/exp_libs.sh, C3 mix).
set -o pipefail
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
TFBS_DEBUG_OVER=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > gpurun_out/$T/diag.json 2> gpurun_out/$T/diag.err || { tail -5 gpurun_out/$T/diag.err; exit 1; }
grep "regions left\|assembly: spill" gpurun_out/$T/diag.err | tail -3
bash tools/exp_libs.sh ${T}_x 3 "$@"
