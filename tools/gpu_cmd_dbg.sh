set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/rs2
TFBS_DEBUG_OVER=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > gpurun_out/rs2/b.json 2> gpurun_out/rs2/b.err || exit 1
grep tfbs_scan gpurun_out/rs2/b.err | tail -2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rs2/prof -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/rs2/prof.log 2>&1 || exit 1
head -6 gpurun_out/rs2/prof/trace_kernel_stats.csv | cut -c1-160
