# Round-3 bench lines of the other BASELINE configs, a kernel trace of the C3 bench with its
# end-to-end leg, and the BGZF kernels' SQ counters.
set -o pipefail
T=${1:-r3b}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for w in C2 C4 C5; do
  timeout -k 10 400 python3 bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 4 > $O/bench_$(echo $w | tr C c).json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/e2e -o trace --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/e2e_trace.log 2>&1 || { echo "e2e trace failed"; exit 1; }
cp "$(find $O/e2e -name '*kernel_stats.csv' | head -1)" $O/kernel_stats_c3_e2e.csv
bash tools/pmc_bgzf.sh ${T}_bgzf || exit 1
