# Round-4 A/B: the key-assembly and BGZF GPU tests, assembly diagnostics, the bench
# step of the in-tree build against the probe builds named on the command line, a
# threshold sweep, and the BGZF writer in-tree vs probebzold (phase clocks).
set -o pipefail
T=${1:-ab}; shift
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reuse or synthetic_regions or c3_full or many_variant or reduce or bgzf" > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for lib in base bzold; do
  if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
  TFBS_BGZF_PROF=1 timeout -k 10 300 python3 tools/bgzf_only.py 1000 > gpurun_out/$T/bgzf_prof_$lib.txt 2>&1 || { tail -5 gpurun_out/$T/bgzf_prof_$lib.txt; exit 1; }
  echo "bgzf $lib: $(grep 'bgzf prof' gpurun_out/$T/bgzf_prof_$lib.txt | sed -n 2p)"
  for rep in 1 2; do
    timeout -k 10 300 python3 tools/bgzf_only.py 1000 > gpurun_out/$T/bgzf_$lib.txt 2>&1 || { tail -5 gpurun_out/$T/bgzf_$lib.txt; exit 1; }
    echo "bgzf $lib: $(tail -1 gpurun_out/$T/bgzf_$lib.txt)"
  done
done
unset TFBS_LIB
TFBS_DEBUG_OVER=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > gpurun_out/$T/diag.json 2> gpurun_out/$T/diag.err || { tail -5 gpurun_out/$T/diag.err; exit 1; }
grep "regions left\|assembly: spill" gpurun_out/$T/diag.err | tail -3
for rep in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/$T/step_$lib.json 2>/dev/null || { echo "bench $lib failed"; exit 1; }
    echo "step $lib: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$T/step_$lib.json | head -1) $(grep -o '"step_device_ms": {[^}]*}' gpurun_out/$T/step_$lib.json)"
  done
done
unset TFBS_LIB
for thr in 1e-4 1e-5 1e-6; do
  timeout -k 10 300 python3 bench.py --threshold $thr --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/$T/thr_$thr.json 2>/dev/null || { echo "bench thr $thr failed"; exit 1; }
  echo "threshold $thr: $(grep -o '"step_device_ms": {[^}]*}' gpurun_out/$T/thr_$thr.json)"
done
