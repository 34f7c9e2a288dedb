#!/bin/bash
# Round-5 GPU session steps (each under its own limit, stopping at the first failure).
# Usage: tools/gpu_r5.sh TAG STEP...   steps: tests (GPU suite), tests_nofull (without the
# C3/C4/C5 full-size tests), bench_<W> (bench.py --workload W, no CPU leg), sprof_<W> (the
# scan's per-wave phase stamps: TFBS_SCAN_PROF build probesprof), prof_<W> (tools/profile_round.sh)
set -o pipefail
T=${1:?tag}; shift
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
for st in "$@"; do
  echo "[$(date +%T)] $st"
  case $st in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread --durations=20 > $O/gpu_tests.log 2>&1
      rc=$?; tail -25 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    tests_nofull)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 -k "not (c3_full or c5_full or c4_shards)" > $O/gpu_tests.log 2>&1
      rc=$?; tail -20 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    bench_*)
      w=${st#bench_}
      timeout -k 10 400 python3 bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['ms_per_step'], d['step_device_ms'], d['roofline']['frac'], d['end_to_end']['regions_per_s'])" ;;
    sprof_*)
      w=${st#sprof_}
      rm -f /tmp/scan_$w.prof
      TFBS_LIB=find-tfbs_amd/lib/probesprof/libtfbs_amd.so TFBS_SCAN_PROF=/tmp/scan_$w.prof timeout -k 10 300 python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-e2e > $O/sprof_$w.json 2> $O/sprof_$w.err || { tail -20 $O/sprof_$w.err; exit 1; }
      python3 tools/scan_prof.py /tmp/scan_$w.prof $O/scan_prof_$w.json > /dev/null || exit 1
      python3 -c "
import json;d=json.load(open('$O/scan_prof_$w.json'))
for l in d['launches']: print(l['launch'], l['workgroups'], {k:round(v,3) for k,v in l['phase_share'].items()}, l['pairs_per_wave'], round(l['cycles_per_pair_in_loop']), l['span_us'], l['tail_us'])" ;;
    prof_*)
      w=${st#prof_}
      bash tools/profile_round.sh ${T}_prof_$w --workload $w || exit 1 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done"
