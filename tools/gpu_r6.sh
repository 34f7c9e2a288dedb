#!/bin/bash
# Round-6 GPU session steps (each under its own limit, stopping at the first failure).
# Usage: tools/gpu_r5.sh TAG STEP...   steps: tests (GPU suite), tests_nofull (without the
# C3/C4/C5 full-size tests), bench_<W> (bench.py --workload W, no CPU leg), sprof_<W> (the
# scan's per-wave phase stamps: TFBS_SCAN_PROF build probesprof; rprof_<W>: probe rprof, the
# rounds' clock split), stall_<W>[:<variant>] (two SQ stall passes over the scan kernel), prof_<W> (tools/profile_round.sh)
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
    k_*)  # k_<expr>: the GPU tests selected by pytest -k <expr>
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${st#k_}" > $O/gpu_tests_k.log 2>&1
      rc=$?; tail -15 $O/gpu_tests_k.log; [ $rc -eq 0 ] || exit $rc ;;
    tests_nofull)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --durations=15 -k "not (c3_full or c5_full or c4_shards)" > $O/gpu_tests.log 2>&1
      rc=$?; tail -20 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    bench_*)
      w=${st#bench_}
      timeout -k 10 400 python3 bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['ms_per_step'], d['step_device_ms'], d['roofline']['frac'], d['end_to_end']['regions_per_s'])" ;;
    sprof_*)  # sprof_<W>[:VAR=VAL]: the probesprof build's per-wave phase stamps (env VAR=VAL)
      spec=${st#sprof_}; w=${spec%%:*}; envv=""; [ "$spec" != "$w" ] && envv=${spec#*:}
      tag=$w${envv:+_${envv//=/}}
      rm -f /tmp/scan_$tag.prof
      env $envv TFBS_LIB=find-tfbs_amd/lib/probesprof/libtfbs_amd.so TFBS_SCAN_PROF=/tmp/scan_$tag.prof timeout -k 10 300 python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-e2e > $O/sprof_$tag.json 2> $O/sprof_$tag.err || { tail -20 $O/sprof_$tag.err; exit 1; }
      python3 tools/scan_prof.py /tmp/scan_$tag.prof $O/scan_prof_$tag.json > /dev/null || exit 1
      python3 -c "
import json;d=json.load(open('$O/scan_prof_$tag.json'))
for l in d['launches']: print('$tag', l['launch'], l['workgroups'], {k:round(v) for k,v in l['phase_cycles_mean_per_wave'].items()}, l['pairs_per_wave']['mean'], round(l['cycles_per_pair_in_loop']), l['candidates_per_wave']['mean'], l['span_us'], l['tail_us'])" ;;
    pmc_*)  # pmc_<W>[:<variant>]: one SQ counter pass over the MFMA phase (variant: a probe name or e.VAR=VAL)
      spec=${st#pmc_}; w=${spec%%:*}; v=base; [ "$spec" != "$w" ] && v=${spec#*:}
      unset TFBS_LIB; envv=""
      case $v in base) ;; e.*) envv=${v#e.} ;; *) export TFBS_LIB=find-tfbs_amd/lib/probe$v/libtfbs_amd.so ;; esac
      d=$O/pmc_${w}_${v//=/}
      env $envv timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $d -o pmc -- python3 bench.py --workload $w --steps 2 --warmup 0 --no-cpu --no-e2e > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
      unset TFBS_LIB
      python3 tools/pmc_summary.py $d > /dev/null || exit 1
      python3 -c "
import json;q=json.load(open('$d/pmc_summary.json'));m=q['SQ_INSTS_MFMA']
print('$w $v', q['_kernels'], 'MFMA %.3g VALU/MFMA %.2f SALU/MFMA %.2f LDS/MFMA %.2f conflicts/LDS %.2f mfma_busy_cycles %.3g' % (m, q['SQ_INSTS_VALU']/m, q['SQ_INSTS_SALU']/m, q['SQ_INSTS_LDS']/m, q['SQ_LDS_BANK_CONFLICT']/q['SQ_INSTS_LDS'], q['SQ_VALU_MFMA_BUSY_CYCLES']))" ;;
    ab_*)  # ab_<W>:<probe>,<probe>: bench.py steps of the in-tree build and probe builds, interleaved twice
      spec=${st#ab_}; w=${spec%%:*}; libs=${spec#*:}
      for rep in 1 2; do
        for lib in base ${libs//,/ }; do
          unset TFBS_LIB; envv=""
          case $lib in base) ;; e.*) envv=${lib#e.} ;; *) export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so ;; esac
          env $envv timeout -k 10 300 python3 bench.py --workload $w --no-cpu --no-e2e --steps 10 > $O/ab_${w}_${lib}_$rep.json 2> $O/ab_${w}_${lib}_$rep.err || { tail -20 $O/ab_${w}_${lib}_$rep.err; exit 1; }
          python3 -c "import json;d=json.load(open('$O/ab_${w}_${lib}_$rep.json'));print('$w $lib rep$rep ms/step %.3f' % d['ms_per_step'], {k: round(v, 3) for k, v in d['step_device_ms'].items()}, 'scanned %.3g' % d['config']['scanned_windows_per_step'])"
        done
      done
      unset TFBS_LIB ;;
    run_*)  # run_<regions>[:<devices>]: tools/bench_run.py at 50 000 samples (BCF decode in the clock)
      spec=${st#run_}; n=${spec%%:*}; dv=""; [ "$spec" != "$n" ] && dv="--devices ${spec#*:}"
      tag=run_${n}${dv:+_$(echo ${spec#*:} | tr , _)}
      timeout -k 10 900 python3 -u tools/bench_run.py --samples 50000 --regions $n $dv --oracle-seconds 0 > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
      grep tfbs_run_timing $O/$tag.err; python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', {k: d.get(k) for k in ('run_s','regions_per_s','device_warmup_s','regions_per_s_with_device_warmup','bcf_decode_alone_s','dataset_gen_s','rows','records')})" ;;
    bgzf_*)  # bgzf_<regions>[:<probe>,...]: tools/bgzf_only.py per build, phase clocks (TFBS_BGZF_PROF) then timing
      spec=${st#bgzf_}; n=${spec%%:*}; libs=""; [ "$spec" != "$n" ] && libs=${spec#*:}
      for rep in 1 2; do
        for lib in base ${libs//,/ }; do
          unset TFBS_LIB; [ $lib = base ] || export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so
          TFBS_BGZF_PROF=1 timeout -k 10 300 python3 tools/bgzf_only.py $n > $O/bgzf_${lib}_prof_$rep.txt 2>&1 || { tail -20 $O/bgzf_${lib}_prof_$rep.txt; exit 1; }
          grep "bgzf prof" $O/bgzf_${lib}_prof_$rep.txt | tail -1
          timeout -k 10 300 python3 tools/bgzf_only.py $n > $O/bgzf_${lib}_$rep.txt 2>&1 || { tail -20 $O/bgzf_${lib}_$rep.txt; exit 1; }
          echo "$lib rep$rep $(tail -1 $O/bgzf_${lib}_$rep.txt)"
        done
      done
      unset TFBS_LIB ;;
    bpmc_*)  # bpmc_<regions>[:<probe>]: two SQ counter passes over tools/bgzf_only.py (bgzf_wave_kernel's last dispatch)
      spec=${st#bpmc_}; n=${spec%%:*}; v=base; [ "$spec" != "$n" ] && v=${spec#*:}
      unset TFBS_LIB; [ $v = base ] || export TFBS_LIB=find-tfbs_amd/lib/probe$v/libtfbs_amd.so
      for pass in a b; do
        d=$O/bpmc_${v}_$pass
        if [ $pass = a ]; then c="SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
        else c="SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_INSTS_VMEM_RD"; fi
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $d -o pmc -- python3 tools/bgzf_only.py $n > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
        python3 tools/pmc_summary.py $d bgzf_wave_kernel > /dev/null || exit 1
        python3 -c "import json;q=json.load(open('$d/pmc_summary_bgzf_wave_kernel.json'));print('$v $pass', {k: v for k, v in q.items() if not k.startswith('_')})"
      done
      unset TFBS_LIB ;;
    kfpmc_*)  # kfpmc_<W>: key_fast_kernel's phase clocks (TFBS_KF_PROF, the slowest regions = the tail) and two SQ passes
      w=${st#kfpmc_}; d=$O/kf_$w; mkdir -p $d
      TFBS_KF_PROF=1 timeout -k 10 300 python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-e2e > $d/bench.json 2> $d/kf_prof.err || { tail -20 $d/kf_prof.err; exit 1; }
      grep "kf prof" $d/kf_prof.err > $d/kf_prof.txt; head -3 $d/kf_prof.txt | cut -c1-300
      for pass in stall1:"SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAVE_CYCLES" stall2:"SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"; do
        name=${pass%%:*}; counters=${pass#*:}
        timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $d/pmc_$name -o pmc -- python3 bench.py --workload $w --steps 2 --warmup 0 --no-cpu --no-e2e > $d/pmc_$name.log 2>&1 || { tail -20 $d/pmc_$name.log; exit 1; }
        python3 tools/pmc_summary.py $d/pmc_$name key_fast_kernel > /dev/null || exit 1
      done ;;
    rprof_*)  # rprof_<W>: the probe rprof build (TFBS_SCAN_PROF + TFBS_ROUND_PROF): phases and the rounds' clock split
      w=${st#rprof_}
      rm -f /tmp/rscan_$w.prof
      TFBS_LIB=find-tfbs_amd/lib/proberprof/libtfbs_amd.so TFBS_SCAN_PROF=/tmp/rscan_$w.prof timeout -k 10 300 python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-e2e > $O/rprof_$w.json 2> $O/rprof_$w.err || { tail -20 $O/rprof_$w.err; exit 1; }
      python3 tools/scan_prof.py /tmp/rscan_$w.prof $O/round_prof_$w.json | tail -60 ;;
    stall_*)  # stall_<W>[:<variant>]: two SQ counter passes over the scan kernel's last dispatch (stall reasons)
      spec=${st#stall_}; w=${spec%%:*}; v=base; [ "$spec" != "$w" ] && v=${spec#*:}
      unset TFBS_LIB; envv=""
      case $v in base) ;; e.*) envv=${v#e.} ;; *) export TFBS_LIB=find-tfbs_amd/lib/probe$v/libtfbs_amd.so ;; esac
      for pass in stall1:"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS" stall2:"SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" stall3:"SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_IFETCH"; do
        name=${pass%%:*}; counters=${pass#*:}
        d=$O/stall_${w}_${v//=/}_$name
        env $envv timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $d -o pmc -- python3 bench.py --workload $w --steps 2 --warmup 0 --no-cpu --no-e2e > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
        python3 tools/pmc_summary.py $d > /dev/null || exit 1
        python3 -c "import json;q=json.load(open('$d/pmc_summary.json'));print('$w $v $name', {k: '%.4g' % v for k, v in q.items() if not k.startswith('_')})"
      done
      unset TFBS_LIB ;;
    tl_*)  # tl_<W>: kernel + memory-copy trace of bench.py (graph-replayed steps), the last steps' timelines
      w=${st#tl_}
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/tl_$w -o tl --output-format csv -- python3 bench.py --workload $w --steps 12 --warmup 3 --no-cpu --no-e2e > $O/tl_$w.json 2> $O/tl_$w.err || { tail -20 $O/tl_$w.err; exit 1; }
      kt=$(find $O/tl_$w -name '*kernel_trace.csv' | head -1); mt=$(find $O/tl_$w -name '*memory_copy_trace.csv' | head -1)
      python3 tools/step_timeline.py $kt $mt 3 > $O/tl_$w.txt; cat $O/tl_$w.txt | head -60 ;;
    probe_scale)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/probe/f4f6_scale.hip -o /tmp/f4f6_scale 2>/dev/null || exit 1
      timeout -k 10 60 /tmp/f4f6_scale > $O/probe_scale.txt 2>&1; rc=$?; cat $O/probe_scale.txt; [ $rc -eq 0 ] || exit $rc ;;
    probe_chain)
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/probe/f4f6_chain.hip -o /tmp/f4f6_chain || exit 1
      timeout -k 10 120 /tmp/f4f6_chain > $O/probe_chain.txt 2>&1 || exit 1
      cat $O/probe_chain.txt ;;
    prof_*)
      w=${st#prof_}
      bash tools/profile_round.sh ${T}_prof_$w --workload $w || exit 1 ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done"
