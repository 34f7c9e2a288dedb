# PMC stall breakdown (two SQ passes) of the in-tree build on the tools/tune.py workload.
# Usage: bash tools/pmc_stalls.sh TAG
OUT=gpurun_out/${1:-pw}; mkdir -p $OUT
export TMPDIR=/tmp TFBS_MFMA=1
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
p2="SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS"
i=0
for set in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i/x -o pmc -- python3 tools/tune.py --regions 2000 --rounds 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/p$i > $OUT/p$i.json && python3 -c "import json;d=json.load(open('$OUT/p$i.json'));print({k:'%.3g'%v for k,v in d.items() if k.startswith('SQ')})"
done
