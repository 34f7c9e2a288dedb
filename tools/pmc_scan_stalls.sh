# PMC stall breakdown of the scan's MFMA phase at the bench's C3 operating point (two
# SQ passes over bench.py, each its own rocprofv3 run); summaries per pass via
# tools/pmc_summary.py (the last step's scan_mfma_kernel dispatches).
# Usage: bash tools/pmc_scan_stalls.sh TAG [bench.py args]
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
p2="SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_MISC"
i=0
for set in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/s$i -o pmc -- python3 bench.py "$@" --steps 2 --warmup 0 --no-cpu --no-e2e > $OUT/s$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/s$i.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/s$i > /dev/null && python3 -c "import json;d=json.load(open('$OUT/s$i/pmc_summary.json'));print({k:'%.4g'%v for k,v in d.items() if k.startswith('SQ')})" || exit 1
  python3 tools/pmc_summary.py $OUT/s$i key_fast_kernel > /dev/null || exit 1
done
