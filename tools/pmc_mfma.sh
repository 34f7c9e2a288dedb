#!/bin/bash
# PMC passes for the MFMA scan (tune.py workload, TFBS_MFMA=1; extra env passes through).
OUT=gpurun_out/${1:-pmc_mfma}
mkdir -p $OUT
export TMPDIR=/tmp TFBS_MFMA=1
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
  n=$(echo $set | cut -c1-12 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/$n -o pmc -- python3 tools/tune.py --regions 2000 --rounds 1 --length-config ${LC:-3} > $OUT/$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $OUT/$n.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
