# SQ counters of the BGZF kernels (tools/bgzf_only.py), one rocprofv3 pass per counter set.
set -o pipefail
O=gpurun_out/${1:-pz}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/bgzf_only.py 1000 > $O/run.log 2>&1 || exit 1
cat $O/run.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc1 -o pmc -- python3 tools/bgzf_only.py 1000 > $O/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc2 -o pmc -- python3 tools/bgzf_only.py 1000 > $O/pmc2.log 2>&1 || exit 1
