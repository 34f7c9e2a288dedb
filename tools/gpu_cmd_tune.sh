# Same-box timing: haplotypes per MFMA workgroup (tools/tune.py, interleaved, counts checked equal), then probe builds.
set -o pipefail
O=gpurun_out/${1:-tn}; shift
mkdir -p $O
timeout -k 10 300 python tools/tune.py --regions 2000 --rounds 4 --length-config 3 TFBS_MFMA_HAPS_PER_BLOCK=64,128,192,256 > $O/hpb.log 2>&1 || { tail -5 $O/hpb.log; exit 1; }
grep -E "median|MISMATCH" $O/hpb.log
[ $# -gt 0 ] && bash tools/ab_probes.sh ${O#gpurun_out/}_p "$@"
exit 0
