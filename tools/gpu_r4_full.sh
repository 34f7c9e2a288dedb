#!/bin/bash
# Round-4 measurement set in one call: the GPU suite and the C3 profile set
# (tools/gpu_final_r4.sh A), then the key assembly's phase clocks and the
# end-to-end kernel traces of C3 and C5.  Usage: tools/gpu_r4_full.sh TAG
set -o pipefail
T=${1:?tag}
bash tools/gpu_final_r4.sh $T A || exit 1
O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
TFBS_KF_PROF=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > $O/kf.json 2> $O/kf.err || { echo "kf prof failed"; exit 1; }
grep "kf prof" $O/kf.err | tail -4 | cut -c1-300
bash tools/trace_e2e.sh ${T}_e2e_c3 || exit 1
bash tools/trace_e2e.sh ${T}_e2e_c5 --workload C5 || exit 1
# A/B of the depth launches' order (shallow class first)
for v in 0 1; do
  TFBS_SCAN_SHALLOW_FIRST=$v timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-e2e > $O/order_$v.json 2> $O/order_$v.err || { echo "order $v failed"; exit 1; }
  echo "shallow_first=$v $(grep -o '"ms_per_step": [0-9.]*' $O/order_$v.json) $(grep -o '"step_device_ms": {[^}]*}' $O/order_$v.json)"
done
