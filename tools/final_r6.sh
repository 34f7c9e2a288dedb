#!/bin/bash
# Round-6 final measurements of the committed library, in two parts (one gpurun call
# each): A = C3 profile (bench line, kernel trace, FETCH/WRITE/SQ passes) + the C3
# scan stall passes + C2 profile; B = the GPU suite, the C5 profile and the run flow at
# 10 000 regions x 50 000 samples with one and two contexts; C = the C4 profile.
# Usage: bash tools/final_r6.sh A|B|C
set -o pipefail
part=${1:?A or B}
case $part in
  A) bash tools/gpu_r6.sh r6final prof_C3 stall_C3 prof_C2 ;;
  B) bash tools/gpu_r6.sh r6final tests prof_C5 run_10000 run_10000:0,0 ;;
  C) bash tools/gpu_r6.sh r6final prof_C4 ;;
esac
