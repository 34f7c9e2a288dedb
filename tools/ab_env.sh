# Same-box timing of environment / library variants on tools/tune.py (C3 lengths).
# Usage: bash tools/ab_env.sh TAG NAME=ENV1,ENV2 ...  (TFBS_LIB=probe<x> selects a probe build)
OUT=gpurun_out/${1:-xe}; shift; mkdir -p $OUT
for rep in 1 2; do for spec in base "$@"; do
  name=${spec%%=*}; envs=""; [ "$spec" != base ] && envs=${spec#*=}
  ( IFS=,; for e in $envs; do case $e in TFBS_LIB=*) export TFBS_LIB=find-tfbs_amd/lib/${e#TFBS_LIB=}/libtfbs_amd.so;; *) export "$e";; esac; done
    timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 4 --length-config 3 ) > $OUT/${name}_$rep.log 2>&1 || exit 1
done; done
for f in $OUT/*.log; do echo "$(basename $f .log): $(grep -h median $f | sed 's/  */ /g')"; done
