# Same-box timing of the in-tree build and tools/probe_build.sh builds on tools/tune.py (C3 lengths).
# Usage: bash tools/ab_probes.sh TAG NAME...   (NAME: find-tfbs_amd/lib/probe<NAME>)
OUT=gpurun_out/${1:-xp}; shift; mkdir -p $OUT
for rep in 1 2; do for lib in base "$@"; do
  if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
  timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 4 --length-config 3 > $OUT/${lib}_$rep.log 2>&1 || exit 1
done; done
for f in $OUT/*.log; do echo "$(basename $f .log): $(grep -h median $f | sed 's/  */ /g')"; done
