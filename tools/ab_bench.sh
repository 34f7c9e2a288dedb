# Same-box A/B of library builds on the C3 bench step (no CPU leg, no end-to-end leg):
# bash tools/ab_bench.sh TAG NAME... (NAME: find-tfbs_amd/lib/probe<NAME>; "base" = the in-tree build)
OUT=gpurun_out/${1:-ab}; shift; mkdir -p $OUT
for rep in 1 2; do for lib in base "$@"; do
  if [ $lib = base ]; then unset TFBS_LIB; else export TFBS_LIB=find-tfbs_amd/lib/probe$lib/libtfbs_amd.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $OUT/${lib}_$rep.json 2> $OUT/${lib}_$rep.err || exit 1
done; done
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('%-12s ms/step %.3f  mfma phase %.3f ms  frac %.3f' % ('$(basename $f .json)', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"; done
