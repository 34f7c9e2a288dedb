# Parity of the scan paths (parity + C3 full batch), then the tune.py timing of the in-tree build.
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py::test_c3_full_batch_vs_oracle tests/test_gpu_fullsize.py::test_c5_full_batch_vs_oracle -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/tune.py --regions 2000 --rounds 4 --length-config 3 > $O/tune.log 2>&1 || exit 1
grep median $O/tune.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['end_to_end']['regions_per_s'])"
