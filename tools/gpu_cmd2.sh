# The device BGZF tests, then the widened full-size parity (progress in the logs as each test ends).
O=gpurun_out/${1:-bg1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bgzf.py -x -v --timeout 240 --timeout-method thread > $O/bgzf.log 2>&1
rc=$?; tail -8 $O/bgzf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread --durations=8 > $O/full.log 2>&1
rc=$?; tail -14 $O/full.log; exit $rc
