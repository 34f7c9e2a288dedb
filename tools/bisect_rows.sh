set -o pipefail
O=gpurun_out/r6bis; mkdir -p $O
timeout -k 10 900 python3 -u tools/bench_run.py --samples 50000 --regions 10000 --oracle-seconds 0 > $O/run_async.json 2> $O/run_async.err || exit 1
grep tfbs_run_timing $O/run_async.err; python3 -c "import json;d=json.load(open('$O/run_async.json'));print('async', d['rows'], d['regions_per_s'])"
TFBS_RUN_ASYNC_WRITE=0 timeout -k 10 900 python3 -u tools/bench_run.py --samples 50000 --regions 10000 --oracle-seconds 0 > $O/run_sync.json 2> $O/run_sync.err || exit 1
python3 -c "import json;d=json.load(open('$O/run_sync.json'));print('sync', d['rows'], d['regions_per_s'])"
