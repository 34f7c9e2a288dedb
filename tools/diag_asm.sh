cd $GRAFT_REPO_ROOT
TFBS_DEBUG_OVER=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > gpurun_out/diag.json 2> gpurun_out/diag.err; tail -30 gpurun_out/diag.err
