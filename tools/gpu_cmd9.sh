# merge phase split (tuning build)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ACC_LIB_PATH=tools/prof/mlprof.so timeout -k 10 200 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu > gpurun_out/mlprof.log 2>&1 || { tail -20 gpurun_out/mlprof.log; exit 1; }
grep ml_prof gpurun_out/mlprof.log | tail -2
