# round-2 closing measurement: config-2 profile, then bench lines for configs 2-5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash profiles/collect.sh r02 2 || exit 1
for cfg in 2 3 4 5; do
    ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_c$cfg.log 2>&1 \
        || { echo "bench c$cfg failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
    tail -1 gpurun_out/bench_c$cfg.log | cut -c1-200
done
