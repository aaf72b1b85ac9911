set -o pipefail
cd $GRAFT_REPO_ROOT
cfg=${1:-2}
ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_c$cfg.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
tail -2 gpurun_out/bench_c$cfg.log
