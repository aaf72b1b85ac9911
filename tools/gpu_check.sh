set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -5 gpurun_out/gpu_tests.log
ACC_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
