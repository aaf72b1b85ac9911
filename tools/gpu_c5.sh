set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_levelise_gpu.py tests/test_merge_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_c5_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/gpu_c5_tests.log; exit 1; }
tail -3 gpurun_out/gpu_c5_tests.log
ACC_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --config 5 > gpurun_out/bench_c5.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -2 gpurun_out/bench_c5.log
