set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_rangedeps_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_rd.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_rd.log
exit $rc
