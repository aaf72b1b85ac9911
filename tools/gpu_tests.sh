# usage: bash tools/gpu_tests.sh <pytest file or dir>... (one pytest process, per-test timeout)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/gpu_tests.log | tail -40
exit $rc
