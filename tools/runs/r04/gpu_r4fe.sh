#!/bin/bash
# fused PartialDeps error path / repeated calls with the concurrent RangeDeps half
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_keydeps_mixed_gpu.py > gpurun_out/r4fe_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4fe_tests.log; exit $rc
