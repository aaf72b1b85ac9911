#!/bin/bash
# CommandsForKey store modes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cfk_deps_gpu.py tests/test_cfk_gpu.py > gpurun_out/r4cs_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r4cs_tests.log; exit $rc
