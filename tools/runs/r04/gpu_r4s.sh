#!/bin/bash
# diagnose: the fused config-4 fixture test with the concurrent RangeDeps half (full stderr, exit status)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PYTHONFAULTHANDLER=1 timeout -k 10 300 python -u -X faulthandler -m pytest -x -v -s --timeout 280 --timeout-method thread -m gpu \
    "tests/test_full_configs_gpu.py::test_config4_fixture_full" > gpurun_out/r4s_out.log 2> gpurun_out/r4s_err.log
echo "rc=$?"
tail -c 3000 gpurun_out/r4s_out.log; echo ----; tail -c 3000 gpurun_out/r4s_err.log
