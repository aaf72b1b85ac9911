#!/bin/bash
# round-end rehearsal: the full GPU suite, smoke(), and the default bench line (what the driver runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > gpurun_out/final_tests.log 2>&1
rc=$?; tail -3 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; tail -1 gpurun_out/final_bench.log | cut -c1-400; exit $rc
