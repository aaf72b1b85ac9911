#!/bin/bash
# run compaction four outputs per thread per round (RangeDeps rd_compact, mixed KeyDeps mx_write): range / mixed
# tests, then config 4 A/B against the previous commit's build (r4c)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_rangedeps_gpu.py \
    tests/test_range_literals.py tests/test_full_configs_gpu.py tests/test_keydeps_mixed_gpu.py > gpurun_out/r4w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4w_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new r4c || exit 1
