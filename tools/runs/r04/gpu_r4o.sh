#!/bin/bash
# RangeDeps tier lists by ballot counts + block-aggregated scatter (no tier sort): tests, config-4 A/B against stpf.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 560 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_rangedeps_gpu.py \
    tests/test_range_literals.py tests/test_keydeps_gpu.py tests/test_keydeps_mixed_gpu.py \
    tests/test_cfk_deps_gpu.py tests/test_cfk_gpu.py tests/test_recovery_gpu.py tests/test_recovery_ranges_gpu.py > gpurun_out/r4_tier.log 2>&1
rc=$?; tail -3 gpurun_out/r4_tier.log; [ $rc -eq 0 ] || exit $rc
ACC_BENCH_MIXED=0 CFGS=4 STEPS=3 bash tools/gpu_abn.sh new stpf
