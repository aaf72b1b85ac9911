#!/bin/bash
# CFK gather unpacks the sorted pair keys (no segment-flags pass): KeyDeps / recovery / mixed tests, configs 2-3 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_keydeps_gpu.py \
    tests/test_recovery_gpu.py tests/test_keydeps_mixed_gpu.py tests/test_cfk_deps_gpu.py > gpurun_out/r4_kd.log 2>&1
rc=$?; tail -3 gpurun_out/r4_kd.log; [ $rc -eq 0 ] || exit $rc
ACC_BENCH_CFK=0 CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new st24
