#!/bin/bash
# RangeDeps 64-lane tier: counting sort variant (tools/prof/rd_rank.so) parity + config-4 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ACC_LIB_PATH=tools/prof/rd_rank.so timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu \
    tests/test_rangedeps_gpu.py tests/test_range_literals.py > gpurun_out/r4_rank.log 2>&1
rc=$?; tail -3 gpurun_out/r4_rank.log; [ $rc -eq 0 ] || exit $rc
ACC_BENCH_MIXED=0 CFGS=4 STEPS=3 bash tools/gpu_abn.sh new rd_rank
