#!/bin/bash
# one-sweep small tiles for mid-size sorts: parity (keydeps / merge / levelise / rangedeps), A/B configs 2 3 5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_keydeps_gpu.py \
    tests/test_merge_gpu.py tests/test_levelise_gpu.py tests/test_rangedeps_gpu.py > gpurun_out/r4_rs.log 2>&1
rc=$?; tail -3 gpurun_out/r4_rs.log; [ $rc -eq 0 ] || exit $rc
ACC_BENCH_CFK=0 CFGS="2 3 5" STEPS=10 bash tools/gpu_abn.sh new new+ACC_RS_SMALL_N=0
