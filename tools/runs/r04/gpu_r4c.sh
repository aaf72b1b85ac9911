#!/bin/bash
# levelise iteration: tests, config-5 (LDS tier default vs windowed), 1M chain timing per poll mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_levelise_gpu.py \
    ${MORE_TESTS:-} > gpurun_out/r4_lv.log 2>&1
rc=$?; tail -3 gpurun_out/r4_lv.log; [ $rc -eq 0 ] || exit $rc
CFGS=5 STEPS=20 bash tools/gpu_abn.sh new new+ACC_LV_WIN=1 || exit 1
for e in "" ACC_LV_POLL=8; do env $e timeout -k 10 300 python tools/lv_time.py || exit 1; done
