#!/bin/bash
# windowed levelise walk: in-wave hops by shuffle (chains resolve within a round): levelise tests, then the 1M-txn
# graph's time per level against r4c, and config 5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_levelise_gpu.py \
    tests/test_full_configs_gpu.py::test_config5_full > gpurun_out/r4lv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4lv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/lv_time.py || exit 1
ACC_LIB_PATH=tools/prof/r4c.so timeout -k 10 300 python tools/lv_time.py || exit 1
CFGS=5 STEPS=20 bash tools/gpu_abn.sh new r4c || exit 1
