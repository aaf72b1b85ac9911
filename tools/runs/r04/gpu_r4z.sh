#!/bin/bash
# merge fit: wave maxima before the global atomics; host syncs polling the stream: merge / levelise tests, config 5 and config 2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_merge_gpu.py \
    tests/test_levelise_gpu.py tests/test_full_configs_gpu.py::test_config5_full > gpurun_out/r4z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4z_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS=5 STEPS=20 bash tools/gpu_abn.sh new r4c || exit 1
# host syncs by polling the stream (ACC_SYNC_BLOCK=1: the blocking wait)
CFGS=2 STEPS=20 bash tools/gpu_abn.sh new new+ACC_SYNC_BLOCK=1 r4c || exit 1
