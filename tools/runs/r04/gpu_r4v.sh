#!/bin/bash
# RangeDeps: tier counts in the size pass (no histogram kernel), range entries as 32-B records for the permuted
# dictionary / class passes: range tests, then config 4 / config 2 A/B against r4base, config-2 timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_rangedeps_gpu.py \
    tests/test_range_literals.py tests/test_full_configs_gpu.py tests/test_recovery_ranges_gpu.py tests/test_rmm_gpu.py \
    tests/test_partial_reduce_gpu.py > gpurun_out/r4v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4v_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new r4base || exit 1
CFGS=2 STEPS=20 bash tools/gpu_abn.sh new r4base || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ACC_BENCH_CFK=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl4 -o run --output-format csv -- \
    python bench.py --config 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/tl4.log 2>&1 || { tail -5 gpurun_out/tl4.log; exit 1; }
f=$(find gpurun_out/tl4 -name "*kernel_trace.csv" | head -1)
python tools/timeline.py "$f" > gpurun_out/tl4_timeline.txt && tail -3 gpurun_out/tl4_timeline.txt
