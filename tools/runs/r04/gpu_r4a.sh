#!/bin/bash
# round-4 check: levelise tiers, world-8 partial reduce, mixed KeyDeps, CFK apply; config 5 A/B (windowed vs LDS
# tier), 1M levelise per tier, config 4 bench (RangeDeps + mixed KeyDeps legs). SKIPT=1: no tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -z "${SKIPT:-}" ]; then
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_levelise_gpu.py \
    tests/test_partial_reduce_gpu.py tests/test_keydeps_mixed_gpu.py tests/test_cfk_deps_gpu.py} > gpurun_out/r4_lv.log 2>&1
rc=$?; tail -3 gpurun_out/r4_lv.log; [ $rc -eq 0 ] || exit $rc
fi
CFGS=5 STEPS=20 bash tools/gpu_abn.sh new new+ACC_LV_LDS=1 || exit 1
for e in "" ACC_LV_WAVES=1 ACC_LV_LDS=1; do env $e timeout -k 10 300 python tools/lv_time.py || exit 1; done
ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/r4_c4.log 2>&1 || { tail -20 gpurun_out/r4_c4.log; exit 1; }
tail -c 3000 gpurun_out/r4_c4.log
