#!/bin/bash
# segment key codes from the apply pass (no separate seg-key kernel): mixed / CFK / recovery tests, mixed A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 560 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_keydeps_mixed_gpu.py \
    tests/test_cfk_deps_gpu.py tests/test_cfk_gpu.py tests/test_recovery_gpu.py tests/test_recovery_ranges_gpu.py \
    tests/test_keydeps_gpu.py tests/test_range_literals.py > gpurun_out/r4_segkey.log 2>&1
rc=$?; tail -3 gpurun_out/r4_segkey.log; [ $rc -eq 0 ] || exit $rc
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new stpf
