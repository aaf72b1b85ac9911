#!/bin/bash
# RangeDeps narrow sorts + mixed piece records: tests, config-4 A/B (32-bit vs 64-bit sorts) with the mixed / fused legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_rangedeps_gpu.py \
    tests/test_range_literals.py tests/test_keydeps_mixed_gpu.py > gpurun_out/r4_rd.log 2>&1
rc=$?; tail -3 gpurun_out/r4_rd.log; [ $rc -eq 0 ] || exit $rc
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new new+ACC_RD_WIDE=1 || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/abn_c4_new_2.log').read().strip().splitlines()[-1])
print('mixed', d.get('keydeps_mixed')); print('fused', d.get('partial_deps'))"
