#!/bin/bash
# configs 2 and 3 bench lines with kernel times; the config-2 stream-pass phase profile (tools/prof/libaccord_amd.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new || exit 1
ACC_LIB_PATH=tools/prof/libaccord_amd.so timeout -k 10 300 python -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu \
    > gpurun_out/r4_phase.log 2>&1 || { tail -5 gpurun_out/r4_phase.log; exit 1; }
grep st_phase gpurun_out/r4_phase.log | tail -2
python -c "
import json; d=json.loads(open('gpurun_out/abn_c2_new_2.log').read().strip().splitlines()[-1])
print('cfk', d.get('cfk_apply'))"
