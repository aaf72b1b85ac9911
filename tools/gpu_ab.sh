#!/bin/bash
# A/B timing of the in-tree library against tools/ab/base.so on one box: bench lines alternate B, A, B, A.
#   CFG=2 STEPS=50 bash tools/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cfg=${CFG:-2}; steps=${STEPS:-50}
for i in 1 2; do
    for v in base new; do
        lib=""; [ $v = base ] && lib=tools/ab/base.so
        ACC_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 5 --no-cpu \
            > gpurun_out/ab_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ab_${v}_$i.log; exit 1; }
        python -c "
import json; d=json.loads(open('gpurun_out/ab_${v}_$i.log').read().strip().splitlines()[-1])
print('$v', d['ms_per_step'], d['roofline']['device_kernel_ms_per_step'])"
    done
done
