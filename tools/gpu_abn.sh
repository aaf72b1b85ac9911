#!/bin/bash
# Same-box timing of several library builds: CFGS="2 3" STEPS=20 bash tools/gpu_abn.sh new base u2 ...
# "new" = the in-tree library ("new+VAR=VALUE": with that environment for bench.py), any other name =
# tools/ab/<name>.so. Two alternating rounds per config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
steps=${STEPS:-20}
for cfg in ${CFGS:-2}; do
    for i in 1 2; do
        for v in "$@"; do
            lib=""; envs=""
            case "$v" in new) ;; new+*) envs="${v#new+}"; envs="${envs//,/ }" ;; *) lib=tools/ab/$v.so ;; esac
            env $envs ACC_BENCH_CFK=0 ACC_BENCH_KERNELS=1 ACC_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --config $cfg --steps $steps --warmup 3 --no-cpu \
                > gpurun_out/abn_c${cfg}_${v}_$i.log 2>&1 || { echo "bench $v c$cfg failed"; tail -20 gpurun_out/abn_c${cfg}_${v}_$i.log; exit 1; }
            python -c "
import json; d=json.loads(open('gpurun_out/abn_c${cfg}_${v}_$i.log').read().strip().splitlines()[-1])
k=d.get('kernels_ms_per_step',{})
top=sorted(k.items(), key=lambda kv: -kv[1])[:6]
mx=d.get('keydeps_mixed',{}).get('ms_per_call'); pd=d.get('partial_deps',{}).get('ms_per_step')
print('c$cfg $v', d['ms_per_step'], d['roofline']['device_kernel_ms_per_step'], ('mixed=%s fused=%s' % (mx, pd)) if mx else '', ' '.join('%s=%.3f' % kv for kv in top))"
        done
    done
done
