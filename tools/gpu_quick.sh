#!/bin/bash
# Quick GPU iteration: the GPU parity tests, then the config-2 and config-3 bench lines.
#   bash tools/gpu_quick.sh [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
sel=${1:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${sel:+-k "$sel"} \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for cfg in ${CFGS:-2 3}; do
    ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg --no-cpu > gpurun_out/bench_c$cfg.log 2>&1 \
        || { echo "bench c$cfg failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('gpurun_out/bench_c$cfg.log').read().strip().splitlines()[-1])
print('c$cfg', d['ms_per_step'], d['value'], d['roofline']['dominant_kernel'], d['roofline']['frac'])
print({k:v for k,v in list(d['kernels_ms_per_step'].items())[:12]})"
done
