#!/bin/bash
# levelise + mixed KeyDeps: tests, config-5 (LDS tier default vs windowed), 1M chain per poll mode, config-4 bench legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
MORE_TESTS=tests/test_keydeps_mixed_gpu.py bash tools/gpu_r4c.sh || exit 1
ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu > gpurun_out/r4_c4.log 2>&1 || { tail -20 gpurun_out/r4_c4.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r4_c4.log').read().strip().splitlines()[-1])
print('c4', d['ms_per_step']); print('mixed', d.get('keydeps_mixed')); print('fused', d.get('partial_deps'))"
