#!/bin/bash
# one-sweep look-back width A/B (8 / 16 / 32 predecessor tiles per step), configs 2, 3, 5
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ACC_BENCH_CFK=0 CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new lb16 lb32
