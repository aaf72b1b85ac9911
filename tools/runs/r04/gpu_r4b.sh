#!/bin/bash
# config-4 RangeDeps probes: the build tier with its sorts / gather removed (wrong results, timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ACC_BENCH_MIXED=0 CFGS=4 STEPS=3 bash tools/gpu_abn.sh new rd_ns1 rd_ns12 rd_ng
