#!/bin/bash
# stream-pass TxnId prefetch A/B (tools/prof/stpf.so), configs 2 and 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
ACC_BENCH_CFK=0 CFGS="2 3" STEPS=10 bash tools/gpu_abn.sh new stpf
