#!/bin/bash
# A/B of the round's latest KeyDeps launch folds against r4base (HEAD~1 build), config-2 timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CFGS=2 STEPS=20 bash tools/gpu_abn.sh new r4base || exit 1
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new r4base || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ACC_BENCH_CFK=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl4 -o run --output-format csv -- \
    python bench.py --config 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/tl4.log 2>&1 || { tail -5 gpurun_out/tl4.log; exit 1; }
f=$(find gpurun_out/tl4 -name "*kernel_trace.csv" | head -1)
python tools/timeline.py "$f" > gpurun_out/tl4_timeline.txt && tail -3 gpurun_out/tl4_timeline.txt
