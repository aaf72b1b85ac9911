#!/bin/bash
# config-2 kernel timeline (rocprofv3 kernel trace of a short bench run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ACC_BENCH_CFK=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl2 -o run --output-format csv -- \
    python bench.py --config 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/tl2.log 2>&1 || { tail -5 gpurun_out/tl2.log; exit 1; }
f=$(find gpurun_out/tl2 -name "*kernel_trace.csv" | head -1)
python tools/timeline.py "$f" > gpurun_out/tl2_timeline.txt && tail -3 gpurun_out/tl2_timeline.txt
