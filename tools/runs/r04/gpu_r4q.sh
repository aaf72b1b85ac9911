#!/bin/bash
# multi-array scans, double-buffered one-sweep status (no memset per sort), one host copy per sync; segment keys
# gathered early in the apply pass: full GPU suite, config 2/3/4 A/B against r4base (HEAD), config-2 timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > gpurun_out/r4q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4q_tests.log; [ $rc -eq 0 ] || exit $rc
CFGS="2 3" STEPS=20 bash tools/gpu_abn.sh new r4base || exit 1
CFGS=4 STEPS=3 bash tools/gpu_abn.sh new r4base || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ACC_BENCH_CFK=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl3 -o run --output-format csv -- \
    python bench.py --config 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/tl3.log 2>&1 || { tail -5 gpurun_out/tl3.log; exit 1; }
f=$(find gpurun_out/tl3 -name "*kernel_trace.csv" | head -1)
python tools/timeline.py "$f" > gpurun_out/tl3_timeline.txt && tail -3 gpurun_out/tl3_timeline.txt
