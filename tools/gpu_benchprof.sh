#!/bin/bash
# Bench lines for configs 2-5, then rocprof collection (kernel trace + FETCH_SIZE + WRITE_SIZE passes) per config:
#   bash tools/gpu_benchprof.sh <tag> [configs-to-profile...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=${1:-r02}
shift
mkdir -p gpurun_out
for cfg in 2 3 4 5; do
    ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_c$cfg.log 2>&1 \
        || { echo "bench c$cfg failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
    tail -1 gpurun_out/bench_c$cfg.log | cut -c1-400
done
for cfg in "$@"; do
    bash profiles/collect.sh "$tag" "$cfg" || exit 1
done
echo done
