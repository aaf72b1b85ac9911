#!/bin/bash
# Round profiles: rocprof kernel trace + FETCH_SIZE + WRITE_SIZE passes for the given configs, then bench lines.
#   bash tools/gpu_prof_all.sh <tag> <configs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
    bash profiles/collect.sh "$tag" "$cfg" || exit 1
    echo "profiled c$cfg"
done
for cfg in "$@"; do
    ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_c$cfg.log 2>&1 \
        || { echo "bench c$cfg failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
    tail -1 gpurun_out/bench_c$cfg.log | cut -c1-300
done
