#!/bin/bash
# bench lines for the round: config 2 (default), then the variants given as "cfg:args" pairs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "$@"; do
    cfg=${spec%%:*}; extra=${spec#*:}; [ "$extra" = "$spec" ] && extra=""
    tagname=$(echo "c${cfg}${extra}" | tr -d ' -')
    ACC_BENCH_KERNELS=1 timeout -k 10 600 python -u bench.py --config $cfg $extra > gpurun_out/bench_${tagname}.log 2>&1 \
        || { echo "bench $spec failed"; tail -30 gpurun_out/bench_${tagname}.log; exit 1; }
    tail -1 gpurun_out/bench_${tagname}.log | cut -c1-600
done
echo done
