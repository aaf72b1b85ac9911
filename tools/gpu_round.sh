#!/bin/bash
# Full round check on the GPU box: GPU parity tests, the three bench configs, then profile collection.
#   bash tools/gpu_round.sh <tag> [configs-to-profile...]
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=${1:-r01}
shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for cfg in 2 3 4 5; do
    ACC_BENCH_KERNELS=1 timeout -k 10 400 python -u bench.py --config $cfg > gpurun_out/bench_c$cfg.log 2>&1 \
        || { echo "bench c$cfg failed"; tail -30 gpurun_out/bench_c$cfg.log; exit 1; }
    tail -1 gpurun_out/bench_c$cfg.log
done
for cfg in "$@"; do
    bash profiles/collect.sh "$tag" "$cfg" || exit 1
done
echo done
