#!/bin/bash
# Round-3 iteration on the GPU box: a test selection, bench lines, an A/B, the N > 1 rehearsal.
#   SEL="pytest -k expr" CFGS="2 5" AB="5:new new+ACC_LV_WALK=1" bash tools/gpu_r03.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFGS="${CFGS:-2}" bash tools/gpu_quick.sh "${SEL:-}" || exit 1
if [ -n "${AB:-}" ]; then
    cfg=${AB%%:*}; vars=${AB#*:}
    CFGS=$cfg STEPS=10 bash tools/gpu_abn.sh $vars || exit 1
fi
if [ -n "${REHEARSE:-}" ]; then
    bash tools/gpu_shard_rehearse.sh || exit 1
fi
echo done
