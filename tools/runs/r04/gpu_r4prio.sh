#!/bin/bash
# context stream at the highest priority (the stream pass ahead of the side-stream window tier): config 2 / 3 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CFGS="2 3" STEPS=20 bash tools/gpu_abn.sh new new+ACC_STREAM_PRIO=1 || exit 1
