#!/bin/bash
# N > 1 bench paths after the round's changes (child context in PartialDeps, launch folds): 4 gloo ranks on GPU 0,
# configs 3 and 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_shard_rehearse.sh 4 3 0.05 && bash tools/gpu_shard_rehearse.sh 4 2 0.25
