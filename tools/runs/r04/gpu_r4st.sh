#!/bin/bash
# the unified CommandsForKey store on the config-2-sized update stream
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/runs/r04/cfk_store_time.py 2>&1 | tail -3
