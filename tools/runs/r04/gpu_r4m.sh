#!/bin/bash
# full GPU test suite + smoke (round-end style), then the N=8 store rehearsal (8 gloo ranks on one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 280 --timeout-method thread -m gpu tests/ > gpurun_out/r4_gputests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -5 gpurun_out/r4_smoke.log; exit 1; }
tail -1 gpurun_out/r4_smoke.log
bash tools/gpu_shard_rehearse.sh 8 3 0.05
