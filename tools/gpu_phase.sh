#!/bin/bash
# Per-phase cycle profile of the KeyDeps stream pass (tools/build_prof.sh library) for the given configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
    ACC_LIB_PATH=tools/prof/libaccord_amd.so timeout -k 10 300 python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu \
        > gpurun_out/phase_c$cfg.log 2>&1 || { echo "phase c$cfg failed"; tail -20 gpurun_out/phase_c$cfg.log; exit 1; }
    grep st_phase gpurun_out/phase_c$cfg.log | tail -2
done
