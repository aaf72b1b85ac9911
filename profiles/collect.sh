#!/bin/bash
# Profile collection for one round, run on the GPU box from the repo root:
#   bash profiles/collect.sh <tag> <config> [variant] [extra bench args...]
# Pass 1: kernel trace + stats (per-kernel durations). Passes 2/3: HBM traffic counters, one TCC counter per
# pass (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2: they cannot share a pass on gfx950).
# Every pass runs under its own time limit; the script stops at the first failure.
set -u
tag=${1:-r02}
cfg=${2:-2}
variant=${3:-}
shift 3 2>/dev/null || shift $#
root=$(pwd)
out=$root/gpurun_out/prof_${tag}_c${cfg}${variant}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
export ACC_BENCH_MIXED=0   # profile the config-4 RangeDeps step alone (the mixed-batch KeyDeps leg runs after it)
export ACC_BENCH_CFK=0     # likewise the config-2 CommandsForKey-update leg
bench="$root/bench.py --config $cfg --steps 5 --warmup 2 --no-cpu $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 $bench > "$out/trace.log" 2>&1 || { echo "trace pass failed: $?"; tail -5 "$out/trace.log"; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 $bench > "$out/fetch.log" 2>&1 || { echo "fetch pass failed: $?"; tail -5 "$out/fetch.log"; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 $bench > "$out/write.log" 2>&1 || { echo "write pass failed: $?"; tail -5 "$out/write.log"; exit 1; }
echo "profiles collected under $out"
