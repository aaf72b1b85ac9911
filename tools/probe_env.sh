#!/bin/bash
# usage: bash tools/probe_env.sh <config> "<ENV=.. ENV2=..>" ... : config-N bench per env setting, prints step ms and the
# top kernels (tuning probes; results go to gpurun_out/probe_*.log)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cfg=$1; shift
i=0
for envs in "$@"; do
    i=$((i+1))
    env $envs ACC_BENCH_KERNELS=1 timeout -k 10 300 python -u bench.py --config $cfg --no-cpu --steps 5 --warmup 2 > gpurun_out/probe_$i.log 2>&1 \
        || { echo "probe [$envs] failed"; tail -20 gpurun_out/probe_$i.log; exit 1; }
    python3 - "$envs" gpurun_out/probe_$i.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = d.get("kernels_ms_per_step", {})
top = sorted(k.items(), key=lambda x: -x[1])[:8]
print(sys.argv[1], "| ms/step", d["ms_per_step"], "|", ", ".join(f"{a}={b}" for a, b in top), "|",
      {a: b for a, b in d.get("path_stats", {}).items() if "txns" in a})
PY
done
