#!/bin/bash
# SQ occupancy/stall counters per kernel for one bench config (diagnostics; one --pmc pass, <= 8 SQ counters):
#   bash tools/prof_sq.sh <config> [bench args...]  -> gpurun_out/sq_c<config>/
set -u
cfg=${1:-2}; shift || true
root=$(pwd)
out=$root/gpurun_out/sq_c$cfg
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS \
    --output-format csv -d "$out" -o run -- python3 $root/bench.py --config $cfg --steps 3 --warmup 1 --no-cpu "$@" > "$out/run.log" 2>&1 \
    || { echo "sq pass failed: $?"; tail -5 "$out/run.log"; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
if not f:
    print("no counter csv"); sys.exit(0)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for row in csv.DictReader(open(f[0])):
    k = row.get("Kernel_Name", "?").split("(")[0].split("<")[0][-40:]
    agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    cnt[(k, row["Counter_Name"])] += 1
tops = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:14]
for k, c in tops:
    w = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{k:40s} waves={c.get('SQ_WAVES',0):.0f} wave_cyc={w:.3g} wait={c.get('SQ_WAIT_ANY',0)/w:.2f} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY',0)/w:.2f} active={c.get('SQ_ACTIVE_INST_ANY',0)/w:.2f} "
          f"busy={c.get('SQ_BUSY_CYCLES',0):.3g} vmem={c.get('SQ_INSTS_VMEM',0):.3g} lds={c.get('SQ_INSTS_LDS',0):.3g}")
PY
