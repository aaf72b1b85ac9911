#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (tools/calib_fetch.hip; one counter per pass).
set -o pipefail
root=$(pwd)
out=$root/gpurun_out/calib
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$root/tools/calib_fetch" > "$out/plain.log" 2>&1 || { echo "plain run failed"; cat "$out/plain.log"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "$root/tools/calib_fetch" > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$out/$c" -o run -- "$root/tools/calib_fetch" > "$out/$c.log" 2>&1 || echo "counter $c unavailable ($?)"
done
cat "$out/plain.log"
echo calib done
