#!/bin/bash
# Tuning build: the library with -DACC_PHASE_PROF (per-phase cycle counters printed to stderr) in tools/ab/prof.so, or
# with other defines: bash tools/build_prof.sh NAME -DFLAG ... -> tools/ab/NAME.so (e.g. lvprof -DACC_LV_PROF).
# Use with ACC_LIB_PATH=tools/ab/<name>.so; never the product build.
set -e
cd "$(dirname "$0")/.."
name=${1:-prof}
shift || true
defs=${*:--DACC_PHASE_PROF}
mkdir -p tools/prof/build_$name tools/ab
for f in cassandra-accord_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -c "$f" -o tools/prof/build_$name/$(basename "$f" .hip).o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o tools/ab/$name.so tools/prof/build_$name/*.o
