#!/bin/bash
# Tuning build: the library with -DACC_PHASE_PROF (per-phase cycle counters printed to stderr) in tools/ab/prof.so.
# Use with ACC_LIB_PATH=tools/ab/prof.so; never the product build.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/prof/build
for f in cassandra-accord_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DACC_PHASE_PROF -c "$f" -o tools/prof/build/$(basename "$f" .hip).o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o tools/ab/prof.so tools/prof/build/*.o
