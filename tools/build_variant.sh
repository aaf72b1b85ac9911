#!/bin/bash
# Tuning builds: tools/build_variant.sh <name> <extra hipcc flags...> -> tools/ab/<name>.so (A/B probes via
# ACC_LIB_PATH; never the product build)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/prof/build_$name
for f in cassandra-accord_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c "$f" -o tools/prof/build_$name/$(basename "$f" .hip).o &
done
wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -o tools/ab/$name.so tools/prof/build_$name/*.o
