#!/bin/bash
# Build a compile-time variant of the library for an A/B (tools/ab.sh):
#   tools/variant.sh NAME "-DMACRO=1" [source.hip ...]   -> scratch/NAME.so
# The named sources (default pfdr_quadratic.hip) are recompiled with the
# extra flags; every other object is the in-tree build's.
set -eu
NAME=$1; FLAGS=$2; shift 2
SRCS=${*:-pfdr_quadratic.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/cp_pfdr_graph_d1_amd/csrc
T=$(mktemp -d)
make -s -C "$C" >/dev/null
cp "$C"/*.o "$T"/
for s in $SRCS; do
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
        -fno-gpu-flush-denormals-to-zero --offload-arch=gfx950 -munsafe-fp-atomics $FLAGS \
        -c -o "$T/${s%.hip}.o" "$C/$s"
done
mkdir -p "$ROOT/scratch"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/scratch/$NAME.so" "$T"/*.o \
    -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl -lpthread
rm -rf "$T"
echo "scratch/$NAME.so"
