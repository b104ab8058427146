#!/bin/bash
# Build a compile-time variant of the library for an A/B (tools/ab.sh):
#   tools/variant.sh NAME "-DMACRO=1" [source.hip ...]          -> scratch/NAME.so
#   SED='s/xcd_e_ = 64/xcd_e_ = 128/' tools/variant.sh NAME ""   (edit a copy of the sources)
# The named sources (default pfdr_quadratic.hip) are recompiled with the
# extra flags -- from a copy of csrc/ edited by the sed expression SED when
# given (the product sources stay untouched); every other object is the
# in-tree build's.
set -eu
NAME=$1; FLAGS=$2; shift 2
SRCS=${*:-pfdr_quadratic.hip}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/cp_pfdr_graph_d1_amd/csrc
T=$(mktemp -d)
make -s -C "$C" >/dev/null
cp "$C"/*.o "$T"/
S=$C
if [ -n "${SED:-}" ]; then
    S=$T/src; mkdir -p "$S"
    cp "$C"/*.hip "$C"/*.hpp "$C"/*.cpp "$S"/
    sed -i -e "$SED" "$S"/*.hip "$S"/*.hpp
    diff -r "$C" "$S" | grep -c '^[<>]' | sed 's/^/changed lines: /' >&2 || true
fi
for s in $SRCS; do
    /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
        -fno-gpu-flush-denormals-to-zero --offload-arch=gfx950 -munsafe-fp-atomics -I"$C" $FLAGS \
        -c -o "$T/${s%.hip}.o" "$S/$s"
done
mkdir -p "$ROOT/scratch"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/scratch/$NAME.so" "$T"/*.o \
    -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl -lpthread
rm -rf "$T"
echo "scratch/$NAME.so"
