#!/bin/bash
# Build an experimental variant of libswarmgpu.so (extra -D flags) into tools/variants/<name>/,
# for A/B timing on the GPU box (tools/ab.sh swaps it in on the box's scratch copy only).
#   bash tools/build_variant.sh <name> "-DFLAG=1 ..."
set -e
NAME=$1; shift
FLAGS="$*"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/variants/$NAME
mkdir -p "$OUT/obj"
cd "$ROOT/swarm_amd/csrc"
pids=()
for f in *.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable $FLAGS \
      -c "$f" -o "$OUT/obj/${f%.hip}.o" & pids+=($!)
done
for f in *.cpp; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC $FLAGS -c "$f" -o "$OUT/obj/${f%.cpp}.cpp.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libswarmgpu.so" "$OUT"/obj/*.o
rm -rf "$OUT/obj"
echo "built $OUT/libswarmgpu.so ($FLAGS)"
