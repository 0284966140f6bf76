#!/bin/bash
# A/B timing on the GPU box: for each variant (tools/variants/<name>/libswarmgpu.so, or
# "base" = the tree's own build) swap the library into this scratch copy and run one probe.
#   gpurun -- 'bash tools/ab.sh <tag> "<probe command>" base v1 v2 ...'
set -o pipefail
TAG=$1; CMD=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cp swarm_amd/libswarmgpu.so "$OUT/.base.so"
for v in "$@"; do
  if [ "$v" = base ]; then cp "$OUT/.base.so" swarm_amd/libswarmgpu.so; else cp "tools/variants/$v/libswarmgpu.so" swarm_amd/libswarmgpu.so; fi
  echo "[$(date +%T)] variant $v: $CMD"
  timeout -k 10 300 bash -c "$CMD" > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -20 "$OUT/$v.err"; cp "$OUT/.base.so" swarm_amd/libswarmgpu.so; exit 1; }
  tail -c 1500 "$OUT/$v.json"; echo
done
cp "$OUT/.base.so" swarm_amd/libswarmgpu.so
rm -f "$OUT/.base.so"
