#!/bin/bash
# Kernel experiments on the GPU box: the C2 pipeline per kernel (tools/c2_probe.py) under
# each given environment setting (only switches that keep results correct).
set -o pipefail
OUT=gpurun_out/${1:-probe}
shift
mkdir -p "$OUT"
for m in "NONE=1" "$@"; do
  env $m timeout -k 10 120 python tools/c2_probe.py >> "$OUT/probe.jsonl" 2>> "$OUT/probe.err" || exit 1
  tail -1 "$OUT/probe.jsonl"
done
