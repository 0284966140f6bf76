#!/bin/bash
# Kernel experiments on the GPU box: the C2 pipeline per kernel (tools/c2_probe.py).
set -o pipefail
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
timeout -k 10 120 python tools/c2_probe.py >> "$OUT/probe.jsonl" 2>> "$OUT/probe.err" || exit 1
tail -1 "$OUT/probe.jsonl"
