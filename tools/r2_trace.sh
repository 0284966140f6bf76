#!/bin/bash
# Kernel trace of the C2 step: per-step busy time vs wall (launch gaps / host syncs).
#   gpurun -- 'bash tools/r2_trace.sh <tag> [bench args]'
set -o pipefail
TAG=${1:-r2trace}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] rocprofv3 kernel trace: bench.py $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py "$@" \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 tools/trace_gaps.py "$OUT/trace" > "$OUT/gaps.txt" && cat "$OUT/gaps.txt"
echo "[$(date +%T)] done"
