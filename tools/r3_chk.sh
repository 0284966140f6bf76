#!/bin/bash
# One group of GPU test files, bounded (round-end evidence split in small calls).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] pytest $*"
timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 \
    || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
echo "[$(date +%T)] done"
