#!/bin/bash
# Full GPU suite + default line (no GNU baselines).
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
step "bench default (no GNU)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-gnu > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_default.json" default
step done
