#!/bin/bash
# Full GPU suite + C3, X1, C4 and fields legs (no GNU baselines).
set -o pipefail
TAG=${1:-full3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
for wl in c3 x1 c4 fields; do
  step "bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
step done
