#!/bin/bash
# Dedup-path GPU tests + C2, X1, URLs, C5 legs (no GNU baselines).
set -o pipefail
TAG=${1:-ks}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest dedup/fused/sharded"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_fused.py tests/test_gpu_sharded.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for wl in c2 x1 urls c5; do
  step "bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
step done
