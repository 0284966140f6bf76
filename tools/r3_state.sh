#!/bin/bash
# State-of-the-tree benches (no tests): default line (no GNU baselines), fields, c4.
#   gpurun --timeout 900 -- 'bash tools/r3_state.sh <tag>'
set -o pipefail
TAG=${1:-state}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "bench default (no GNU)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-gnu > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_default.json" default
for wl in fields c4; do
  step "bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
step done
