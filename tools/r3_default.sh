#!/bin/bash
# The driver's default bench line (GNU baselines included), then the C3, C4 and fields legs.
set -o pipefail
TAG=${1:-def}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] bench default"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_default.json" default
for wl in c3 c4 fields; do
  echo "[$(date +%T)] bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
echo "[$(date +%T)] done"
