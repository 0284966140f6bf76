#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r2y}
mkdir -p "$OUT"
export TMPDIR=/tmp
for B in ${BUCKETS:-0 1}; do
  SG_BUCKET=$B timeout -k 10 300 python -u bench.py --workload x1 --no-cpu-baseline --steps 5 --warmup 2 ${BENCHARGS:-} > "$OUT/x1_b$B.json" 2> "$OUT/x1_b$B.err" || { tail -20 "$OUT/x1_b$B.err"; exit 1; }
  python3 tools/jsum.py "$OUT/x1_b$B.json" "B=$B"
done
