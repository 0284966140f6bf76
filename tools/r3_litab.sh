#!/bin/bash
# Literal-filter A/B: matcher parity tests on the tree's build, then C3 and X1 legs per variant.
#   gpurun -- 'bash tools/r3_litab.sh <tag> base v1 ...'
set -o pipefail
TAG=${1:-litab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] pytest match/fused"
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for wl in c3 x1; do
  bash tools/ab.sh "$TAG/$wl" "python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu --no-cpu-baseline" "$@" \
      > "$OUT/ab_$wl.log" 2>&1 || { tail -20 "$OUT/ab_$wl.log"; exit 1; }
  for v in "$@"; do python3 tools/jsum.py "$OUT/$wl/$v.json" "$wl $v" | head -2; done
done
echo "[$(date +%T)] done"
