#!/bin/bash
# Literal filter check: match/fused tests, then C4 (auto vs the old build), C3, X1, fields.
set -o pipefail
TAG=${1:-litchk}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fused.py tests/test_gpu_templates.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for wl in c4 c3 x1 fields; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu --no-cpu-baseline > "$OUT/$wl.json" \
      2> "$OUT/$wl.err" || { tail -20 "$OUT/$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/$wl.json" $wl | head -2
done
if [ -d tools/variants/old ]; then
  bash tools/ab.sh "$TAG/old" "python -u bench.py --workload c4 --steps 10 --warmup 3 --no-gnu --no-cpu-baseline" old > /dev/null 2>&1 || exit 1
  python3 tools/jsum.py "$OUT/old/old.json" c4-old | head -2
fi
