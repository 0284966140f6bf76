#!/bin/bash
# Literal-filter session: matcher parity tests, then C3 / X1 / C4 legs.
#   gpurun --timeout 900 -- 'bash tools/r3_lit.sh <tag>'
set -o pipefail
TAG=${1:-lit}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest match/fused/templates/post/formats"
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_fused.py tests/test_gpu_templates.py \
    tests/test_gpu_post.py tests/test_gpu_formats.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for wl in c3 x1 c4; do
  step "bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
step done
