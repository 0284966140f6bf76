#!/bin/bash
# httpx -json fields session: format/template parity tests, then the fields leg.
#   gpurun --timeout 900 -- 'bash tools/r3_fields.sh <tag>'
set -o pipefail
TAG=${1:-fields}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest formats/templates/post"
timeout -k 10 400 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_templates.py tests/test_gpu_post.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
step "bench fields"
timeout -k 10 300 python -u bench.py --workload fields --steps 5 --warmup 2 > "$OUT/bench_fields.json" \
    2> "$OUT/bench_fields.err" || { tail -20 "$OUT/bench_fields.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_fields.json" fields
step done
