#!/bin/bash
# Bucket-path iteration: its parity tests, the dedup tests, then the C2 bench line.
set -o pipefail
TAG=${1:-r2b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest bucket"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bucket.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/bucket_tests.log" 2>&1 || { tail -40 "$OUT/bucket_tests.log"; exit 1; }
tail -3 "$OUT/bucket_tests.log"
step "pytest dedup"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/dedup_tests.log" 2>&1 || { tail -40 "$OUT/dedup_tests.log"; exit 1; }
tail -3 "$OUT/dedup_tests.log"
step "bench c2"
SG_BK_DEBUG=${BKDBG:-0} timeout -k 10 300 python -u bench.py ${BENCHARGS:-} > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
step done
grep "bk_" "$OUT/bench_c2.err" | tail -5
