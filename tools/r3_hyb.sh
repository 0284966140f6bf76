#!/bin/bash
# Hybrid-sort session: new hybrid tests + dedup parity, then the C2 probe and the default line.
set -o pipefail
TAG=${1:-hyb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest hybrid"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup.py -m gpu -x -q -k hybrid --timeout 120 --timeout-method thread \
    > "$OUT/tests_hyb.log" 2>&1 || { tail -40 "$OUT/tests_hyb.log"; exit 1; }
tail -2 "$OUT/tests_hyb.log"
step "c2 probe"
timeout -k 10 200 python -u tools/c2_probe.py > "$OUT/c2_probe.json" 2> "$OUT/c2_probe.err" || { tail -20 "$OUT/c2_probe.err"; exit 1; }
cat "$OUT/c2_probe.json"
step "pytest dedup/sharded/fused/post/ingest/distributed"
timeout -k 10 500 python -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_sharded.py tests/test_gpu_fused.py \
    tests/test_gpu_post.py tests/test_gpu_ingest.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
step "bench default (no GNU)"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-gnu > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_default.json" default
step done
