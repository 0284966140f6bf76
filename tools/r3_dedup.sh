#!/bin/bash
# Dedup-path session: dedup/sharded/fused/distributed parity tests, then the C2 (+urls, x1)
# default line without the slow sub-legs, and C5.
#   gpurun --timeout 1100 -- 'bash tools/r3_dedup.sh <tag> [c5]'
set -o pipefail
TAG=${1:-dd}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest dedup/sharded/fused/post/ingest/distributed"
timeout -k 10 500 python -u -m pytest tests/test_gpu_dedup.py tests/test_gpu_sharded.py tests/test_gpu_fused.py \
    tests/test_gpu_post.py tests/test_gpu_ingest.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
step "bench default line (c2 + urls, x1, c1, c3, c5 sub-legs; no GNU baselines)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-gnu > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" \
    || { tail -20 "$OUT/bench_c2.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_c2.json" c2
if [ "$2" = c5 ]; then
  step "bench c5 ips"
  timeout -k 10 400 python -u bench.py --workload c5 --c5-data ips --steps 5 --warmup 2 --no-gnu --no-cpu-baseline \
      > "$OUT/bench_c5ips.json" 2> "$OUT/bench_c5ips.err" || { tail -20 "$OUT/bench_c5ips.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_c5ips.json" c5ips
fi
step done
