#!/bin/bash
# Round-3 GPU session: parity tests, the driver's default bench command, and a 2-rank gloo
# rehearsal of the N > 1 default (C5 strong scaling, round-pipelined exchange).
#   gpurun --timeout 1200 -- 'bash tools/r3_run.sh <tag> [tests|notests] [rehearse|norehearse]'
set -o pipefail
TAG=${1:-r3}
MODE=${2:-tests}
REH=${3:-rehearse}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ "$MODE" = tests ]; then
  step "pytest -m gpu"
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi
step "bench default (driver command)"
SECONDS=0; timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" \
    2> "$OUT/bench_default.err" || { tail -30 "$OUT/bench_default.err"; exit 1; }
echo "bench wall ${SECONDS}s"
python3 tools/jsum.py "$OUT/bench_default.json" || true
if [ "$REH" = rehearse ]; then
  step "bench --gpus 2 gloo rehearsal (C5 strong, 200M records)"
  timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --c5-records 200000000 --steps 3 --warmup 1 \
      > "$OUT/bench_n2_gloo.json" 2> "$OUT/bench_n2_gloo.err" || { tail -30 "$OUT/bench_n2_gloo.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_n2_gloo.json" || true
fi
step done
