#!/bin/bash
# Round-2 first GPU session: parity tests, the default bench line, and SQ counter passes
# for the matching kernels. gpurun -- 'bash tools/r2_early.sh <tag>'
set -o pipefail
TAG=${1:-r2a}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -3 "$OUT/gpu_tests.log"
step "bench c2"
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
step "sq c3"
timeout -k 10 400 bash tools/pmc_sq.sh "$TAG/sq_c3" bench.py --workload c3 --lines 20000000 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
step "sq c4"
timeout -k 10 400 bash tools/pmc_sq.sh "$TAG/sq_c4" bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
python3 tools/pmc_sq.py "$OUT/sq_c3" "$OUT/sq_c3.md" > /dev/null
python3 tools/pmc_sq.py "$OUT/sq_c4" "$OUT/sq_c4.md" > /dev/null
step done
