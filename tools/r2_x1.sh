#!/bin/bash
# Fused-step parity tests and the default bench line (C2 + X1).
set -o pipefail
TAG=${1:-r2x}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest fused"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread \
    > "$OUT/fused_tests.log" 2>&1 || { tail -40 "$OUT/fused_tests.log"; exit 1; }
tail -3 "$OUT/fused_tests.log"
step "bench default"
timeout -k 10 600 python -u bench.py ${BENCHARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); x=d['fused_x1']
print('C2', d['ms_per_step'], d['value'], d['dedup_path'])
print('X1', json.dumps(x)[:1500])"
step done
