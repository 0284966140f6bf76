#!/bin/bash
set -o pipefail
TAG=${1:-hyb2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest hybrid + dedup"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedup.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/ab.sh "$TAG/ab" "python -u tools/c2_probe.py" base t3584 t2560
step done
