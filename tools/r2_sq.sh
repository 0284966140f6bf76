#!/bin/bash
# SQ counter passes over the C2 bench (bucket path kernels). gpurun -- 'bash tools/r2_sq.sh <tag>'
set -o pipefail
TAG=${1:-r2sq}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 400 bash tools/pmc_sq.sh "$TAG/sq_c2" bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-x1 || exit 1
python3 tools/pmc_sq.py "gpurun_out/$TAG/sq_c2" "gpurun_out/$TAG/sq_c2.md" > /dev/null
cat "gpurun_out/$TAG/sq_c2.md"
