#!/bin/bash
# smoke() then the rocprofv3 kernel stats + PMC passes of the given legs.
set -o pipefail
TAG=${1:-sp}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
bash tools/r3_profile.sh "$TAG" "$@"
