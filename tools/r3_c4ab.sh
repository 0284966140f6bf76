#!/bin/bash
# C4 prefilter scheme check: forced two-class, forced joint, automatic, and the old build.
set -o pipefail
TAG=${1:-c4ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
C="python -u bench.py --workload c4 --steps 10 --warmup 3 --no-gnu --no-cpu-baseline"
for mode in 0 1 auto; do
  echo "[$(date +%T)] scheme $mode"
  if [ $mode = auto ]; then timeout -k 10 300 $C > "$OUT/auto.json" 2> "$OUT/auto.err" || { tail -20 "$OUT/auto.err"; exit 1; }
  else SG_LIT_SCHEME=$mode timeout -k 10 300 $C > "$OUT/s$mode.json" 2> "$OUT/s$mode.err" || { tail -20 "$OUT/s$mode.err"; exit 1; }; fi
done
bash tools/ab.sh "$TAG/old" "$C" old > /dev/null 2>&1 || exit 1
for f in s0 s1 auto old/old; do python3 tools/jsum.py "$OUT/$f.json" $f | head -3; done
