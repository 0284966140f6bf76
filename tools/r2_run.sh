#!/bin/bash
# Generic: run the given pytest files (GPU) and then optional bench commands.
#   TESTS="tests/a.py tests/b.py" BENCH="--workload x1 ...;VAR=1 --workload c4" bash tools/r2_run.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r2run}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  echo "[$(date +%T)] pytest $TESTS"
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
i=0
IFS=';' read -ra BL <<< "${BENCH:-}"
for b in "${BL[@]}"; do
  [ -z "$b" ] && continue
  i=$((i+1))
  echo "[$(date +%T)] bench $b"
  pre="${b%%--*}"; args="--${b#*--}"  # optional leading VAR=value settings
  timeout -k 10 600 env $pre python -u bench.py $args > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" || { tail -20 "$OUT/bench$i.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench$i.json" "[$b]"
done
echo "[$(date +%T)] done"
