#!/bin/bash
# Round-end evidence: full GPU suite, smoke(), the driver's default bench line (with the GNU
# baselines) and the C3, C4 and fields legs.
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
step "smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step "bench default"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" \
    || { tail -20 "$OUT/bench_default.err"; exit 1; }
python3 tools/jsum.py "$OUT/bench_default.json" default
for wl in c3 c4 fields; do
  step "bench $wl"
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --no-gnu > "$OUT/bench_$wl.json" \
      2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  python3 tools/jsum.py "$OUT/bench_$wl.json" $wl
done
step done
