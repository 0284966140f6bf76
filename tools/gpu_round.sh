#!/bin/bash
# One GPU-box session: parity tests, both bench legs, rocprofv3 kernel stats of the C2 bench,
# and the HBM traffic counters (one counter per pass, as MI355X_MICROARCH.md prescribes).
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh <tag> [tests|notests]'
set -o pipefail
TAG=${1:-run}
MODE=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }

if [ "$MODE" = tests ]; then
  step "pytest -m gpu"
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
  tail -3 "$OUT/gpu_tests.log"
fi

step "bench c2"
timeout -k 10 300 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
cat "$OUT/bench_c2.json"
step "bench c3"
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { tail -20 "$OUT/bench_c3.err"; exit 1; }
cat "$OUT/bench_c3.json"

step "bench c4"
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { tail -20 "$OUT/bench_c4.err"; exit 1; }
cat "$OUT/bench_c4.json"

step "bench fields"
timeout -k 10 300 python -u bench.py --workload fields --steps 3 --warmup 1 > "$OUT/bench_fields.json" 2> "$OUT/bench_fields.err" || { tail -20 "$OUT/bench_fields.err"; exit 1; }
cat "$OUT/bench_fields.json"

step "bench c5"
timeout -k 10 600 python -u bench.py --workload c5 --steps 3 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" || { tail -20 "$OUT/bench_c5.err"; exit 1; }
cat "$OUT/bench_c5.json"

step "rocprofv3 stats c2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_c2" -o c2 --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof_c2.json" 2> "$OUT/prof_c2.err" || { tail -20 "$OUT/prof_c2.err"; exit 1; }
step "rocprofv3 stats c3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_c3" -o c3 --output-format csv -- \
    python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err" || { tail -20 "$OUT/prof_c3.err"; exit 1; }

step "rocprofv3 stats c4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_c4" -o c4 --output-format csv -- \
    python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err" || { tail -20 "$OUT/prof_c4.err"; exit 1; }

step "rocprofv3 stats fields"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_fields" -o fields --output-format csv -- \
    python3 bench.py --workload fields --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/prof_fields.json" 2> "$OUT/prof_fields.err" || { tail -20 "$OUT/prof_fields.err"; exit 1; }

step "rocprofv3 stats c5"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_c5" -o c5 --output-format csv -- \
    python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c5.json" 2> "$OUT/prof_c5.err" || { tail -20 "$OUT/prof_c5.err"; exit 1; }

for ctr in FETCH_SIZE WRITE_SIZE; do
  step "pmc $ctr c2"
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_c2_$ctr" -o p --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_c2_$ctr.json" 2> "$OUT/pmc_c2_$ctr.err" || { tail -20 "$OUT/pmc_c2_$ctr.err"; exit 1; }
  step "pmc $ctr c3"
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_c3_$ctr" -o p --output-format csv -- \
      python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_c3_$ctr.json" 2> "$OUT/pmc_c3_$ctr.err" || { tail -20 "$OUT/pmc_c3_$ctr.err"; exit 1; }
  step "pmc $ctr c4"
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_c4_$ctr" -o p --output-format csv -- \
      python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_c4_$ctr.json" 2> "$OUT/pmc_c4_$ctr.err" || { tail -20 "$OUT/pmc_c4_$ctr.err"; exit 1; }
  step "pmc $ctr fields"
  timeout -s KILL 240 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_fields_$ctr" -o p --output-format csv -- \
      python3 bench.py --workload fields --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fields_$ctr.json" 2> "$OUT/pmc_fields_$ctr.err" || { tail -20 "$OUT/pmc_fields_$ctr.err"; exit 1; }
done
step "done"
