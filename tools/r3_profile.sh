#!/bin/bash
# Round-3 profiles: rocprofv3 kernel stats and the HBM traffic counters (FETCH_SIZE and
# WRITE_SIZE, one counter per pass as MI355X_MICROARCH.md prescribes) per leg; summaries with
#   python3 tools/pmc_summary.py gpurun_out/<tag> profiles/r03/<name> c2 x1 ...
#   gpurun --timeout 1200 -- 'bash tools/r3_profile.sh <tag> [legs...]'
set -o pipefail
TAG=${1:-r3prof}; shift
LEGS=${*:-c2 x1 urls c3 c4 c5 fields}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
args_of() {
  case $1 in
    c2) echo "--steps 5 --warmup 2 --no-cpu-baseline --no-sub" ;;
    x1) echo "--workload x1 --steps 5 --warmup 2 --no-cpu-baseline" ;;
    urls) echo "--workload urls --steps 5 --warmup 2 --no-cpu-baseline" ;;
    c3) echo "--workload c3 --steps 3 --warmup 1 --no-cpu-baseline" ;;
    c4) echo "--workload c4 --steps 2 --warmup 1 --no-cpu-baseline" ;;
    c5) echo "--workload c5 --steps 1 --warmup 1 --no-cpu-baseline" ;;
    c5r) echo "--workload c5 --c5-path rounds --c5-records 125000000 --steps 3 --warmup 1 --no-cpu-baseline" ;;
    fields) echo "--workload fields --steps 2 --warmup 1 --no-cpu-baseline" ;;
  esac
}
for wl in $LEGS; do
  A=$(args_of $wl)
  step "rocprofv3 stats $wl"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$wl" -o $wl --output-format csv -- \
      python3 bench.py $A > "$OUT/prof_$wl.json" 2> "$OUT/prof_$wl.err" || { tail -20 "$OUT/prof_$wl.err"; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step "pmc $ctr $wl"
    timeout -s KILL 400 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_${wl}_$ctr" -o p --output-format csv -- \
        python3 bench.py $A > "$OUT/pmc_${wl}_$ctr.json" 2> "$OUT/pmc_${wl}_$ctr.err" || { tail -20 "$OUT/pmc_${wl}_$ctr.err"; exit 1; }
  done
done
step done
