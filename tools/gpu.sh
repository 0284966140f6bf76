#!/bin/bash
# One GPU-box session, as a list of steps (replaces the per-round r2_*/r3_* scripts):
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh <tag> <step> [<step> ...]'
# Steps (outputs under gpurun_out/<tag>/):
#   tests[:<pytest paths>]    pytest -m gpu (all of tests/ by default)
#   bench:<leg>[@label]       bench.py for a leg (table below) -> bench_<leg>[@label].json
#   prof:<leg>                rocprofv3 --kernel-trace --stats of the leg -> prof_<leg>/
#   pmc:<leg>                 FETCH_SIZE and WRITE_SIZE passes (one counter per pass) -> pmc_<leg>_*/
#   sq:<leg>[@label]          two SQ/TCC counter passes over the leg -> sq_<leg>[@label]_p{1,2}/
#   py:<script>[,args]        python3 <script> args -> py_<name>.log
#   bin:<exe>[,args]          a built program (tools/bin) -> bin_<name>.log
#   VAR=value                 exported for the following steps (e.g. SG_LIT_SCHEME=1)
# Every GPU step runs under its own timeout and the session stops at the first failure.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
args_of() {
  case $1 in
    default) echo "--gpus 1 --steps 20 --warmup 5" ;;
    c2) echo "--steps 10 --warmup 3 --no-sub" ;;
    c2p) echo "--steps 5 --warmup 2 --no-cpu-baseline --no-sub" ;;
    x1) echo "--workload x1 --steps 10 --warmup 3" ;;
    x1p) echo "--workload x1 --steps 5 --warmup 2 --no-cpu-baseline" ;;
    urls) echo "--workload urls --steps 10 --warmup 3" ;;
    urlsp) echo "--workload urls --steps 5 --warmup 2 --no-cpu-baseline" ;;
    c3) echo "--workload c3 --steps 5 --warmup 2" ;;
    c3p) echo "--workload c3 --steps 3 --warmup 1 --no-cpu-baseline" ;;
    c4) echo "--workload c4 --steps 3 --warmup 1" ;;
    c4p) echo "--workload c4 --steps 2 --warmup 1 --no-cpu-baseline" ;;
    c5) echo "--workload c5 --steps 3 --warmup 1" ;;
    c5p) echo "--workload c5 --steps 1 --warmup 1 --no-cpu-baseline" ;;
    c5pb1g) echo "--workload c5 --steps 3 --warmup 1 --no-cpu-baseline --c5-part-bytes 1073741824" ;;
    c5pb512m) echo "--workload c5 --steps 3 --warmup 1 --no-cpu-baseline --c5-part-bytes 536870912" ;;
    c5r) echo "--workload c5 --c5-path rounds --c5-records 125000000 --steps 3 --warmup 1 --no-cpu-baseline" ;;
    c5rnccl) echo "--workload c5 --c5-path rounds --dist-backend nccl --steps 3 --warmup 1" ;;
    c5rp) echo "--workload c5 --c5-path rounds --dist-backend nccl --steps 1 --warmup 1 --no-cpu-baseline" ;;
    fields) echo "--workload fields --steps 3 --warmup 1" ;;
    fieldsp) echo "--workload fields --steps 2 --warmup 1 --no-cpu-baseline" ;;
    n2gloo) echo "--gpus 2 --dist-backend gloo --c5-records 200000000 --steps 3 --warmup 1" ;;
    *) echo "unknown leg $1" >&2; return 1 ;;
  esac
}
SQ1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQ2="SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM TCC_HIT TCC_MISS"
for s in "$@"; do
  kind=${s%%:*}; arg=${s#*:}
  case $s in
    *=*) if [ "$kind" = "$s" ]; then export "$s"; step "env $s"; continue; fi ;;
  esac
  case $kind in
    tests)
      paths=tests; [ "$arg" != "$s" ] && paths=${arg//,/ }
      step "pytest -m gpu $paths"
      timeout -k 10 900 python -u -m pytest $paths -m gpu -x -q --timeout 240 --timeout-method thread \
          > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
      tail -3 "$OUT/tests.log" ;;
    bench)
      A=$(args_of "${arg%%@*}") || exit 1
      step "bench $arg: $A"
      SECONDS=0
      timeout -k 10 900 python -u bench.py $A > "$OUT/bench_$arg.json" 2> "$OUT/bench_$arg.err" \
          || { tail -30 "$OUT/bench_$arg.err"; exit 1; }
      echo "bench $arg wall ${SECONDS}s"
      python3 tools/jsum.py "$OUT/bench_$arg.json" || true ;;
    prof)
      A=$(args_of "$arg") || exit 1
      step "rocprofv3 stats $arg"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$arg" -o $arg --output-format csv -- \
          python3 bench.py $A > "$OUT/prof_$arg.json" 2> "$OUT/prof_$arg.err" || { tail -20 "$OUT/prof_$arg.err"; exit 1; } ;;
    pmc)
      A=$(args_of "$arg") || exit 1
      for ctr in FETCH_SIZE WRITE_SIZE; do
        step "pmc $ctr $arg"
        timeout -s KILL 600 rocprofv3 --pmc $ctr -T -d "$OUT/pmc_${arg}_$ctr" -o p --output-format csv -- \
            python3 bench.py $A > "$OUT/pmc_${arg}_$ctr.json" 2> "$OUT/pmc_${arg}_$ctr.err" \
            || { tail -20 "$OUT/pmc_${arg}_$ctr.err"; exit 1; }
      done ;;
    sq)
      A=$(args_of "${arg%%@*}") || exit 1
      i=1
      for P in "$SQ1" "$SQ2"; do
        step "sq pass $i $arg"
        timeout -s KILL 400 rocprofv3 --pmc $P -T -d "$OUT/sq_${arg}_p$i" -o p --output-format csv -- \
            python3 bench.py $A > "$OUT/sq_${arg}_p$i.log" 2>&1 || { tail -5 "$OUT/sq_${arg}_p$i.log"; exit 1; }
        i=$((i+1))
      done ;;
    py)
      scr=${arg%%,*}; rest=""; [ "$scr" != "$arg" ] && rest=${arg#*,}
      name=$(basename "$scr" .py)
      step "python3 $scr ${rest//,/ }"
      timeout -k 10 600 python3 -u "$scr" ${rest//,/ } > "$OUT/py_$name.log" 2>&1 || { tail -30 "$OUT/py_$name.log"; exit 1; }
      tail -40 "$OUT/py_$name.log" ;;
    bin)
      exe=${arg%%,*}; rest=""; [ "$exe" != "$arg" ] && rest=${arg#*,}
      name=$(basename "$exe")
      step "$exe ${rest//,/ }"
      timeout -k 10 300 "$exe" ${rest//,/ } > "$OUT/bin_$name.log" 2>&1 || { tail -30 "$OUT/bin_$name.log"; exit 1; }
      tail -20 "$OUT/bin_$name.log" ;;
    *) echo "unknown step $s"; exit 1 ;;
  esac
done
step done
