#!/bin/bash
# SQ/TCC counter passes over the C2 probe (one pass per counter group, MI355X slot limits:
# 8 SQ, 4 TCC per pass). Usage: bash tools/pmc_sq.sh <tag> [probe.py [args...]]
# (default probe: tools/c2_probe.py; e.g. bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline)
set -o pipefail
OUT=gpurun_out/${1:-sq}
PROBE=${2:-tools/c2_probe.py}
shift 2 2>/dev/null || shift $#
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM TCC_HIT TCC_MISS"
i=1
for P in "$P1" "$P2"; do
  echo "[$(date +%T)] pass $i"
  timeout -s KILL 240 rocprofv3 --pmc $P -T -d "$OUT/p$i" -o p --output-format csv -- python3 $PROBE "$@" > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; exit 1; }
  i=$((i+1))
done
echo done
