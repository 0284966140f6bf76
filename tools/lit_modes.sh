#!/bin/bash
# k_lit_scan pass split on C3 and the C4 prefilter: normal, skip verify (1), skip probes (2),
# skip both (3), and the candidate counters (8).
#   gpurun -- 'bash tools/lit_modes.sh <tag>'
set -o pipefail
OUT=gpurun_out/${1:-litmodes}
mkdir -p "$OUT"
for mode in -1 1 2 3 8; do
  if [ "$mode" = -1 ]; then E=""; else E="SG_LIT_DEBUG=$mode"; fi
  echo "[$(date +%T)] c3 mode $mode"
  timeout -k 10 200 env $E python3 tools/c3_probe.py 20000000 >> "$OUT/c3.log" 2>&1 || { tail -5 "$OUT/c3.log"; exit 1; }
  echo "[$(date +%T)] c4 mode $mode"
  timeout -k 10 200 env $E python3 tools/c4_probe.py 4000000 bench >> "$OUT/c4.log" 2>&1 || { tail -5 "$OUT/c4.log"; exit 1; }
done
tail -n 12 "$OUT/c3.log" "$OUT/c4.log"
