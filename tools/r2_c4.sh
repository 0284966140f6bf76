#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r2c4}
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in ${VS:-1 0}; do
  SG_VERIFY_SORT=$V timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c4_v$V.json" 2> "$OUT/c4_v$V.err" || { tail -20 "$OUT/c4_v$V.err"; exit 1; }
  python3 tools/jsum.py "$OUT/c4_v$V.json" "vsort=$V"
done
for V in ${VS:-1 0}; do
  SG_VERIFY_SORT=$V timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_v$V" -o p --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_v$V.log" 2>&1 || { tail -5 "$OUT/pmc_v$V.log"; exit 1; }
  python3 - "$OUT/pmc_v$V" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:6]:
    print("   %-20s fetch MB/launch (x2 corr) %.1f" % (k[:20], 2 * sum(v) / len(v) / 1e3))
PY
done
