#!/usr/bin/env python3
"""Per-kernel averages of the SQ/TCC counter passes written by tools/gpu.sh sq:<leg>.
  python tools/pmc_sq.py gpurun_out/<tag>/sq_<leg> [out.md]   (reads sq_<leg>_p*/)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    src = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(src + "_p*/p_counter_collection.csv") + glob.glob(os.path.join(src, "p*", "p_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    cols = ["SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
            "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_LEVEL_WAVES", "TCC_HIT", "TCC_MISS"]
    lines = ["| kernel | " + " | ".join(c.replace("SQ_", "").lower() for c in cols) + " | wait% | l2hit% |",
             "|" + "---|" * (len(cols) + 3)]
    rows = []
    for k, d in acc.items():
        avg = {c: (sum(d[c]) / len(d[c]) if d.get(c) else 0.0) for c in cols}
        tot = avg["SQ_WAIT_ANY"] + avg["SQ_WAIT_INST_ANY"] + avg["SQ_ACTIVE_INST_ANY"]
        wait = 100.0 * avg["SQ_WAIT_ANY"] / tot if tot else 0.0
        h = avg["TCC_HIT"] + avg["TCC_MISS"]
        rows.append((avg["SQ_BUSY_CYCLES"], k, avg, wait, 100.0 * avg["TCC_HIT"] / h if h else 0.0))
    for _, k, avg, wait, hit in sorted(rows, reverse=True):
        lines.append("| %s | " % k + " | ".join("%.3g" % avg[c] for c in cols) + " | %.0f | %.0f |" % (wait, hit))
    text = "\n".join(lines) + "\n"
    print(text)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)


if __name__ == "__main__":
    main()
