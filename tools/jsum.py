#!/usr/bin/env python3
"""One-line summary of a bench JSON file: ms/step, dedup path, records and the top kernels.
  python3 tools/jsum.py <bench.json> [label]"""
import json
import sys

d = json.load(open(sys.argv[1]))
lab = sys.argv[2] if len(sys.argv) > 2 else ""
print(lab, d.get("ms_per_step"), d.get("dedup_path"), d.get("records"))
print("  ", [(k, v.get("ms_total")) for k, v in list(d.get("kernels", {}).items())[:14]])
x = d.get("fused_x1")
if x:
    print("  X1", x.get("ms_per_step"), x.get("dedup_path"), x.get("records"))
    print("    ", [(k, v.get("ms_total")) for k, v in list((x.get("kernels_top") or {}).items())])
