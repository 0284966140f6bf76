#!/usr/bin/env python3
"""One-line summary of a bench JSON file: ms/step, records, roofline and the top kernels of
the headline and of every sub-leg.
  python3 tools/jsum.py <bench.json> [label]"""
import json
import sys

lines = [ln for ln in open(sys.argv[1]) if ln.startswith("{")]
d = json.loads(lines[-1])
lab = sys.argv[2] if len(sys.argv) > 2 else ""


def show(name, x):
    if not isinstance(x, dict):
        return
    if "error" in x:
        print("  %s ERROR %s" % (name, x["error"]))
        return
    rf = x.get("roofline") or {}
    print("  %-8s %s ms/step value %s n_gpus %s hbm_frac %s | %s %s frac %s | %s" % (
        name, x.get("ms_per_step"), x.get("value"), x.get("n_gpus"), x.get("hbm_frac_step"), rf.get("kernel"),
        rf.get("avg_launch_us"), rf.get("frac"), x.get("records")))
    cb = x.get("cpu_baseline") or {}
    if cb:
        print("           cpu %s %s" % (cb.get("value"), {k: v for k, v in cb.items() if "exact" in k}))
    kt = x.get("kernels_top") or x.get("kernels") or {}
    print("           ", [(k, v.get("ms_total")) for k, v in list(kt.items())[:12]])


print(lab)
show("head", d)
for k in ("c1", "c3", "c5", "fused_x1", "urls", "c2_weak"):
    show(k, d.get(k))
