#!/usr/bin/env python3
"""Summarise one tools/gpu.sh session's prof:<leg> and pmc:<leg> steps: rocprofv3 kernel
stats + the FETCH_SIZE / WRITE_SIZE passes.

  python tools/pmc_summary.py gpurun_out/<tag> profiles/r04/<name>  [leg[:workload] ...]

(leg: the gpu.sh leg, e.g. c3p; workload: the key bench.py looks the traffic up under, e.g. c3.)

Writes <name>_<wl>_kernels.csv (rocprofv3 --stats, verbatim), <name>_<wl>_summary.md and
updates profiles/pmc_traffic.json (per-kernel HBM bytes per launch, read by bench.py).

Counter units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE
are reported in KiB; on gfx950 FETCH_SIZE counts a wide coalesced streaming read at exactly
half its bytes (128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores. Other access widths are uncalibrated (noted in the summary).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


# Kernels launched once per step over the whole input (the matching engines): their per-launch
# traffic is averaged over FULL-SIZE dispatches only, so a smaller launch of the same symbol
# (a sample check on a slice) cannot pull it below the real launches'. Kernels a step launches
# at several sizes (the cur and prior parse, C5's per-part passes) average every dispatch.
FULL_SIZE = {"k_lit_scan", "k_verify", "k_dfa_match", "k_dfa_multi", "k_ac_match", "k_json_scan_t", "k_json_emit"}


def per_kernel_counter(path, counter, used=None):
    """Per kernel: the counter's average per dispatch (FULL_SIZE kernels: over the dispatches
    at the largest grid the kernel ran with and at least half its longest duration there).
    used[kernel] = (dispatches averaged, all)."""
    rows = defaultdict(list)
    if not os.path.exists(path):  # no PMC pass for this workload: stats only
        return {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            dur = float(row.get("End_Timestamp") or 0) - float(row.get("Start_Timestamp") or 0)
            rows[row["Kernel_Name"]].append((int(row.get("Grid_Size") or 0), dur, float(row["Counter_Value"]) * 1024.0))
    out = {}
    for k, rs in rows.items():
        full = rs
        if k.split("<")[0] in FULL_SIZE:
            g = max(r[0] for r in rs)
            at = [r for r in rs if r[0] == g]
            dmax = max(r[1] for r in at)
            full = [r for r in at if r[1] >= 0.5 * dmax] or at
        out[k] = sum(r[2] for r in full) / len(full)
        if used is not None:
            used[k] = (len(full), len(rs))
    return out


def stats(path):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            out[row["Name"]] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3, float(row["Percentage"]))
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    wls = sys.argv[3:] or ["c2", "c3"]
    tfile = os.path.join(os.path.dirname(dst), "..", "pmc_traffic.json")
    tfile = os.path.normpath(tfile)
    traffic = json.load(open(tfile)) if os.path.exists(tfile) else {}
    for spec in wls:
        wl, key = (spec.split(":") + [spec])[:2] if ":" in spec else (spec, spec)
        ks = os.path.join(src, "prof_" + wl, wl + "_kernel_stats.csv")
        if not os.path.exists(ks):
            continue
        shutil.copy(ks, "%s_%s_kernels.csv" % (dst, key))
        st = stats(ks)
        used = {}
        fe = per_kernel_counter(os.path.join(src, "pmc_%s_FETCH_SIZE" % wl, "p_counter_collection.csv"), "FETCH_SIZE",
                                used)
        wr = per_kernel_counter(os.path.join(src, "pmc_%s_WRITE_SIZE" % wl, "p_counter_collection.csv"), "WRITE_SIZE")
        lines = ["# %s — rocprofv3 kernel stats + HBM traffic (%s, leg %s)" % (key.upper(), os.path.basename(src), wl), "",
                 "FETCH_SIZE doubled (gfx950 wide-read correction), WRITE_SIZE as reported; both KiB→bytes, "
                 "per launch, averaged over the PMC pass's dispatches (the matching engines: over their full-size "
                 "dispatches only, the largest grid and at least half the longest duration there; `pmc launches` = "
                 "averaged / all). Traffic GB/s = "
                 "(fetch+write) / avg duration (rocprofv3 stats, all calls).", "",
                 "| kernel | calls | avg µs | % time | fetch MB/launch | write MB/launch | traffic GB/s | pmc launches |",
                 "|---|---|---|---|---|---|---|---|"]
        if fe or wr:  # a fresh PMC pass replaces the workload's rows (no stale kernels survive)
            traffic[key] = {}
        for k, (calls, avg_us, pct) in sorted(st.items(), key=lambda kv: -kv[1][2]):
            f = fe.get(k)
            w = wr.get(k)
            tb = (2.0 * f if f is not None else 0.0) + (w or 0.0)
            gbs = tb / (avg_us * 1e-6) / 1e9 if avg_us > 0 and (f is not None or w is not None) else None
            lines.append("| %s | %d | %.2f | %.2f | %s | %s | %s | %s |" % (
                k, calls, avg_us, pct,
                "%.2f" % (2.0 * f / 1e6) if f is not None else "-",
                "%.2f" % (w / 1e6) if w is not None else "-",
                "%.0f" % gbs if gbs is not None else "-",
                "%d/%d" % used[k] if k in used else "-"))
            if (f is not None or w is not None) and key in traffic:
                traffic[key][k] = {"fetch_bytes": round(2.0 * f) if f is not None else None,
                                  "write_bytes": round(w) if w is not None else None,
                                  "bytes": round(tb), "avg_us": round(avg_us, 2),
                                  "source": os.path.join(os.path.basename(os.path.dirname(dst)),
                                                         os.path.basename(dst) + "_" + key + "_summary.md")}
        with open("%s_%s_summary.md" % (dst, key), "w") as f:
            f.write("\n".join(lines) + "\n")
        print("\n".join(lines[:16]))
    with open(tfile, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
