"""Per-step busy time vs wall from a rocprofv3 kernel trace (CSV): steps are delimited by
the launches of a marker kernel (default k_rs_hist, once per C2 step). Prints the median
step span, the kernel busy time in it, and the largest idle gaps with the kernels around
them."""
import csv
import glob
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_rs_hist"
    files = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(marks) < 3:
        print("fewer than 3 steps found for marker", marker)
        return
    spans, busies, gaps = [], [], {}
    for a, b in zip(marks[-12:-1], marks[-11:]):
        seg = rows[a:b]
        span = rows[b][0] - rows[a][0]
        busy = sum(e - s for s, e, _ in seg)
        spans.append(span)
        busies.append(busy)
        for (s0, e0, n0), (s1, e1, n1) in zip(seg, seg[1:] + [rows[b]]):
            gaps.setdefault((n0, n1), []).append(s1 - e0)
    print("steps analysed: %d; median step span %.1f us, kernel busy %.1f us (%.0f%%), kernels/step %d" % (
        len(spans), statistics.median(spans) / 1e3, statistics.median(busies) / 1e3,
        100 * statistics.median(busies) / statistics.median(spans), marks[-1] - marks[-2]))
    top = sorted(((statistics.median(v), k) for k, v in gaps.items()), reverse=True)[:15]
    print("largest median gaps (us) between consecutive kernels:")
    for g, (a, b) in top:
        print("  %8.1f  %s -> %s" % (g / 1e3, a, b))
    tot = sum(statistics.median(v) for v in gaps.values())
    print("sum of median gaps per step: %.1f us" % (tot / 1e3))


if __name__ == "__main__":
    main()
