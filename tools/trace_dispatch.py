#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace CSV per (kernel, grid size): calls, mean and total
duration, plus the dispatch sequence of the last outer iteration's kernels in order
(consecutive repeats collapsed).  Usage: tools/trace_dispatch.py <kernel_trace.csv>"""
import csv
import sys
from collections import OrderedDict


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = OrderedDict()
    for r in rows:
        name = r["Kernel_Name"].split("(")[0][:70]
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        key = (name, grid)
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        a = agg.setdefault(key, [0, 0.0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print("total %.2f ms over %d dispatches" % (tot, len(rows)))
    for (name, grid), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%-70s grid %-10s %5d calls %9.3f ms avg %9.2f ms tot" % (name, grid, n, t / n, t))
    print("\nlast 120 dispatches (name, grid, ms):")
    seq = []
    for r in rows[-120:]:
        name = r["Kernel_Name"].split("(")[0][:60]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        seq.append("%-60s %-10s %8.3f" % (name, r.get("Grid_Size", "?"), d))
    print("\n".join(seq))


if __name__ == "__main__":
    main(sys.argv[1])
