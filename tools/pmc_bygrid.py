#!/usr/bin/env python3
"""Per-(kernel, grid size) means of rocprofv3 --pmc per-dispatch CSVs (plain or .gz):
  python tools/pmc_bygrid.py file.csv[.gz] ...   (prints one line per kernel/grid)"""
import collections
import csv
import gzip
import io
import sys


def rows(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        yield from csv.DictReader(io.StringIO(f.read()))


agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(dict)
for p in sys.argv[1:]:
    for r in rows(p):
        k = (r["Kernel_Name"].split("(")[0].split("::")[-1], int(r["Grid_Size"]))
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for k in sorted(agg, key=lambda k: -sum(dur[k].values())):
    d = {c: sum(v) / len(v) for c, v in agg[k].items()}
    n = len(dur[k])
    print(f"{k[0]} grid={k[1]} dispatches={n} avg_ms={1e3 * sum(dur[k].values()) / n:.3f}")
    print("   " + " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
