#!/usr/bin/env python3
"""One line per ccsc kernel of a rocprofv3 --stats kernel_stats.csv: calls, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tag = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if "ccsc::" in r["Name"]:
        name = r["Name"].split("(")[0].replace("void ", "")
        print(f"{tag:8s} {name[:48]:48s} n={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:10.1f} us")
