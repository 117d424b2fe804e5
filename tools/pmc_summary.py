#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs per kernel: mean counter value per dispatch."""
import collections
import csv
import hashlib
import os
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "ccsc_code_iccv2017_amd", "csrc")


# the sources the dominant kernel (the register-line z-step) is built from
ZKERNEL_SOURCES = ("zline.hip", "zline.hpp", "fft_fixed.hpp", "slice.hpp", "common.hpp")


def source_hash():
    """sha256 over the dominant kernel's sources: a PMC summary taken from other
    sources is stale (bench.py reports traffic_stale)."""
    h = hashlib.sha256()
    for f in ZKERNEL_SOURCES:
        h.update(f.encode())
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()


def summarize(path, match=("ccsc::",)):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in rows:
        name = r["Kernel_Name"]
        if not any(m in name for m in match):
            continue
        k = name.split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {}
    for k, d in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]["dispatches"] = len(dur[k])
        out[k]["avg_s"] = sum(dur[k].values()) / max(len(dur[k]), 1)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--json":
        # --json OUT N_LOCAL csv...: one merged {kernel: {counter: mean per dispatch}} file
        import json
        out, n_local = args[1], int(args[2])
        merged = {"n_local": n_local, "units": "FETCH_SIZE/WRITE_SIZE in kB per dispatch (raw)",
                  "src_sha256": source_hash()}
        for p in args[3:]:
            for k, d in summarize(p).items():
                m = merged.setdefault(k, {})
                if any(c.startswith("SQ_") for c in d):
                    # the SQ pass's own kernel time (its clock = GRBM_GUI_ACTIVE / 8 / time)
                    d = dict(d)
                    d["sq_avg_s"] = d.pop("avg_s")
                    d.pop("dispatches", None)
                m.update(d)
        json.dump(merged, open(out, "w"), indent=1)
        sys.exit(0)
    for p in args:
        for k, d in summarize(p).items():
            print(p.split("/")[-1], k, {a: f"{b:.4g}" for a, b in d.items()})
