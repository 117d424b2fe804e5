#!/usr/bin/env python3
"""Seconds per outer iteration of the non-headline BASELINE.json configs on one MI355X
(the same leg bench.py runs after the C2 line; definitions in bench.CONFIGS).

  python tools/bench_configs.py [--configs C1,C3,C4,C5] [--steps 1]

One untimed warm-up outer iteration, then `steps` timed ones.  One JSON line per config.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ccsc_code_iccv2017_amd import learners as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C3,C4,C5")
    ap.add_argument("--steps", type=int, default=1)
    a = ap.parse_args()
    want = set(a.configs.split(","))
    with E.Context(0) as ctx:
        for key, label, variant, shape, ks, lam, kind in bench.CONFIGS:
            if key in want:
                r = bench.run_config(ctx, key, label, variant, shape, ks, lam, kind, a.steps)
                print(json.dumps({"config": key, **r}), flush=True)


if __name__ == "__main__":
    main()
