#!/usr/bin/env python3
"""Seconds per outer iteration of every BASELINE.json config on one MI355X.

  python tools/bench_configs.py [--configs C1,C3,C4,C5] [--steps 2]

C1: 2D dParallel, K=100 11x11, n=1000 100x100 patches, 10 blocks.
C3: 2-3D hyperspectral (admm_learn), K=100 11x11x31, n=64 100x100x31 cubes.
C4: 3D, K=49 11x11x11, n=64 64x64x32 clips (ni = 8).
C5: 4D light field, K=49 11x11x5x5, n=64 64x64 5x5-view patches (ni = 8).
(C2, the headline workload, is bench.py.)  Synthetic standard-normal data
(C3: uniform, so max(b) > 0 as gamma_heuristic needs, L23:36); one untimed
warm-up outer iteration, then `steps` timed ones (objective excluded where the
learner allows it; C3 evaluates it every inner iteration, as the reference's
rollback test needs).  One JSON line per config.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ccsc_code_iccv2017_amd import learners as E  # noqa: E402
from ccsc_code_iccv2017_amd import _lib as L  # noqa: E402


def run(name, ctx, variant, b_shape, ks, steps, smooth=False, lam=1.0):
    rng = np.random.default_rng(7)
    b = rng.random(b_shape) if smooth else rng.standard_normal(b_shape)
    p = E.make_problem(variant, b_shape, ks, 1.0, lam, steps + 1, 0.0, "none", seed=11)
    sm = 0.5 * rng.random(b_shape) if smooth else None
    t0 = time.perf_counter()
    s = E.Session(ctx, p, b, smooth_init=sm)
    setup = time.perf_counter() - t0
    s.step(1)
    t0 = time.perf_counter()
    s.step(steps)
    dt = (time.perf_counter() - t0) / steps
    n = b_shape[-1]
    s.close()
    print(json.dumps({"config": name, "s_per_outer_iteration": dt, "patch_iters_per_s": n / dt,
                      "n": n, "setup_s": setup, "steps": steps}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C3,C4,C5")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    want = set(a.configs.split(","))
    with E.Context(0) as ctx:
        if "C1" in want:
            run("C1 2D dParallel K=100 n=1000", ctx, L.CCSC_DPAR, (100, 100, 1000),
                [11, 11, 100], a.steps)
        if "C3" in want:
            run("C3 2-3D hyperspectral K=100 W=31 n=64", ctx, L.CCSC_HS23, (100, 100, 31, 64),
                [11, 11, 31, 100], a.steps, smooth=True)
        if "C4" in want:
            p = (64, 64, 32, 64)
            run("C4 3D K=49 n=64 64x64x32", ctx, L.CCSC_L3D, p, [11, 11, 11, 49], a.steps,
                lam=0.1)
        if "C5" in want:
            run("C5 4D K=49 5x5 views n=64", ctx, L.CCSC_L4D, (64, 64, 5, 5, 64),
                [11, 11, 5, 5, 49], a.steps)


if __name__ == "__main__":
    main()
