#!/usr/bin/env python3
"""Benchmark of the reconstruction solvers (ccsc_solve) at the reference's sizes.

One JSON line per solver: ADMM iterations per second of one image (tol = 0 so the
iteration count is fixed; setup and output formation excluded: the device time of the
iteration loop from the solver's own HIP events), the whole-iteration HBM roofline, and
the float64 NumPy oracle (oracle/ccsc_solvers.py) timed on the host for a bounded
number of iterations as the CPU baseline.

Workloads (synthetic data of the reference's shapes, seeded; random unit-norm filters
of the shipped filter banks' shapes):
  inpaint   2D/Inpainting: 256 x 256 test images, 100 filters 11 x 11 (Filters_ours_2D_large)
  poisson   2D/Poisson_deconv: 512 x 384 images, 100 filters + dirac
  demosaic  2-3D/Demosaicing: 100 x 100 x 31 cube, filters [11, 11, 31, 100]
  lightfield 4D/ViewSynthesis: 5 x 5 views of 128 x 128 as 25 channels, filters [11, 11, 25, 49]
  video     3D/Deblurring: 64 x 64 x 32 clip, 49 filters 11^3 + dirac, 3 x 3 blur psf

Algorithmic bytes per iteration (each pass reads and writes its operands once):
codes  Kc * (4 * 8 P  [z, d2 read + write]  + 4 passes * 2 * 16 F)
data   W  * (2 * 8 P  [d1] + 2 * 8 P [M, Mb] + 8 P [smooth] + 4 passes * 2 * 16 F)
with P grid voxels and F half-spectrum bins per slice.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0


def unit(k):
    return k / np.sqrt(np.sum(k ** 2, axis=tuple(range(k.ndim - 1)), keepdims=True))


def workload(name, rng):
    if name == "inpaint":
        x = rng.uniform(size=(256, 256))
        mask = (rng.uniform(size=x.shape) < 0.5).astype(float)
        return dict(variant=0, b=x * mask, mask=mask, smooth_init=x * 0.9, x_orig=x,
                    kernels=unit(rng.standard_normal((11, 11, 100))), lam=(5.0, 2.0), grid=(266, 266, 1),
                    Kc=100, W=1)
    if name == "poisson":
        x = rng.uniform(0.05, 1, size=(512, 384))
        return dict(variant=1, b=rng.poisson(x * 1000) / 1000.0, mask=np.ones(x.shape), x_orig=x,
                    kernels=unit(rng.standard_normal((11, 11, 100))), lam=(20000.0, 1.0),
                    grid=(522, 394, 1), Kc=101, W=1)
    if name == "demosaic":
        x = rng.uniform(size=(100, 100, 31))
        mask = (rng.uniform(size=x.shape) < 1 / 31).astype(float)
        return dict(variant=2, b=x * mask, mask=mask, smooth_init=x * 0.9,
                    kernels=unit(rng.standard_normal((11, 11, 31, 100))), lam=(100000.0, 1.0),
                    grid=(100, 100, 1), Kc=100, W=31)
    if name == "lightfield":
        x = rng.standard_normal((128, 128, 25))
        mask = np.zeros(x.shape)
        mask[:, :, ::2] = 1
        return dict(variant=2, b=x * mask, mask=mask, smooth_init=x * 0.5,
                    kernels=unit(rng.standard_normal((11, 11, 25, 49))), lam=(10000.0, 1.0),
                    grid=(128, 128, 1), Kc=49, W=25)
    if name == "video":
        x = rng.standard_normal((64, 64, 32))
        psf = np.zeros((3, 3, 3))
        psf[:, :, 1] = 1 / 9
        return dict(variant=3, b=x, mask=np.ones(x.shape), smooth_init=x * 0.5, psf=psf,
                    kernels=unit(rng.standard_normal((11, 11, 11, 49))), lam=(10000.0, 0.125),
                    grid=(74, 74, 42), Kc=50, W=1)
    raise KeyError(name)


def alg_bytes(w):
    X, Y, T = w["grid"]
    P = X * Y * T
    F = (X // 2 + 1) * Y * T
    return w["Kc"] * (4 * 8 * P + 8 * 16 * F) + w["W"] * (5 * 8 * P + 8 * 16 * F)


def cpu_iters_per_s(w, iters):
    from solver_cases import run_oracle
    names = {0: "solve_inpaint", 1: "solve_poisson", 2: "solve_multich", 3: "solve_video"}
    inp = dict(b=w["b"], kernels=w["kernels"], mask=w["mask"], smooth_init=w.get("smooth_init"),
               psf=w.get("psf"), x_orig=w.get("x_orig"), lambda_residual=w["lam"][0],
               lambda_prior=w["lam"][1], max_it=iters, tol=0.0)
    t0 = time.perf_counter()
    run_oracle(names[w["variant"]], inp, verbose="none")
    t1 = time.perf_counter()
    inp["max_it"] = 0
    run_oracle(names[w["variant"]], inp, verbose="none")
    t2 = time.perf_counter()
    return iters / max((t1 - t0) - (t2 - t1), 1e-9), t1 - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solvers", default="inpaint,poisson,demosaic,lightfield,video")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--cpu-iters", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    from ccsc_code_iccv2017_amd import solvers as SV
    from ccsc_code_iccv2017_amd.learners import Context
    ctx = Context(0)
    rng = np.random.default_rng(2017)
    for name in args.solvers.split(","):
        w = workload(name, rng)
        run = lambda it: SV.solve(w["variant"], w["b"], w["kernels"], w["mask"], w["lam"][0],  # noqa: E731
                                  w["lam"][1], it, 0.0, "none", smooth_init=w.get("smooth_init"),
                                  psf=w.get("psf"), x_orig=w.get("x_orig"), ctx=ctx)
        run(2)   # warm-up (code objects, allocator)
        z, res, log = run(args.iters)
        assert np.all(np.isfinite(res)), "non-finite reconstruction"
        sec = log["seconds"]
        B = alg_bytes(w)
        gbs = B * args.iters / sec / 1e9
        line = {"solver": name, "metric": "ADMM iterations/s (one image)",
                "value": args.iters / sec, "unit": "iters/s", "ms_per_iter": sec * 1e3 / args.iters,
                "iters": args.iters, "dtype": "f64", "data": "synthetic",
                "config": {"grid": w["grid"], "codes": w["Kc"], "channels": w["W"],
                           "image": list(w["b"].shape)},
                "roofline": {"bound": "hbm", "scope": "whole iteration (all kernels)",
                             "alg_bytes_per_iter": B, "achieved": gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS}}
        if not args.no_cpu_baseline:
            v, t = cpu_iters_per_s(w, args.cpu_iters)
            line["cpu_baseline"] = {"value": v, "unit": "iters/s", "cores": os.cpu_count(),
                                    "kind": "port", "sample": f"{args.cpu_iters} iterations of "
                                    f"oracle/ccsc_solvers.py (NumPy float64), {t:.1f} s"}
            line["speedup_vs_cpu"] = line["value"] / v
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
