#!/usr/bin/env python3
"""Where the learned filters' norms sit after 20 outer iterations, on the float64 oracle
(CPU, reduced sizes of the C4 and C3 shapes) -- the pin for tests/test_gpu_configs.py's
unit-sphere bounds (VERDICT r03 "what's weak" 1).

C4 (L3): d_res is block 1's local d-solve output D{1} (L3:141,226-227), NOT the projected
consensus u = Pi(mean D + mean y) (L3:118): its norms sit off the sphere by the ADMM primal
residual D{1} - u.  Printed per outer iteration: the norm range of crop(D{1}) and of crop(u).
C3 (L23): d_res is the d-solve output d = real(ifft2(d_hat)) (L23:126,231), whose splitting
partner v2 = d is projected every inner iteration (L23:113).

  python tools/norm_offset.py [--c4] [--c3]  > profiles/r04/norm_offset.txt
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ccsc_oracle as O  # noqa: E402
from ccsc_code_iccv2017_amd import synth  # noqa: E402


def rng_norms(a, axes):
    n = np.sqrt((a ** 2).sum(axis=axes))
    return n.min(), n.max(), n.mean()


def c4(n=16, sb=(24, 24, 12), K=49, psf=11, iters=20):
    b = synth.clips_3d(n, sb, K=K, psf=psf, device="cpu")
    r = psf // 2
    sp = [s + 2 * r for s in sb]
    rng = np.random.default_rng(44)
    init = {"d": rng.standard_normal((psf,) * 3 + (K,)),
            "z": rng.standard_normal(sp + [K, n])}
    t0 = time.time()
    d_res, *_, tr = O.learn_3d(b, [psf] * 3 + [K], 1.0, 1.0, iters, 0.0, "none", init)
    print(f"C4-shaped oracle run: sb {sb}, K {K}, n {n} (ni {int(np.sqrt(n))}), {iters} outer "
          f"iterations, {time.time() - t0:.0f} s")
    for i, (D1, U) in enumerate(zip(tr["D1"], tr["U"])):
        a = rng_norms(O.crop_filters(D1, 3, r), (0, 1, 2))
        u = rng_norms(O.crop_filters(U, 3, r), (0, 1, 2))
        print(f"  outer {i + 1:2d}: |crop D1| {a[0]:.6f} .. {a[1]:.6f} (mean {a[2]:.6f})   "
              f"|crop u| {u[0]:.6f} .. {u[1]:.6f}")
    fin = rng_norms(d_res, (0, 1, 2))
    print(f"  d_res norms after {iters}: {fin[0]:.6f} .. {fin[1]:.6f} (mean {fin[2]:.6f})")
    return {"case": "C4-shaped", "sb": list(sb), "K": K, "n": n, "psf": psf, "iters": iters,
            "b": "synth.clips_3d(n, sb, K=K, psf=psf, device='cpu')",
            "init": "numpy default_rng(44): d ~ randn(psf^3, K), then z ~ randn(sp + [K, n])",
            "d_res_norms": np.sqrt((d_res ** 2).sum(axis=(0, 1, 2))).tolist(),
            "d1_norms_per_outer": [np.sqrt((O.crop_filters(D1, 3, r) ** 2).sum(axis=(0, 1, 2))).tolist()
                                   for D1 in tr["D1"]],
            "u_norms_last": np.sqrt((O.crop_filters(tr["U"][-1], 3, r) ** 2).sum(axis=(0, 1, 2))).tolist()}


def c3(n=4, sb=(40, 40), W=31, K=100, psf=11, iters=20):
    rng = np.random.default_rng(5)
    b = rng.random(sb + (W, n))
    sm = 0.5 * rng.random(sb + (W, n))
    r = psf // 2
    init = {"d": rng.standard_normal((psf, psf, K)),
            "z": rng.standard_normal((sb[0] + 2 * r, sb[1] + 2 * r, K, n))}
    t0 = time.time()
    d_res, z, Dz, obj, tr = O.learn_hs23(b, [psf, psf, W, K], 1.0, 1.0, iters, 0.0, "none",
                                         init, sm)
    nr = rng_norms(d_res, (0, 1))
    print(f"C3-shaped oracle run: sb {sb}, W {W}, K {K}, n {n}, {tr['outer']} outer iterations "
          f"(rolled back: {tr['rolled_back']}), {time.time() - t0:.0f} s")
    print(f"  d_res per (w, k) norms: {nr[0]:.6f} .. {nr[1]:.6f} (mean {nr[2]:.6f})")
    return {"case": "C3-shaped", "sb": list(sb), "W": W, "K": K, "n": n, "psf": psf,
            "iters": iters, "outer": tr["outer"], "rolled_back": tr["rolled_back"],
            "b": "numpy default_rng(5): b ~ U[0,1) sb+(W,n), smooth_init ~ 0.5 U[0,1)",
            "init": "same rng: d ~ randn(psf, psf, K), z ~ randn(X, Y, K, n)",
            "d_res_norms_min_max_mean": list(map(float, nr))}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--c3", action="store_true")
    ap.add_argument("--json", help="write the results (a test fixture) here")
    ap.add_argument("--sb", help="C4 clip size, e.g. 44,44,22 (default 24,24,12)")
    ap.add_argument("--n", type=int, default=16, help="C4 clips (a perfect square)")
    ap.add_argument("--iters", type=int, default=20, help="C4 outer iterations")
    a = ap.parse_args()
    res = []
    if a.c4 or not a.c3:
        sb = tuple(int(x) for x in a.sb.split(",")) if a.sb else (24, 24, 12)
        res.append(c4(n=a.n, sb=sb, iters=a.iters))
    if a.c3 or not a.c4:
        res.append(c3())
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res if len(res) > 1 else res[0], f, indent=1)
