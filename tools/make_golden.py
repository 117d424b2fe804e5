#!/usr/bin/env python3
"""Generate tests/golden/ fixtures.

1. Small learner fixtures from the float64 oracle (inputs + expected outputs):
   they pin the oracle against regressions and give the GPU tests fixed inputs.
2. reference_filter_norms.json: per-filter norms of the learned filters the
   reference ships (2D/Filters/*.mat, 3D/Filters/*.mat, 4D/Filters/*.mat), read
   with scipy.io.loadmat (MAT v5, data only).  Only these numbers are committed,
   not the reference's files.  Needs /root/reference (this container only).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import ccsc_oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"


def learner_fixture(name, variant, sb, psf, K, n, ni, max_it, seed):
    rng = np.random.default_rng(seed)
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], n))
    d0 = rng.standard_normal((psf, psf, K))
    z0 = rng.standard_normal((X, Y, K, ni if variant == "dz" else n))
    fn = O.learn_2d_dparallel if variant == "dp" else O.learn_2d_dzparallel
    d, z, DZ, it, tr = fn(b, [psf, psf, K], 1.0, 1.0, max_it, 0.0, "brief", {"d": d0, "z": z0},
                          ni=ni, trace_objective=True)
    meta = {"variant": variant, "kernel_size": [psf, psf, K], "ni": ni, "max_it": max_it,
            "generator": "tools/make_golden.py (oracle/ccsc_oracle.py, float64)"}
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), b=b, d0=d0, z0=z0, d_res=d,
                        trace_obj_d=np.array(tr["obj_d"]), trace_obj_z=np.array(tr["obj_z"]),
                        obj_vals_z=np.array(it["obj_vals_z"]), z_sum=np.array(z.sum()),
                        DZ_sum=np.array(DZ.sum()), meta=np.array(json.dumps(meta)))


def hs_fixture(name, sb, W, psf, K, n, lam, max_it, seed):
    """2-3D learner (L23): inputs, final filters, per-iteration objectives, Dz checksum."""
    rng = np.random.default_rng(seed)
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.random(sb + (W, n))
    sm = 0.5 * rng.random(sb + (W, n))
    d0 = rng.standard_normal((psf, psf, K))
    z0 = rng.standard_normal((X, Y, K, n))
    d, z, Dz, obj, tr = O.learn_hs23(b, [psf, psf, W, K], 1.0, lam, max_it, 0.0, "none",
                                     {"d": d0, "z": z0}, sm)
    meta = {"variant": "hs23", "kernel_size": [psf, psf, W, K], "lambda": lam,
            "max_it": max_it, "generator": "tools/make_golden.py (oracle/ccsc_oracle.py, float64)"}
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), b=b, smooth_init=sm, d0=d0, z0=z0,
                        d_res=d, trace_obj_d=np.array(tr["obj_d"]),
                        trace_obj_z=np.array(tr["obj_z"]), obj=np.array(obj),
                        Dz_sum=np.array(Dz.sum()), meta=np.array(json.dumps(meta)))


def reference_norms():
    from scipy.io import loadmat
    out = {}
    spec = {
        "2D/Filters/Filters_ours_2D_large.mat": (2, 0.01),
        "3D/Filters/3D_video_filters.mat": (3, 0.01),
        "4D/Filters/4d_filters_lightfield.mat": (2, 0.01),
        # the 2-3D learner projects every (wavelength, atom) 11x11 slice (L23:246); its
        # d_res is the d-solve output (L23:126, 231), not the projected split, so it
        # spreads wider around the sphere (0.9954 .. 1.0250)
        "2-3D/Filters/2D-3D-Hyperspectral.mat": (2, 0.03),
    }
    for rel, (nsp, tol) in spec.items():
        path = os.path.join(REF, rel)
        if not os.path.exists(path):
            continue
        d = np.asarray(loadmat(path)["d"], dtype=np.float64)
        norms = np.sqrt((d ** 2).sum(axis=tuple(range(nsp)))).ravel()
        out[rel] = {"shape": list(d.shape), "norms": [round(float(x), 6) for x in norms],
                    "tol": tol}
    return out


def write_reference_norms():
    norms = reference_norms()
    if norms:
        json.dump(norms, open(os.path.join(GOLD, "reference_filter_norms.json"), "w"), indent=0)


def solver_fixture(name):
    """Reconstruction-solver fixture: the oracle (oracle/ccsc_solvers.py) on the seeded
    case of tests/solver_cases.py -> z, res and the per-iterate objective trace."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from solver_cases import solver_case
    z, res, log = solver_case(name)
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), z=z, res=res,
                        obj=np.array(log["obj"]), iters=np.array(log["iters"]),
                        meta=np.array(json.dumps({"generator": "tools/make_golden.py "
                                                  "(oracle/ccsc_solvers.py, float64)"})))


if __name__ == "__main__":
    os.makedirs(GOLD, exist_ok=True)
    for nm in ("solve_inpaint", "solve_poisson", "solve_multich", "solve_video"):
        solver_fixture(nm)
    if "--solvers" in sys.argv:
        sys.exit(0)
    if "--norms" in sys.argv:
        write_reference_norms()
        sys.exit(0)
    learner_fixture("dp_small", "dp", (12, 12), 5, 3, 4, 2, 2, 101)
    learner_fixture("dz_small", "dz", (12, 12), 5, 3, 4, 2, 2, 102)
    learner_fixture("dp_odd", "dp", (11, 10), 5, 3, 6, 3, 2, 103)
    learner_fixture("dz_110", "dz", (100, 100), 11, 2, 2, 1, 1, 104)
    hs_fixture("hs_small", (10, 9), 3, 5, 4, 3, 1.0, 2, 105)
    write_reference_norms()
    print("fixtures:", sorted(os.listdir(GOLD)))
