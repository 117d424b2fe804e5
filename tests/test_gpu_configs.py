"""GPU: the configurations C3, C4 and C5 of BASELINE.json on their real grids.

* Oracle parity on C4's and C5's grids with the D-factor form the engine picks for
  their block shape: ni << K selects the Woodbury factor (kernels.hpp woodbury_fits;
  ccsc_resolve reports it), the reference's own pinv(rho I + A A^H) form (dP:230-236,
  L3:258-273, L4:243-263).  K = 49 filters as in learn_kernels_3D.m:71 /
  learn_kernels_4D.m:61; n = 4 (ni = 2, two consensus blocks) keeps the float64
  oracle to seconds.
* Full-size runs (n = 64 as SURVEY.md §8(d) proposes) on seeded synthetic data of
  the reference's kind (synth.clips_3d / lightfields_4d / cubes_23), for the
  reference drivers' 20 outer iterations (learn_kernels_3D.m:85, learn_kernels_4D.m:77;
  the 2-3D driver's 40, learn_hyperspectral.m:22, halved): the iteration-0 objective
  matches its closed-form expectation over the random init (z0 ~ randn drawn on the
  device, d0 given), the objective is finite and decreases, and the learned filters
  sit on the unit sphere like the reference's shipped ones (tests/golden/
  reference_filter_norms.json: 3D 0.9991 .. 1.0014, 4D 1.0000 +- 2e-5 per (u, v, k)
  slice, 2-3D 0.995 .. 1.025).
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import ccsc_oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    return np.linalg.norm((np.asarray(a) - np.asarray(b)).ravel()) / np.linalg.norm(np.asarray(b).ravel())


def _ref_norms(key):
    return json.load(open(os.path.join(GOLD, "reference_filter_norms.json")))[key]


def test_c4_grid_woodbury_matches_oracle(gpu_ctx):
    """L3 on C4's 74x74x42 grid (64x64x32 clips, 11^3 filters), K = 49, n = 4: two blocks
    of ni = 2 -> the Woodbury D-factor, against the oracle's pinv form."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    sb, psf, K, n = (64, 64, 32), 11, 49, 4
    ks = [psf] * 3 + [K]
    p = E.resolve(E.make_problem(L.CCSC_L3D, sb + (n,), ks, 1.0, 0.1, 2, 0.0, "all"))
    assert p.ni == 2 and p.dfactor == L.DFACTOR["woodbury"]
    rng = np.random.default_rng(74)
    g = tuple(s + 2 * (psf // 2) for s in sb)
    b = rng.standard_normal(sb + (n,))
    init = {"d": rng.standard_normal((psf,) * 3 + (K,)), "z": rng.standard_normal(g + (K, n))}
    kw = dict(max_it_d=2, max_it_z=1)
    d_o, z_o, DZ_o, obj_o, _, _ = O.learn_3d(b, ks, 1.0, 0.1, 2, 0.0, "all", init,
                                            factored=True, **kw)
    d_e, z_e, DZ_e, obj_e, _ = E.admm_learn_conv3D_large(b, ks, 1.0, 0.1, 2, 0.0, "all", init,
                                                        ctx=gpu_ctx, **kw)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)


def test_c5_grid_woodbury_matches_oracle(gpu_ctx):
    """L4 on C5's grid (64x64 patches, 5x5 views, 11x11 filters -> 74x74 planes),
    K = 49, n = 4: the Woodbury D-factor shared by the 25 views, against the oracle."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    sb, UV, psf, K, n = (64, 64), 5, 11, 49, 4
    ks = [psf, psf, UV, UV, K]
    p = E.resolve(E.make_problem(L.CCSC_L4D, sb + (UV, UV, n), ks, 1.0, 1.0, 2, 0.0, "all"))
    assert p.ni == 2 and p.dfactor == L.DFACTOR["woodbury"]
    rng = np.random.default_rng(75)
    r = psf // 2
    b = rng.standard_normal(sb + (UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((sb[0] + 2 * r, sb[1] + 2 * r, 1, 1, K, n))}
    kw = dict(max_it_d=3, max_it_z=2)
    d_o, z_o, DZ_o, obj_o, _, _ = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init, **kw)
    d_e, z_e, DZ_e, obj_e, _ = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all",
                                                             init, ctx=gpu_ctx, **kw)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)


def _run_session(ctx, p, b, d0, outer, smooth_init=None):
    """Objective of the random init, then after every outer iteration (outside the
    learner's own timing); the cropped filters at the end."""
    from ccsc_code_iccv2017_amd import learners as E
    s = E.Session(ctx, p, b, d0=d0, smooth_init=smooth_init)
    try:
        objs = [s.objective()]
        for _ in range(outer):
            done = s.step(1)
            objs.append(s.objective())
            if done:
                break
        d_res = s.results(want_z=False, want_DZ=False)[0]
    finally:
        s.close()
    return np.array(objs), d_res


def _check_objective(objs, expect0, what, strict=True, rtol0=2e-3):
    """rtol0 ~ 5 standard deviations of the iteration-0 objective over the random init
    (Monte Carlo on the host with the same d0: C5's 17M code entries through 25 views
    of one fixed filter set spread 1.1e-3; C2/C3/C4 draw 10^8 - 10^9 entries)."""
    print(f"{what}: objective {objs[0]:.6e} (closed form {expect0:.6e}) -> {objs[-1]:.6e} "
          f"after {len(objs) - 1} outer iterations")
    assert np.all(np.isfinite(objs))
    assert abs(objs[0] / expect0 - 1) < rtol0, (objs[0], expect0)
    assert objs[1] < objs[0], objs
    assert objs[-1] < objs[1] if strict else objs[-1] <= objs[1], objs


def test_c4_fullsize_20_iterations(gpu_ctx):
    """C4: 3D learner, K = 49 11^3 filters, n = 64 synthetic 64x64x32 local-CN clips
    (ni = 8 -> 8 blocks, Woodbury D-factor), lambda = 1 (learn_kernels_3D.m:72-73)."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    sb, psf, K, n = (64, 64, 32), 11, 49, 64
    b = synth.clips_3d(n, sb, K=K, psf=psf, device="cuda:0")
    p = E.make_problem(L.CCSC_L3D, b.shape, [psf] * 3 + [K], 1.0, 1.0, 20, 0.0, "none", seed=43)
    assert E.resolve(p).dfactor == L.DFACTOR["woodbury"]
    d0 = np.random.default_rng(44).standard_normal((psf,) * 3 + (K,))
    objs, d_res = _run_session(gpu_ctx, p, b, d0, 20)
    P = np.prod([s + 2 * (psf // 2) for s in sb])
    expect0 = 0.5 * (n * np.prod(sb) * float((d0 ** 2).sum()) + float((b ** 2).sum())) \
        + math.sqrt(2 / math.pi) * n * K * P
    _check_objective(objs, expect0, "C4")
    norms = np.sqrt((d_res ** 2).sum(axis=(0, 1, 2)))
    ref = np.array(_ref_norms("3D/Filters/3D_video_filters.mat")["norms"])
    print(f"C4 filter norms {norms.min():.6f} .. {norms.max():.6f} "
          f"(reference 3D {ref.min():.6f} .. {ref.max():.6f})")
    # d_res is block 1's local d-solve output D{1} (L3:141, 226-227), which leaves the
    # sphere its projected consensus u lies on outward by the ADMM primal residual, a
    # drift that grows over the outer iterations and with the block's data weight
    # (test_c4_reduced_norm_offset_matches_oracle pins the same drift on the oracle at
    # 1/9 the size: +0.016% after 20 iterations); at full C4 it measures +0.35 .. +0.40%
    assert np.all(norms > 1.0) and np.all(norms < 1.006), (norms.min(), norms.max())


def test_c5_fullsize_20_iterations(gpu_ctx):
    """C5: 4D light-field learner, K = 49 11x11 filters over 5x5 views, n = 64 synthetic
    local-CN light fields of 64x64 (ni = 8, Woodbury), lambda = 1 (learn_kernels_4D.m:62-63)."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    sb, UV, psf, K, n = (64, 64), 5, 11, 49, 64
    b = synth.lightfields_4d(n, sb, views=UV, K=K, psf=psf, device="cuda:0")
    p = E.make_problem(L.CCSC_L4D, b.shape, [psf, psf, UV, UV, K], 1.0, 1.0, 20, 0.0, "none",
                       seed=45)
    assert E.resolve(p).dfactor == L.DFACTOR["woodbury"]
    d0 = np.random.default_rng(46).standard_normal((psf, psf, UV, UV, K))
    objs, d_res = _run_session(gpu_ctx, p, b, d0, 20)
    X = sb[0] + 2 * (psf // 2)
    expect0 = 0.5 * (n * sb[0] * sb[1] * float((d0 ** 2).sum()) + float((b ** 2).sum())) \
        + math.sqrt(2 / math.pi) * n * K * X * X
    _check_objective(objs, expect0, "C5", rtol0=6e-3)
    norms = np.sqrt((d_res ** 2).sum(axis=(0, 1)))              # per (u, v, k) slice (L4:224-225)
    ref = np.array(_ref_norms("4D/Filters/4d_filters_lightfield.mat")["norms"])
    print(f"C5 filter norms {norms.min():.6f} .. {norms.max():.6f} "
          f"(reference 4D {ref.min():.6f} .. {ref.max():.6f})")
    assert np.all(np.abs(norms - 1) < 1e-2)


def test_c3_fullsize_20_iterations(gpu_ctx):
    """C3: 2-3D hyperspectral learner, K = 100 11x11 filters over W = 31 wavelengths,
    n = 64 synthetic 100x100x31 cubes with the 13x13 Gaussian smooth_init
    (learn_hyperspectral.m:2-16), lambda = 1; the rollback test (L23:204-213) may stop
    it early, so the objective never increases."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    sb, W, psf, K, n = (100, 100), 31, 11, 100, 64
    b, sm = synth.cubes_23(n, sb, W=W, K=K, psf=psf, device="cuda:0")
    p = E.make_problem(L.CCSC_HS23, b.shape, [psf, psf, W, K], 1.0, 1.0, 20, 0.0, "none",
                       seed=47)
    d0 = np.random.default_rng(48).standard_normal((psf, psf, K))
    objs, d_res = _run_session(gpu_ctx, p, b, d0, 20, smooth_init=sm)
    X = sb[0] + 2 * (psf // 2)
    expect0 = 0.5 * (W * n * sb[0] * sb[1] * float((d0 ** 2).sum()) + float(((sm - b) ** 2).sum())) \
        + W * math.sqrt(2 / math.pi) * n * K * X * X
    _check_objective(objs, expect0, "C3", strict=False)
    assert np.all(np.diff(objs) <= 1e-12 * np.abs(objs[:-1])), objs
    norms = np.sqrt((d_res ** 2).sum(axis=(0, 1)))              # per (w, k) slice (L23:246)
    ref = np.array(_ref_norms("2-3D/Filters/2D-3D-Hyperspectral.mat")["norms"])
    print(f"C3 filter norms {norms.min():.6f} .. {norms.max():.6f} "
          f"(reference 2-3D {ref.min():.6f} .. {ref.max():.6f})")
    # d_res is the d-solve output d (L23:126, 231), not a projection: on this data the
    # constraint split (rho = gamma_D ratio 5000, L23:93) holds it on the sphere to 1e-6
    # (round 3: 1.000000 .. 1.000000); test_c3_reduced_norms_match_oracle shows the same
    # quantity leaving the sphere (0.87 .. 1.001) where the data term dominates
    assert np.all(np.abs(norms - 1) < 1e-4), (norms.min(), norms.max())


@pytest.mark.parametrize("fixture", ["c4_reduced_norms.json", "c4_third_norms.json"])
def test_c4_reduced_norm_offset_matches_oracle(gpu_ctx, fixture):
    """The norm offset of C4's d_res is the algorithm's own: on C4-shaped problems (K = 49
    11^3 filters, n = 16 synthetic clips -> ni = 4, Woodbury) of 24x24x12 (1/19 of a C4 clip's
    volume) and 44x44x22 (1/3), 20 outer iterations, the engine reproduces the float64
    oracle's per-filter norms of d_res = crop(D{1}) (the 1/3 case exactly at 8 iterations and as a
    band at 20, see pin_note; tests/golden/c4_*_norms.json,
    tools/norm_offset.py: 1.000000 .. 1.000162 and 1.000001 .. 1.000036, the projected
    consensus u at exactly 1; profiles/r04/norm_offset_c4.txt, profiles/r06/norm_offset_c4_third.txt)."""
    from ccsc_code_iccv2017_amd import learners as E
    from ccsc_code_iccv2017_amd import synth
    g = json.load(open(os.path.join(GOLD, fixture)))
    sb, K, n, psf, iters = tuple(g["sb"]), g["K"], g["n"], g["psf"], g["iters"]
    b = synth.clips_3d(n, sb, K=K, psf=psf, device="cpu")
    r = psf // 2
    sp = [s + 2 * r for s in sb]

    def run(it):
        rng = np.random.default_rng(44)
        init = {"d": rng.standard_normal((psf,) * 3 + (K,)), "z": rng.standard_normal(sp + [K, n])}
        d_e, *_ = E.admm_learn_conv3D_large(b, [psf] * 3 + [K], 1.0, 1.0, it, 0.0, "none", init,
                                           ctx=gpu_ctx)
        return np.sqrt((d_e ** 2).sum(axis=(0, 1, 2)))

    norms = run(iters)
    print(f"C4-shaped engine norms {norms.min():.6f} .. {norms.max():.6f}")
    if "pin_iters" in g:
        # the 1/3-volume problem amplifies rounding-level differences ~10^2-10^3x per outer
        # iteration past iteration 8 (g["pin_note"], profiles/r06/c4_third_divergence.txt):
        # pinned where both are still exact, the 20-iteration norms compared as a band
        np.testing.assert_allclose(run(g["pin_iters"]), np.array(g["pin_norms"]), rtol=1e-10)
        np.testing.assert_allclose(norms, np.array(g["d_res_norms"]), rtol=0, atol=1e-4)
    else:
        np.testing.assert_allclose(norms, np.array(g["d_res_norms"]), rtol=1e-8)
    assert norms.max() > 1.0 + 1e-5   # the outward drift, not round-off


def test_c3_reduced_norms_match_oracle(gpu_ctx):
    """C3's d_res is the d-solve output: on a C3-shaped problem (K = 100, W = 31, 40x40
    uniform-noise cubes, n = 4) whose data term dominates, the oracle's d leaves the
    sphere (0.868 .. 1.001 after the rollback at outer iteration 8,
    tests/golden/c3_reduced_norms.json) and the engine reproduces it."""
    from ccsc_code_iccv2017_amd import learners as E
    g = json.load(open(os.path.join(GOLD, "c3_reduced_norms.json")))
    sb, W, K, n, psf, iters = tuple(g["sb"]), g["W"], g["K"], g["n"], g["psf"], g["iters"]
    rng = np.random.default_rng(5)
    b = rng.random(sb + (W, n))
    sm = 0.5 * rng.random(sb + (W, n))
    r = psf // 2
    init = {"d": rng.standard_normal((psf, psf, K)),
            "z": rng.standard_normal((sb[0] + 2 * r, sb[1] + 2 * r, K, n))}
    d_e, _, _, _, log = E.admm_learn(b, [psf, psf, W, K], 1.0, 1.0, iters, 0.0, "none", init, sm,
                                     ctx=gpu_ctx, return_log=True)
    assert log["outer"] == g["outer"] and log["rolled_back"] == g["rolled_back"]
    norms = np.sqrt((d_e ** 2).sum(axis=(0, 1)))
    mn, mx, me = g["d_res_norms_min_max_mean"]
    print(f"C3-shaped engine norms {norms.min():.6f} .. {norms.max():.6f} (mean {norms.mean():.6f})")
    np.testing.assert_allclose([norms.min(), norms.max(), norms.mean()], [mn, mx, me], rtol=1e-8)
