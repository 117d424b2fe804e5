"""GPU parity: the HIP engine (through the C-ABI) against the float64 oracle.

Tolerances: both sides compute in float64; they differ only in FFT form
(half-spectrum R2C/C2R vs full complex), in the per-frequency inverse
(Cholesky vs the reference's Woodbury/pinv form) and in summation order, so
objectives must agree to 1e-9 relative and filters to 1e-7 (far inside the
north-star gate of 1e-4 relative objective / 0.999 cosine).
"""
import numpy as np
import pytest

from oracle import ccsc_oracle as O

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    return np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300)


@pytest.mark.parametrize("X,Y", [(16, 16), (110, 110), (15, 14), (14, 15), (24, 20), (74, 74),
                                 (26, 37), (60, 60), (62, 41), (38, 34), (58, 46), (110, 106)])
def test_fft2d_r2c_c2r(gpu_ctx, X, Y):
    from ccsc_code_iccv2017_amd.learners import fft2d_test
    rng = np.random.default_rng(X * 1000 + Y)
    a = rng.standard_normal((X, Y, 5))
    hs, rt = fft2d_test(gpu_ctx, a)
    ref = np.fft.fft2(a, axes=(0, 1))[: X // 2 + 1]
    assert np.abs(hs - ref).max() / np.abs(ref).max() < 1e-13
    assert np.abs(rt - a).max() < 1e-12


def _case(variant, sb, psf, K, n, ni, seed):
    rng = np.random.default_rng(seed)
    b = rng.standard_normal((sb[0], sb[1], n))
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    d0 = rng.standard_normal((psf, psf, K))
    if variant == "dz":
        z0 = rng.standard_normal((X, Y, K, ni))
    else:
        z0 = rng.standard_normal((X, Y, K, n))
    return b, d0, z0


@pytest.mark.parametrize("variant", ["dp", "dz"])
@pytest.mark.parametrize("sb,psf,K,n,ni", [((12, 12), 5, 3, 4, 2), ((100, 100), 11, 4, 4, 2),
                                           ((11, 10), 5, 3, 6, 3),
                                           # prime grid lengths (71 x 73: generic passes)
                                           ((61, 63), 11, 3, 4, 2),
                                           # Woodbury D-factor (ni << K): K <= 64, K > 64, ni = 8
                                           ((12, 12), 5, 8, 4, 2), ((12, 12), 5, 70, 4, 2),
                                           ((12, 12), 5, 32, 16, 8),
                                           # Cholesky D-factor, 9 <= K <= 64, ni > K / 4
                                           ((12, 12), 5, 24, 24, 12),
                                           # the headline block shape K = ni = 100 (C1/C2):
                                           # 13 Cholesky panels, RPL = 2 d-solve, 2 blocks
                                           ((12, 12), 5, 100, 200, 100),
                                           # K > 112: the 8-tile (K = 128, two-sweep d-solve)
                                           # and 12-tile (K = 170, RPL = 3) MFMA factor
                                           ((12, 12), 5, 128, 256, 128),
                                           ((12, 12), 5, 170, 170, 170),
                                           # K > 192: the HBM-resident Gram + left-looking
                                           # Cholesky (gramchol_big.hip), d-solve RPL = 4, 5, 7;
                                           # K = 400 = 25 tiles, the largest supported (few
                                           # patches per block keep the oracle in seconds)
                                           ((12, 12), 5, 200, 24, 12),
                                           ((12, 12), 5, 260, 6, 3),
                                           ((12, 12), 5, 400, 4, 2),
                                           # K > 400: the reference's Woodbury form on the
                                           # ni x ni factor (wbig.hip), ni = 2 and 12
                                           ((6, 6), 5, 420, 4, 2),
                                           ((6, 6), 5, 450, 24, 12)])
def test_learn_2d_matches_oracle(gpu_ctx, variant, sb, psf, K, n, ni):
    from ccsc_code_iccv2017_amd import learners as E
    b, d0, z0 = _case(variant, sb, psf, K, n, ni, seed=7)
    ks = [psf, psf, K]
    init = {"d": d0, "z": z0}
    max_it = 2
    if variant == "dp":
        o = O.learn_2d_dparallel(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init, ni=ni,
                                 trace_objective=True)
        e = E.admm_learn_conv2D_large_dParallel(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init,
                                                ni=ni, trace_objective=True, ctx=gpu_ctx)
    else:
        o = O.learn_2d_dzparallel(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init, ni=ni,
                                  trace_objective=True)
        e = E.admm_learn_conv2D_large_dzParallel(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init,
                                                 ni=ni, trace_objective=True, ctx=gpu_ctx)
    d_o, z_o, DZ_o, it_o, tr_o = o
    d_e, z_e, DZ_e, it_e = e
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    np.testing.assert_allclose(it_e["obj_vals_d"], it_o["obj_vals_d"], rtol=1e-9)
    np.testing.assert_allclose(it_e["obj_vals_z"], it_o["obj_vals_z"], rtol=1e-9)
    np.testing.assert_allclose(it_e["trace"]["obj_d"], np.array(tr_o["obj_d"]), rtol=1e-9)
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("variant", ["dp", "dz"])
@pytest.mark.parametrize("sb", [(252, 6), (6, 252), (211, 6)])
def test_learn_2d_generic_prime_grids_match_oracle(gpu_ctx, variant, sb):
    """Padded grids whose lengths need generic prime passes beyond the old planner
    (VERDICT r04 missing item 2, reference crops any size, dP:16): 262 = 2 x 131 in x and
    in y, 221 = 13 x 17 (two generic passes)."""
    from ccsc_code_iccv2017_amd import learners as E
    psf, K, n, ni = 11, 3, 4, 2
    b, d0, z0 = _case(variant, sb, psf, K, n, ni, seed=17)
    ks = [psf, psf, K]
    init = {"d": d0, "z": z0}
    if variant == "dp":
        o = O.learn_2d_dparallel(b, ks, 1.0, 1.0, 2, 0.0, "brief", init, ni=ni,
                                 trace_objective=True)
        e = E.admm_learn_conv2D_large_dParallel(b, ks, 1.0, 1.0, 2, 0.0, "brief", init, ni=ni,
                                                trace_objective=True, ctx=gpu_ctx)
    else:
        o = O.learn_2d_dzparallel(b, ks, 1.0, 1.0, 2, 0.0, "brief", init, ni=ni,
                                  trace_objective=True)
        e = E.admm_learn_conv2D_large_dzParallel(b, ks, 1.0, 1.0, 2, 0.0, "brief", init, ni=ni,
                                                 trace_objective=True, ctx=gpu_ctx)
    d_o, z_o, DZ_o, it_o, tr_o = o
    d_e, z_e, DZ_e, it_e = e
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("variant", ["dp", "dz"])
@pytest.mark.parametrize("sb,verbose,tol", [((150, 150), "brief", 0.0),
                                            ((150, 150), "none", 0.0),
                                            ((150, 150), "brief", 1e-3),
                                            # 262 = 2 x 131 by 160: a generic line pass too
                                            ((252, 150), "brief", 0.0)])
def test_learn_2d_grids_past_lds_match_oracle(gpu_ctx, variant, sb, verbose, tol):
    """Learner grids larger than one CU's LDS (VERDICT r04 missing item 1; the reference
    poses the problem on any sb + 2r grid, dP:16,23-24): 150 x 150 patches (a 160 x 160
    fp64 slice, 205 KB) run on the global line passes of the solvers (recon.hip) with the
    elementwise stages of gslice.hip -- d, z, DZ, the objective trace and the tol path
    against the oracle."""
    from ccsc_code_iccv2017_amd import learners as E
    psf, K, n, ni = 11, 3, 4, 2
    b, d0, z0 = _case(variant, sb, psf, K, n, ni, seed=19)
    ks = [psf, psf, K]
    init = {"d": d0, "z": z0}
    trace = verbose != "none"
    if variant == "dp":
        o = O.learn_2d_dparallel(b, ks, 1.0, 1.0, 2, tol, verbose, init, ni=ni,
                                 trace_objective=trace)
        e = E.admm_learn_conv2D_large_dParallel(b, ks, 1.0, 1.0, 2, tol, verbose, init, ni=ni,
                                                trace_objective=trace, ctx=gpu_ctx)
    else:
        o = O.learn_2d_dzparallel(b, ks, 1.0, 1.0, 2, tol, verbose, init, ni=ni,
                                  trace_objective=trace)
        e = E.admm_learn_conv2D_large_dzParallel(b, ks, 1.0, 1.0, 2, tol, verbose, init, ni=ni,
                                                 trace_objective=trace, ctx=gpu_ctx)
    d_o, z_o, DZ_o, it_o, tr_o = o
    d_e, z_e, DZ_e, it_e = e
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    if trace:
        np.testing.assert_allclose(it_e["obj_vals_z"], it_o["obj_vals_z"], rtol=1e-9)
    if tol > 0:
        np.testing.assert_array_equal(it_e["trace"]["n_z"], np.array(tr_o["n_z"]))
    elif trace:
        np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


def test_learn_4d_tile_dsolve_many_views_matches_oracle(gpu_ctx):
    """The tile d-solve over several right-hand sides (dstep.hip k_dsolve_tile, NV = 4 views,
    K = 72 on the Cholesky factor with inverted diagonal tiles) against the oracle and
    against the two-sweep k_dsolve (CCSC_DS_TILE=0)."""
    import os
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(13)
    sb, UV, psf, K, n = (10, 9), 2, 5, 72, 4
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                   trace_objective=True)
    outs = {}
    for tile in ("1", "0"):
        os.environ["CCSC_DS_TILE"] = tile
        try:
            outs[tile] = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                        trace_objective=True, ctx=gpu_ctx,
                                                        dfactor="cholesky")
        finally:
            del os.environ["CCSC_DS_TILE"]
    for e in outs.values():
        assert _rel(e[0], d_o) < 1e-7
        assert _rel(e[1].real, z_o.real) < 1e-7
        np.testing.assert_allclose(e[4]["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)
    assert _rel(outs["1"][0], outs["0"][0]) < 1e-9


def test_woodbury_staged_matches_per_lane(gpu_ctx):
    """The LDS-staged many-view Woodbury d-solve (k_dsolve_wbs, h in Ch's layout) against the
    per-lane form (CCSC_WB_STAGE=0: k_dsolve_wbv) and the oracle: 4D, 3 x 3 views, K = 24,
    ni = 4 (Woodbury), two blocks."""
    import os
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(31)
    sb, UV, psf, K, n = (10, 9), 3, 5, 24, 16
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                   trace_objective=True)
    outs = {}
    for stage in ("1", "0"):
        os.environ["CCSC_WB_STAGE"] = stage
        try:
            outs[stage] = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                         trace_objective=True, ctx=gpu_ctx,
                                                         dfactor="woodbury")
        finally:
            del os.environ["CCSC_WB_STAGE"]
    for e in outs.values():
        assert _rel(e[0], d_o) < 1e-7
        assert _rel(e[1].real, z_o.real) < 1e-7
        np.testing.assert_allclose(e[4]["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)
    assert _rel(outs["1"][0], outs["0"][0]) < 1e-10


def test_learn_4d_cholesky_many_views_matches_oracle(gpu_ctx):
    """The K x K D-factor with many right-hand sides per frequency (4D, 16 views, K = 20,
    CCSC_DFACTOR_CHOLESKY): K NV = 320 > 256 takes gramchol.hip's eight h slots per thread
    (HP = 8) beside the Gauss Gram (NV <= 16: the MFMA kernel; more views take the VALU
    k_gram_chol); against the oracle's pinv form."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(12)
    sb, UV, psf, K, n = (8, 8), 4, 3, 20, 4
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                   trace_objective=True)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all",
                                                                 init, trace_objective=True,
                                                                 ctx=gpu_ctx, dfactor="cholesky")
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("sb,UV,psf,K,n", [((10, 9), 2, 5, 3, 4), ((9, 9), 3, 5, 2, 9),
                                           ((64, 64), 5, 11, 4, 4),
                                           ((10, 9), 2, 5, 8, 4),      # Woodbury, 4 views
                                           # Woodbury d-solve over the views (dstep.hip
                                           # k_dsolve_wbv): 36 views = whole-wave lanes
                                           # (H = 1), K = 40 = two row segments of 20
                                           ((8, 8), 6, 3, 8, 4), ((8, 8), 6, 3, 40, 4),
                                           ((8, 7), 2, 3, 40, 4)])
def test_learn_4d_matches_oracle(gpu_ctx, sb, UV, psf, K, n):
    """4D light-field learner (L4:1-212): spatial-only convolution over U x V views,
    per-view D-solves sharing one factor, diagonal z-solve (Q7), per-slice projection (Q10)."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(11)
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    d0 = rng.standard_normal((psf, psf, UV, UV, K))
    z0 = rng.standard_normal((X, Y, 1, 1, K, n))
    ks = [psf, psf, UV, UV, K]
    init = {"d": d0, "z": z0}
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                   trace_objective=True)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all",
                                                                 init, trace_objective=True,
                                                                 ctx=gpu_ctx)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    assert np.abs(z_o.imag).max() < 1e-9 * np.abs(z_o.real).max()   # Q8: round-off only
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)
    np.testing.assert_allclose(it_e["trace"]["obj_d"], np.array(tr_o["obj_d"]), rtol=1e-9)
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("variant", ["dp", "dz"])
@pytest.mark.parametrize("K,n,ni,max_it", [(100, 40, 20, 2), (280, 100, 100, 1)])
def test_learn_2d_woodbury_many_patches_matches_oracle(gpu_ctx, variant, K, n, ni, max_it):
    """The Woodbury D-factor past k_gram_wb's ni <= 8 (wbig.hip: A_f and the Cholesky factor
    of rho I + A_f A_f^H, ni x ni up to the reference's ni = 100, dP:11,230-236), forced with
    dfactor='woodbury' on shapes the K x K Cholesky also runs -- against the oracle."""
    from ccsc_code_iccv2017_amd import learners as E
    sb, psf = (12, 12) if K <= 100 else (6, 6), 5
    b, d0, z0 = _case(variant, sb, psf, K, n, ni, seed=37)
    ks = [psf, psf, K]
    init = {"d": d0, "z": z0}
    fo = O.learn_2d_dparallel if variant == "dp" else O.learn_2d_dzparallel
    fe = (E.admm_learn_conv2D_large_dParallel if variant == "dp"
          else E.admm_learn_conv2D_large_dzParallel)
    d_o, z_o, DZ_o, it_o, tr_o = fo(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init, ni=ni,
                                    trace_objective=True)
    d_e, z_e, DZ_e, it_e = fe(b, ks, 1.0, 1.0, max_it, 0.0, "brief", init, ni=ni,
                              trace_objective=True, ctx=gpu_ctx, dfactor="woodbury")
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("dfactor,n", [("auto", 4), ("cholesky", 4), ("cholesky", 36)])
def test_learn_4d_many_filter_views_match_oracle(gpu_ctx, dfactor, n):
    """K = 100 filters over 5 x 5 views (K NV = 2500 right-hand sides per f: VERDICT r05
    missing item 3, the reference takes any K, learn_kernels_4D.m:61): the Woodbury factor
    (ni = 2), and the Cholesky factor with h = A^H b formed by the per-bin GEMM (the MFMA Gram
    with no right-hand sides, then the tile d-solve over the 25 views), ni = 2 and ni = 6."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(31)
    sb, UV, psf, K = (6, 5), 5, 3, 100
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "all", init,
                                                   trace_objective=True)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "all",
                                                                 init, trace_objective=True,
                                                                 ctx=gpu_ctx, dfactor=dfactor)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)
    np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("tol", [0.0, 1e-3])
def test_learn_4d_grid_past_lds_matches_oracle(gpu_ctx, tol):
    """4D learner on a 160 x 160 grid (150 x 150 views + 2r): the global-pass slices of
    gslice.hip with the diagonal z-solve against the view correlations (L4:310-347) and the
    per-view objective / cropped DZ (L4:205-206, 349-369) -- VERDICT r04 missing item 1."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(21)
    sb, UV, psf, K, n = (150, 150), 2, 11, 3, 4
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_4d(b, ks, 1.0, 1.0, 2, tol, "all", init,
                                                   trace_objective=True)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, tol, "all",
                                                                 init, trace_objective=True,
                                                                 ctx=gpu_ctx)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)
    if tol > 0:
        np.testing.assert_array_equal(it_e["trace"]["n_z"], np.array(tr_o["n_z"]))
    else:
        np.testing.assert_allclose(it_e["trace"]["obj_z"], np.array(tr_o["obj_z"]), rtol=1e-9)


@pytest.mark.parametrize("sb,psf,K,n,tol", [((8, 9, 7), 3, 3, 4, 0.0), ((10, 10, 6), 5, 4, 9, 0.0),
                                            ((10, 10, 6), 5, 4, 9, 2e-2),
                                            ((20, 20, 12), 11, 8, 4, 0.0),   # Woodbury
                                            ((64, 64, 32), 11, 2, 1, 0.0)])   # C4 grid 74x74x42
def test_learn_3d_matches_oracle(gpu_ctx, sb, psf, K, n, tol):
    """3D learner (L3:1-230): plane R2C/C2R + t-direction FFT, Sherman-Morrison z-solve,
    psf^3 support projection; odd/even and ragged grid extents."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(21)
    r = psf // 2
    g = tuple(s + 2 * r for s in sb)
    b = rng.standard_normal(sb + (n,))
    init = {"d": rng.standard_normal((psf, psf, psf, K)), "z": rng.standard_normal(g + (K, n))}
    ks = [psf, psf, psf, K]
    lam = 0.1     # lambda_prior 1 zeroes z on the small grids (|z| ~ 1e-17): no signal to compare
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_3d(b, ks, 1.0, lam, 3, tol, "all", init,
                                                   trace_objective=True)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv3D_large(b, ks, 1.0, lam, 3, tol, "all", init,
                                                            trace_objective=True, ctx=gpu_ctx)
    assert d_e.shape == d_o.shape and z_e.shape == z_o.shape and DZ_e.shape == DZ_o.shape
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)
    tr = it_e["trace"]
    np.testing.assert_array_equal(tr["n_d"], np.array(tr_o["n_d"]))
    np.testing.assert_array_equal(tr["n_z"], np.array(tr_o["n_z"]))
    for i, (od, oz) in enumerate(zip(tr_o["obj_d"], tr_o["obj_z"])):
        np.testing.assert_allclose(tr["obj_d"][i, :len(od)], od, rtol=1e-9)
        np.testing.assert_allclose(tr["obj_z"][i, :len(oz)], oz, rtol=1e-9)
    if tol > 0:
        for i, (dd, zd) in enumerate(zip(tr_o["d_diff"], tr_o["z_diff"])):
            np.testing.assert_allclose(tr["d_diff"][i, :len(dd)], dd, rtol=1e-6)
            np.testing.assert_allclose(tr["z_diff"][i, :len(zd)], zd, rtol=1e-6)


@pytest.mark.parametrize("sb,psf,K,n", [((10, 10, 6), 5, 4, 9),
                                        ((20, 20, 12), 11, 8, 4),     # Woodbury
                                        ((64, 64, 32), 11, 2, 1),     # C4 grid 74x74x42
                                        # K T = 8400 > 8 * 1024: no k_tsolve3 plan fits
                                        # (tsolve_tc = 0), the three-kernel z-solve
                                        ((6, 6, 40), 3, 200, 1)])
def test_learn_3d_production_path_matches_oracle(gpu_ctx, sb, psf, K, n):
    """The benchmarked 3D path: verbose 'none' and no objective trace, so the
    z-iterations skip the z store, fuse the next forward plane transform into k_plane_inv
    and reuse its spectra (c_ready); only the last z-iteration stores z.  d, z and DZ
    against the oracle."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(23)
    r = psf // 2
    g = tuple(s + 2 * r for s in sb)
    b = rng.standard_normal(sb + (n,))
    init = {"d": rng.standard_normal((psf, psf, psf, K)), "z": rng.standard_normal(g + (K, n))}
    ks = [psf, psf, psf, K]
    d_o, z_o, DZ_o, _, _, _ = O.learn_3d(b, ks, 1.0, 0.1, 2, 0.0, "none", init)
    d_e, z_e, DZ_e, _, _ = E.admm_learn_conv3D_large(b, ks, 1.0, 0.1, 2, 0.0, "none", init,
                                                      ctx=gpu_ctx)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7


@pytest.mark.parametrize("sb,psf,K,n,tol,verbose", [
    ((120, 120, 32), 11, 2, 1, 0.0, "all"),    # 130^2 planes: past one CU's LDS
    ((64, 64, 242), 11, 2, 1, 0.0, "none"),    # T = 252 = 4 * 63: past the t-tile kernels
    ((150, 150, 4), 3, 2, 4, 5e-2, "all"),     # 152^2 x 6, two blocks, tol breaks (n_z 10, 4)
])
def test_learn_3d_grids_past_lds_match_oracle(gpu_ctx, sb, psf, K, n, tol, verbose):
    """3D clips the LDS plane / t-tile kernels cannot hold (VERDICT r05 missing item 1: the
    reference crops any clip, L3:16,23-26, learn_kernels_3D.m:31-44) run on the global line
    passes (x rows, y lines per plane, t lines; gslice.hip's 3D prologue / epilogue): d, z and
    DZ at 1e-7, the objective trace at 1e-9, the tol path's inner-iteration counts exact."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(29)
    r = psf // 2
    g = tuple(s + 2 * r for s in sb)
    b = rng.standard_normal(sb + (n,))
    init = {"d": rng.standard_normal((psf, psf, psf, K)), "z": rng.standard_normal(g + (K, n))}
    ks = [psf, psf, psf, K]
    trace = verbose != "none"
    d_o, z_o, DZ_o, obj_o, it_o, tr_o = O.learn_3d(b, ks, 1.0, 0.1, 2, tol, verbose, init,
                                                   trace_objective=trace)
    d_e, z_e, DZ_e, obj_e, it_e = E.admm_learn_conv3D_large(b, ks, 1.0, 0.1, 2, tol, verbose, init,
                                                            trace_objective=trace, ctx=gpu_ctx)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7
    assert abs(obj_e - obj_o) <= 1e-9 * abs(obj_o)
    if trace:
        tr = it_e["trace"]
        np.testing.assert_array_equal(tr["n_z"], np.array(tr_o["n_z"]))
        np.testing.assert_array_equal(tr["n_d"], np.array(tr_o["n_d"]))
        for i, oz in enumerate(tr_o["obj_z"]):
            np.testing.assert_allclose(tr["obj_z"][i, :len(oz)], oz, rtol=1e-9)


@pytest.mark.parametrize("sb,UV,psf,K,n", [((10, 9), 2, 5, 3, 4),
                                           ((64, 64), 5, 11, 4, 4),    # C5 grid 74x74, 25 views
                                           ((8, 8), 6, 3, 40, 4)])     # Woodbury over the views
def test_learn_4d_production_path_matches_oracle(gpu_ctx, sb, UV, psf, K, n):
    """The benchmarked 4D path: verbose 'none', no objective trace (z stored only by the
    last z-iteration); d, z and DZ against the oracle."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(24)
    r = psf // 2
    X, Y = sb[0] + 2 * r, sb[1] + 2 * r
    b = rng.standard_normal((sb[0], sb[1], UV, UV, n))
    init = {"d": rng.standard_normal((psf, psf, UV, UV, K)),
            "z": rng.standard_normal((X, Y, 1, 1, K, n))}
    ks = [psf, psf, UV, UV, K]
    d_o, z_o, DZ_o, _, _, _ = O.learn_4d(b, ks, 1.0, 1.0, 2, 0.0, "none", init)
    d_e, z_e, DZ_e, _, _ = E.admm_learn_conv4D_lightfield(b, ks, 1.0, 1.0, 2, 0.0, "none", init,
                                                          ctx=gpu_ctx)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e.real, z_o.real) < 1e-7
    assert _rel(DZ_e, DZ_o) < 1e-7


@pytest.mark.parametrize("verbose", ["brief", "none"])
@pytest.mark.parametrize("variant", ["dp", "dz"])
def test_headline_block_on_110_grid_matches_port(gpu_ctx, variant, verbose):
    """C1/C2's exact block: 100x100 patches (110x110 grid, the compile-time-planned z-step
    kernel), K = ni = 100, 2 consensus blocks; checked against the half-spectrum port
    (pinned to the literal oracle by tests/test_oracle.py) since the literal oracle's
    12,100 pinv's per block take minutes.  Inner counts reduced to keep the CPU side short."""
    from ccsc_code_iccv2017_amd import learners as E
    from oracle.ccsc_port import DzPort
    K, n, ni, mid, miz = 100, 200, 100, 3, 3
    rng = np.random.default_rng(110)
    b = rng.standard_normal((100, 100, n))
    d0 = rng.standard_normal((11, 11, K))
    z0 = rng.standard_normal((110, 110, K, ni if variant == "dz" else n))
    init = {"d": d0, "z": z0}
    if variant == "dz":
        cst = dict(rho_d=5000.0, rho_z=1.0, theta_div=1.0)
        fn = E.admm_learn_conv2D_large_dzParallel
    else:
        cst = dict(rho_d=500.0, rho_z=50.0, theta_div=50.0)
        fn = E.admm_learn_conv2D_large_dParallel
    d_e, z_e, DZ_e, it_e = fn(b, [11, 11, K], 1.0, 1.0, 2, 0.0, verbose, init, ni=ni,
                              max_it_d=mid, max_it_z=miz, ctx=gpu_ctx)
    port = DzPort(b, d0, z0, 1.0, ni=ni, max_it_d=mid, max_it_z=miz,
                  replicate_z0=(variant == "dz"), **cst)
    port.outer()
    port.outer()
    assert _rel(d_e, O.crop_filters(port.D[0], 2, 5)) < 1e-7
    assert _rel(z_e, port.z) < 1e-7
    if verbose != "none":   # 'none': z-iterations run on the state without (z, y) in between
        obj = O.objective_2d(port.z, port.dhat_full(), b, 1.0, 1.0, 5)
        assert abs(it_e["obj_vals_z"][-1] - obj) <= 1e-9 * abs(obj)


@pytest.mark.parametrize("rho_d", [500.0, 5000.0])
def test_dfactor_forms_agree(gpu_ctx, rho_d):
    """CCSC_DFACTOR_WOODBURY and _CHOLESKY (the two D-factor forms, kernels.hpp
    woodbury_ok) give the oracle's iterate on the same input, with large-magnitude codes
    (|Zhat|^2 >> rho_D: the Woodbury solve's cancellation regime)."""
    from ccsc_code_iccv2017_amd import learners as E
    b, d0, z0 = _case("dp", (12, 12), 5, 32, 16, 8, seed=23)
    z0 = 30.0 * z0
    init = {"d": d0, "z": z0}
    o = O.learn_2d_dparallel(b, [5, 5, 32], 1.0, 1.0, 2, 0.0, "brief", init, ni=8, rho_d=rho_d,
                             trace_objective=True)
    outs = {}
    for form in ("woodbury", "cholesky"):
        outs[form] = E.admm_learn_conv2D_large_dParallel(b, [5, 5, 32], 1.0, 1.0, 2, 0.0, "brief",
                                                         init, ni=8, rho_d=rho_d, dfactor=form,
                                                         trace_objective=True, ctx=gpu_ctx)
    for form, e in outs.items():
        assert _rel(e[0], o[0]) < 1e-7, form
        assert _rel(e[1], o[1]) < 1e-7, form
        np.testing.assert_allclose(e[3]["trace"]["obj_z"], np.array(o[4]["obj_z"]), rtol=1e-9)
    assert _rel(outs["woodbury"][0], outs["cholesky"][0]) < 1e-8


@pytest.mark.parametrize("K", [72, 100])
def test_dsolve_tile_matches_two_sweep_and_oracle(gpu_ctx, K, monkeypatch):
    """The tile d-solve (dstep.hip k_dsolve_tile on a factor whose diagonal tiles are
    inverted by k_invert_diag; NV = 1, 64 < K <= 112 -- the C1/C2 block shape) and the
    two-sweep k_dsolve (CCSC_DS_TILE=0) give the oracle's iterate (dP:252-276); K = 72
    leaves a partial last tile (Tn = 5)."""
    from ccsc_code_iccv2017_amd import learners as E
    b, d0, z0 = _case("dz", (12, 12), 5, K, 2 * K, K, seed=41)
    init = {"d": d0, "z": z0}
    o = O.learn_2d_dzparallel(b, [5, 5, K], 1.0, 1.0, 2, 0.0, "brief", init, ni=K,
                              trace_objective=True)
    outs = {}
    for tile in ("1", "0"):
        monkeypatch.setenv("CCSC_DS_TILE", tile)
        outs[tile] = E.admm_learn_conv2D_large_dzParallel(b, [5, 5, K], 1.0, 1.0, 2, 0.0,
                                                          "brief", init, ni=K,
                                                          trace_objective=True, ctx=gpu_ctx)
    for tile, e in outs.items():
        assert _rel(e[0], o[0]) < 1e-7, tile
        assert _rel(e[1], o[1]) < 1e-7, tile
        np.testing.assert_allclose(e[3]["trace"]["obj_z"], np.array(o[4]["obj_z"]), rtol=1e-9)
    assert _rel(outs["1"][0], outs["0"][0]) < 1e-9


def test_dfactor_woodbury_rejected_when_blocks_too_large(gpu_ctx):
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    b, d0, z0 = _case("dz", (12, 12), 5, 8, 24, 12, seed=3)
    with pytest.raises(L.CCSCError) as ei:
        E.admm_learn_conv2D_large_dzParallel(b, [5, 5, 8], 1.0, 1.0, 1, 0.0, "none",
                                             {"d": d0, "z": z0}, ni=12, dfactor="woodbury",
                                             ctx=gpu_ctx)
    assert ei.value.code == L.CCSC_E_UNSUPPORTED


def test_k_above_400_runs_woodbury_and_ni_above_100_is_rejected(gpu_ctx):
    """K > 400 runs on the Woodbury factor (wbig.hip; ni = 1 here) and matches the oracle; a
    block of more than 100 patches past K = 400 is a clean CCSC_E_UNSUPPORTED."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    b, d0, z0 = _case("dz", (6, 6), 3, 401, 2, 1, seed=4)
    init = {"d": d0, "z": z0}
    d_e, z_e, DZ_e, _ = E.admm_learn_conv2D_large_dzParallel(b, [3, 3, 401], 1.0, 1.0, 1, 0.0,
                                                             "none", init, ni=1, ctx=gpu_ctx)
    d_o, z_o, DZ_o, _, _ = O.learn_2d_dzparallel(b, [3, 3, 401], 1.0, 1.0, 1, 0.0, "none", init,
                                                 ni=1)
    assert _rel(d_e, d_o) < 1e-7
    assert _rel(z_e, z_o) < 1e-7
    b2, d2, z2 = _case("dz", (6, 6), 3, 401, 202, 101, seed=4)
    with pytest.raises(L.CCSCError) as ei:
        E.admm_learn_conv2D_large_dzParallel(b2, [3, 3, 401], 1.0, 1.0, 1, 0.0, "none",
                                             {"d": d2, "z": z2}, ni=101, ctx=gpu_ctx)
    assert ei.value.code == L.CCSC_E_UNSUPPORTED


@pytest.mark.parametrize("miz", [1, 2, 4])
def test_zline_state_path_matches_port(gpu_ctx, miz):
    """The register-line z-step's steady state (zline.hip mode 2: state order, bin-slot
    spectra, the corr C2R, k_zhat_split from the state) -- reached only when no objective
    forces (z, y) between z-iterations (verbose 'none'), as in the bench -- against the
    port on C2's 110x110 grid."""
    from ccsc_code_iccv2017_amd import learners as E
    from oracle.ccsc_port import DzPort
    K, n, ni = 4, 4, 2
    rng = np.random.default_rng(55)
    b = rng.standard_normal((100, 100, n))
    d0 = rng.standard_normal((11, 11, K))
    z0 = rng.standard_normal((110, 110, K, ni))
    d_e, z_e, DZ_e, _ = E.admm_learn_conv2D_large_dzParallel(
        b, [11, 11, K], 1.0, 1.0, 2, 0.0, "none", {"d": d0, "z": z0}, ni=ni, max_it_d=2,
        max_it_z=miz, ctx=gpu_ctx)
    port = DzPort(b, d0, z0, 1.0, ni=ni, max_it_d=2, max_it_z=miz)
    port.outer()
    port.outer()
    assert _rel(z_e, port.z) < 1e-7
    assert _rel(d_e, O.crop_filters(port.D[0], 2, 5)) < 1e-7


@pytest.mark.parametrize("verbose", ["none", "brief"])
@pytest.mark.parametrize("variant", ["dz", "dp"])
def test_zline_tol_matches_port(gpu_ctx, variant, verbose):
    """tol > 0 on C2's 110x110 grid (the reference driver runs tol = 1e-3,
    learn_kernels_2D_large.m:24) through the register-line z-step, which keeps z_old in
    the y buffer (no third z-sized buffer): 'none' takes the one-launch-late test with
    the speculative launch rolled back when it fires, 'brief' the objective's
    materialisation.  Inner counts, d/z diffs and the iterate match the port, whose
    tol branches are pinned to the literal oracle (tests/test_oracle.py); the tol is
    picked >= 5% away from every diff, so no break decision sits on round-off."""
    from ccsc_code_iccv2017_amd import learners as E
    from oracle.ccsc_port import DzPort
    from tests.test_oracle import pick_tol
    K, n, ni, mid, miz = 4, 4, 2, 3, 8
    rng = np.random.default_rng(77)
    b = rng.standard_normal((100, 100, n))
    d0 = rng.standard_normal((11, 11, K))
    z0 = rng.standard_normal((110, 110, K, ni if variant == "dz" else n))
    if variant == "dz":
        cst, fn = dict(), E.admm_learn_conv2D_large_dzParallel
    else:
        cst = dict(rho_d=500.0, rho_z=50.0, theta_div=50.0, replicate_z0=False)
        fn = E.admm_learn_conv2D_large_dParallel
    p0 = DzPort(b, d0, z0, 1.0, ni=ni, max_it_d=mid, max_it_z=miz, **cst)
    p0.outer()
    tol = pick_tol(p0.trace["z_diff"][0], p0.trace["d_diff"][0], at=3)
    port = DzPort(b, d0, z0, 1.0, ni=ni, max_it_d=mid, max_it_z=miz, tol=tol, **cst)
    for _ in range(3):
        if not port.finished:
            port.outer()
    assert port.trace["n_z"][0] < miz          # a z break fires in outer iteration 1
    d_e, z_e, DZ_e, it_e = fn(b, [11, 11, K], 1.0, 1.0, 3, tol, verbose, {"d": d0, "z": z0},
                              ni=ni, max_it_d=mid, max_it_z=miz, ctx=gpu_ctx)
    tr = it_e["trace"]
    np.testing.assert_array_equal(tr["n_z"], port.trace["n_z"])
    np.testing.assert_array_equal(tr["n_d"], port.trace["n_d"])
    for i, (dd, zd) in enumerate(zip(port.trace["d_diff"], port.trace["z_diff"])):
        np.testing.assert_allclose(tr["d_diff"][i, :len(dd)], dd, rtol=1e-6)
        np.testing.assert_allclose(tr["z_diff"][i, :len(zd)], zd, rtol=1e-6)
    assert _rel(z_e, port.z) < 1e-7
    assert _rel(d_e, O.crop_filters(port.D[0], 2, 5)) < 1e-7


@pytest.mark.parametrize("variant", ["dZ", "dP"])
def test_zline_two_stream_phase_is_exact(gpu_ctx, monkeypatch, variant):
    """With tol = 0 and >= 512 patches on the 110 grid the engine splits every z-launch of a
    phase over two streams (patches [0, np/2) and the rest, engine.cpp zsplit_ok); the
    per-patch arithmetic is the same kernel's, so the result equals the one-stream run
    bit for bit -- for dZ (the bench workload) and dP (C1's 1000 patches take this path)."""
    from ccsc_code_iccv2017_amd import learners as E
    K, n, ni = 3, 1024, 512
    rng = np.random.default_rng(1024)
    b = rng.standard_normal((100, 100, n))
    d0 = rng.standard_normal((11, 11, K))
    z0 = rng.standard_normal((110, 110, K, ni if variant == "dZ" else n))
    learn = (E.admm_learn_conv2D_large_dzParallel if variant == "dZ"
             else E.admm_learn_conv2D_large_dParallel)
    out = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("CCSC_ZSPLIT2", flag)
        out[flag] = learn(b, [11, 11, K], 1.0, 1.0, 2, 0.0, "none", {"d": d0, "z": z0}, ni=ni,
                          max_it_d=2, max_it_z=3, ctx=gpu_ctx)
    assert np.array_equal(out["1"][0], out["0"][0])
    assert np.array_equal(out["1"][1], out["0"][1])
