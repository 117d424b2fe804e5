"""Known-answer tests of the reconstruction-solver oracle (oracle/ccsc_solvers.py) and the
host-side checks of ccsc_solve (CPU only).

The reference ships no fixtures for these solvers (parity unpinned), so the
restatement is pinned analytically: psf2otf is centred circular convolution, the
Sherman-Morrison z-solve solves the per-frequency normal equations, the Poisson prox is
the stationary point of its objective, the diagonal solve is b / (rho + s).  The golden
fixtures (tests/golden/solve_*.npz, tools/make_golden.py) freeze the oracle's outputs."""
import os

import numpy as np
import pytest

from oracle import ccsc_solvers as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def test_psf2otf_is_centred_circular_convolution():
    rng = np.random.default_rng(1)
    k = rng.standard_normal((5, 3))
    x = rng.standard_normal((12, 9))
    y = np.real(np.fft.ifft2(S.psf2otf(k, x.shape) * np.fft.fft2(x)))
    ref = np.zeros_like(x)
    for i in range(12):
        for j in range(9):
            for a in range(5):
                for b in range(3):
                    ref[i, j] += k[a, b] * x[(i - (a - 2)) % 12, (j - (b - 1)) % 9]
    np.testing.assert_allclose(y, ref, atol=1e-12)


def test_psf2otf_drops_roundoff_imaginary_part():
    d = np.zeros((11, 11))
    d[5, 5] = 1
    otf = S.psf2otf(d, (30, 40))
    assert np.all(otf.imag == 0) and np.allclose(otf.real, 1)
    t = S.psf2otf(np.array([[1.0, -1.0]]), (6, 8))
    np.testing.assert_allclose(np.abs(t) ** 2,
                               np.tile(2 - 2 * np.cos(2 * np.pi * np.arange(8) / 8), (6, 1)),
                               atol=1e-12)


def test_sm_solve_is_the_normal_equations():
    rng = np.random.default_rng(2)
    X, Y, K = 6, 5, 4
    dhat = np.fft.fft2(rng.standard_normal((X, Y, K)), axes=(0, 1))
    xi1 = np.fft.fft2(rng.standard_normal((X, Y)))
    xi2 = np.fft.fft2(rng.standard_normal((X, Y, K)), axes=(0, 1))
    gam = [0.3, 2.1]
    rho = gam[1] / gam[0]
    zh = S.solve_conv_term_sm(dhat.reshape(X * Y, K, order="F"), xi1, xi2, gam, (X, Y, K))
    for i in range(X):
        for j in range(Y):
            d = dhat[i, j]
            A = np.outer(np.conj(d), d) + rho * np.eye(K)
            rhs = np.conj(d) * xi1[i, j] + rho * xi2[i, j]
            np.testing.assert_allclose(zh[i, j], np.linalg.solve(A, rhs), rtol=1e-10, atol=1e-12)


def test_poisson_solve_equals_sm_where_tg_vanishes():
    rng = np.random.default_rng(3)
    X, Y, K = 6, 6, 3
    dhat = np.fft.fft2(rng.standard_normal((X, Y, K)), axes=(0, 1))
    xi1 = np.fft.fft2(rng.standard_normal((X, Y)))
    xi2 = np.fft.fft2(rng.standard_normal((X, Y, K)), axes=(0, 1))
    gam = [1.0, 5.0]
    flat = dhat.reshape(X * Y, K, order="F")
    a = S.solve_conv_term_poisson(flat, xi1, xi2, gam, (X, Y, K))
    b = S.solve_conv_term_sm(flat, xi1, xi2, gam, (X, Y, K))
    np.testing.assert_allclose(a[0, 0], b[0, 0], rtol=1e-12)      # TG(0, 0) = 0
    assert not np.allclose(a[1, 2], b[1, 2])                      # the smoothness weight acts


def test_poisson_prox_stationarity():
    rng = np.random.default_rng(4)
    u = rng.standard_normal(50) * 3
    I = rng.uniform(0.1, 2, 50)
    th = 0.7
    x = S.prox_poisson(u, th, np.ones(50), I)
    # x minimises th * (x - I log x) + (x - u)^2 / 2
    np.testing.assert_allclose(th * (1 - I / x) + (x - u), 0, atol=1e-10)
    m = np.zeros(50)
    np.testing.assert_array_equal(S.prox_poisson(u, th, m, I), u)


def test_diag_solve_formula():
    rng = np.random.default_rng(5)
    dhat = rng.standard_normal((4, 3, 2, 5)) + 1j * rng.standard_normal((4, 3, 2, 5))
    x1 = rng.standard_normal((4, 3, 2)) + 1j * rng.standard_normal((4, 3, 2))
    x2 = rng.standard_normal((4, 3, 5)) + 1j * rng.standard_normal((4, 3, 5))
    rho = 2.0
    s = np.sum(np.abs(dhat) ** 2, axis=(2, 3))[..., None]
    b = np.einsum("xywk,xyw->xyk", np.conj(dhat), x1) + rho * x2
    np.testing.assert_allclose(S.solve_conv_term_diag(dhat, x1, x2, rho), b / (rho + s), rtol=1e-12)


@pytest.mark.parametrize("name", ["solve_inpaint", "solve_poisson", "solve_multich", "solve_video"])
def test_oracle_reproduces_golden(name):
    from solver_cases import solver_case
    g = np.load(os.path.join(GOLD, f"{name}.npz"))
    z, res, log = solver_case(name)
    np.testing.assert_allclose(z, g["z"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(res, g["res"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(np.asarray(log["obj"]), g["obj"], rtol=1e-10)
    assert int(log["iters"]) == int(g["iters"])


def _abi():
    from ccsc_code_iccv2017_amd import _lib as L
    return L


def _problem(L, variant, sb, K=4, k=5, nch=1, n=1, psf=(3, 3, 3)):
    p = L.SolveProblem()
    p.variant = variant
    for i in range(3):
        p.sb[i] = sb[i] if i < len(sb) else 1
        p.ksize[i] = k
        p.psf_size[i] = psf[i]
    p.nch, p.n, p.K = nch, n, K
    p.lambda_residual, p.lambda_prior, p.max_it, p.tol = 5.0, 2.0, 10, 1e-3
    return p


@pytest.mark.parametrize("variant,sb,ok", [
    (0, (256, 256), True),          # the inpainting test images (266 x 266 grid)
    (1, (512, 384), True),          # the Poisson dataset (522 x 394 = 2 * 197: generic radix)
    (2, (100, 100, 31), True),
    (3, (64, 64, 32), True),
    (0, (30020, 10), False),        # 30030 = 2*3*5*7*11*13: no 4-pass plan within the budgets
])
def test_solve_supported(variant, sb, ok):
    L = _abi()
    p = _problem(L, variant, sb, k=11, nch=sb[2] if variant == 2 else 1)
    eb = L.errbuf()
    rc = L.lib().ccsc_solve_supported(p, eb, len(eb))
    assert (rc == 0) == ok, eb.value


def test_solve_rejects_bad_problems():
    L = _abi()
    eb = L.errbuf()
    p = _problem(L, 2, (20, 20, 3), nch=0)
    assert L.lib().ccsc_solve_supported(p, eb, len(eb)) == L.CCSC_E_INVALID
    p = _problem(L, 0, (20, 20))
    p.lambda_prior = 0
    assert L.lib().ccsc_solve_supported(p, eb, len(eb)) == L.CCSC_E_INVALID
    p = _problem(L, 7, (20, 20))
    assert L.lib().ccsc_solve_supported(p, eb, len(eb)) == L.CCSC_E_INVALID
