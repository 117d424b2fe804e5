"""CPU baseline "port": vectorised float64 NumPy/SciPy restatement of the 2D
dzParallel learner (2D/admm_learn_conv2D_large_dzParallel.m:90-194).

TEST / BASELINE INFRASTRUCTURE ONLY -- imported by tests/ and by bench.py's
``cpu_baseline`` leg, never by the product path.

The literal oracle (``ccsc_oracle.py``) restates the reference formulas
one-to-one (full spectra, pinv per frequency) and is far too slow to time at
the benchmark size (12,100 pinv's of 100x100 per block).  This port computes
the same iteration with the algebra a competent CPU implementation would use:
half-spectrum real FFTs (scipy.fft, all cores), one batched LAPACK inverse of
A^H A + rho I per frequency, and the closed-form Sherman-Morrison z-solve.
tests/test_oracle.py pins it to the literal oracle.
"""
from __future__ import annotations

import os

import numpy as np
import scipy.fft as sfft

from .ccsc_oracle import embed_filters, kernel_constraint_proj


def _r2c(a, workers):
    # real transform along MATLAB dim 1 (x), complex along dim 2 (y)
    return sfft.rfftn(a, axes=(1, 0), workers=workers)


def _c2r(a, X, Y, workers):
    return sfft.irfftn(a, s=(Y, X), axes=(1, 0), workers=workers)


class DzPort:
    """State of the dzParallel learner with tol = 0 (fixed inner counts)."""

    def __init__(self, b, d0, z0, lambda_prior, *, ni, rho_d=5000.0, rho_z=1.0, theta_div=1.0,
                 max_it_d=5, max_it_z=10, workers=None):
        self.w = workers if workers is not None else (os.cpu_count() or 1)
        b = np.asarray(b, dtype=np.float64)
        psf = d0.shape[0]
        self.r = r = psf // 2
        self.K = K = d0.shape[-1]
        self.n = n = b.shape[-1]
        self.ni = ni
        self.N = n // ni
        self.X, self.Y = b.shape[0] + 2 * r, b.shape[1] + 2 * r
        self.rho_d, self.rho_z = rho_d, rho_z
        self.theta = lambda_prior / theta_div
        self.mid, self.miz = max_it_d, max_it_z
        B = np.pad(b, ((r, r), (r, r), (0, 0)))
        self.Bh = _r2c(B, self.w)                                   # [Xh, Y, n]
        d = embed_filters(np.asarray(d0, float), [self.X, self.Y], 2, r)
        self.D = [d.copy() for _ in range(self.N)]
        self.yD = [np.zeros_like(d) for _ in range(self.N)]
        self.Dbar = np.zeros_like(d)
        self.Udbar = np.zeros_like(d)
        z0 = np.asarray(z0, float)
        self.z = np.concatenate([z0] * self.N, axis=3)             # dZ:44-47
        self.yz = np.zeros_like(self.z)
        self.dhat = None

    def outer(self):
        X, Y, K, ni, w = self.X, self.Y, self.K, self.ni, self.w
        # precompute (dZ:96-100): S_f = (A^H A + rho I)^-1, h_f = A^H b_f
        Zh = _r2c(self.z, w)                                        # [Xh, Y, K, n]
        S, h = [], []
        for nn in range(self.N):
            A = Zh[..., nn * ni:(nn + 1) * ni].reshape(-1, K, ni).transpose(0, 2, 1)   # [F, ni, K]
            AH = np.conj(A.transpose(0, 2, 1))
            G = AH @ A
            G[:, range(K), range(K)] += self.rho_d
            S.append(np.linalg.inv(G))
            bb = self.Bh[..., nn * ni:(nn + 1) * ni].reshape(-1, ni)
            h.append(np.einsum("fkp,fp->fk", AH, bb))
        # D iterations (dZ:104-135)
        for _ in range(self.mid):
            u = kernel_constraint_proj(self.Dbar + self.Udbar, self.r, 2)
            for nn in range(self.N):
                self.yD[nn] = self.yD[nn] + (self.D[nn] - u)
                C = _r2c(u - self.yD[nn], w).reshape(-1, K)
                x = np.einsum("fkj,fj->fk", S[nn], h[nn] + self.rho_d * C)
                xh = x.reshape(X // 2 + 1, Y, K)
                if nn == 0:
                    self.dhat = xh
                self.D[nn] = _c2r(xh, X, Y, w)
            self.Dbar = sum(self.D) / self.N
            self.Udbar = sum(self.yD) / self.N
        # Z iterations (dZ:147-172) with the simplified Sherman-Morrison solve
        dh = self.dhat                                              # [Xh, Y, K]
        s = np.sum(np.abs(dh) ** 2, axis=2)
        for _ in range(self.miz):
            a = self.z + self.yz
            aa = np.abs(a)
            with np.errstate(divide="ignore", invalid="ignore"):
                u = np.where(aa > self.theta, 1.0 - self.theta / aa, 0.0) * a
            self.yz = self.yz + (self.z - u)
            c = u - self.yz
            Ch = _r2c(c, w)                                         # [Xh, Y, K, n]
            rr = np.einsum("xyk,xykn->xyn", dh, Ch)
            wv = (self.Bh - rr) / (self.rho_z + s)[..., None]
            Zh = Ch + np.conj(dh)[..., None] * wv[:, :, None, :]
            self.z = _c2r(Zh, X, Y, w)
        return self
