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


def shard(N, rank, world):
    """Contiguous block split (same rule as ccsc_shard in the engine)."""
    base, rem = divmod(N, world)
    nb = base + (1 if rank < rem else 0)
    return rank * base + min(rank, rem), nb


class DzPort:
    """State of the dzParallel learner with tol = 0 (fixed inner counts).

    ``replicate_z0=False`` restates dParallel's iteration instead (dP:89-190:
    z0 is the full size_z, not one block replicated; pass dP's constants
    rho_d=500, rho_z=50, theta_div=50, max_it_d=10).  The z-step's filter
    spectrum is block 1's d-solve output D1^ in both (dP:143 takes fft2(D{1})
    = D1^ up to round-off, since D{1} = real(ifft2(D1^)) of a Hermitian D1^).

    Multi-rank restatement: with ``world > 1`` this instance
    owns the contiguous blocks ``shard(N, rank, world)`` (``b`` is then the
    rank-local patches) and the two exchanges of the engine are injected:
    ``allreduce(x)`` sums the support-restricted sum_j (D_j + y_j) over ranks
    (KernelConstraintProj reads only the support, dP:208-209) and
    ``bcast(x)`` ships rank 0's block-1 filter spectrum to every rank
    (the z-step uses block 1's D, dP:143).
    """

    def __init__(self, b, d0, z0, lambda_prior, *, ni, rho_d=5000.0, rho_z=1.0, theta_div=1.0,
                 max_it_d=5, max_it_z=10, workers=None, N=None, rank=0, world=1,
                 allreduce=None, bcast=None, replicate_z0=True, tol=0.0):
        self.w = workers if workers is not None else (os.cpu_count() or 1)
        b = np.asarray(b, dtype=np.float64)
        psf = d0.shape[0]
        self.r = r = psf // 2
        self.K = K = d0.shape[-1]
        self.n = n = b.shape[-1]
        self.ni = ni
        self.Nloc = n // ni
        self.N = N if N is not None else self.Nloc          # global block count
        self.rank, self.world = rank, world
        self.allreduce = allreduce or (lambda x: x)
        self.bcast = bcast or (lambda x: x)
        self.X, self.Y = b.shape[0] + 2 * r, b.shape[1] + 2 * r
        self.rho_d, self.rho_z = rho_d, rho_z
        self.theta = lambda_prior / theta_div
        self.mid, self.miz = max_it_d, max_it_z
        B = np.pad(b, ((r, r), (r, r), (0, 0)))
        self.Bh = _r2c(B, self.w)                                   # [Xh, Y, n]
        d = embed_filters(np.asarray(d0, float), [self.X, self.Y], 2, r)
        self.D = [d.copy() for _ in range(self.Nloc)]
        self.yD = [np.zeros_like(d) for _ in range(self.Nloc)]
        self.u = np.zeros_like(d)                                    # Pi(Dbar + Udbar), Q2
        z0 = np.asarray(z0, float)
        self.z = np.concatenate([z0] * self.Nloc, axis=3) if replicate_z0 else z0.copy()  # dZ:44-47 / dP:45
        self.yz = np.zeros_like(self.z)
        self.dhat = None
        # tol > 0 (single rank): the d / z break tests dZ:125-132, 163-169 (dP:125-132,
        # 156-167) and the outer termination dZ:186-188; per outer iteration the
        # relative changes and the inner counts
        self.tol = tol
        self.trace = {"d_diff": [], "z_diff": [], "n_d": [], "n_z": []}
        self.finished = False

    def dhat_full(self):
        """Block 1's filter spectrum on the full X x Y grid (the objective's dup{1})."""
        return np.fft.fft2(_c2r(self.dhat, self.X, self.Y, self.w), axes=(0, 1))

    def outer(self):
        X, Y, K, ni, w = self.X, self.Y, self.K, self.ni, self.w
        # precompute (dZ:96-100): S_f = (A^H A + rho I)^-1, h_f = A^H b_f
        Zh = _r2c(self.z, w)                                        # [Xh, Y, K, n]
        S, h = [], []
        for nn in range(self.Nloc):
            A = Zh[..., nn * ni:(nn + 1) * ni].reshape(-1, K, ni).transpose(0, 2, 1)   # [F, ni, K]
            AH = np.conj(A.transpose(0, 2, 1))
            G = AH @ A
            G[:, range(K), range(K)] += self.rho_d
            S.append(np.linalg.inv(G))
            bb = self.Bh[..., nn * ni:(nn + 1) * ni].reshape(-1, ni)
            h.append(np.einsum("fkp,fp->fk", AH, bb))
        # D iterations (dZ:104-135)
        r, s = self.r, 2 * self.r + 1
        sup = (np.r_[X - r:X, 0:r + 1][:, None], np.r_[Y - r:Y, 0:r + 1][None, :])
        dh_loc = None
        dds, zds = [], []
        for _ in range(self.mid):
            d_old = self.D[0]
            u = self.u
            for nn in range(self.Nloc):
                self.yD[nn] = self.yD[nn] + (self.D[nn] - u)
                C = _r2c(u - self.yD[nn], w).reshape(-1, K)
                x = np.einsum("fkj,fj->fk", S[nn], h[nn] + self.rho_d * C)
                xh = x.reshape(X // 2 + 1, Y, K)
                if nn == 0:
                    dh_loc = xh
                self.D[nn] = _c2r(xh, X, Y, w)
            # consensus (dP:114-121, 106): only the support of Dbar + Udbar is read
            loc = sum((Dj + yj)[sup[0], sup[1]] for Dj, yj in zip(self.D, self.yD))
            tot = self.allreduce(np.ascontiguousarray(loc))
            full = np.zeros_like(u)
            full[sup[0], sup[1]] = tot / self.N
            self.u = kernel_constraint_proj(full, r, 2)
            dds.append(np.linalg.norm(self.D[0] - d_old) / np.linalg.norm(self.D[0]))
            if self.tol > 0 and dds[-1] < self.tol:
                break
        self.dhat = self.bcast(np.ascontiguousarray(dh_loc))         # block 1 lives on rank 0
        # Z iterations (dZ:147-172) with the simplified Sherman-Morrison solve
        dh = self.dhat                                              # [Xh, Y, K]
        s = np.sum(np.abs(dh) ** 2, axis=2)
        for _ in range(self.miz):
            z_old = self.z
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
            zds.append(np.linalg.norm(self.z - z_old) / np.linalg.norm(self.z))
            if self.tol > 0 and zds[-1] < self.tol:
                break
        for key, v in (("d_diff", dds), ("z_diff", zds), ("n_d", len(dds)), ("n_z", len(zds))):
            self.trace[key].append(v)
        if self.tol > 0 and zds[-1] < self.tol and dds[-1] < self.tol:
            self.finished = True
        return self
