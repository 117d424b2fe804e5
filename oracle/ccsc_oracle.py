"""CPU oracle: float64 NumPy restatement of the CCSC consensus-ADMM learners.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``libccsc.so`` via
``ccsc_code_iccv2017_amd``) never calls into it.

PARITY STATUS: *parity unpinned by the reference*.  The reference is MATLAB
(R2016b) and neither MATLAB nor Octave exists in this container or on the GPU
box; the reference ships no tests, fixtures or golden vectors for this path
(SURVEY.md §4, §8c).  This restatement is therefore pinned by analytic
known-answer tests (tests/test_oracle.py: per-frequency normal equations,
Sherman-Morrison == dense solve, half == full spectrum, FFT objective == direct
convolution objective, projection idempotence, one-block consensus == plain
ADMM) and by the one external invariant the reference ships (its learned
filters sit on the unit sphere).

Every function follows the reference *literally* (full-spectrum FFTs, the
Woodbury/pinv form of the per-frequency inverse, column-major reshapes), so
that the HIP engine -- which uses half-spectrum R2C/C2R FFTs, Cholesky
factors and the algebraically simplified z-solve -- is checked against the
reference's own formulation rather than against itself.

Array conventions: NumPy arrays carry the MATLAB shapes ([X, Y, K, n] etc.)
and MATLAB axis meaning; ``np.reshape(..., order='F')`` restates MATLAB
``reshape``.  Short names used in citations (paths relative to the reference):

  dP  = 2D/admm_learn_conv2D_large_dParallel.m
  dZ  = 2D/admm_learn_conv2D_large_dzParallel.m
  L3  = 3D/admm_learn_conv3D_large.m
  L4  = 4D/admm_learn_conv4D_lightfield.m
  L23 = 2-3D/DictionaryLearning/admm_learn.m

Deviations (all documented in DESIGN.md):
  * ``init`` is honoured (the reference ignores it, Q11) so runs are
    reproducible: ``init = {'d': kernel_size array, 'z': size_z array}``.
  * dZ's objective subtracts every block of ``b`` (the reference subtracts the
    last block only and crashes for N > 1, Q5).
  * ``verbose='none'`` does not crash (the reference reads an undefined
    variable, Q6); objectives are then NaN in ``iterations``.
  * 4D ``z`` is kept complex exactly as the reference (Q8).
"""

from __future__ import annotations

import math
import numpy as np

__all__ = [
    "kernel_constraint_proj",
    "precompute_H_hat_D",
    "precompute_H_hat_Z",
    "solve_conv_term_D",
    "solve_conv_term_Z",
    "prox_sparse",
    "objective_2d",
    "learn_2d_dparallel",
    "learn_2d_dzparallel",
    "learn_3d",
    "learn_4d",
    "learn_hs23",
    "solve_conv_term_D_hs",
    "solve_conv_term_Z_hs",
    "objective_hs",
    "prox_data_masked",
    "pad_symmetric_2d",
    "embed_filters",
    "crop_filters",
]


def _F(a, shape):
    """MATLAB reshape (column-major)."""
    return np.reshape(a, shape, order="F")


def prox_sparse(u, theta):
    """ProxSparse = @(u, theta) max(0, 1 - theta./abs(u)) .* u   (dP:32)."""
    a = np.abs(u)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = np.maximum(0.0, 1.0 - theta / a)
    s = np.where(a == 0, 0.0, s)
    return s * u


# ----------------------------------------------------------------------------
# Kernel constraint projection.  dP:201-219 (2D), L3:232-256 (3D per filter),
# L4:214-241 (4D per (u, v, k) spatial slice).
# ----------------------------------------------------------------------------
def kernel_constraint_proj(u, psf_radius, ndim_spatial):
    """Project onto {support (2r+1)^d around the origin, ||d_k|| <= 1}.

    u: [X, Y, (T | U, V), K] real.  ``ndim_spatial`` = number of leading dims
    that are circularly shifted (2 for 2D and 4D, 3 for 3D).  The norm is taken
    over the spatial support of every trailing index (per filter in 2D/3D, per
    (u, v, k) slice in 4D, L4:224-225).
    """
    r = psf_radius
    s = 2 * r + 1
    shift = [r] * ndim_spatial + [0] * (u.ndim - ndim_spatial)
    up = np.roll(u, shift, axis=tuple(range(u.ndim)))            # circshift(u, +r)
    sl = tuple([slice(0, s)] * ndim_spatial)
    up = up[sl].copy()                                            # crop 1:2r+1
    nrm = np.sum(up ** 2, axis=tuple(range(ndim_spatial)), keepdims=True)
    mask = np.broadcast_to(nrm >= 1, up.shape)
    den = np.broadcast_to(np.sqrt(nrm), up.shape)
    up[mask] = up[mask] / den[mask]
    pad = [(0, u.shape[i] - s) for i in range(ndim_spatial)] + [(0, 0)] * (u.ndim - ndim_spatial)
    up = np.pad(up, pad)                                          # padarray post
    return np.roll(up, [-x for x in shift], axis=tuple(range(u.ndim)))  # circshift -r


def embed_filters(d_small, size_spatial, ndim_spatial, psf_radius):
    """d = circshift(padarray(d0, size_x - ksize, 0, 'post'), -r)   (dP:38-39)."""
    pad = [(0, size_spatial[i] - d_small.shape[i]) for i in range(ndim_spatial)]
    pad += [(0, 0)] * (d_small.ndim - ndim_spatial)
    d = np.pad(d_small, pad)
    shift = [-psf_radius] * ndim_spatial + [0] * (d_small.ndim - ndim_spatial)
    return np.roll(d, shift, axis=tuple(range(d.ndim)))


def crop_filters(D, ndim_spatial, psf_radius):
    """d_res = circshift(D, +r); d_res(1:2r+1, ...)   (dP:195-196)."""
    shift = [psf_radius] * ndim_spatial + [0] * (D.ndim - ndim_spatial)
    d = np.roll(D, shift, axis=tuple(range(D.ndim)))
    s = 2 * psf_radius + 1
    return d[tuple([slice(0, s)] * ndim_spatial)].copy()


# ----------------------------------------------------------------------------
# Per-frequency solves (literal restatements).
# ----------------------------------------------------------------------------
def precompute_H_hat_D(z_hat_block, ss, k, ni, rho, rep_views=1, factored=False):
    """dP:221-237.  Returns (zhat_mat [ss, ni, k], zhat_inv_mat [ss, k, k]).

    zhat_mat{f} = permute(reshape(z_hat, [ss, k, ni]), [3,2,1]) -> ni x k.
    zhat_inv_mat{f} = 1/rho*eye(k) - 1/rho*A'*pinv(rho*eye(ni) + A*A')*A.
    ``rep_views`` > 1 restates L4:252 (repmat over the 5x5 views: the same
    matrix repeated once per view, frequency index = spatial + ss_sp*view).
    ``factored``: zhat_inv_mat is kept as the reference's own factors (rho, pinv(rho I
    + A A')) and applied right to left in solve_conv_term_D -- the same formula without
    the ss x k x k array (8.8 GB on C4's 74x74x42 grid at K = 49).
    """
    zh = _F(z_hat_block, (ss, k, ni))
    A = np.transpose(zh, (0, 2, 1))                     # [ss, ni, k]
    AH = np.conj(np.transpose(A, (0, 2, 1)))            # [ss, k, ni]
    M = rho * np.eye(ni)[None] + A @ AH                 # [ss, ni, ni]
    P = np.linalg.pinv(M)
    if factored:
        assert rep_views == 1
        return A, ("pinv", rho, P)
    inv = (np.eye(k)[None] - AH @ P @ A) / rho          # [ss, k, k]
    if rep_views > 1:
        A = np.concatenate([A] * rep_views, axis=0)
        inv = np.concatenate([inv] * rep_views, axis=0)
    return A, inv


def solve_conv_term_D(zhat_mat, zhat_inv_mat, d_rhs_hat, B_block_hat, rho, spatial_shape, k, ni):
    """dP:252-276: x_f = Sinv_f * (A_f' * b_f + rho * c_f)."""
    ss = zhat_mat.shape[0]
    xi1 = _F(B_block_hat, (ss, ni))                     # b_f = row f
    xi2 = _F(d_rhs_hat, (ss, k))
    AH = np.conj(np.transpose(zhat_mat, (0, 2, 1)))
    rhs = np.einsum("fkp,fp->fk", AH, xi1) + rho * xi2
    if isinstance(zhat_inv_mat, tuple):                 # factored: (I - A' P A) rhs / rho
        _, rho_f, P = zhat_inv_mat
        t = np.einsum("fpk,fk->fp", zhat_mat, rhs)
        t = np.einsum("fpq,fq->fp", P, t)
        x = (rhs - np.einsum("fkp,fp->fk", AH, t)) / rho_f
    else:
        x = np.einsum("fkj,fj->fk", zhat_inv_mat, rhs)
    return _F(x, tuple(spatial_shape) + (k,))


def precompute_H_hat_Z(dhat, ss):
    """dP:239-250: dhat_flat = reshape(dhat, ss, []); dhatTdhat = sum |dhat|^2."""
    dflat = _F(dhat, (ss, -1))
    return dflat, np.sum(np.conj(dflat) * dflat, axis=1)


def solve_conv_term_Z(dhat_flat, dhatTdhat, z_rhs_hat, B_hat, rho, size_z):
    """dP:278-303 (Sherman-Morrison rank-1 solve per frequency and patch).

    b = conj(dhat) .* B + rho .* zhat_rhs ;
    z_hat = 1/rho*b - 1/rho * 1/(rho + dhatTdhat) .* conj(dhat) .* sum(dhat .* b, k)
    """
    ni = size_z[-1]
    k = size_z[-2]
    ss = int(np.prod(size_z[:-2]))
    dT = np.conj(dhat_flat.T)[:, :, None]               # [k, ss, 1]
    Bf = _F(B_hat, (ss, 1, ni)).transpose(1, 0, 2)      # [1, ss, ni]
    zf = _F(z_rhs_hat, (ss, k, ni)).transpose(1, 0, 2)  # [k, ss, ni]
    b = dT * Bf + rho * zf
    sc = 1.0 / (rho + dhatTdhat)[None, :, None]
    zh = b / rho - (1.0 / rho) * sc * dT * np.sum(np.conj(dT) * b, axis=0, keepdims=True)
    return _F(zh.transpose(1, 0, 2), size_z)


def objective_2d(z, dhat, b, lambda_residual, lambda_prior, psf_radius):
    """dP:305-324 with d given by its spectrum (dZ:310-331 passes dup{1}).

    Dz = real(ifft2(sum(fft2(z) .* dhat, 3))); crop; 1/2||Dz - b||^2 + lambda*|z|_1.
    z: [X, Y, K, n]; dhat: [X, Y, K]; b: [x, y, n].
    """
    r = psf_radius
    zh = np.fft.fft2(z, axes=(0, 1))
    Dz = np.real(np.fft.ifft2(np.sum(zh * dhat[:, :, :, None], axis=2), axes=(0, 1)))
    Dz = Dz[r:Dz.shape[0] - r, r:Dz.shape[1] - r, :]
    f_z = lambda_residual * 0.5 * np.sum((Dz - b) ** 2)
    g_z = lambda_prior * np.sum(np.abs(z))
    return float(f_z + g_z)


def _rel(diff, ref):
    nr = np.linalg.norm(ref.ravel())
    return np.linalg.norm(diff.ravel()) / nr if nr > 0 else np.inf


def _want_obj(verbose, which):
    return verbose in which


def _new_trace():
    return {"obj_d": [], "obj_z": [], "d_diff": [], "z_diff": [], "D1": [], "n_d": [], "n_z": [],
            "U": []}


# ----------------------------------------------------------------------------
# 2D dParallel   (dP:1-199)
# ----------------------------------------------------------------------------
def learn_2d_dparallel(b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                       verbose, init, *, ni=100, max_it_d=10, max_it_z=10,
                       rho_d=500.0, rho_z=50.0, theta_div=50.0, trace_objective=False):
    """Restatement of admm_learn_conv2D_large_dParallel (dP:1-199).

    Returns (d_res, z_res, DZ, iterations, trace).  ``trace`` holds the
    objective after every inner iteration when ``trace_objective`` is set
    (used by the parity tests; the reference only prints these for 'brief').
    """
    b = np.asarray(b, dtype=np.float64)
    psf_s = kernel_size[0]
    k = kernel_size[-1]
    sb = b.shape
    n = sb[-1]
    N = n // ni                                                   # dP:12 (Q13)
    r = psf_s // 2                                                # dP:15
    size_x = [sb[0] + 2 * r, sb[1] + 2 * r, n]                    # dP:16
    size_z = [size_x[0], size_x[1], k, n]                         # dP:17
    size_z_crop = [size_x[0], size_x[1], k, ni]
    size_d_full = [size_x[0], size_x[1], k]
    ss = size_x[0] * size_x[1]

    B = np.pad(b, ((r, r), (r, r), (0, 0)))                       # dP:23
    B_hat = np.fft.fft2(B, axes=(0, 1))                           # dP:24
    Bh = [B_hat[:, :, nn * ni:(nn + 1) * ni] for nn in range(N)]  # dP:26-28

    d0 = np.asarray(init["d"], dtype=np.float64)
    d = embed_filters(d0, size_x[:2], 2, r)                       # dP:38-39
    dup = [np.fft.fft2(d, axes=(0, 1)) for _ in range(N)]         # dP:41-42
    D = [d.copy() for _ in range(N)]                              # dP:43
    z = np.array(init["z"], dtype=np.float64).reshape(size_z, order="F")  # dP:45
    z_hat = np.fft.fft2(z, axes=(0, 1))                           # dP:46

    objective = lambda z_, d_: objective_2d(z_, np.fft.fft2(d_, axes=(0, 1)), b,
                                            lambda_residual, lambda_prior, r)
    trace = _new_trace()
    obj_val = objective(z, d) if (verbose in ("brief", "all") or trace_objective) else float("nan")
    obj_val_filter = obj_val_z = obj_val
    iterations = {"obj_vals_d": [obj_val_filter], "obj_vals_z": [obj_val_z], "tim_vals": [0.0]}
    trace["obj0"] = obj_val

    Dbar = np.zeros(size_d_full)
    Udbar = np.zeros(size_d_full)
    d_D = [np.zeros(size_d_full) for _ in range(N)]               # dP:82
    d_Z = np.zeros(size_z)                                        # dP:85
    d_diff = z_diff = None
    for i in range(max_it):                                       # dP:89
        zm, zi = [], []
        for nn in range(N):                                       # dP:95-99
            zup = z_hat[:, :, :, nn * ni:(nn + 1) * ni]
            A, S = precompute_H_hat_D(zup, ss, k, ni, rho_d)
            zm.append(A)
            zi.append(S)
        od, zd = [], []
        for i_d in range(max_it_d):                               # dP:103
            d_old = D[0]
            u_D2 = kernel_constraint_proj(Dbar + Udbar, r, 2)     # dP:106
            for nn in range(N):                                   # dP:107-113
                d_D[nn] = d_D[nn] + (D[nn] - u_D2)
                ud = np.fft.fft2(u_D2 - d_D[nn], axes=(0, 1))
                dup[nn] = solve_conv_term_D(zm[nn], zi[nn], ud, Bh[nn], rho_d, size_x[:2], k, ni)
                D[nn] = np.real(np.fft.ifft2(dup[nn], axes=(0, 1)))
            Dbar = sum(D) / N                                     # dP:114-121
            Udbar = sum(d_D) / N
            dd = _rel(D[0] - d_old, D[0])
            zd.append(dd)
            d_diff = dd
            if verbose == "brief":                                # dP:126-129
                obj_val_filter = objective(z, D[0])
            if trace_objective:
                od.append(objective(z, D[0]))
            if d_diff < tol:
                break
        trace["obj_d"].append(od)
        trace["d_diff"].append(zd)
        trace["n_d"].append(len(zd))

        dhat_flat, dTd = precompute_H_hat_Z(np.fft.fft2(D[0], axes=(0, 1)), ss)   # dP:143
        oz, zz = [], []
        for i_z in range(max_it_z):                               # dP:147
            z_old = z
            u_Z2 = prox_sparse(z + d_Z, lambda_prior / theta_div)   # dP:150
            d_Z = d_Z + (z - u_Z2)                                # dP:151
            ud_Z = np.fft.fft2(u_Z2 - d_Z, axes=(0, 1))           # dP:152
            z_hat = solve_conv_term_Z(dhat_flat, dTd, ud_Z, B_hat, rho_z, size_z)
            z = np.real(np.fft.ifft2(z_hat, axes=(0, 1)))         # dP:154
            z_diff = _rel(z - z_old, z)
            zz.append(z_diff)
            if verbose == "brief":
                obj_val_z = objective(z, D[0])
            if trace_objective:
                oz.append(objective(z, D[0]))
            if z_diff < tol:
                break
        trace["obj_z"].append(oz)
        trace["z_diff"].append(zz)
        trace["n_z"].append(len(zz))
        trace["D1"].append(D[0].copy())
        iterations["obj_vals_d"].append(obj_val_filter)          # dP:174-176
        iterations["obj_vals_z"].append(obj_val_z)
        iterations["tim_vals"].append(0.0)
        if z_diff < tol and d_diff < tol:                         # dP:186
            break

    DZ = np.real(np.fft.ifft2(np.sum(z_hat * dup[0][:, :, :, None], axis=2, keepdims=True),
                              axes=(0, 1)))                       # dP:193
    d_res = crop_filters(D[0], 2, r)                              # dP:195-196
    return d_res, z, DZ, iterations, trace


# ----------------------------------------------------------------------------
# 2D dzParallel   (dZ:1-206)
# ----------------------------------------------------------------------------
def learn_2d_dzparallel(b, kernel_size, lambda_residual, lambda_prior, max_it, tol,
                        verbose, init, *, ni=100, max_it_d=5, max_it_z=10,
                        rho_d=5000.0, rho_z=1.0, theta_div=1.0, trace_objective=False):
    """Restatement of admm_learn_conv2D_large_dzParallel (dZ:1-206).

    z0 (init['z'], shape size_z_crop = [X, Y, K, ni]) is replicated into every
    block (dZ:44-47, Q4).  Objective: intended form, all blocks (Q5).
    """
    b = np.asarray(b, dtype=np.float64)
    psf_s = kernel_size[0]
    k = kernel_size[-1]
    sb = b.shape
    n = sb[-1]
    N = n // ni
    r = psf_s // 2
    size_x = [sb[0] + 2 * r, sb[1] + 2 * r, n]
    size_z_crop = [size_x[0], size_x[1], k, ni]
    size_d_full = [size_x[0], size_x[1], k]
    ss = size_x[0] * size_x[1]

    B = np.pad(b, ((r, r), (r, r), (0, 0)))
    B_hat = np.fft.fft2(B, axes=(0, 1))
    Bh = [B_hat[:, :, nn * ni:(nn + 1) * ni] for nn in range(N)]

    d0 = np.asarray(init["d"], dtype=np.float64)
    d = embed_filters(d0, size_x[:2], 2, r)
    D = [d.copy() for _ in range(N)]                              # dZ:40
    dup = [np.fft.fft2(d, axes=(0, 1)) for _ in range(N)]         # dZ:41-42
    z = np.array(init["z"], dtype=np.float64).reshape(size_z_crop, order="F")  # dZ:44
    Z = [z.copy() for _ in range(N)]                              # dZ:45
    Z_hat = [np.fft.fft2(z, axes=(0, 1)) for _ in range(N)]       # dZ:46-47

    def objective(Zl, dh):                                        # dZ:310-331 (Q5 fixed)
        zt = np.concatenate(Zl, axis=3)
        return objective_2d(zt, dh, b[:, :, :N * ni], lambda_residual, lambda_prior, r)

    trace = _new_trace()
    obj_val = objective(Z, dup[0]) if (verbose in ("brief", "all") or trace_objective) else float("nan")
    obj_val_filter = obj_val_z = obj_val
    iterations = {"obj_vals_d": [obj_val_filter], "obj_vals_z": [obj_val_z], "tim_vals": [0.0]}
    trace["obj0"] = obj_val

    Dbar = np.zeros(size_d_full)
    Udbar = np.zeros(size_d_full)
    d_D = [np.zeros(size_d_full) for _ in range(N)]
    d_Z = [np.zeros(size_z_crop) for _ in range(N)]
    d_diff = z_diff = None
    for i in range(max_it):                                       # dZ:90
        zm, zi = [], []
        for nn in range(N):                                       # dZ:96-100
            A, S = precompute_H_hat_D(Z_hat[nn], ss, k, ni, rho_d)
            zm.append(A)
            zi.append(S)
        od, zd = [], []
        for i_d in range(max_it_d):                               # dZ:104
            d_old = D[0]
            u_D2 = kernel_constraint_proj(Dbar + Udbar, r, 2)
            for nn in range(N):
                d_D[nn] = d_D[nn] + (D[nn] - u_D2)
                ud = np.fft.fft2(u_D2 - d_D[nn], axes=(0, 1))
                dup[nn] = solve_conv_term_D(zm[nn], zi[nn], ud, Bh[nn], rho_d, size_x[:2], k, ni)
                D[nn] = np.real(np.fft.ifft2(dup[nn], axes=(0, 1)))
            Dbar = sum(D) / N
            Udbar = sum(d_D) / N
            d_diff = _rel(D[0] - d_old, D[0])
            zd.append(d_diff)
            if verbose in ("brief", "all"):
                obj_val_filter = objective(Z, dup[0])
            if trace_objective:
                od.append(objective(Z, dup[0]))
            if d_diff < tol:
                break
        trace["obj_d"].append(od)
        trace["d_diff"].append(zd)
        trace["n_d"].append(len(zd))

        dhat_flat, dTd = precompute_H_hat_Z(dup[0], ss)          # dZ:143
        oz, zz = [], []
        for i_z in range(max_it_z):                               # dZ:147
            Z_old = [x for x in Z]
            for nn in range(N):                                   # dZ:150-158
                u = prox_sparse(Z[nn] + d_Z[nn], lambda_prior / theta_div)
                d_Z[nn] = d_Z[nn] + (Z[nn] - u)
                ud_Z = np.fft.fft2(u - d_Z[nn], axes=(0, 1))
                Z_hat[nn] = solve_conv_term_Z(dhat_flat, dTd, ud_Z, Bh[nn], rho_z, size_z_crop)
                Z[nn] = np.real(np.fft.ifft2(Z_hat[nn], axes=(0, 1)))
            zt = np.concatenate(Z, axis=3)
            zt_old = np.concatenate(Z_old, axis=3)
            z_diff = _rel(zt - zt_old, zt)                        # dZ:164
            zz.append(z_diff)
            if verbose in ("brief", "all"):
                obj_val_z = objective(Z, dup[0])
            if trace_objective:
                oz.append(objective(Z, dup[0]))
            if z_diff < tol:
                break
        trace["obj_z"].append(oz)
        trace["z_diff"].append(zz)
        trace["n_z"].append(len(zz))
        trace["D1"].append(D[0].copy())
        iterations["obj_vals_d"].append(obj_val_filter)
        iterations["obj_vals_z"].append(obj_val_z)
        iterations["tim_vals"].append(0.0)
        if z_diff < tol and d_diff < tol:
            break

    z_t = np.concatenate(Z, axis=3)
    DZ = np.real(np.fft.ifft2(np.sum(np.fft.fft2(z_t, axes=(0, 1)) * dup[0][:, :, :, None],
                                     axis=2, keepdims=True), axes=(0, 1)))   # dZ:197
    d_res = crop_filters(D[0], 2, r)
    return d_res, z_t, DZ, iterations, trace


# ----------------------------------------------------------------------------
# 3D   (L3:1-230)
# ----------------------------------------------------------------------------
def _objective_nd(z, dhat, b, lambda_residual, lambda_prior, r, nsp):
    """L3:341-380 (fftn per slice == fftn over the spatial axes)."""
    ax = tuple(range(nsp))
    zh = np.fft.fftn(z, axes=ax)
    Dz = np.real(np.fft.ifftn(np.sum(zh * dhat[..., None], axis=nsp), axes=ax))
    sl = tuple(slice(r, Dz.shape[i] - r) for i in range(nsp))
    Dz = Dz[sl]
    return float(lambda_residual * 0.5 * np.sum((Dz - b) ** 2) + lambda_prior * np.sum(np.abs(z)))


def learn_3d(b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init, *,
             ni=None, max_it_d=10, max_it_z=10, rho_d=5000.0, rho_z=1.0, theta_div=1.0,
             trace_objective=False, factored=False):
    """Restatement of admm_learn_conv3D_large (L3:1-230).  ni = sqrt(n) (L3:11)."""
    b = np.asarray(b, dtype=np.float64)
    k = kernel_size[-1]
    n = b.shape[-1]
    if ni is None:
        ni = int(round(math.sqrt(n)))
    N = n // ni
    r = kernel_size[0] // 2
    sp = [b.shape[i] + 2 * r for i in range(3)]                   # L3:16
    size_z = sp + [k, n]
    size_z_crop = sp + [k, ni]
    size_d_full = sp + [k]
    ss = int(np.prod(sp))
    ax = (0, 1, 2)

    B = np.pad(b, ((r, r), (r, r), (r, r), (0, 0)))               # L3:23
    B_hat = np.fft.fftn(B, axes=ax)                               # L3:24-26
    Bh = [B_hat[..., nn * ni:(nn + 1) * ni] for nn in range(N)]

    d = embed_filters(np.asarray(init["d"], dtype=np.float64), sp, 3, r)   # L3:39-40
    D = [d.copy() for _ in range(N)]
    d_hat = np.fft.fftn(d, axes=ax)                               # L3:42-45
    D_hat = [d_hat.copy() for _ in range(N)]
    z = np.array(init["z"], dtype=np.float64).reshape(size_z, order="F")   # L3:48
    z_hat = np.fft.fftn(z, axes=ax)                               # L3:49-55

    objective = lambda z_, d_: _objective_nd(z_, np.fft.fftn(d_, axes=ax), b,
                                             lambda_residual, lambda_prior, r, 3)
    trace = _new_trace()
    trace["obj0"] = objective(z, d) if (verbose in ("brief", "all") or trace_objective) else float("nan")

    Dbar = np.zeros(size_d_full)
    Udbar = np.zeros(size_d_full)
    d_D = [np.zeros(size_d_full) for _ in range(N)]
    d_Z = np.zeros(size_z)
    d_diff = z_diff = None
    for i in range(max_it):                                       # L3:100
        zm, zi = [], []
        for nn in range(N):                                       # L3:106-110
            A, S = precompute_H_hat_D(z_hat[..., nn * ni:(nn + 1) * ni], ss, k, ni, rho_d,
                                      factored=factored)
            zm.append(A)
            zi.append(S)
        od, zd = [], []
        for i_d in range(max_it_d):                               # L3:114
            d_old = d
            u_D2 = kernel_constraint_proj(Dbar + Udbar, r, 3)     # L3:118
            for nn in range(N):
                d_D[nn] = d_D[nn] + (D[nn] - u_D2)
                ud = np.fft.fftn(u_D2 - d_D[nn], axes=ax)
                D_hat[nn] = solve_conv_term_D(zm[nn], zi[nn], ud, Bh[nn], rho_d, sp, k, ni)
                D[nn] = np.real(np.fft.ifftn(D_hat[nn], axes=ax))
            Dbar = sum(D) / N
            Udbar = sum(d_D) / N
            d = D[0]
            d_hat = D_hat[0]                                      # L3:141-142
            d_diff = _rel(d - d_old, d)
            zd.append(d_diff)
            if trace_objective:
                od.append(objective(z, d))
            if d_diff < tol:
                break
        trace["obj_d"].append(od)
        trace["d_diff"].append(zd)
        trace["n_d"].append(len(zd))
        trace["U"].append(u_D2)                                   # the projected consensus
        dhat_flat, dTd = precompute_H_hat_Z(d_hat, ss)            # L3:161
        oz, zz = [], []
        for i_z in range(max_it_z):                               # L3:164
            z_old = z
            u_Z2 = prox_sparse(z + d_Z, lambda_prior / theta_div)   # L3:168
            d_Z = d_Z + (z - u_Z2)
            ud_Z = np.fft.fftn(u_Z2 - d_Z, axes=ax)
            z_hat = solve_conv_term_Z(dhat_flat, dTd, ud_Z, B_hat, rho_z, size_z)
            z = np.real(np.fft.ifftn(z_hat, axes=ax))
            z_diff = _rel(z - z_old, z)
            zz.append(z_diff)
            if trace_objective:
                oz.append(objective(z, d))
            if z_diff < tol:
                break
        trace["obj_z"].append(oz)
        trace["z_diff"].append(zz)
        trace["n_z"].append(len(zz))
        trace["D1"].append(D[0].copy())
        if z_diff < tol and d_diff < tol:                         # L3:211
            break

    DZ = np.real(np.fft.ifftn(np.sum(z_hat * d_hat[..., None], axis=3), axes=ax))   # L3:218-224
    d_res = crop_filters(d, 3, r)                                 # L3:226-227
    obj_val = objective(z, d)                                     # L3:229
    iterations = {"obj_vals_d": [], "obj_vals_z": [], "tim_vals": [], "it_vals": []}
    return d_res, z, DZ, obj_val, iterations, trace


# ----------------------------------------------------------------------------
# 4D light field   (L4:1-212)
# ----------------------------------------------------------------------------
def learn_4d(b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init, *,
             ni=None, max_it_d=10, max_it_z=10, rho_d=500.0, rho_z=50.0, theta_div=50.0,
             trace_objective=False):
    """Restatement of admm_learn_conv4D_lightfield (L4:1-212).

    b: [x, y, U, V, n]; kernel_size = [s, s, U, V, K].  Convolution is spatial
    only; the z-solve is the reference's diagonal form b/(rho + sum|dhat|^2)
    (L4:327-332, Q7); z is complex (L4:164, Q8).  Requires U == V (the
    reference swaps sw1/sw2, Q9).
    """
    b = np.asarray(b, dtype=np.float64)
    k = kernel_size[-1]
    U, V = kernel_size[2], kernel_size[3]
    if U != V or b.shape[2] != U or b.shape[3] != V:
        raise ValueError("4D learner requires square view grids matching kernel_size (Q9)")
    n = b.shape[-1]
    if ni is None:
        ni = int(round(math.sqrt(n)))
    N = n // ni
    r = kernel_size[0] // 2
    X, Y = b.shape[0] + 2 * r, b.shape[1] + 2 * r
    size_z = [X, Y, 1, 1, k, n]
    size_d_full = [X, Y, U, V, k]
    ss_sp = X * Y
    ax = (0, 1)

    B = np.pad(b, ((r, r), (r, r), (0, 0), (0, 0), (0, 0)))      # L4:25
    B_hat = np.fft.fft2(B, axes=ax)
    Bh = [B_hat[..., nn * ni:(nn + 1) * ni] for nn in range(N)]

    d = embed_filters(np.asarray(init["d"], dtype=np.float64), [X, Y], 2, r)   # L4:39-40
    D = [d.copy() for _ in range(N)]
    D_hat = [np.fft.fft2(d, axes=ax) for _ in range(N)]
    z = np.array(init["z"], dtype=np.complex128).reshape(size_z, order="F")   # L4:46
    z_hat = np.fft.fft2(z, axes=ax)

    def objective(z_, d_hat_):                                    # L4:349-369
        zh = np.fft.fft2(z_, axes=ax)                             # [X,Y,1,1,K,n]
        Dz = np.real(np.fft.ifft2(np.sum(zh * d_hat_[..., None], axis=4), axes=ax))
        Dz = Dz[r:X - r, r:Y - r]
        return float(lambda_residual * 0.5 * np.sum((Dz - b) ** 2)
                     + lambda_prior * np.sum(np.abs(z_)))

    trace = _new_trace()
    trace["obj0"] = objective(z, D_hat[0]) if (verbose in ("brief", "all") or trace_objective) else float("nan")

    Dbar = np.zeros(size_d_full)
    Udbar = np.zeros(size_d_full)
    d_D = [np.zeros(size_d_full) for _ in range(N)]
    d_Z = np.zeros(size_z, dtype=np.complex128)
    d_diff = z_diff = None
    for i in range(max_it):                                       # L4:96
        zm, zi = [], []
        for nn in range(N):                                       # L4:102-106, 243-263
            zup = z_hat[..., nn * ni:(nn + 1) * ni]               # [X,Y,1,1,K,ni]
            A, S = precompute_H_hat_D(zup, ss_sp, k, ni, rho_d)   # identical for every view
            zm.append(A)
            zi.append(S)
        od, zd = [], []
        for i_d in range(max_it_d):                               # L4:110
            d_old = D[0]
            u_D2 = kernel_constraint_proj(Dbar + Udbar, r, 2)     # per (u,v,k) slice (Q10)
            for nn in range(N):
                d_D[nn] = d_D[nn] + (D[nn] - u_D2)
                ud = np.fft.fft2(u_D2 - d_D[nn], axes=ax)         # [X,Y,U,V,K]
                out = np.empty_like(ud)
                for iu in range(U):                               # L4:281-308 per view
                    for iv in range(V):
                        out[:, :, iu, iv, :] = solve_conv_term_D(
                            zm[nn], zi[nn], ud[:, :, iu, iv, :], Bh[nn][:, :, iu, iv, :],
                            rho_d, [X, Y], k, ni)
                D_hat[nn] = out
                D[nn] = np.real(np.fft.ifft2(D_hat[nn], axes=ax))
            Dbar = sum(D) / N
            Udbar = sum(d_D) / N
            d_diff = _rel(D[0] - d_old, D[0])
            zd.append(d_diff)
            if trace_objective:
                od.append(objective(z, D_hat[0]))
            if d_diff < tol:
                break
        trace["obj_d"].append(od)
        trace["d_diff"].append(zd)
        trace["n_d"].append(len(zd))

        dh = D_hat[0]                                             # [X,Y,U,V,K]
        s = np.sum(np.abs(dh) ** 2, axis=(2, 3, 4))               # L4:277 + L4:330
        Eb = np.einsum("xyuvk,xyuvn->xykn", np.conj(dh), B_hat)   # L4:327 first term
        oz, zz = [], []
        for i_z in range(max_it_z):                               # L4:154
            z_old = z
            u_Z2 = prox_sparse(z + d_Z, lambda_prior / theta_div)   # L4:159
            d_Z = d_Z + (z - u_Z2)
            ud_Z = np.fft.fft2(u_Z2 - d_Z, axes=ax)[:, :, 0, 0]   # [X,Y,K,n]
            bb = Eb + rho_z * ud_Z
            x = bb / rho_z - (1.0 / rho_z) * (1.0 / (rho_z + s))[:, :, None, None] * s[:, :, None, None] * bb
            z_hat = x[:, :, None, None]                           # L4:335
            z = np.fft.ifft2(z_hat, axes=ax)                      # L4:164 (complex, Q8)
            z_diff = _rel(z - z_old, z)
            zz.append(z_diff)
            if trace_objective:
                oz.append(objective(z, D_hat[0]))
            if z_diff < tol:
                break
        trace["obj_z"].append(oz)
        trace["z_diff"].append(zz)
        trace["n_z"].append(len(zz))
        trace["D1"].append(D[0].copy())
        if z_diff < tol and d_diff < tol:
            break

    d_hat = D_hat[0]
    Dz = np.real(np.fft.ifft2(np.sum(z_hat * d_hat[..., None], axis=4), axes=ax))   # L4:205
    DZ = Dz[r:X - r, r:Y - r]
    d_res = crop_filters(D[0], 2, r)                              # L4:208-209
    obj_val = objective(z, D_hat[0])                              # L4:211
    iterations = {"obj_vals_d": [], "obj_vals_z": [], "tim_vals": [], "it_vals": []}
    return d_res, z, DZ, obj_val, iterations, trace


# ----------------------------------------------------------------------------
# 2-3D hyperspectral   (L23 = 2-3D/DictionaryLearning/admm_learn.m:1-343)
# ----------------------------------------------------------------------------
def pad_symmetric_2d(a, r):
    """padarray(a, [r, r, 0, 0], 'symmetric', 'both')   (L23:19)."""
    pad = [(r, r), (r, r)] + [(0, 0)] * (a.ndim - 2)
    return np.pad(a, pad, mode="symmetric")


def prox_data_masked(u, theta, M, Mtb):
    """ProxDataMasked = @(u, theta) (Mtb + 1/theta*u) ./ (M + 1/theta*ones)   (L23:26)."""
    return (Mtb + (1.0 / theta) * u) / (M + (1.0 / theta) * np.ones(u.shape))


def solve_conv_term_D_hs(z_hat, xi_hat1, xi_hat2, rho):
    """L23:273-300.  Per spatial frequency i: opt = 1/rho*I - 1/rho*Z'*pinv(rho*I + Z*Z')*Z
    (Z = zhat_mat{i}, n x k), then x = opt*(Z'*xi1(i,w,:) + rho*xi2(i,w,:)) for every
    wavelength w.  z_hat [X, Y, 1, K, n]; xi_hat1 [X, Y, W, n]; xi_hat2 [X, Y, W, K]."""
    X, Y, _, K, n = z_hat.shape
    W = xi_hat1.shape[2]
    ss = X * Y
    zm = _F(z_hat, (ss, K, n)).transpose(0, 2, 1)       # zhat_mat{i} = [n, k]   (L23:285)
    ZH = np.conj(zm.transpose(0, 2, 1))                  # [ss, k, n]
    opt = (np.eye(K)[None] - ZH @ np.linalg.pinv(rho * np.eye(n)[None] + zm @ ZH) @ zm) / rho
    x1 = _F(xi_hat1, (ss, W, n))                         # xi_hat_1_cell{ind}, ind = i + ss*(w-1)
    x2 = _F(xi_hat2, (ss, W, K))
    rhs = np.einsum("fkn,fwn->fwk", ZH, x1) + rho * x2   # L23:293
    out = np.einsum("fkj,fwj->fwk", opt, rhs)
    return _F(out, (X, Y, W, K))                          # L23:298


def solve_conv_term_Z_hs(dhat, xi_hat1, xi_hat2, gamma_ratio, W):
    """L23:302-324, the diagonal form (Q7): b = sum_w conj(dhat) .* xi1 + rho .* xi2,
    x = 1/rho*b - 1/rho * 1/(rho + s) .* s .* b with s = sum_{w,k}|dhat|^2 and
    rho = W * gamma_Z(2)/gamma_Z(1).  dhat [X, Y, W, K]; xi_hat1 [X, Y, W, n];
    xi_hat2 [X, Y, K, n] -> z_hat [X, Y, K, n]."""
    rho = W * gamma_ratio                                 # L23:311
    s = np.sum(np.abs(dhat) ** 2, axis=(2, 3))            # sum(dhatTdhat, 2)   (L23:267, 317)
    b = np.einsum("xywk,xywn->xykn", np.conj(dhat), xi_hat1) + rho * xi_hat2   # L23:314
    sc = (1.0 / (rho + s))[:, :, None, None]
    return b / rho - (1.0 / rho) * sc * s[:, :, None, None] * b                # L23:319


def objective_hs(z, dhat, b, lambda_residual, lambda_prior, r, smoothinit):
    """L23:326-343: z repeated over the W wavelengths (z2), Dz = ifft2(sum_k dhat .* fft2(z2))
    + smoothinit; f = lambda_res/2 ||crop(Dz) - b||^2 + lambda * sum|z2| (= W sum|z|)."""
    W = dhat.shape[2]
    zh = np.fft.fft2(z, axes=(0, 1))                      # [X, Y, K, n]
    Dz = np.real(np.fft.ifft2(np.einsum("xywk,xykn->xywn", dhat, zh), axes=(0, 1))) + smoothinit
    X, Y = Dz.shape[:2]
    f_z = lambda_residual * 0.5 * np.sum((Dz[r:X - r, r:Y - r] - b) ** 2)
    g_z = lambda_prior * W * np.sum(np.abs(z))
    return float(f_z + g_z)


def learn_hs23(b, kernel_size, lambda_residual, lambda_prior, max_it, tol, verbose, init,
               smooth_init, *, max_it_d=10, max_it_z=10):
    """Restatement of admm_learn (2-3D/DictionaryLearning/admm_learn.m, "L23").

    b, smooth_init: [x, y, W, n]; kernel_size = [s, s, W, K].  Non-consensus ADMM:
    v1 = H x (masked data prox) and v2 = x (kernel constraint in the D-phase,
    sparsity in the Z-phase).  ``init = {'d': [s, s, K], 'z': [X, Y, K, n]}``
    follows the reference's own draw (L23:54-57: one [s, s, K] array replicated
    over W, then z = randn(size_z), L23:69); the reference's init branch
    (L23:50-52) leaves d empty and cannot run.  The objective is evaluated after
    every inner iteration, as in the reference: it drives the rollback test
    (L23:204-213, Q16).  ``verbose`` only prints in the reference.

    Returns (d_res [s,s,W,K], z [X,Y,K,n], Dz [X,Y,W,n], obj_val, trace); trace
    holds obj0, obj_d / obj_z per inner iteration, d_diff, z_diff, rolled_back.
    """
    b = np.asarray(b, dtype=np.float64)
    smooth_init = np.asarray(smooth_init, dtype=np.float64)
    psf_s = kernel_size[0]
    k = kernel_size[3]                                            # L23:8
    n = b.shape[3]
    W = b.shape[2]
    r = psf_s // 2                                                # L23:12
    X, Y = b.shape[0] + 2 * r, b.shape[1] + 2 * r
    size_x = [X, Y, W, n]                                         # L23:13
    size_z = [X, Y, k, n]
    size_k_full = [X, Y, W, k]
    ax = (0, 1)

    smoothinit = pad_symmetric_2d(smooth_init, r)                 # L23:19
    M = np.pad(np.ones(b.shape), ((r, r), (r, r), (0, 0), (0, 0)))  # L23:255-258
    Mtb = np.pad(b, ((r, r), (r, r), (0, 0), (0, 0))) * M - smoothinit * M

    def objective(z_, dh):                                        # L23:22
        return objective_hs(z_, dh, b, lambda_residual, lambda_prior, r, smoothinit)

    lam = [lambda_residual, lambda_prior]                         # L23:35-38
    gamma_h = 60.0 * lambda_prior / np.max(b)
    gD = [gamma_h / 5000.0, gamma_h]
    gZ = [gamma_h / 500.0, gamma_h]

    d_D = [np.zeros(size_x), np.zeros(size_k_full)]               # L23:41-47
    d0 = np.asarray(init["d"], dtype=np.float64)                  # [s, s, K]
    d = embed_filters(d0, [X, Y], 2, r)                           # L23:54-55
    d = np.repeat(d[:, :, None, :], W, axis=2)                    # L23:56 -> [X, Y, W, K]
    d_hat = np.fft.fft2(d, axes=ax)                               # L23:57
    d_Z = [np.zeros(size_x), np.zeros(size_z)]                    # L23:61-67
    z = np.array(init["z"], dtype=np.float64).reshape(size_z, order="F")   # L23:69

    obj_val = objective(z, d_hat)                                 # L23:72
    trace = {"obj0": obj_val, "obj_d": [], "obj_z": [], "d_diff": [], "z_diff": [],
             "rolled_back": False, "outer": 0}
    obj_val_filter = obj_val_z = obj_val                          # L23:82-83
    for i in range(max_it):                                       # L23:86
        rho = gD[1] / gD[0]                                       # L23:93
        obj_val_min = min(obj_val_filter, obj_val_z)              # L23:94
        d_old = d
        d_hat_old = d_hat
        z_hat = np.fft.fft2(z, axes=ax)[:, :, None]               # L23:100 -> [X, Y, 1, K, n]
        od = []
        for i_d in range(max_it_d):                               # L23:102
            v1 = np.real(np.fft.ifft2(np.einsum("xywk,xykn->xywn", d_hat, z_hat[:, :, 0]),
                                      axes=ax))                   # L23:108
            v2 = d                                                # L23:109
            u1 = prox_data_masked(v1 - d_D[0], lam[0] / gD[0], M, Mtb)   # L23:112
            u2 = kernel_constraint_proj(v2 - d_D[1], r, 2)        # L23:113 (per (w, k), L23:246)
            d_D[0] = d_D[0] - (v1 - u1)                           # L23:117
            d_D[1] = d_D[1] - (v2 - u2)
            xi1 = np.fft.fft2(u1 + d_D[0], axes=ax)               # L23:120-121
            xi2 = np.fft.fft2(u2 + d_D[1], axes=ax)
            d_hat = solve_conv_term_D_hs(z_hat, xi1, xi2, rho)    # L23:125
            d = np.real(np.fft.ifft2(d_hat, axes=ax))             # L23:126
            obj_val = objective(z, d_hat)                         # L23:132
            od.append(obj_val)
        trace["obj_d"].append(od)
        obj_val_filter = obj_val                                  # L23:139
        d_diff = _rel(d - d_old, d)                               # L23:142-146
        trace["d_diff"].append(d_diff)

        z_hat = np.fft.fft2(z, axes=ax)                           # L23:158
        z_old = z
        z_hat_old = z_hat
        oz = []
        for i_z in range(max_it_z):                               # L23:165
            v1 = np.real(np.fft.ifft2(np.einsum("xywk,xykn->xywn", d_hat, z_hat), axes=ax))  # L23:171
            v2 = z
            u1 = prox_data_masked(v1 - d_Z[0], lam[0] / gZ[0], M, Mtb)   # L23:175
            u2 = prox_sparse(v2 - d_Z[1], lam[1] / gZ[1])         # L23:176
            d_Z[0] = d_Z[0] - (v1 - u1)                           # L23:180
            d_Z[1] = d_Z[1] - (v2 - u2)
            xi1 = np.fft.fft2(u1 + d_Z[0], axes=ax)               # L23:183-184
            xi2 = np.fft.fft2(u2 + d_Z[1], axes=ax)
            z_hat = solve_conv_term_Z_hs(d_hat, xi1, xi2, gZ[1] / gZ[0], W)   # L23:188
            z = np.real(np.fft.ifft2(z_hat, axes=ax))             # L23:189
            obj_val = objective(z, d_hat)                         # L23:195
            oz.append(obj_val)
        trace["obj_z"].append(oz)
        obj_val_z = obj_val                                       # L23:202
        trace["outer"] = i + 1

        if obj_val_min <= obj_val_filter and obj_val_min <= obj_val_z:   # L23:204-213 (Q16)
            z = np.real(np.fft.ifft2(z_hat_old, axes=ax))
            d_hat = d_hat_old
            d = np.real(np.fft.ifft2(d_hat, axes=ax))
            obj_val = objective(z, d_hat)
            trace["rolled_back"] = True
            break
        z_diff = _rel(z - z_old, z)                               # L23:216-220
        trace["z_diff"].append(z_diff)
        if z_diff < tol and d_diff < tol:                         # L23:223
            break

    d_res = crop_filters(d, 2, r)                                 # L23:231-232
    Dz = np.real(np.fft.ifft2(np.einsum("xywk,xykn->xywn", d_hat, np.fft.fft2(z, axes=ax)),
                              axes=ax)) + smoothinit              # L23:234-235
    return d_res, z, Dz, obj_val, trace
