"""Python mirror of the reference's reconstruction solvers over the libccsc C-ABI
(``ccsc_solve``, include/ccsc.h).  Same names, argument order and meaning, and the
same ``[z, res]`` return as the MATLAB functions:

  z, res = admm_solve_conv2D_weighted_sampling(b, kernels, mask, lambda_residual,
      lambda_prior, smooth_init, max_it, tol, x_orig, verbose)
                      # 2D/Inpainting/admm_solve_conv2D_weighted_sampling.m:1-4
  z, res = admm_solve_conv_poisson(b, kmat, mask, lambda_residual, lambda_prior,
      max_it, tol, x_orig, verbose)   # 2D/Poisson_deconv/admm_solve_conv_poisson.m:1-2
  z, res = admm_solve_conv23D_weighted_sampling(b, kmat, mask, lambda_residual,
      lambda_prior, max_it, tol, _, verbose, smooth_init)
                      # 2-3D/Demosaicing/admm_solve_conv23D_weighted_sampling.m:1-2
  z, res = admm_solve_conv_weighted_sampling_lf(...)     # 4D/ViewSynthesis (same text)
  z, res = admm_solve_video_weighted_sampling(b, kmat, mask, lambda_residual,
      lambda_prior, max_it, tol, verbose, psf, smooth_init)
                      # 3D/Deblurring/admm_solve_video_weighted_sampling.m:1-2

Arrays carry the MATLAB shapes and are exchanged column-major.  A trailing image
axis (``batch=True``) solves several images of one shape in one call, each with
its own gamma heuristic and tol test (the reference's callers loop over images).
The verbose trace (objective / PSNR / relative change per iterate) is returned by
``solve`` instead of printed.  There is no CPU fallback: the HIP engine is the
product path.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .learners import Context


def _f64(a):
    return None if a is None else np.asfortranarray(a, dtype=np.float64)


def solve(variant, b, kernels, mask, lambda_residual, lambda_prior, max_it, tol, verbose="none",
          smooth_init=None, psf=None, x_orig=None, batch=False, ctx=None, want_z=True,
          want_res=True):
    """One ccsc_solve call.  Returns (z, res, log) with log = {'iters', 'obj', 'psnr',
    'diff', 'seconds'} (per-image arrays; trace entries are NaN unless verbose asks)."""
    own = ctx is None
    if own:
        ctx = Context(0)
    try:
        lib = L.lib()
        b = _f64(b)
        kernels = _f64(kernels)
        mask = _f64(mask)
        v3 = variant == L.CCSC_SOLVE_VIDEO3D
        multi = variant == L.CCSC_SOLVE_MULTICH
        nimg_axes = (3 if (v3 or multi) else 2)
        if batch:
            if b.ndim != nimg_axes + 1:
                raise ValueError(f"batched b must have {nimg_axes + 1} dims")
            n = b.shape[-1]
        else:
            if b.ndim != nimg_axes:
                raise ValueError(f"b must have {nimg_axes} dims")
            n = 1
        p = L.SolveProblem()
        p.variant = variant
        sb = list(b.shape[:2]) + ([b.shape[2]] if v3 else [1])
        for i in range(3):
            p.sb[i] = sb[i]
        p.nch = b.shape[2] if multi else 1
        p.n = n
        kd = 3 if v3 else 2
        ks = list(kernels.shape[:kd]) + [1] * (3 - kd)
        for i in range(3):
            p.ksize[i] = ks[i]
        p.K = kernels.shape[-1] if kernels.ndim > kd + (1 if multi else 0) else 1
        if multi and kernels.shape[2] != p.nch:
            raise ValueError("kernels must be [k, k, W, K] with W = size(b, 3)")
        if v3:
            if psf is None:
                raise ValueError("the video solver needs the blur psf")
            psf = _f64(psf)
            ps = list(psf.shape) + [1] * (3 - psf.ndim)
            for i in range(3):
                p.psf_size[i] = ps[i]
        p.lambda_residual = lambda_residual
        p.lambda_prior = lambda_prior
        p.max_it = max_it
        p.tol = tol
        p.verbose = L.VERBOSE[verbose] if isinstance(verbose, str) and verbose in L.VERBOSE else 0
        eb = L.errbuf()
        L.check(lib.ccsc_solve_supported(p, eb, len(eb)), eb)
        if mask.shape != b.shape:
            raise ValueError("mask must have the shape of b")
        inp = L.SolveInputs()
        smooth_init = _f64(smooth_init)
        x_orig = _f64(x_orig)
        # the library copies exactly b.size doubles of smooth_init and b.size / W of x_orig
        if smooth_init is not None and smooth_init.size != b.size:
            raise ValueError("smooth_init must have the size of b")
        if x_orig is not None and x_orig.size != b.size // p.nch:
            raise ValueError("x_orig must have the size of one channel of b")

        keep = [b, kernels, mask, smooth_init, psf, x_orig]
        inp.b, inp.kernels, inp.mask = L.dptr(b), L.dptr(kernels), L.dptr(mask)
        inp.smooth_init, inp.psf, inp.x_orig = L.dptr(smooth_init), L.dptr(psf), L.dptr(x_orig)
        rx, ry = (0, 0) if multi else (ks[0] // 2, ks[1] // 2)
        rt = ks[2] // 2 if v3 else 0
        X, Y = sb[0] + 2 * rx, sb[1] + 2 * ry
        T = sb[2] + 2 * rt
        Kc = p.K + (1 if variant in (L.CCSC_SOLVE_POISSON2D, L.CCSC_SOLVE_VIDEO3D) else 0)
        zshape = [X, Y] + ([T] if v3 else []) + [Kc] + ([n] if batch else [])
        if multi:
            rshape = [sb[0], sb[1], p.nch] + ([n] if batch else [])
        else:
            rshape = sb[:2] + ([sb[2]] if v3 else []) + ([n] if batch else [])
        z = np.zeros(zshape, order="F") if want_z else None
        res = np.zeros(rshape, order="F") if want_res else None
        out = L.SolveOutputs()
        out.z, out.res = L.dptr(z), L.dptr(res)
        cap = max_it + 1
        iters = np.zeros(n, dtype=np.int32)
        obj = np.full((n, cap), np.nan)
        psnr = np.full((n, cap), np.nan)
        diff = np.full((n, cap), np.nan)
        secs = np.zeros(1)
        lg = L.SolveLog()
        lg.capacity = cap
        lg.iters, lg.obj, lg.psnr, lg.diff = L.iptr(iters), L.dptr(obj), L.dptr(psnr), L.dptr(diff)
        lg.seconds = L.dptr(secs)
        L.check(lib.ccsc_solve(ctx.ptr, p, inp, out, lg, eb, len(eb)), eb)
        del keep
        log = {"iters": iters, "obj": obj, "psnr": psnr, "diff": diff, "seconds": float(secs[0])}
        return z, res, log
    finally:
        if own:
            ctx.close()


def admm_solve_conv2D_weighted_sampling(b, kernels, mask, lambda_residual, lambda_prior,
                                        smooth_init, max_it, tol, x_orig=None, verbose="none",
                                        *, ctx=None, batch=False):
    """SI:1-4 (2D inpainting)."""
    z, res, _ = solve(L.CCSC_SOLVE_INPAINT2D, b, kernels, mask, lambda_residual, lambda_prior,
                      max_it, tol, verbose, smooth_init=smooth_init, x_orig=x_orig, batch=batch,
                      ctx=ctx)
    return z, res


def admm_solve_conv_poisson(b, kmat, mask, lambda_residual, lambda_prior, max_it, tol,
                            x_orig=None, verbose="none", *, ctx=None, batch=False):
    """SP:1-2 (2D Poisson deconvolution)."""
    z, res, _ = solve(L.CCSC_SOLVE_POISSON2D, b, kmat, mask, lambda_residual, lambda_prior,
                      max_it, tol, verbose, x_orig=x_orig, batch=batch, ctx=ctx)
    return z, res


def admm_solve_conv23D_weighted_sampling(b, kmat, mask, lambda_residual, lambda_prior, max_it,
                                         tol, _unused=None, verbose="none", smooth_init=None, *,
                                         ctx=None, batch=False):
    """SD:1-2 (2-3D demosaicing)."""
    z, res, _ = solve(L.CCSC_SOLVE_MULTICH, b, kmat, mask, lambda_residual, lambda_prior, max_it,
                      tol, verbose, smooth_init=smooth_init, batch=batch, ctx=ctx)
    return z, res


def admm_solve_conv_weighted_sampling_lf(b, kmat, mask, lambda_residual, lambda_prior, max_it,
                                         tol, _unused=None, verbose="none", smooth_init=None, *,
                                         ctx=None, batch=False):
    """4D/ViewSynthesis/admm_solve_conv_weighted_sampling_lf.m:1-2 (the text of SD; the
    views of the light field are its channels, reconstruct_subsampling_lightfield.m:53-56)."""
    return admm_solve_conv23D_weighted_sampling(b, kmat, mask, lambda_residual, lambda_prior,
                                                max_it, tol, _unused, verbose, smooth_init,
                                                ctx=ctx, batch=batch)


def admm_solve_video_weighted_sampling(b, kmat, mask, lambda_residual, lambda_prior, max_it, tol,
                                       verbose="none", psf=None, smooth_init=None, *, ctx=None,
                                       batch=False):
    """SV:1-2 (3D video deblurring)."""
    z, res, _ = solve(L.CCSC_SOLVE_VIDEO3D, b, kmat, mask, lambda_residual, lambda_prior, max_it,
                      tol, verbose, smooth_init=smooth_init, psf=psf, batch=batch, ctx=ctx)
    return z, res
