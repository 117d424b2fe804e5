"""Seeded input cases of the reconstruction solvers (shared by the oracle fixtures,
tools/make_golden.py, and the GPU parity tests).  Shapes follow the reference's callers
at reduced size: 2D/Inpainting/reconstruct_2D_subsampling.m (random 50% mask, smooth
offset), 2D/Poisson_deconv/reconstruct_poisson_noise.m (Poisson counts, full mask),
2-3D/Demosaicing/reconstruct_subsampling_hyperspectral.m (one sample per channel in
each sb x sb cell), 3D/Deblurring/reconstruct_subsampling_video.m (3x3 blur in the
middle frame of a 3-frame psf, full mask)."""
import numpy as np


def _unit(k):
    n = np.sqrt(np.sum(k ** 2, axis=tuple(range(k.ndim - 1)), keepdims=True))
    return k / n


def _blur(a, axes=(0, 1)):
    out = a.copy()
    for ax in axes:
        out = (np.roll(out, 1, ax) + 2 * out + np.roll(out, -1, ax)) / 4
    return out


def solver_inputs(name, seed=None, n=None, scale=1):
    """Inputs of case `name` (dict of keyword arguments of the oracle function).  `n`
    stacks that many images along a trailing axis (the batched ccsc_solve)."""
    rng = np.random.default_rng(seed if seed is not None else
                                {"solve_inpaint": 11, "solve_poisson": 12,
                                 "solve_multich": 13, "solve_video": 14}[name])
    imgs = []
    for _ in range(n or 1):
        if name == "solve_inpaint":
            sb = (20 * scale, 18 * scale)
            x = _blur(rng.standard_normal(sb)) + 0.5
            mask = (rng.uniform(size=sb) < 0.5).astype(float)
            imgs.append(dict(b=x * mask, mask=mask, smooth_init=_blur(_blur(x * mask)), x_orig=x))
        elif name == "solve_poisson":
            sb = (16 * scale, 14 * scale)
            x = np.abs(_blur(rng.standard_normal(sb))) + 0.2
            counts = rng.poisson(x * 200) / 200.0
            imgs.append(dict(b=counts, mask=np.ones(sb), x_orig=x))
        elif name == "solve_multich":
            W, cell = 4, 2
            sb = (12 * scale, 10 * scale, W)
            x = _blur(rng.standard_normal(sb)) + 1.0
            mask = np.zeros(sb)
            c = 0
            for m in range(cell):
                for q in range(cell):
                    mask[m::cell, q::cell, c] = 1
                    c += 1
            imgs.append(dict(b=x * mask, mask=mask, smooth_init=_blur(x)))
        elif name == "solve_video":
            sb = (10 * scale, 9 * scale, 8)
            x = _blur(rng.standard_normal(sb), axes=(0, 1, 2))
            imgs.append(dict(b=x + 1.0, mask=np.ones(sb), smooth_init=_blur(x + 1.0)))
        else:
            raise KeyError(name)
    out = {k: (np.stack([d[k] for d in imgs], axis=-1) if n else imgs[0][k]) for k in imgs[0]}
    if name == "solve_inpaint":
        out.update(kernels=_unit(rng.standard_normal((5, 5, 4))), lambda_residual=5.0,
                   lambda_prior=2.0, max_it=15, tol=0.0)
    elif name == "solve_poisson":
        out.update(kernels=_unit(rng.standard_normal((5, 5, 3))), lambda_residual=200.0,
                   lambda_prior=1.0, max_it=12, tol=0.0)
    elif name == "solve_multich":
        out.update(kernels=_unit(rng.standard_normal((5, 5, 4, 5))), lambda_residual=1000.0,
                   lambda_prior=1.0, max_it=10, tol=0.0)
    else:
        psf = np.zeros((3, 3, 3))
        psf[:, :, 1] = rng.uniform(0.5, 1.0, (3, 3))
        psf /= psf.sum()
        out.update(kernels=_unit(rng.standard_normal((3, 3, 3, 3))), psf=psf,
                   lambda_residual=1000.0, lambda_prior=0.125, max_it=8, tol=0.0)
    return out


def run_oracle(name, inp, verbose="brief"):
    """The oracle on one image of `inp` (unbatched)."""
    from oracle import ccsc_solvers as S
    if name == "solve_inpaint":
        return S.admm_solve_conv2D_weighted_sampling(
            inp["b"], inp["kernels"], inp["mask"], inp["lambda_residual"], inp["lambda_prior"],
            inp["smooth_init"], inp["max_it"], inp["tol"], inp.get("x_orig"), verbose)
    if name == "solve_poisson":
        return S.admm_solve_conv_poisson(
            inp["b"], inp["kernels"], inp["mask"], inp["lambda_residual"], inp["lambda_prior"],
            inp["max_it"], inp["tol"], inp.get("x_orig"), verbose)
    if name == "solve_multich":
        return S.admm_solve_conv23D_weighted_sampling(
            inp["b"], inp["kernels"], inp["mask"], inp["lambda_residual"], inp["lambda_prior"],
            inp["max_it"], inp["tol"], None, verbose, inp["smooth_init"])
    return S.admm_solve_video_weighted_sampling(
        inp["b"], inp["kernels"], inp["mask"], inp["lambda_residual"], inp["lambda_prior"],
        inp["max_it"], inp["tol"], verbose, inp["psf"], inp["smooth_init"])


def solver_case(name):
    return run_oracle(name, solver_inputs(name))
