"""Synthetic learner inputs -- the reference's drivers read
image/video/light-field datasets that are not available here, so the bench and
tests use seeded synthetic data of the same shapes:

  * ground-truth filters: K random psf^d arrays, zero mean, unit norm
  * codes: Bernoulli(density) * N(0, 1) per pixel per filter
  * b_raw = sum_k d*_k (*) z*_k + noise * N(0, 1)      ('valid' convolution)
  * local contrast normalisation + zero mean, restating the 'local_cn' branch
    of image_helpers/CreateImages.m:299-369 (13x13 Gaussian, sigma 3*1.591,
    reflection padding of image_helpers/rconv2.m:22-58, std floored at its
    median) and the ZERO_MEAN branch CreateImages.m:652-657.  Like the
    reference, the normalised image is stored as single then widened to double
    (CreateImages.m:367, :711).

On a GPU the local contrast normalisation runs in libccsc's hand-written kernel
(ccsc_local_cn_dev, csrc/localcn.hip: one workgroup per image, LDS-resident 13x13
convolutions, radix-select median); the torch restatement below serves CPU tensors
(tests, the CPU baseline).  PyTorch draws the synthetic codes and noise.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as Fnn


def fspecial_gaussian(size: int = 13, sigma: float = 3 * 1.591) -> np.ndarray:
    """MATLAB fspecial('gaussian', [size size], sigma)."""
    h = (size - 1) / 2.0
    x = np.arange(-h, h + 1)
    g = np.exp(-(x[:, None] ** 2 + x[None, :] ** 2) / (2.0 * sigma * sigma))
    g[g < np.finfo(float).eps * g.max()] = 0
    return g / g.sum()


def rconv2(large: torch.Tensor, small: np.ndarray) -> torch.Tensor:
    """image_helpers/rconv2.m:22-58 on a batch [n, H, W]: reflect about the edge
    pixels (edge not repeated), then conv2(..., 'valid')."""
    sy, sx = small.shape
    py, px = (sy - 1) // 2, (sx - 1) // 2
    t = large[:, None]
    t = Fnn.pad(t, (px, sx - 1 - px, py, sy - 1 - py), mode="reflect")
    k = torch.as_tensor(np.ascontiguousarray(small[::-1, ::-1]), dtype=t.dtype, device=t.device)
    return Fnn.conv2d(t, k[None, None])[:, 0]


def local_cn_gpu(imgs: torch.Tensor) -> torch.Tensor:
    """local_cn on the GPU through the C-ABI (ccsc_local_cn_dev); imgs [n, H, W] on a
    CUDA device.  No fallback: a missing libccsc raises."""
    from . import _lib as L
    from .learners import Context
    n, H, W = imgs.shape
    x = imgs.to(torch.float64).transpose(1, 2).contiguous()   # [n, W, H] = column-major [H, W]
    out = torch.empty_like(x)
    dev = imgs.device.index if imgs.device.index is not None else torch.cuda.current_device()
    torch.cuda.synchronize(imgs.device)
    with Context(dev) as ctx:   # one stream for this call (no context outlives it)
        eb = L.errbuf()
        L.check(L.lib().ccsc_local_cn_dev(ctx.ptr, x.data_ptr(), out.data_ptr(), n, H, W, eb,
                                          len(eb)), eb)
    return out.transpose(1, 2)


def local_cn(imgs: torch.Tensor) -> torch.Tensor:
    """CreateImages.m:299-369 ('local_cn') then :652-657 (ZERO_MEAN) per image.

    imgs: [n, H, W] float64 (rows = MATLAB dim 1).  Returns float64 values that
    went through the reference's single-precision storage.  CUDA tensors go through
    the HIP kernel (local_cn_gpu); this torch restatement serves CPU tensors.
    """
    if imgs.is_cuda:
        return local_cn_gpu(imgs)
    k = fspecial_gaussian(13, 3 * 1.591)
    lmn = rconv2(imgs, k)
    lmnsq = rconv2(imgs * imgs, k)
    lvar = torch.clamp(lmnsq - lmn * lmn, min=0)
    lstd = torch.sqrt(lvar)
    n = imgs.shape[0]
    flat = lstd.reshape(n, -1)
    q = torch.sort(flat, dim=1).values
    lq = int(math.floor(flat.shape[1] / 2 + 0.5))            # MATLAB round(length/2), 1-based
    th = q[:, lq - 1].clone()
    zero = th == 0
    if bool(zero.any()):                                       # CI:337-345: median of nonzeros
        for i in torch.nonzero(zero).flatten().tolist():
            nz = q[i][q[i] != 0]
            th[i] = nz[int(math.floor(nz.numel() / 2 + 0.5)) - 1] if nz.numel() else 0
    lstd = torch.maximum(lstd, th[:, None, None])
    lstd = torch.where(lstd == 0, torch.full_like(lstd, np.finfo(float).eps), lstd)
    out = ((imgs - lmn) / lstd).to(torch.float32)              # I{image} = single(temp)
    out = out - out.mean(dim=(1, 2), keepdim=True)             # ZERO_MEAN, in single
    return out.to(torch.float64)


def make_filters(K: int, psf: int, ndim: int, rng: np.random.Generator) -> np.ndarray:
    d = rng.standard_normal((K,) + (psf,) * ndim)
    d -= d.reshape(K, -1).mean(1).reshape((K,) + (1,) * ndim)
    d /= np.linalg.norm(d.reshape(K, -1), axis=1).reshape((K,) + (1,) * ndim)
    return d


def images_2d(n: int, size=(100, 100), K: int = 100, psf: int = 11, seed: int = 2017,
              density: float = 0.002, noise: float = 0.01, device: str = "cpu",
              chunk: int = 100, local_cn_on: bool = True, first: int = 0) -> np.ndarray:
    """Synthetic contrast-normalised images, MATLAB layout [x, y, n] float64.

    Patches first .. first+n-1 of the global sequence; chunk c (global patches
    c*chunk ..) draws from its own seeded stream on `device`, so a rank that
    generates only its shard gets exactly the single-GPU data.
    """
    rng = np.random.default_rng(seed)
    d = make_filters(K, psf, 2, rng)                         # [K, psf, psf]  (x, y)
    dw = torch.as_tensor(np.ascontiguousarray(d[:, ::-1, ::-1]), dtype=torch.float32,
                         device=device)[None]                # conv2d weight [1, K, psf, psf]
    H, W = size
    out = np.empty((H, W, n), order="F")
    if first % chunk:
        raise ValueError("first must be chunk-aligned")
    for c0 in range(first, first + n, chunk):
        m = min(chunk, first + n - c0)
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + c0 // chunk)
        shape = (m, K, H + psf - 1, W + psf - 1)
        mask = torch.rand(shape, generator=g, device=device) < density
        codes = torch.randn(shape, generator=g, device=device) * mask
        raw = Fnn.conv2d(codes.to(torch.float32), dw)[:, 0].double()
        del codes, mask
        raw = raw + noise * torch.randn(raw.shape, generator=g, device=device, dtype=torch.float64)
        img = local_cn(raw) if local_cn_on else raw
        out[:, :, c0 - first:c0 - first + m] = img.permute(1, 2, 0).cpu().numpy()
    return out


def init_2d(kernel_size, size_z, seed: int = 7):
    """d0 = randn(kernel_size); z0 = randn(size_z) (dP:38,45 draw order)."""
    rng = np.random.default_rng(seed)
    d0 = rng.standard_normal(tuple(kernel_size))
    z0 = rng.standard_normal(tuple(size_z))
    return {"d": d0, "z": z0}
