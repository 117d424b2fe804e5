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


def _sparse_codes(shape, density, g, device):
    mask = torch.rand(shape, generator=g, device=device) < density
    return (torch.randn(shape, generator=g, device=device) * mask).to(torch.float32)


def _single(t: torch.Tensor) -> torch.Tensor:
    """Stored as single, then widened (the reference's datasets are single: CI:367,
    learn_kernels_4D_extract_patches.m:16-53)."""
    return t.to(torch.float32).to(torch.float64)


def clips_3d(n: int, size=(64, 64, 32), K: int = 49, psf: int = 11, seed: int = 2017 + 3,
             density: float = 0.002, noise: float = 0.01, device: str = "cpu",
             chunk: int = 8) -> np.ndarray:
    """Synthetic video clips for the 3D learner (config C4), MATLAB layout [x, y, t, n].

    b_raw = sum_k d*_k (*) z*_k + noise ('valid' 3D convolution of sparse codes with K
    zero-mean unit-norm psf^3 filters), then the local contrast normalisation of every
    frame -- the reference's clips are crops of a frame-wise local-CN movie
    (learn_kernels_3D.m:12, extractContrastNormalizatonMovie.m:30)."""
    rng = np.random.default_rng(seed)
    d = make_filters(K, psf, 3, rng)                         # [K, x, y, t]
    X, Y, T = size
    G = (T + psf - 1, Y + psf - 1, X + psf - 1)               # codes' support, torch order (t, y, x)
    # the 'valid' 3D convolution as a circular one on the codes' grid (its outputs at
    # indices >= psf - 1 never wrap): filters zero-padded to G, one rfftn each
    dpad = np.zeros((K,) + G)
    dpad[:, :psf, :psf, :psf] = d.transpose(0, 3, 2, 1)
    dh = torch.fft.rfftn(torch.as_tensor(dpad, device=device), dim=(1, 2, 3))
    out = np.empty((X, Y, T, n), order="F")
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + c0 // chunk)
        codes = _sparse_codes((m, K) + G, density, g, device).double()
        zh = torch.fft.rfftn(codes, dim=(2, 3, 4))
        del codes
        full = torch.fft.irfftn((zh * dh[None]).sum(dim=1), s=G, dim=(1, 2, 3))
        del zh
        raw = full[:, psf - 1:, psf - 1:, psf - 1:]           # [m, T, Y, X]
        raw = raw + noise * torch.randn(raw.shape, generator=g, device=device, dtype=torch.float64)
        frames = raw.reshape(m * T, Y, X).transpose(1, 2)     # [m T, X(rows), Y]
        cn = local_cn(frames.contiguous()).reshape(m, T, X, Y)
        out[:, :, :, c0:c0 + m] = cn.permute(2, 3, 1, 0).cpu().numpy()
    return out


def lightfields_4d(n: int, size=(64, 64), views: int = 5, K: int = 49, psf: int = 11,
                   seed: int = 2017 + 4, density: float = 0.002, noise: float = 0.01,
                   device: str = "cpu", chunk: int = 16) -> np.ndarray:
    """Synthetic light fields for the 4D learner (config C5), MATLAB layout
    [x, y, U, V, n], single precision widened to double like the reference's patches.

    Every view (u, v) sees the same sparse codes through its own slice of the K
    filters d*_k(x, y, u, v) (spatial convolution only, the model of L4:18-21); each
    view image is then locally contrast normalised (the reference's light fields are
    local-CN data, learn_kernels_4D.m:10-12)."""
    rng = np.random.default_rng(seed)
    U = V = views
    d = rng.standard_normal((K, psf, psf, U, V))
    d -= d.mean(axis=(1, 2), keepdims=True)
    d /= np.sqrt((d ** 2).sum(axis=(1, 2), keepdims=True))  # unit norm per (u, v, k) slice
    # conv2d weight [U V, K, y, x] (output channel = view, u fastest as MATLAB's layout)
    wt = d.transpose(4, 3, 0, 2, 1).reshape(V * U, K, psf, psf)[:, :, ::-1, ::-1]
    w = torch.as_tensor(np.ascontiguousarray(wt), dtype=torch.float32, device=device)
    X, Y = size
    out = np.empty((X, Y, U, V, n), order="F")
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + c0 // chunk)
        codes = _sparse_codes((m, K, Y + psf - 1, X + psf - 1), density, g, device)
        raw = Fnn.conv2d(codes, w).double()                   # [m, V U, Y, X]
        del codes
        raw = raw + noise * torch.randn(raw.shape, generator=g, device=device, dtype=torch.float64)
        imgs = raw.reshape(m * U * V, Y, X).transpose(1, 2).contiguous()
        cn = _single(local_cn(imgs)).reshape(m, V, U, X, Y)
        out[..., c0:c0 + m] = cn.permute(3, 4, 2, 1, 0).cpu().numpy()
    return out


def gauss_symmetric(b: np.ndarray, size: int = 13, sigma: float = 3 * 1.591,
                    device: str = "cpu") -> np.ndarray:
    """imfilter(b, fspecial('gaussian', 13, 3*1.591), 'same', 'conv', 'symmetric') over
    the first two dims of b (learn_hyperspectral.m:15-16): mirror padding that repeats
    the edge sample."""
    k = fspecial_gaussian(size, sigma)
    h = (size - 1) // 2
    X, Y = b.shape[:2]
    rest = b.shape[2:]
    t = torch.as_tensor(np.ascontiguousarray(b.reshape(X, Y, -1, order="F").transpose(2, 1, 0)),
                        device=device)                        # [m, Y, X]
    ix = torch.as_tensor(np.pad(np.arange(X), h, mode="symmetric"), device=device)
    iy = torch.as_tensor(np.pad(np.arange(Y), h, mode="symmetric"), device=device)
    t = t[:, iy][:, :, ix]
    kk = torch.as_tensor(np.ascontiguousarray(k.T[::-1, ::-1]), dtype=t.dtype, device=device)
    o = Fnn.conv2d(t[:, None], kk[None, None])[:, 0]          # [m, Y, X]
    return np.asfortranarray(o.permute(2, 1, 0).cpu().numpy().reshape((X, Y) + rest, order="F"))


def cubes_23(n: int, size=(100, 100), W: int = 31, K: int = 100, psf: int = 11,
             seed: int = 2017 + 2, density: float = 0.002, noise: float = 0.01,
             device: str = "cpu", chunk: int = 8):
    """Synthetic hyperspectral cubes for the 2-3D learner (config C3), MATLAB layout
    [x, y, W, n], and their smooth_init.  b(x, y, w) = sum_k d*_k(., ., w) (*) z*_k(x, y)
    + noise (one code map per atom shared by the W wavelengths, the model of
    L23:302-324), shifted and scaled to [0.05, 1]: "similarly normalized but not
    contrast normalized" nonnegative data (learn_hyperspectral.m:9-11), so max(b) > 0
    as gamma_heuristic needs (L23:36).  smooth_init = the 13x13 Gaussian low-pass of b
    with symmetric padding (learn_hyperspectral.m:15-16)."""
    rng = np.random.default_rng(seed)
    d = rng.standard_normal((K, psf, psf, W))
    d -= d.mean(axis=(1, 2, 3), keepdims=True)
    d /= np.sqrt((d ** 2).sum(axis=(1, 2, 3), keepdims=True))
    wt = d.transpose(3, 0, 2, 1)[:, :, ::-1, ::-1]           # [W, K, y, x]
    w = torch.as_tensor(np.ascontiguousarray(wt), dtype=torch.float32, device=device)
    X, Y = size
    raw = np.empty((X, Y, W, n), order="F")
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + c0 // chunk)
        codes = _sparse_codes((m, K, Y + psf - 1, X + psf - 1), density, g, device)
        r_ = Fnn.conv2d(codes, w).double()                    # [m, W, Y, X]
        del codes
        r_ = r_ + noise * torch.randn(r_.shape, generator=g, device=device, dtype=torch.float64)
        raw[..., c0:c0 + m] = r_.permute(3, 2, 1, 0).cpu().numpy()
    lo, hi = raw.min(), raw.max()
    b = np.asfortranarray(0.05 + 0.95 * (raw - lo) / (hi - lo))
    return b, gauss_symmetric(b, device=device)


def init_2d(kernel_size, size_z, seed: int = 7):
    """d0 = randn(kernel_size); z0 = randn(size_z) (dP:38,45 draw order)."""
    rng = np.random.default_rng(seed)
    d0 = rng.standard_normal(tuple(kernel_size))
    z0 = rng.standard_normal(tuple(size_z))
    return {"d": d0, "z": z0}
