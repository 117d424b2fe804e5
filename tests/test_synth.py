"""Synthetic-input generator against a loop-level NumPy
restatement of the reference's preprocessing:

  * image_helpers/rconv2.m:22-58 -- reflection about the edge pixels (edge not
    repeated), built with the reference's own 1-based index ranges, then
    conv2(..., 'valid') as an explicit sum over the flipped kernel;
  * image_helpers/CreateImages.m:299-369 -- 'local_cn': 13x13 Gaussian
    (sigma 3*1.591), lvar clamp, std floored at the median of the sorted
    stds (round(length/2), 1-based), the zero-median branch CI:340-347 (median
    of the nonzeros, or 0 when there are none), zero stds -> eps, single storage;
  * CreateImages.m:652-657 -- ZERO_MEAN on the single image.

The restatement is pure test infrastructure (CPU, small sizes)."""
import math

import numpy as np
import pytest
import torch

from ccsc_code_iccv2017_amd import synth

EPS = np.finfo(float).eps


def fspecial_gaussian_loop(n, sigma):
    """MATLAB fspecial('gaussian', [n n], sigma): exp, eps*max cut, normalise."""
    h = np.empty((n, n))
    c = (n - 1) / 2.0
    for i in range(n):
        for j in range(n):
            h[i, j] = math.exp(-((i - c) ** 2 + (j - c) ** 2) / (2 * sigma * sigma))
    h[h < EPS * h.max()] = 0
    return h / h.sum()


def rconv2_loop(large, small):
    """rconv2.m:35-58 with MATLAB's index ranges (1-based, inclusive)."""
    ly, lx = large.shape
    sy, sx = small.shape
    sy2, sx2 = (sy - 1) // 2, (sx - 1) // 2           # ctr = 0 (rconv2.m:24,43-44)

    def rng(a, b):                                      # MATLAB a:-1:b -> 0-based list
        return [i - 1 for i in range(a, b - 1, -1)]
    top, bot = rng(sy - sy2, 2), rng(ly - 1, ly - sy2)
    left, right = rng(sx - sx2, 2), rng(lx - 1, lx - sx2)
    rows = top + list(range(ly)) + bot
    cols = left + list(range(lx)) + right
    cl = large[np.ix_(rows, cols)]                      # rconv2.m:47-53
    H, W = cl.shape[0] - sy + 1, cl.shape[1] - sx + 1   # conv2 'valid' (rconv2.m:58)
    out = np.zeros((H, W))
    for y in range(H):
        for x in range(W):
            acc = 0.0
            for u in range(sy):
                for v in range(sx):
                    acc += cl[y + u, x + v] * small[sy - 1 - u, sx - 1 - v]
            out[y, x] = acc
    return out


def local_cn_loop(dim):
    """CreateImages.m:306-369 then :652-657 for one single-colour image."""
    k = fspecial_gaussian_loop(13, 3 * 1.591)
    lmn = rconv2_loop(dim, k)
    lmnsq = rconv2_loop(dim ** 2, k)
    lvar = lmnsq - lmn ** 2
    lvar[lvar < 0] = 0
    lstd = np.sqrt(lvar)
    q = np.sort(lstd.flatten(order="F"))
    lq = int(math.floor(len(q) / 2 + 0.5))              # round(length(q)/2)
    th = q[lq - 1]
    if th == 0:                                          # CI:340-347
        q = q[q != 0]
        th = q[int(math.floor(len(q) / 2 + 0.5)) - 1] if len(q) else 0.0
    lstd[lstd <= th] = th
    lstd[lstd == 0] = EPS
    out = ((dim - lmn) / lstd).astype(np.float32)       # I{image} = single(temp)
    out = out - out.mean(dtype=np.float32)              # ZERO_MEAN (single)
    return out.astype(np.float64)


def test_fspecial_matches_loop():
    np.testing.assert_allclose(synth.fspecial_gaussian(13, 3 * 1.591),
                               fspecial_gaussian_loop(13, 3 * 1.591), rtol=0, atol=1e-17)


@pytest.mark.parametrize("shape", [(16, 16), (17, 20), (21, 14), (13, 13)])
def test_rconv2_matches_loop(shape):
    rng = np.random.default_rng(sum(shape))
    a = rng.standard_normal(shape)
    k = fspecial_gaussian_loop(13, 3 * 1.591)
    got = synth.rconv2(torch.as_tensor(a)[None], k)[0].numpy()
    np.testing.assert_allclose(got, rconv2_loop(a, k), rtol=1e-12, atol=1e-14)


def test_rconv2_asymmetric_kernel_orientation():
    """conv2 (not correlation) and the reflection ranges with a non-symmetric kernel."""
    rng = np.random.default_rng(5)
    a = rng.standard_normal((15, 18))
    k = rng.standard_normal((5, 7))
    got = synth.rconv2(torch.as_tensor(a)[None], k)[0].numpy()
    np.testing.assert_allclose(got, rconv2_loop(a, k), rtol=1e-12, atol=1e-13)


def _cases():
    rng = np.random.default_rng(3)
    smooth = rng.standard_normal((18, 23))
    spot = np.zeros((40, 40))                            # most local stds are exactly 0
    spot[3:5, 4:6] = 1.0
    const = np.full((16, 16), 0.25)                      # every std 0, no nonzeros: th = 0 -> eps
    return [("random_even", rng.standard_normal((16, 16))),
            ("random_odd", smooth),
            ("zero_median", spot),
            ("constant", const)]


@pytest.mark.parametrize("name,img", _cases(), ids=[c[0] for c in _cases()])
def test_local_cn_matches_loop(name, img):
    want = local_cn_loop(img)
    got = synth.local_cn(torch.as_tensor(img)[None])[0].numpy()
    # single storage: every output value is a float32
    assert np.array_equal(got.astype(np.float32).astype(np.float64), got)
    # float32 rounding of (dim - lmn) / lstd and of the single-precision mean
    scale = max(np.abs(want).max(), 1.0)
    np.testing.assert_allclose(got, want, rtol=0, atol=4e-7 * scale)
    if name == "constant":
        assert np.all(got == 0)


def test_zero_median_branch_taken():
    """The spot image really exercises CI:340-347 (median std is 0, nonzeros exist)."""
    img = _cases()[2][1]
    k = fspecial_gaussian_loop(13, 3 * 1.591)
    lstd = np.sqrt(np.maximum(rconv2_loop(img ** 2, k) - rconv2_loop(img, k) ** 2, 0))
    q = np.sort(lstd.ravel())
    assert q[int(math.floor(len(q) / 2 + 0.5)) - 1] == 0 and np.any(q > 0)


def test_images_2d_shape_layout_and_sharding():
    """MATLAB layout [x, y, n]; a chunk-aligned shard reproduces the full draw."""
    full = synth.images_2d(6, size=(20, 20), K=4, psf=5, chunk=2, seed=11)
    part = synth.images_2d(2, size=(20, 20), K=4, psf=5, chunk=2, seed=11, first=4)
    assert full.shape == (20, 20, 6) and full.flags.f_contiguous
    np.testing.assert_array_equal(full[:, :, 4:], part)
    # every patch is zero-mean (in single) and contrast-normalised
    assert np.all(np.abs(full.mean(axis=(0, 1))) < 1e-6)
    raw = synth.images_2d(2, size=(20, 20), K=4, psf=5, chunk=2, seed=11, local_cn_on=False)
    np.testing.assert_allclose(synth.local_cn(torch.as_tensor(np.moveaxis(raw, 2, 0)))
                               .numpy(), np.moveaxis(full[:, :, :2], 2, 0), rtol=0, atol=2e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(100, 100), (17, 23), (24, 9)])
def test_local_cn_gpu_kernel_matches_loop(shape):
    """csrc/localcn.hip (through ccsc_local_cn_dev) == the loop restatement of
    CreateImages.m:306-369 + :652-657; single-precision output, so agreement to the
    float32 rounding of the last step (the mean's summation order is not MATLAB's)."""
    rng = np.random.default_rng(5)
    imgs = [rng.standard_normal(shape), np.ones(shape) * 3.0,            # constant: zero-median branch
            np.where(rng.uniform(size=shape) < 0.7, 0.0, rng.standard_normal(shape))]
    t = torch.as_tensor(np.stack(imgs), dtype=torch.float64, device="cuda")
    got = synth.local_cn(t).cpu().numpy()
    for i, im in enumerate(imgs):
        ref = local_cn_loop(im)
        np.testing.assert_allclose(got[i], ref, rtol=0, atol=2e-6 * max(1.0, np.abs(ref).max()))


@pytest.mark.gpu
def test_local_cn_host_entry_point(gpu_ctx):
    """ccsc_local_cn (host arrays, column-major [H, W, n]) == the device entry point."""
    from ccsc_code_iccv2017_amd import _lib as L
    rng = np.random.default_rng(6)
    b = np.asfortranarray(rng.standard_normal((30, 28, 5)))
    out = np.zeros_like(b, order="F")
    eb = L.errbuf()
    L.check(L.lib().ccsc_local_cn(gpu_ctx.ptr, L.dptr(b), L.dptr(out), 5, 30, 28, eb, len(eb)), eb)
    for i in range(5):
        np.testing.assert_allclose(out[:, :, i], local_cn_loop(b[:, :, i]), rtol=0, atol=2e-6)
