"""GPU parity of the reconstruction solvers (ccsc_solve through the C-ABI) against the
float64 oracle (oracle/ccsc_solvers.py) on the seeded cases of tests/solver_cases.py.

Bar: z and res within 1e-8 relative (Frobenius), the per-iterate objective / PSNR /
relative-change trace within 1e-8 relative, iteration counts exact (tol cases stop at
the same iterate).  Grids: the small fixture shapes, odd and even extents, the Poisson
dataset's 522 x 394 grid (394 = 2 * 197, a generic-radix pass) and the inpainting
test set's 266 x 266 grid at reduced iteration counts; batched calls where images stop
at different iterates."""
import numpy as np
import pytest

from solver_cases import run_oracle, solver_inputs

CASES = ["solve_inpaint", "solve_poisson", "solve_multich", "solve_video"]


def _gpu(name, inp, ctx, batch=False, verbose="brief"):
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import solvers as SV
    var = {"solve_inpaint": L.CCSC_SOLVE_INPAINT2D, "solve_poisson": L.CCSC_SOLVE_POISSON2D,
           "solve_multich": L.CCSC_SOLVE_MULTICH, "solve_video": L.CCSC_SOLVE_VIDEO3D}[name]
    return SV.solve(var, inp["b"], inp["kernels"], inp["mask"], inp["lambda_residual"],
                    inp["lambda_prior"], inp["max_it"], inp["tol"], verbose,
                    smooth_init=inp.get("smooth_init"), psf=inp.get("psf"),
                    x_orig=inp.get("x_orig"), batch=batch, ctx=ctx)


def _rel(a, b):
    return np.linalg.norm((np.asarray(a) - np.asarray(b)).ravel()) / max(
        np.linalg.norm(np.asarray(b).ravel()), 1e-300)


def _check(name, z, res, log, zo, reso, lo, img=0):
    assert int(log["iters"][img]) == lo["iters"]
    n = lo["iters"] + 1
    np.testing.assert_allclose(log["obj"][img, :n], lo["obj"], rtol=1e-8)
    np.testing.assert_allclose(log["diff"][img, 1:n], lo["diff"][1:], rtol=1e-7)
    if name in ("solve_inpaint", "solve_poisson") and not np.isnan(lo["psnr"][0]):
        np.testing.assert_allclose(log["psnr"][img, :n], lo["psnr"], rtol=1e-8)
    assert _rel(z, zo) < 1e-8, _rel(z, zo)
    assert _rel(res, reso) < 1e-8, _rel(res, reso)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_solver_matches_oracle(gpu_ctx, name):
    inp = solver_inputs(name)
    zo, reso, lo = run_oracle(name, inp)
    z, res, log = _gpu(name, inp, gpu_ctx)
    _check(name, z, res, log, zo, reso, lo)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_solver_golden_fixture_on_gpu(gpu_ctx, name):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz"))
    z, res, log = _gpu(name, solver_inputs(name), gpu_ctx)
    assert _rel(z, g["z"]) < 1e-8 and _rel(res, g["res"]) < 1e-8
    np.testing.assert_allclose(log["obj"][0, :len(g["obj"])], g["obj"], rtol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("name,scale", [("solve_inpaint", 3), ("solve_poisson", 2),
                                        ("solve_multich", 3), ("solve_video", 2)])
def test_solver_odd_and_larger_grids(gpu_ctx, name, scale):
    inp = solver_inputs(name, seed=99, scale=scale)
    inp["max_it"] = 6
    zo, reso, lo = run_oracle(name, inp)
    z, res, log = _gpu(name, inp, gpu_ctx)
    _check(name, z, res, log, zo, reso, lo)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_solver_batch_with_tol(gpu_ctx, name):
    """Three images in one call; tol stops them at their own iterates (SI:136)."""
    inp = solver_inputs(name, seed=5, n=3)
    inp["max_it"] = 40
    outs = []
    for i in range(3):
        one = {k: (v[..., i] if isinstance(v, np.ndarray) and k not in ("kernels", "psf") else v)
               for k, v in inp.items()}
        outs.append(run_oracle(name, one))
    # a tol between the images' relative changes at their middle iterates
    diffs = [o[2]["diff"] for o in outs]
    inp["tol"] = 1.001 * float(np.median([d[min(12, len(d) - 1)] for d in diffs]))
    outs = []
    for i in range(3):
        one = {k: (v[..., i] if isinstance(v, np.ndarray) and k not in ("kernels", "psf") else v)
               for k, v in inp.items()}
        outs.append(run_oracle(name, one))
    z, res, log = _gpu(name, inp, gpu_ctx, batch=True)
    for i in range(3):
        zo, reso, lo = outs[i]
        _check(name, z[..., i], res[..., i], log, zo, reso, lo, img=i)
    assert len({o[2]["iters"] for o in outs}) >= 1


@pytest.mark.gpu
def test_poisson_dataset_grid(gpu_ctx):
    """The Poisson set's 512 x 384 images: 522 x 394 grid, 394 = 2 * 197 (generic pass)."""
    rng = np.random.default_rng(7)
    inp = solver_inputs("solve_poisson")
    x = np.abs(rng.standard_normal((512, 384))) * 0.3 + 0.1
    inp.update(b=rng.poisson(x * 100) / 100.0, mask=np.ones((512, 384)), x_orig=x, max_it=3,
               kernels=inp["kernels"])
    zo, reso, lo = run_oracle("solve_poisson", inp)
    z, res, log = _gpu("solve_poisson", inp, gpu_ctx)
    _check("solve_poisson", z, res, log, zo, reso, lo)


@pytest.mark.gpu
def test_inpaint_test_set_grid(gpu_ctx):
    """The inpainting test images (256 x 256, 11 x 11 filters: 266 x 266 grid)."""
    rng = np.random.default_rng(8)
    x = rng.standard_normal((256, 256)) * 0.2 + 0.5
    mask = (rng.uniform(size=x.shape) < 0.5).astype(float)
    k = rng.standard_normal((11, 11, 8))
    k /= np.sqrt((k ** 2).sum(axis=(0, 1)))
    inp = dict(b=x * mask, mask=mask, smooth_init=x * 0.9, x_orig=x, kernels=k,
               lambda_residual=5.0, lambda_prior=2.0, max_it=3, tol=0.0)
    zo, reso, lo = run_oracle("solve_inpaint", inp)
    z, res, log = _gpu("solve_inpaint", inp, gpu_ctx)
    _check("solve_inpaint", z, res, log, zo, reso, lo)


@pytest.mark.gpu
def test_solver_max_it_zero_and_quiet(gpu_ctx):
    """max_it = 0 returns z = 0 and res = crop(smoothinit); verbose 'none' leaves the
    trace NaN but still runs the tol test."""
    inp = solver_inputs("solve_inpaint")
    inp["max_it"] = 0
    zo, reso, lo = run_oracle("solve_inpaint", inp)
    z, res, log = _gpu("solve_inpaint", inp, gpu_ctx)
    assert np.all(z == 0)
    assert _rel(res, reso) < 1e-12
    inp = solver_inputs("solve_inpaint")
    inp["tol"] = 1e-2
    zo, reso, lo = run_oracle("solve_inpaint", inp, verbose="none")
    z, res, log = _gpu("solve_inpaint", inp, gpu_ctx, verbose="none")
    assert int(log["iters"][0]) == lo["iters"]
    assert np.all(np.isnan(log["obj"]))
    assert _rel(z, zo) < 1e-8
