function [ z, res ] = admm_solve_video_weighted_sampling(b, kmat, mask, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, psf, smooth_init)
% Drop-in for 3D/Deblurring/admm_solve_video_weighted_sampling.m (same signature): video
% deblurring with 3D filters plus a dirac (prepended, as the reference) under the blur psf.
    [z, res] = ccsc_solve_call(nargout, 3, b, kmat, mask, lambda_residual, lambda_prior, ...
        max_it, tol, verbose, smooth_init, psf, []);
end
