function [ z, res ] = admm_solve_conv23D_weighted_sampling(b, kmat, mask, ...
                    lambda_residual, lambda_prior, max_it, tol, ~, verbose, smooth_init)
% Drop-in for 2-3D/Demosaicing/admm_solve_conv23D_weighted_sampling.m (same signature):
% multichannel reconstruction, b = [x, y, W], kmat = [k, k, W, K], no padding.
    [z, res] = ccsc_solve_call(nargout, 2, b, kmat, mask, lambda_residual, lambda_prior, ...
        max_it, tol, verbose, smooth_init, [], []);
end
