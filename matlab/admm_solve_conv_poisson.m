function [ z, res ] = admm_solve_conv_poisson(b, kmat, mask, ...
                    lambda_residual, lambda_prior, max_it, tol, x_orig, verbose)
% Drop-in for 2D/Poisson_deconv/admm_solve_conv_poisson.m (same signature): Poisson
% deconvolution with the learned filters plus a dirac (appended last, as the reference).
    if nargin < 8, x_orig = []; end
    if nargin < 9, verbose = 'none'; end
    [z, res] = ccsc_solve_call(nargout, 1, b, kmat, mask, lambda_residual, lambda_prior, ...
        max_it, tol, verbose, [], [], x_orig);
end
