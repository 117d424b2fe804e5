function [ z, res ] = admm_solve_conv2D_weighted_sampling(b, kernels, mask, ...
                    lambda_residual, lambda_prior, smooth_init, max_it, tol, x_orig, verbose)
% Drop-in for 2D/Inpainting/admm_solve_conv2D_weighted_sampling.m (same signature):
% the sparse-coding inpainting ADMM on the GPU of ccsc_device() through ccsc_solve_mex /
% libccsc.  res is only formed when the caller takes it.
    if nargin < 9, x_orig = []; end
    if nargin < 10, verbose = 'none'; end
    [z, res] = ccsc_solve_call(nargout, 0, b, kernels, mask, lambda_residual, lambda_prior, ...
        max_it, tol, verbose, smooth_init, [], x_orig);
end
