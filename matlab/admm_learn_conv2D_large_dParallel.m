function [ d_res, z_res, DZ, iterations ] = admm_learn_conv2D_large_dParallel(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 2D/admm_learn_conv2D_large_dParallel.m (same signature): runs the
% consensus-ADMM learner on the GPUs of ccsc_device() (one or several MI355X)
% through ccsc_mex / libccsc.  init (ignored by the reference) may carry .d
% (kernel_size) and .z (size_z); when empty, d0 and z0 are drawn here with randn
% in the reference's order.  Only the outputs the caller takes are computed.
    [d0, z0] = ccsc_init(b, kernel_size, init, false);
    o = ccsc_call([1 3 4 2], nargout, 0, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
    d_res = o{1};
    if nargout > 1, z_res = o{3}; end
    if nargout > 2, DZ = o{4}; end
    if nargout > 3, iterations = o{2}; end
end
