function [ d_res, z_res, DZ, iterations ] = admm_learn_conv2D_large_dzParallel(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 2D/admm_learn_conv2D_large_dzParallel.m (same signature).
% z0 is size_z_crop = [X, Y, K, 100] and is replicated into every block (dZ:44-47).
    [d0, z0] = ccsc_init(b, kernel_size, init, true);
    o = ccsc_call([1 3 4 2], nargout, 1, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
    d_res = o{1};
    if nargout > 1, z_res = o{3}; end
    if nargout > 2, DZ = o{4}; end
    if nargout > 3, iterations = o{2}; end
end
