function [ d_res, z_res, DZ, iterations ] = admm_learn_conv2D_large_dzParallel(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 2D/admm_learn_conv2D_large_dzParallel.m (same signature).
% z0 is size_z_crop = [X, Y, K, 100] and is replicated into every block (dZ:44-47).
    [d0, z0] = ccsc_init(b, kernel_size, init, true);
    [d_res, z_res, DZ, ~, iterations] = ccsc_mex(1, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
end
