function [ d_res, z_res, DZ, iterations ] = admm_learn_conv2D_large_dParallel(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 2D/admm_learn_conv2D_large_dParallel.m (same signature): runs the
% consensus-ADMM learner on an MI355X through ccsc_mex / libccsc.
% init (ignored by the reference) may carry .d (kernel_size) and .z (size_z);
% when empty, d0 and z0 are drawn here with randn in the reference's order.
    [d0, z0] = ccsc_init(b, kernel_size, init, false);
    [d_res, z_res, DZ, ~, iterations] = ccsc_mex(0, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
end
