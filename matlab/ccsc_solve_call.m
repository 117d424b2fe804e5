function [z, res] = ccsc_solve_call(nout, variant, b, kernels, mask, lambda_residual, ...
                                    lambda_prior, max_it, tol, verbose, smooth_init, psf, x_orig)
% Call ccsc_solve_mex on the first GPU of ccsc_device(), asking for res only when the
% wrapper's caller takes it.
    devs = ccsc_device();
    args = {variant, b, kernels, mask, lambda_residual, lambda_prior, max_it, tol, ...
            verbose, smooth_init, psf, x_orig, devs(1)};
    if nout > 1
        [z, res] = ccsc_solve_mex(args{:});
    else
        z = ccsc_solve_mex(args{:});
        res = [];
    end
end
