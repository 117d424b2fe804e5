function [ z, res ] = admm_solve_conv_weighted_sampling_lf(b, kmat, mask, ...
                    lambda_residual, lambda_prior, max_it, tol, ~, verbose, smooth_init)
% Drop-in for 4D/ViewSynthesis/admm_solve_conv_weighted_sampling_lf.m, whose text is the
% 2-3D demosaicing solver's: the U*V views are the channels (b = [x, y, U*V],
% kmat = [k, k, U*V, K], reconstruct_subsampling_lightfield.m:53-56).
    [z, res] = ccsc_solve_call(nargout, 2, b, kmat, mask, lambda_residual, lambda_prior, ...
        max_it, tol, verbose, smooth_init, [], []);
end
