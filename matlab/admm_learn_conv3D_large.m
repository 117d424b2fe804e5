function [ d_res, z_res, DZ, obj_val, iterations ] = admm_learn_conv3D_large(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 3D/admm_learn_conv3D_large.m (function admm_learn_convND_large, same
% signature): the 3D consensus learner on an MI355X through ccsc_mex / libccsc.
% b: [x, y, t, n]; kernel_size = [s, s, s, K].  init (ignored by the reference)
% may carry .d and .z; otherwise d0 = randn(kernel_size), z0 = randn(size_z) in
% the reference's draw order (L3:39, L3:48).
    r = floor(kernel_size(1) / 2);
    sb = size(b);
    if numel(sb) < 4, sb(4) = 1; end
    size_z = [sb(1:3) + 2 * r, kernel_size(end), sb(4)];
    if ~isempty(init) && isfield(init, 'd'), d0 = init.d; else, d0 = randn(kernel_size); end
    if ~isempty(init) && isfield(init, 'z'), z0 = init.z; else, z0 = randn(size_z); end
    o = ccsc_call([1 3 4 5 2], nargout, 2, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
    d_res = o{1};
    if nargout > 1, z_res = o{3}; end
    if nargout > 2, DZ = o{4}; end
    if nargout > 3, obj_val = o{5}; end
    if nargout > 4, iterations = o{2}; end
end
