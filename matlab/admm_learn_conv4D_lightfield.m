function [ d_res, z_res, DZ, obj_val, iterations ] = admm_learn_conv4D_lightfield(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init)
% Drop-in for 4D/admm_learn_conv4D_lightfield.m (same signature) on an MI355X.
% b: [x, y, U, V, n] (single in the reference driver: widened to double here);
% kernel_size = [s, s, U, V, K].  z_res is returned complex like the reference
% (L4:164); its imaginary part is round-off there and zero here (Q8).
    b = double(b);
    r = floor(kernel_size(1) / 2);
    sb = size(b);
    if numel(sb) < 5, sb(5) = 1; end
    size_z = [sb(1:2) + 2 * r, 1, 1, kernel_size(end), sb(5)];
    if ~isempty(init) && isfield(init, 'd'), d0 = init.d; else, d0 = randn(kernel_size); end
    if ~isempty(init) && isfield(init, 'z'), z0 = real(init.z); else, z0 = randn(size_z); end
    o = ccsc_call([1 3 4 5 2], nargout, 3, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, ccsc_device());
    d_res = o{1};
    if nargout > 1, z_res = o{3}; end
    if nargout > 2, DZ = o{4}; end
    if nargout > 3, obj_val = o{5}; end
    if nargout > 4, iterations = o{2}; end
    if nargout > 1, z_res = complex(z_res); end
end
