function [ d_res, z_res, Dz, obj_val ] = admm_learn(b, kernel_size, ...
                    lambda_residual, lambda_prior, max_it, tol, verbose, init, smooth_init)
% Drop-in for 2-3D/DictionaryLearning/admm_learn.m (same signature): the
% hyperspectral learner on an MI355X through ccsc_mex / libccsc.
% b, smooth_init: [x, y, W, n]; kernel_size = [s, s, W, K].  Without init, the
% filters are drawn as the reference does (L23:54-56: randn([s s K]), one per
% atom, replicated over W) and then z = randn(size_z) (L23:69); init may carry
% .d ([s s K]) and .z ([X Y K n]).
    r = floor(kernel_size(1) / 2);
    sb = size(b);
    if numel(sb) < 4, sb(4) = 1; end
    size_z = [sb(1:2) + 2 * r, kernel_size(4), sb(4)];
    if ~isempty(init) && isfield(init, 'd'), d0 = init.d; else, d0 = randn(kernel_size([1 2 4])); end
    if ~isempty(init) && isfield(init, 'z'), z0 = init.z; else, z0 = randn(size_z); end
    % one GPU: the d-solve couples every image per frequency (L23:289-295), so the
    % 2-3D learner does not shard; with CCSC_DEVICES listing several GPUs it takes the first
    devs = ccsc_device();
    o = ccsc_call([1 3 4 5], nargout, 4, b, kernel_size, lambda_residual, ...
        lambda_prior, max_it, tol, verbose, d0, z0, devs(1), smooth_init);
    d_res = o{1};
    if nargout > 1, z_res = o{3}; end
    if nargout > 2, Dz = o{4}; end
    if nargout > 3, obj_val = o{5}; end
end
