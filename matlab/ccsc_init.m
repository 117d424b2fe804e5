function [d0, z0] = ccsc_init(b, kernel_size, init, crop)
% d = randn(kernel_size) then z = randn(size_z) -- the reference's draw order
% (dP:38,45; dZ:38,44), so the same rng state reproduces its initialisation.
    psf_radius = floor(kernel_size(1) / 2);
    sb = size(b);
    k = kernel_size(end);
    ni = 100;
    if crop, nz = ni; else, nz = sb(end); end
    size_z = [sb(1:2) + 2 * psf_radius, k, nz];
    if ~isempty(init) && isfield(init, 'd'), d0 = init.d; else, d0 = randn(kernel_size); end
    if ~isempty(init) && isfield(init, 'z'), z0 = init.z; else, z0 = randn(size_z); end
end
