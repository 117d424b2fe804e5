function o = ccsc_call(slots, nout, varargin)
% Call ccsc_mex asking only for the outputs the wrapper's caller takes.
% slots(i) = the ccsc_mex output index of the wrapper's i-th output
% (ccsc_mex returns [d_res, iterations, z_res, DZ, obj_val]); outputs the caller
% does not take are never allocated or copied (z_res is ~97 GB at C2).
    k = max(slots(1:max(nout, 1)));
    o = cell(1, k);
    [o{:}] = ccsc_mex(varargin{:});
end
