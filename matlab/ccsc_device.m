function devs = ccsc_device()
% GPU indices for ccsc_mex: env CCSC_DEVICES (e.g. '0,1,2,3,4,5,6,7': one call
% runs the learner over all of them, blocks sharded across the GPUs), else
% CCSC_DEVICE (one index), default 0.
    s = getenv('CCSC_DEVICES');
    if ~isempty(s)
        devs = str2double(strsplit(s, ','));
        return;
    end
    s = getenv('CCSC_DEVICE');
    if isempty(s), devs = 0; else, devs = str2double(s); end
end
