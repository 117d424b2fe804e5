function dev = ccsc_device()
% GPU index for ccsc_mex (env CCSC_DEVICE, default 0).
    s = getenv('CCSC_DEVICE');
    if isempty(s), dev = 0; else, dev = str2double(s); end
end
