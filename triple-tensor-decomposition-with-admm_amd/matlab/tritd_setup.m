function tritd_setup()
%TRITD_SETUP  Put the MI355X drop-in ahead of the reference on the MATLAB path.
%   Call after the drivers' addpath(genpath(pwd)) (traffic_triple_comparison.m:3,
%   video_triple_comparison.m:2); addpath prepends, so this folder then
%   shadows fast_robust_triple_tensor/triple_decomp_ADMM.m and triple_product.m.
here = fileparts(mfilename('fullpath'));
addpath(here);
end
