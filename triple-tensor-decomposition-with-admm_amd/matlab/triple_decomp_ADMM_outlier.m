function [A, B, C, O, errHist, E] = triple_decomp_ADMM_outlier(D, r, opts)
%TRIPLE_DECOMP_ADMM_OUTLIER  Name called by video_triple_comparison.m:54.
%   In the reference this name exists only as an internal function name and
%   does not resolve; here it is the same GPU solver as triple_decomp_ADMM.
[A, B, C, O, errHist, E] = triple_decomp_ADMM(D, r, opts);
end
