function [A, B, C, O, errHist, E] = triple_decomp_ADMM_outlier(D, r, varargin)
%TRIPLE_DECOMP_ADMM_OUTLIER  Name called by video_triple_comparison.m:54.
%   triple_decomp_ADMM_outlier(D, r, opts): in the reference this name exists
%   only as an internal function name (origin_triple_tensor/triple_decomp_ADMM.m:1)
%   and does not resolve; here it is the same GPU solver as triple_decomp_ADMM.
%
%   triple_decomp_ADMM_outlier(X, r, rho, lambda, gamma_A, epsilon, p, theta,
%   maxIter, tol) is the signature of fast_robust_triple_tensor/test.m:1, the
%   nonconvex variant (outlier ADMM with duals Lambda/Gamma, ALS factors with a
%   reweighted shrink on A); it runs on the GPU through tritd_mex('ncvx', ...).
%   The initial factors are drawn with randn in the order of test.m:24-26.
if numel(varargin) == 1
    [A, B, C, O, errHist, E] = triple_decomp_ADMM(D, r, varargin{1});
    return;
end
if numel(varargin) ~= 8
    error('triple_decomp_ADMM_outlier: use (D, r, opts) or (X, r, rho, lambda, gamma_A, epsilon, p, theta, maxIter, tol)');
end
[n1, n2, n3] = size(D);
A0 = randn(n1, r, r);
B0 = randn(r, n2, r);
C0 = randn(r, r, n3);
[A, B, C, O, errHist] = tritd_mex('ncvx', double(D), r, varargin{:}, A0, B0, C0);
E = [];
end
