function [A, B, C, O, errHist, E] = triple_decomp_ADMM(D, r, opts)
%TRIPLE_DECOMP_ADMM  MI355X drop-in for fast_robust_triple_tensor/triple_decomp_ADMM.m.
%   [A,B,C,O,errHist] = triple_decomp_ADMM(D, r, opts) runs the robust
%   triple-decomposition ADMM on the GPU (libtritd.so via tritd_mex) with the
%   reference's inputs, outputs, opts fields and stopping rule.  A sixth
%   output E (the sparse copy) is available; the reference never returns it.
%
%   The initial factors are drawn here with randn in the reference's order
%   (A, then B, then C), so the global RNG stream and the starting point are
%   those of the reference run.  A single D keeps its class (the fp32 path:
%   O and E single, A, B, C and errHist double, as MATLAB's class rules give
%   the reference); any other class is processed in double.  Use
%   tritd_devices(idx) to shard D over several GPUs.
%
%   opts.model = 'qi' (optional; this build's own field) swaps the executed
%   rank-r^2 CP builders for the Qi-model design matrices of
%   origin_triple_tensor/buildF.m, buildG.m, buildH.m (3-index triple
%   product; reconstruct with triple_product(A, B, C, 'qi')).  Double D only.
[n1, n2, n3] = size(D);
A0 = randn(n1, r, r);
B0 = randn(r, n2, r);
C0 = randn(r, r, n3);
if ~isa(D, 'single')
    D = double(D);
end
[A, B, C, O, errHist, E] = tritd_mex('admm', D, r, opts, A0, B0, C0);
end
