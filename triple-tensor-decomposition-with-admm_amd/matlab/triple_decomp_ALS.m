function [A, B, C, errHist] = triple_decomp_ALS(X, r, opts)
%TRIPLE_DECOMP_ALS  MI355X drop-in for fast_robust_triple_tensor/triple_decomp_ALS.m.
%   [A,B,C,errHist] = triple_decomp_ALS(X, r, opts) runs the ALS fit of the
%   triple (rank-r^2 CP) model on the GPU (libtritd.so via tritd_mex) with the
%   reference's inputs, outputs and stopping rule: only opts.maxIter and
%   opts.tol are read, errHist(k) is the relative fit error before the
%   update of iteration k, every mode uses the ridge 1e-9, and the line
%   'Iteration %d, relative error = %.4e' is printed every 5 iterations.
%
%   The initial factors are drawn here with randn in the reference's order
%   (A, then B, then C).  X is processed in double.  tritd_devices(idx)
%   shards X over several GPUs.
[n1, n2, n3] = size(X);
A0 = randn(n1, r, r);
B0 = randn(r, n2, r);
C0 = randn(r, r, n3);
[A, B, C, errHist] = tritd_mex('als', double(X), r, opts, A0, B0, C0);
end
