function Xhat = triple_product(A, B, C, model)
%TRIPLE_PRODUCT  MI355X drop-in for fast_robust_triple_tensor/triple_product.m:
%   Xhat(i,j,t) = sum_{p,q} A(i,p,q) B(p,j,q) C(p,q,t).
%   triple_product(A, B, C, 'qi') is Qi's 3-index product
%   sum_{p,q,s} A(i,q,s) B(p,j,s) C(p,q,t) (origin_triple_tensor/triple_product.m:8-19,
%   origin_triple_tensor/buildF.m:2-6), the model of opts.model = 'qi'.
if nargin < 4
    Xhat = tritd_mex('triple_product', double(A), double(B), double(C));
else
    Xhat = tritd_mex('triple_product', double(A), double(B), double(C), model);
end
end
