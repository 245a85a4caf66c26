function Xhat = triple_product(A, B, C)
%TRIPLE_PRODUCT  MI355X drop-in for fast_robust_triple_tensor/triple_product.m:
%   Xhat(i,j,t) = sum_{p,q} A(i,p,q) B(p,j,q) C(p,q,t).
Xhat = tritd_mex('triple_product', double(A), double(B), double(C));
end
