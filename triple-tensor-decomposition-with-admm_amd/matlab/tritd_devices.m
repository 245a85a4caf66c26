function tritd_devices(idx)
%TRITD_DEVICES  GPUs the next triple_decomp_ADMM calls shard D over.
%   tritd_devices([0 1 2 3]) splits D along mode 1 over HIP devices 0..3
%   (0-based ordinals, as rocm-smi lists them); the library drives them all
%   from MATLAB's thread and sums the per-iteration partial products with
%   RCCL.  tritd_devices([]) returns to one GPU.
tritd_mex('devices', double(idx(:)'));
end
