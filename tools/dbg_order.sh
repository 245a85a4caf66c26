#!/bin/bash
# which earlier GPU test file leaves the device-form product failing
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dbg
for f in test_gpu_als test_gpu_configs test_gpu_determinism; do
  timeout -k 10 300 python -u -m pytest tests/$f.py tests/test_gpu_devprod.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dbg/$f.log 2>&1
  echo "$f: $(tail -1 gpurun_out/dbg/$f.log)"; grep -m2 "TritdError:" gpurun_out/dbg/$f.log
done
