#!/bin/bash
# which test of test_gpu_configs.py leaves the device-form product failing
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dbg
for t in ${TESTS}; do
  timeout -k 10 200 python -u -m pytest "tests/test_gpu_configs.py::$t" tests/test_gpu_devprod.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/dbg/b_$t.log 2>&1
  echo "$t: $(tail -1 gpurun_out/dbg/b_$t.log) $(grep -m1 'TritdError:\|RuntimeError:' gpurun_out/dbg/b_$t.log)"
done
