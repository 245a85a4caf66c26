#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dbg
for f in test_gpu_als test_gpu_determinism; do
  timeout -k 10 300 python -u tools/dbg_stale.py tests/$f.py > gpurun_out/dbg/stale_$f.log 2>&1
  grep -E "^==|torch " gpurun_out/dbg/stale_$f.log
done
