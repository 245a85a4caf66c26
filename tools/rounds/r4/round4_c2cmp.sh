#!/bin/bash
# Round 4: config 2 bench, the in-tree build against $OLD (TRITD_LIB), twice each.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for l in "" ${OLD:-}; do
    v=$(TRITD_LIB=${l:-triple-tensor-decomposition-with-admm_amd/tritd/libtritd.so} timeout -k 10 120 python3 bench.py --config ${CFG:-2} --no-cpu --no-e2e --no-prims 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("%.1f it/s  %.4f ms" % (d["value"], d["ms_per_step"]))') || exit 1
    echo "config ${CFG:-2} ${l:-in-tree} rep $rep: $v" | tee -a gpurun_out/c2cmp.log
  done
done
