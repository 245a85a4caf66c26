#!/bin/bash
# Round 4: config 2 bench at several K5 t-split counts (TRITD_K5_TSPLIT).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for ts in ${SPLITS:-9 18 36 72}; do
  for rep in 1 2; do
    v=$(TRITD_K5_TSPLIT=$ts timeout -k 10 120 python3 bench.py --config 2 --no-cpu --no-e2e --no-prims 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print("%.1f it/s  %.4f ms" % (d["value"], d["ms_per_step"]))') || exit 1
    echo "tsplit $ts rep $rep: $v" | tee -a gpurun_out/c2_tsplit.log
  done
done
