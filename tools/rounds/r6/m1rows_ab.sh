#!/bin/bash
# Round 6: whole-row M1 (k_m1_rows, partial sets summed by apply A) — parity at config 4 / 256-row
# shards / config 3 with the sets on, the iteration A/B over the set count, and a kernel trace per count.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_m1rows; mkdir -p $O
TRITD_M1_Q=4 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_fullsize.py tests/test_gpu_configs.py -k "config4 or config3 or repeat" \
    tests/test_gpu_determinism.py > $O/parity_q4.txt 2>&1
timeout -k 10 400 python3 tools/ab_env.py TRITD_M1_Q -,2,4,8 3 20 > $O/ab.txt 2>&1
for q in 2 4 8; do
  TRITD_M1_Q=$q timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace$q -o run -- \
      python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 2 > $O/trace$q.log 2>&1
  python3 tools/trace_iter.py $O/trace$q/run_kernel_trace.csv 3 > $O/iter$q.txt
done
echo done
