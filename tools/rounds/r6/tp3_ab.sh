#!/bin/bash
# Round 6: k_tp3 (C^T chunk staged once, no barriers in the walk) vs k_tp2 — parity with it on, A/B.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_tp3b; mkdir -p $O
TRITD_TP3=4 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_devprod.py -k "triple or product or devprod or destroyed" \
    > $O/parity_tp3.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 tools/ab_tp.py TRITD_TP3 -,2,4,16 2 > $O/ab.txt 2>&1
grep -E "k_tp" $O/prof/run_kernel_stats.csv > $O/tp_stats.csv || true
timeout -k 10 300 python3 tools/ab_tp.py TRITD_TP3 -,2,4,8,16 5 > $O/ab_noprof.txt 2>&1
echo done
