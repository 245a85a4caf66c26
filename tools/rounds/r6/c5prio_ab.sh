#!/bin/bash
# Round 6: config-5 K5 (k5_f32s) with wave priority 1 for the W-heavy h = 1 wave over the walk (pr1)
# or for the chain wave over its elementwise chain (pr2) — timing only (results identical: priority
# changes no arithmetic); interleaved A/B at config 5.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_c5prio; mkdir -p $O
AB_CFG=5 timeout -k 10 300 python3 -u tools/ab_same.py ab6/base.so,ab6/pr1.so,ab6/pr2.so 0 16 4 > $O/same_c5.txt 2>&1
AB_CFG=5 timeout -k 10 700 python3 -u tools/ab_lib.py ab6/base.so,ab6/pr1.so,ab6/pr2.so 3 6 > $O/ab_c5.txt 2>&1
echo done
