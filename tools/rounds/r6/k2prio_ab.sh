#!/bin/bash
# Round 6: K2 (k_m3_cp) with wave priority 1 over the first 4/8 or 6/8 of each walk (A/B; results identical).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_k2prio; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/p4.so,ab6/p6.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 600 python3 tools/ab_lib.py ab6/base.so,ab6/p4.so,ab6/p6.so 5 20 > $O/ab_c4.txt 2>&1
echo done
