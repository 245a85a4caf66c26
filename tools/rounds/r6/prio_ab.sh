#!/bin/bash
# Round 6: K5 with a static wave priority by dispatch round (A/B, timing only: results identical).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_prio; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/base.so,ab6/prio.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 500 python3 tools/ab_lib.py ab6/base.so,ab6/prio.so 6 20 > $O/ab_c4.txt 2>&1
echo done
