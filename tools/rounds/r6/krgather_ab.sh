#!/bin/bash
# Round 6: unconditional Khatri-Rao gathers (no per-element branch + wait) — bitwise equality,
# iteration A/B (config 4 and 5), primitive A/B (triple product), and a K5 kernel-stats pass.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_krg; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/old.so,ab6/new.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 400 python3 tools/ab_lib.py ab6/old.so,ab6/new.so 4 20 > $O/ab_c4.txt 2>&1
timeout -k 10 300 python3 tools/ab_prims.py ab6/old.so ab6/new.so 4 > $O/ab_prims.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --no-cpu --no-e2e --no-prims --no-c5 > $O/stats.log 2>&1
AB_CFG=5 timeout -k 10 600 python3 tools/ab_lib.py ab6/old.so,ab6/new.so 2 5 > $O/ab_c5.txt 2>&1
echo done
