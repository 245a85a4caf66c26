#!/bin/bash
# Round 5 diagnosis of K5 (config 4): placement strategies, timing-only K5
# variants (ab/*.so, tools/build_k5_variants.sh), SQ counters, P=8 shard.
set -uo pipefail
O=gpurun_out/r5_diag; mkdir -p $O
timeout -k 10 200 tools/placement.bin 8 > $O/placement.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/ab_lib.py ab/base.so,ab/nobar.so,ab/lsplit.so,ab/noce.so,ab/now.so,ab/nol.so 3 10 \
    > $O/ab_diag.txt 2>&1 || exit $?
bash tools/rounds/r5/k5_sq.sh
