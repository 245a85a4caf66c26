#!/bin/bash
# Round 6: K5 prologue order (slices, tile, then the KR gather; 32-bit index math) — bitwise
# equality with the previous build and an interleaved iteration A/B at config 4.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_k5pro; mkdir -p $O
timeout -k 10 300 python3 tools/ab_same.py ab6/new.so,ab6/pro.so 256 8 12 > $O/same.txt 2>&1
timeout -k 10 300 python3 tools/ab_same.py ab6/new.so,ab6/pro.so 96 5 12 > $O/same_small.txt 2>&1
timeout -k 10 500 python3 tools/ab_lib.py ab6/old.so,ab6/new.so,ab6/pro.so 5 20 > $O/ab_c4.txt 2>&1
echo done
