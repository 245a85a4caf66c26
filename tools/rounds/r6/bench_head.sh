#!/bin/bash
# Round 6, last commit: the default bench line on another box (box-to-box spread of the final build).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_bench_head; mkdir -p $O
timeout -k 10 600 python3 -u bench.py > $O/bench_line.json 2> $O/bench.err
echo done
