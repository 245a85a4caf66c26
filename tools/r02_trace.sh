#!/bin/bash
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02/trace
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 > $O/bench.log 2>&1
echo ok
