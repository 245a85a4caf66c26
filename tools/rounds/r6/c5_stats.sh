#!/bin/bash
# Round 6, last build: rocprofv3 --kernel-trace --stats of the config-5 bench leg (per-kernel averages).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_c5stats; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --steps 5 --warmup 1 > $O/bench.log 2>&1
echo done
