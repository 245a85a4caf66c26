#!/bin/bash
# Round 6, final build: P = 8 / 4 / 2 shard timing (one-rank RCCL communicator) and a P = 8 kernel trace.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_shard_final; mkdir -p $O
timeout -k 10 300 python3 tools/shard_timing.py 8 4 2 > $O/shard.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/shard_timing.py 8 > $O/trace.log 2>&1
echo done
