#!/bin/bash
# Round 5: P = 8/4/2 shard timing (one-rank RCCL) under a kernel trace, then
# the default bench line (config 4 + the config-5 leg).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5_shard_bench}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- \
    python3 tools/shard_timing.py 8 > $O/shard.txt 2>&1 || exit $?
timeout -k 10 200 python3 tools/shard_timing.py 4 2 >> $O/shard.txt 2>&1 || exit $?
timeout -k 10 500 python3 -u bench.py > $O/bench.txt 2>&1
