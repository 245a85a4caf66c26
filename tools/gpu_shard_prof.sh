#!/bin/bash
# Per-rank compute of the mode-1 sharded schedule (one-rank RCCL communicator,
# TRITD_SHOV=1) at P = 1, 2, 4, 8 row shards of config 4, then a rocprofv3
# kernel-trace of the P = 8 shard (what one rank of the 8-GPU bench runs).
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/shard
SHARD_MODES=rccl-sharded timeout -k 10 300 python3 tools/shard_timing.py 1 2 4 8 > gpurun_out/shard/timing.log 2>&1 || exit $?
cat gpurun_out/shard/timing.log | grep "P="
SHARD_MODES=rccl-sharded timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shard/p8 -o run -- \
    python3 tools/shard_timing.py 8 > gpurun_out/shard/p8.log 2>&1 || exit $?
echo done
