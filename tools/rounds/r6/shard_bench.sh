# Round 6: P = 8 / 4 shard timing with the host enqueue time, one P = 8 kernel trace, and the
# default bench line (session-path / PCIe breakdown of the one-shot call).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_shard; mkdir -p $O
timeout -k 10 300 python3 tools/shard_timing.py 8 4 > $O/shard.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/shard_timing.py 8 > $O/trace.log 2>&1
timeout -k 10 500 python3 bench.py > $O/bench_line.json 2> $O/bench.err
echo done
