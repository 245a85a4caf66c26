#!/bin/bash
# Config-5 kernel trace: one iteration's sequence (tools/trace_iter.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_c5trace; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/line.json 2> $O/err.txt &&
python3 tools/trace_iter.py $(ls $O/stats/*/run_kernel_trace.csv 2>/dev/null || ls $O/stats/run_kernel_trace.csv) 3 "k5_f32s<" > $O/iter.txt
