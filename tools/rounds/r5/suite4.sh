#!/bin/bash
# Round 5: config-5 trace of the current build, then the full GPU suite, smoke and the default bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_suite4; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/line.json 2> $O/err.txt || exit $?
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 3 "k5_f32s<" > $O/iter.txt
bash tools/rounds/r5/suite.sh r5_suite4/suite
