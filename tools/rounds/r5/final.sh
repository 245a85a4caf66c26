#!/bin/bash
# Round 5 final: config-5 trace of the final build, full GPU suite, smoke, default bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5_final}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_f32.py -x -q --timeout 300 --timeout-method thread > $O/f32_tests.txt 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- \
    python3 bench.py --config 5 --no-cpu --no-e2e --no-prims --no-c5 --steps 10 --warmup 3 > $O/c5_line.json 2> $O/c5_err.txt || exit $?
python3 tools/trace_iter.py $O/stats/run_kernel_trace.csv 3 "k5_f32s<" > $O/c5_iter.txt
bash tools/rounds/r5/suite.sh ${1:-r5_final}/suite
