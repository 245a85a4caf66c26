#!/bin/bash
# GPU suite, default bench line, and a one-iteration kernel timeline at P=1
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/r03/bench4.json 2> gpurun_out/r03/bench4.err || exit $?
cat gpurun_out/r03/bench4.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03/p1trace -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03/p1trace.log 2>&1 || exit $?
python3 tools/trace_iter.py gpurun_out/r03/p1trace/run_kernel_trace.csv 60
