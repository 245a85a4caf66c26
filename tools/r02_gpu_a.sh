#!/bin/bash
# round-2 GPU check: counter list, the GPU suite, the default bench line
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02
timeout -k 10 60 rocprofv3 -L > gpurun_out/r02/counters.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err || exit $?
cat gpurun_out/r02/bench.json
