#!/bin/bash
# Round-5 first GPU pass: GPU suite (with the full-size oracle tests), smoke, bench line.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cut -c1-600 gpurun_out/bench4.json
