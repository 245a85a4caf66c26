#!/bin/bash
# Round 4: GPU suite + smoke + one default bench line (the round-end sequence).
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
cut -c1-700 gpurun_out/bench_c4.json
