#!/bin/bash
# Round 4: quick GPU check — the N-rank bench launch test and one bench line.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 380 --timeout-method thread -p no:cacheprovider > gpurun_out/launch_test.log 2>&1
rc=$?; tail -3 gpurun_out/launch_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --no-e2e > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
cut -c1-600 gpurun_out/bench_c4.json
