#!/bin/bash
# Round 4: GPU suite on the in-tree build, then an interleaved K5 A/B of ab/*.so.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_lib.py ${AB_LIBS} 6 10 > gpurun_out/ab.log 2>&1 || exit $?
tail -4 gpurun_out/ab.log
timeout -k 10 300 python3 bench.py --no-e2e > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
cut -c1-700 gpurun_out/bench_c4.json
