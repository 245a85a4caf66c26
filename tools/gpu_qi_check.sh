#!/bin/bash
# GPU round trip for the §8f rank-4 rows (opts.model='qi', the test.m solver),
# then the whole GPU suite and the default bench line (no CPU leg).
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_qi_model.py tests/test_ncvx.py tests/test_mex_gateway.py \
    -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/rank4_tests.log 2>&1
rc=$?; tail -30 gpurun_out/rank4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cat gpurun_out/bench4.json
