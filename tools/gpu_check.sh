#!/bin/bash
# One GPU round trip: the GPU test suite, then the config-4 and config-5 bench
# lines, the ALS line and the primitive rooflines (outputs under gpurun_out/).
# Run through gpurun on one MI355X.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench4.json 2> gpurun_out/bench4.err || exit $?
cat gpurun_out/bench4.json
timeout -k 10 400 python3 bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/bench5.json \
    2> gpurun_out/bench5.err || exit $?
cat gpurun_out/bench5.json
timeout -k 10 300 python3 bench.py --algo als --steps 20 --warmup 3 > gpurun_out/bench_als.json \
    2> gpurun_out/bench_als.err || exit $?
cat gpurun_out/bench_als.json
timeout -k 10 200 python3 tools/bench_prims.py > gpurun_out/prims.json 2> gpurun_out/prims.err || exit $?
cat gpurun_out/prims.json
