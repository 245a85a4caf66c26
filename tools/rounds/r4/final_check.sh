#!/bin/bash
# Round-end evidence in one GPU call: GPU tests, smoke(), config-4 profiles
# (PMC traffic in the timed window, kernel stats, bench line with CPU
# baseline, primitive kernels), config-5 profiles and bench line, ALS line.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/smoke.log
bash tools/refresh_profiles.sh r01 > gpurun_out/refresh_c4.log 2>&1 || exit $?
tail -3 gpurun_out/refresh_c4.log | cut -c1-300
bash tools/refresh_profiles_c5.sh r01 > gpurun_out/refresh_c5.log 2>&1 || exit $?
tail -1 gpurun_out/refresh_c5.log | cut -c1-300
timeout -k 10 300 python3 bench.py --algo als --steps 20 --warmup 3 > gpurun_out/bench_als.json 2> gpurun_out/bench_als.err || exit $?
cut -c1-300 gpurun_out/bench_als.json
