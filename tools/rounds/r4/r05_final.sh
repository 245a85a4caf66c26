#!/bin/bash
# Round-5 evidence in one GPU call: the whole GPU suite, smoke(), config-4
# profiles (PMC traffic, SQ MFMA pass, kernel stats, bench line with CPU
# baseline and end-to-end, primitives), config-5 profiles and bench line, ALS line.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash tools/refresh_profiles.sh r05 > gpurun_out/refresh_c4.log 2>&1 || exit $?
tail -3 gpurun_out/refresh_c4.log | cut -c1-400
bash tools/refresh_profiles_c5.sh r05 > gpurun_out/refresh_c5.log 2>&1 || exit $?
tail -1 gpurun_out/refresh_c5.log | cut -c1-400
timeout -k 10 300 python3 bench.py --algo als --steps 20 --warmup 3 > gpurun_out/bench_als.json 2> gpurun_out/bench_als.err || exit $?
cut -c1-300 gpurun_out/bench_als.json
timeout -k 10 60 tools/coexec > gpurun_out/coexec.log 2>&1 || exit $?
cat gpurun_out/coexec.log
