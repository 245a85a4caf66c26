#!/bin/bash
# Final-build check: the whole GPU suite and smoke(), then the config-5
# evidence (tools/refresh_profiles_c5.sh r05)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash tools/refresh_profiles_c5.sh r05 > gpurun_out/refresh_c5.log 2>&1 || exit $?
tail -1 gpurun_out/refresh_c5.log | cut -c1-400
