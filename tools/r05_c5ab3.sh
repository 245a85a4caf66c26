#!/bin/bash
# config 5: deferred-W K5 pairs (ab/defer.so) and the register-row M2 — parity and A/B
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_base.log 2>&1
rc=$?; echo "base: $(tail -1 gpurun_out/f32_base.log)"; [ $rc -eq 0 ] || exit $rc
TRITD_LIB=$PWD/ab/defer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_defer.log 2>&1
rc=$?; echo "defer: $(tail -1 gpurun_out/f32_defer.log)"; [ $rc -eq 0 ] || exit $rc
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_lib.py ab/base.so,ab/defer.so 4 8 > gpurun_out/ab_defer.log 2>&1 || exit $?
tail -2 gpurun_out/ab_defer.log
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_env.py TRITD_M2V -,1 3 8 > gpurun_out/ab_m2w.log 2>&1 || exit $?
tail -2 gpurun_out/ab_m2w.log
