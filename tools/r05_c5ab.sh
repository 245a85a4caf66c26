#!/bin/bash
# fp32 tests + config-5 A/B of the round-5 K2 / M1-M2 kernels + co-execution probe
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32.log 2>&1
rc=$?; tail -1 gpurun_out/f32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/coexec > gpurun_out/coexec.log 2>&1 || exit $?
cat gpurun_out/coexec.log
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_env.py TRITD_M3F_OLD -,1 3 8 > gpurun_out/ab_m3.log 2>&1 || exit $?
tail -2 gpurun_out/ab_m3.log
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_env.py TRITD_M1M2_OLD -,1 3 8 > gpurun_out/ab_m12.log 2>&1 || exit $?
tail -2 gpurun_out/ab_m12.log
