#!/bin/bash
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/diag_e2e.py > gpurun_out/diag_e2e.log 2>&1 || exit $?
head -3 gpurun_out/diag_e2e.log
TRITD_LIB=$PWD/ab/split.so timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f32_split.log 2>&1
rc=$?; echo "split: $(tail -1 gpurun_out/f32_split.log)"; [ $rc -eq 0 ] || exit $rc
AB_CFG=5 timeout -k 10 400 python3 -u tools/ab_lib.py ab/base.so,ab/split.so 4 8 > gpurun_out/ab_split.log 2>&1 || exit $?
tail -2 gpurun_out/ab_split.log
