#!/bin/bash
# a config-5 K5 variant ab/$1.so: fp32 GPU tests on it, then an interleaved
# config-5 A/B against the in-tree default (ab/base.so)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1
TRITD_LIB=$PWD/ab/$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t5_$V.log 2>&1
rc=$?; echo "$V tests: $(tail -1 gpurun_out/t5_$V.log)"; [ $rc -eq 0 ] || exit $rc
AB_CFG=5 timeout -k 10 500 python3 -u tools/ab_lib.py ab/base.so,ab/$V.so 4 8 > gpurun_out/ab5_$V.log 2>&1 || exit $?
tail -2 gpurun_out/ab5_$V.log
