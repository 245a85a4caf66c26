#!/bin/bash
# a K5 variant ab/$1.so: GPU parity subset on it, then an interleaved config-4
# A/B against the in-tree default (ab/base.so)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
V=$1
TRITD_LIB=$PWD/ab/$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$V.log 2>&1
rc=$?; echo "$V tests: $(tail -1 gpurun_out/t_$V.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/ab_lib.py ab/base.so,ab/$V.so 6 10 > gpurun_out/ab_$V.log 2>&1 || exit $?
tail -2 gpurun_out/ab_$V.log
