#!/bin/bash
# Round 4: a GPU test subset on the in-tree build, then an interleaved K5 A/B of $AB_LIBS.
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_sub.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_sub.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_lib.py ${AB_LIBS} 6 10 > gpurun_out/ab2.log 2>&1 || exit $?
tail -3 gpurun_out/ab2.log
